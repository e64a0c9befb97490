# Round 5: r05d (stress parity, stage1 pipeline trace) then r05c (driver-form
# bench, headline kernel trace + PMC passes) in one box.
set -u
bash tools/runs/r05d.sh; rc=$?
echo "r05d rc=$rc"
bash tools/runs/r05c.sh || exit 1
exit $rc
