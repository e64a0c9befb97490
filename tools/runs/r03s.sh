# Round 3 A/B: transformer tile rows (M2_TFL_RB) on the stage1 pipeline (B=32) and stage2 B=64 / B=8, alternated.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r03s_ab.txt
for rep in 1 2 3; do
  for rb in 0 2 4; do
    if [ $rb = 0 ]; then unset M2_TFL_RB; else export M2_TFL_RB=$rb; fi
    p=$(timeout -k 10 120 python -u bench.py --workload pipeline --no-cpu-baseline --no-extras --steps 200 --warmup 20 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    s=$(timeout -k 10 120 python -u bench.py --workload s2_b64 --no-cpu-baseline --no-extras --steps 100 --warmup 10 2>/dev/null | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "rep $rep rb $rb pipeline $p s2_b64 $s" | tee -a gpurun_out/r03s_ab.txt
  done
done
unset M2_TFL_RB
