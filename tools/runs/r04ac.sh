# Round 4: the full GPU suite and smoke on the exact final library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04ac_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ac_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r04ac_smoke.log
