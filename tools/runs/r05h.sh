# Round 5: the stage1 tail variant vocoder_tailr.hip (M2_TAILR=1):
# parity (test_gpu_tailp.py), then kernel stats of the headline vocoder with
# and without it, alternated twice.
set -u
tag=${1:-r05h}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tailp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for v in r p; do
  if [ $v = r ]; then export M2_TAILR=1; else unset M2_TAILR; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${v}_$i -o run -- \
      python3 bench.py --workload vocoder --steps 100 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${v}_$i.json 2>/dev/null || exit 1
  rm -f gpurun_out/${tag}_${v}_$i/run_kernel_trace.csv
done
done
