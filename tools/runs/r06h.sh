# Round 6: the mailbox fix (first T_max read from a side stream), the pipeline
# tests, the submit host-cost profile, then the stress-flip probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_T.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1 || { tail -n 30 gpurun_out/r06h_tests.log; exit 1; }
tail -n 1 gpurun_out/r06h_tests.log
timeout -k 10 200 python3 -u tools/probe/pipe_host.py --profile > gpurun_out/r06h_submit_prof.txt 2>&1 || { tail -n 30 gpurun_out/r06h_submit_prof.txt; exit 1; }
head -45 gpurun_out/r06h_submit_prof.txt
bash tools/runs/r06f.sh
