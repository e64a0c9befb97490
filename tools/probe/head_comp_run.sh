set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_head_comp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hc_tests.log 2>&1 || { tail -n 30 gpurun_out/hc_tests.log; exit 1; }
tail -n 1 gpurun_out/hc_tests.log
bash tools/probe/head_comp_ab2.sh
