# Round 4: after pruning the masked instantiations of forms 5-10 (host maps
# them to 3): every tile test, the parity and device-T files.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_parity.py tests/test_gpu_device_T.py tests/test_gpu_sharding_streaming.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04u_tests.log; [ $rc -eq 0 ] || exit $rc
