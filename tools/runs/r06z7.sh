# The exact-f32 head's composed input conv o ConvT1 (M2_F32_COMP): form tests,
# then an in-process A/B on the strict line's shape.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06z7
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_f32_forms.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -3 ${O}_tests.log
timeout -k 10 150 python3 -u tools/probe/voc_env_ab.py M2_F32_COMP 0,1 1 s1 32 500 8 40 > ${O}_comp.txt 2>&1 || exit 1
cat ${O}_comp.txt
