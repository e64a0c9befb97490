set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06z3
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_f32_forms.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > ${O}_tests.log 2>&1 || { tail -30 ${O}_tests.log; exit 1; }
tail -3 ${O}_tests.log
timeout -k 10 150 python3 -u tools/probe/voc_env_ab.py M2_F32_PAIR 0,1 1 s1 32 500 8 40 > ${O}_pair.txt 2>&1 || exit 1
cat ${O}_pair.txt
M2_F32_PAIR=1 timeout -k 10 150 python3 -u tools/probe/voc_env_ab.py M2_F32_MT 0,1,2,3 1 s1 32 500 6 40 > ${O}_mt.txt 2>&1 || exit 1
cat ${O}_mt.txt
