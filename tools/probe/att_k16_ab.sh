# head_dim-48 attention: the last QK^T k-step on the K = 16 MFMA (new) vs the
# zero-padded K = 32 step (old library), and QT = 2 forced (new): the
# attention tests (default and forced QT = 2) first, then att_bench arms
# alternated on one box.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k16_tests.log 2>&1 || { tail -n 30 gpurun_out/k16_tests.log; exit 1; }
tail -n 1 gpurun_out/k16_tests.log
M2_ATT_QT=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k16_tests_qt2.log 2>&1 || { tail -n 30 gpurun_out/k16_tests_qt2.log; exit 1; }
tail -n 1 gpurun_out/k16_tests_qt2.log
S=32x500x64,64x500x96,8x500x96,16x2600x96,128x2600x96
for i in 1 2; do
  M2TTS_HIP_LIB=tools/probe/libm2_att_old.so timeout -k 10 200 python tools/probe/att_bench.py --shapes $S > gpurun_out/k16_old_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python tools/probe/att_bench.py --shapes $S > gpurun_out/k16_new_$i.json 2>/dev/null || exit 1
  M2_ATT_QT=2 timeout -k 10 200 python tools/probe/att_bench.py --shapes $S > gpurun_out/k16_qt2_$i.json 2>/dev/null || exit 1
done
