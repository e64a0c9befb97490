set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_attention.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/att_tests.log 2>&1 &&
timeout -k 10 120 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_stag.json &&
M2_ATT_NWV=8 timeout -k 10 120 python tools/probe/att_bench.py --iters 100 --shapes 32x500x64 > gpurun_out/att_stag_nwv8.json &&
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_vns/libm2tts_hip_vns.so timeout -k 10 120 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_nostag.json &&
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_vns/libm2tts_hip_vns.so M2_ATT_NWV=8 timeout -k 10 120 python tools/probe/att_bench.py --iters 100 --shapes 32x500x64 > gpurun_out/att_nostag_nwv8.json
