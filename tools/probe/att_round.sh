set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/probe/att_check.py > gpurun_out/att_check_default.log 2>&1 &&
timeout -k 10 120 python tools/probe/att_bench.py --iters 100 > gpurun_out/att_new.json &&
M2_ATT_QT=1 timeout -k 10 120 python tools/probe/att_bench.py --iters 100 --shapes 32x500x64 > gpurun_out/att_qt1.json &&
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_ast/libm2tts_hip_ast.so timeout -k 10 120 python tools/probe/att_stamps.py 32x500x64 > gpurun_out/att_stamps.log 2>&1
