# Round 6: phase stamps of form 12 after the out-projection prefetch - the
# per-wave attention-loop times by wave index (which waves finish first).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 300 python -u tools/probe/tfl_stamps.py s2 128x2600 > gpurun_out/r06ao_stamps.txt 2>&1 || { tail -20 gpurun_out/r06ao_stamps.txt; exit 1; }
cat gpurun_out/r06ao_stamps.txt
d=gpurun_out/r06ao_tr_lf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > $d.log 2>&1 || { tail -n 20 $d.log; exit 1; }
python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 3 > gpurun_out/r06ao_tr_lf.txt || exit 1
rm -f $d/run_kernel_trace.csv
cat gpurun_out/r06ao_tr_lf.txt
