# Round 3 checkpoint: CPU quota of the box, the -m gpu suite + driver-form bench,
# kernel stats + PMC passes of the headline vocoder and the B=8 stage2 step.
set -u
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max 2>&1; nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'; } > gpurun_out/r03j_cpu.txt
cat gpurun_out/r03j_cpu.txt
M2TTS_HIP_LIB=m2-tts_amd/csrc/build_tst/libm2tts_hip_tst.so timeout -k 10 120 python -u tools/probe/tfl_stamps.py s2 8x500 64x500 > gpurun_out/r03j_stamps.txt 2>&1 &&
bash tools/gpu_check.sh r03j &&
tools/profile_gpu.sh r03j_vocoder &&
python3 tools/pmc_summary.py gpurun_out/prof_r03j_vocoder > gpurun_out/r03j_vocoder_pmc.txt
