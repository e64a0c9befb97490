# Re-entry check of the restored tree: the -m gpu suite, bench as the driver
# runs it and with its defaults, rocprofv3 stats + PMC of the headline vocoder
# and the stage2 B=8 vocoder (pipelined stage2 tail).
set -u
bash tools/gpu_check.sh r02l &&
tools/profile_gpu.sh r02l_vocoder &&
tools/profile_gpu.sh r02l_s2v_b8 --workload s2_vocoder --s2-shape 8x500
