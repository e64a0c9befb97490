# Round-2 closing records (re-entry session): the -m gpu suite, bench as the
# driver runs it and with its defaults, rocprofv3 kernel stats + PMC passes of
# the headline vocoder, the stage2 B=8 vocoder and the pipeline.
set -u
bash tools/gpu_check.sh r02m &&
tools/profile_gpu.sh r02m_vocoder &&
tools/profile_gpu.sh r02m_s2v_b8 --workload s2_vocoder --s2-shape 8x500 &&
tools/profile_gpu.sh r02m_pipeline --workload pipeline
