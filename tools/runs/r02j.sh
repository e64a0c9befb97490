# Round-2 closing records: the -m gpu suite + bench as the driver runs it and
# with its defaults (tools/gpu_check.sh), then rocprofv3 kernel stats + PMC
# passes of the headline vocoder and the pipeline.
set -u
bash tools/gpu_check.sh r02j &&
tools/profile_gpu.sh r02j_vocoder &&
tools/profile_gpu.sh r02j_pipeline --workload pipeline
