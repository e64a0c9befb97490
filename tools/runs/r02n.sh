# Round-2 final records after the stage2 composed head: the -m gpu suite,
# bench (driver form and defaults), stage2 vocoder kernel stats + PMC at
# B=8 T=500 and B=16 T=2600.
set -u
bash tools/gpu_check.sh r02n &&
tools/profile_gpu.sh r02n_s2v_b8 --workload s2_vocoder --s2-shape 8x500 &&
tools/profile_gpu.sh r02n_s2v_b16 --workload s2_vocoder --s2-shape 16x2600
