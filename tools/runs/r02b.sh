set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02b_bench_n2_gloo.json 2> gpurun_out/r02b_bench_n2_gloo.err &&
tools/profile_gpu.sh r02_s2v_b8 --workload s2_vocoder --s2-shape 8x500 &&
tools/profile_gpu.sh r02_s2v_b16 --workload s2_vocoder --s2-shape 16x2600 &&
tools/profile_gpu.sh r02_pipeline --workload pipeline
