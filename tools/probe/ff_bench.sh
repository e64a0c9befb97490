set -u
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload pipeline --no-extras --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/ff_pipe_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --workload s2_b64 --no-extras --no-cpu-baseline --steps 100 --warmup 20 > gpurun_out/ff_s2b64_$i.json 2>/dev/null || exit 1
done
