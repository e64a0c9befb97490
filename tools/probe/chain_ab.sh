set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for c in 1 0; do
    M2_TF_CHAIN=$c timeout -k 10 120 python bench.py --workload pipeline --no-extras --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/ab_chain${c}_$i.json 2>/dev/null || exit 1
  done
done
