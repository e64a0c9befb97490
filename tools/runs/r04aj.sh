# Round 4: 64-row first-launch tiles (4-wave workgroups) at 4 rounds of
# 16-row tiles: the stage1 pipeline (B=32 T=500) and stage2 B=32 S=100
# (configs[3]'s share at N=2) with M2_TFL_FIRST_RB=4 against the default.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do for v in auto rb4; do
  E=0; [ $v = rb4 ] && E=4
  M2_TFL_FIRST_RB=$E timeout -k 10 300 python3 bench.py --workload pipeline --steps 100 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/r04aj_pipe_${v}$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r04aj_pipe_${v}$i.json').read().strip().splitlines()[-1]);print('pipeline', '$v', d['ms_per_step'])"
done; done
for i in 1 2; do for v in auto rb4; do
  E=0; [ $v = rb4 ] && E=4
  d=gpurun_out/r04aj_b32_${v}$i
  M2_TFL_FIRST_RB=$E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 32 one 100 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
  echo "== b32 $v $i"; grep -E "span|first_kernel" $d.txt
done; done
