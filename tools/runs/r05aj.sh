# Round 5: r05ah (key-split layer tiles) with write-through record stores instead of agent-scope fences, field-major records of the active waves only; A/B only.
# tile, each on half of the keys; M2_TFL_SPLIT=0 turns them off): layer tile
# tests incl. the forced split forms, parity, then in-process A/B at the
# configs[3] B=8 share and a few small-grid shapes, and B=8 kernel traces.
set -u
tag=r05aj
export TMPDIR=/tmp
mkdir -p gpurun_out
true
for bs in "8 100" "4 100" "16 100" "2 520"; do
  timeout -k 10 200 python -u tools/probe/env_ab.py M2_TFL_SPLIT 0,-1 s2 $bs 8 30 >> gpurun_out/${tag}_ab.txt 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/probe/env_ab.py M2_TFL_SPLIT 0,-1 s1 8 100 8 30 >> gpurun_out/${tag}_ab.txt 2>&1 || exit 1
cat gpurun_out/${tag}_ab.txt
for i in 1 2; do
for v in 0 -1; do
  d=gpurun_out/${tag}_tr8_split${v}_$i
  M2_TFL_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/probe/s2_small_trace.py 8 dev 100 > $d.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize $d/run_kernel_trace.csv 20 > $d.txt || exit 1
  rm -f $d/run_kernel_trace.csv
done
done
