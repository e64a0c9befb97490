# Round 5: the stage2 head (CfgS2, grids < 1024 workgroups) with both B
# planes two k-blocks ahead (BP 3, tools/probe/libm2tts_vE.so) against BP 1
# (in-tree): parity, then kernel stats at 8x500 and 16x500, alternated.
set -u
tag=r05s
export TMPDIR=/tmp
mkdir -p gpurun_out
M2TTS_HIP_LIB=tools/probe/libm2tts_vE.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in base vE; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v != base ] && L=tools/probe/libm2tts_$v.so
  for sh in 8x500 16x500; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 50 --warmup 20 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_${sh}_${v}_$i/run_kernel_trace.csv
  done
done
done
