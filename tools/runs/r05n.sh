# Round 5: stage2 mid B-fragment prefetch at four waves per SIMD (a smaller
# weight prefetch depth makes room): vA = CfgS2 BP 1 / PDM 3, Alt BP 2;
# vB = both BP 2 / PDM 3; vC = PDM 3 only (control); base = in-tree.
set -u
tag=r05n
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in vA vB; do
  M2TTS_HIP_LIB=tools/probe/libm2tts_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head_comp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_${v}_tests.log 2>&1 || { tail -n 20 gpurun_out/${tag}_${v}_tests.log; exit 1; }
  tail -n 1 gpurun_out/${tag}_${v}_tests.log
done
for i in 1 2; do
for v in base vA vB vC; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v != base ] && L=tools/probe/libm2tts_$v.so
  for sh in 8x500 16x2600; do
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_${sh}_${v}_$i -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 30 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/${tag}_${sh}_${v}_$i.json 2>/dev/null || exit 1
    rm -f gpurun_out/${tag}_${sh}_${v}_$i/run_kernel_trace.csv
  done
done
done
