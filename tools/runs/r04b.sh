# NNLS convergence test on the GPU (audio tests), range-policy tests with the
# redo grid, and the redo grid A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
# the lean query-split softmax with buffer-descriptor staging and the f16
# overflow test (transformer_layer.hip): every tile form and head_dim first
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py tests/test_gpu_attention.py tests/test_gpu_parity.py tests/test_gpu_head_comp.py tests/test_gpu_sharding_streaming.py tests/test_gpu_device_T.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04b_tf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_audio_features.py tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04b_tests.log; [ $rc -eq 0 ] || exit $rc
M2_REDO_GRID=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_range.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tests_g8.log 2>&1
rc=$?; tail -2 gpurun_out/r04b_tests_g8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe/redo_grid_ab.py > gpurun_out/r04b_redo_ab.txt 2>&1 || exit 1
cat gpurun_out/r04b_redo_ab.txt
# N=2 rehearsal on one GPU (two gloo ranks sharing it): the sharded lines' parity check
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04b_bench_n2_gloo.json 2> gpurun_out/r04b_bench_n2_gloo.err || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04b_bench_n2_gloo.json").read().strip().splitlines()[-1])
print(d["n_gpus"], d["value"], {k: (d[k]["ms_per_step"], d[k].get("parity")) for k in d if isinstance(d[k], dict) and "parity" in d[k]})
PY
# library A/B: the long-form step's decoder layers, new (lean loop without
# per-step address VALU and cmax) against the previous commit's build
OLD=m2-tts_amd/csrc/build_old/libm2tts_hip_old.so
for i in 1 2; do for v in new old; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04b_lf_${v}$i -o run -- python3 tools/probe/s2_small_trace.py 128 one 520 > gpurun_out/r04b_lf_${v}$i.log 2>&1 || exit 1
  python3 tools/probe/s2_small_trace.py --summarize gpurun_out/r04b_lf_${v}$i/run_kernel_trace.csv 3 > gpurun_out/r04b_lf_${v}$i.txt || exit 1
  rm -f gpurun_out/r04b_lf_${v}$i/run_kernel_trace.csv
  echo "== $v $i"; grep -E "span|layer_kernel" gpurun_out/r04b_lf_${v}$i.txt
done; done
for i in 1 2; do for v in new old; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = old ] && L=$OLD
  M2TTS_HIP_LIB=$L timeout -k 10 200 python3 bench.py --workload pipeline --steps 200 --warmup 50 --no-cpu-baseline --no-extras > gpurun_out/r04b_pipe_${v}$i.json 2>/dev/null || exit 1
  echo "pipeline $v $i $(python3 -c "import json;print(json.loads(open('gpurun_out/r04b_pipe_${v}$i.json').read().strip().splitlines()[-1])['ms_per_step'])")"
done; done
# stage2 x3 head / mid: weight k-blocks in flight per item (X3S2_PDM 4 = the
# previous build, 8 = in-tree default, 12)
for i in 1; do for v in 4 8 12; do
  L=m2-tts_amd/csrc/build_ab/libm2tts_hip_pdm$v.so; [ $v = 8 ] && L=m2-tts_amd/src/m2amd/libm2tts_hip.so
  for sh in 8x500 16x2600; do
    M2TTS_HIP_LIB=$L timeout -k 10 200 python3 bench.py --workload s2_vocoder --s2-shape $sh --steps 60 --warmup 10 --no-cpu-baseline --no-extras > gpurun_out/r04b_pdm${v}_${sh}_$i.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r04b_pdm${v}_${sh}_$i.json').read().strip().splitlines()[-1]);print('pdm$v $sh $i', d['ms_per_step'], [(k['kernel'][:28], k['avg_ms']) for k in d['vocoder_kernels']])"
  done
done; done
# split-f16 duration convs against the exact-f32 ones, in-process
: > gpurun_out/r04b_dursplit_ab.txt
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_SPLIT 0,1 s2 8 100 8 40 >> gpurun_out/r04b_dursplit_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe/env_ab.py M2_DUR_SPLIT 0,1 s1 32 100 8 40 >> gpurun_out/r04b_dursplit_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r04b_dursplit_ab.txt | cut -c1-100
