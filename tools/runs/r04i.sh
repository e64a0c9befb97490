# Round 4: a step's staging issued after its K fragment reads (LDS serves its
# queue in order) against the previous order (TFL_STAGE_FIRST=1 build):
# tile tests, decoder alone at the long-form and mid grids, alternated.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tf_layer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_tf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04i_tf_tests.log; [ $rc -eq 0 ] || exit $rc
SF=m2-tts_amd/csrc/build_ab/libm2tts_hip_sf.so
for shp in "128 2600 6" "16 2600 20" "64 500 40"; do
for i in 1 2; do for v in new sf; do
  L=m2-tts_amd/src/m2amd/libm2tts_hip.so; [ $v = sf ] && L=$SF
  tag=$(echo $shp | cut -d' ' -f1-2 | tr ' ' x)_${v}$i
  M2TTS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i_$tag -o run -- python3 tools/probe/dec_time.py $shp > gpurun_out/r04i_$tag.log 2>&1 || exit 1
  rm -f gpurun_out/r04i_$tag/run_kernel_trace.csv
  python3 - gpurun_out/r04i_$tag/run_kernel_stats.csv "$tag $(grep decoder gpurun_out/r04i_$tag.log)" <<'PY'
import csv, sys
print(sys.argv[2], " | ".join(f'{r["Name"].split("(")[0].replace("void m2::tfl::", "")} {float(r["AverageNs"]) / 1e3:.1f}us' for r in csv.DictReader(open(sys.argv[1])) if "layer_kernel" in r["Name"]))
PY
done; done; done
