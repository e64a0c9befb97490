# Round 6: stage2 pipelined tail with the LDS-DMA loader (TAILP2_DMA=1, the
# new build) against the register loader (build_base): tailp2 / range /
# streaming / parity / device-T tests on the new build, then kernel stats at
# B=8 T=500 and B=16 T=2600 and the s2 vocoder lines, alternated twice.
set -u
tag=r06t
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=m2-tts_amd/src/m2amd/libm2tts_hip.so
OLD=m2-tts_amd/csrc/build_base/libm2tts_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_tailp2.py tests/test_gpu_range.py tests/test_gpu_sharding_streaming.py tests/test_gpu_parity.py tests/test_gpu_device_T.py tests/test_gpu_stress.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -n 30 gpurun_out/${tag}_tests.log; exit 1; }
tail -n 1 gpurun_out/${tag}_tests.log
for i in 1 2; do
for v in new old; do
  L=$NEW; [ $v = old ] && L=$OLD
  for shp in 8x500 16x2600; do
    d=gpurun_out/${tag}_${v}_${shp}_$i
    M2TTS_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
        python3 bench.py --workload s2_vocoder --s2-shape $shp --steps 60 --warmup 60 --no-cpu-baseline --no-extras > $d.json 2>/dev/null || exit 1
    rm -f $d/run_kernel_trace.csv
    python3 - "$d" "$v $shp $i" <<'PY'
import csv, sys, json
d, tag = sys.argv[1], sys.argv[2]
rows = {r["Name"].split("(")[0].split("::")[-1][:24]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(d + "/run_kernel_stats.csv")) if "m2::" in r["Name"]}
b = json.loads(open(d + ".json").read().strip().splitlines()[-1])
print(tag, b["ms_per_step"], {k: round(v, 2) for k, v in rows.items()})
PY
  done
done
done
