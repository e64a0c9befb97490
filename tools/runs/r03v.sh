# Round 3: PMC + kernel-stats passes of the headline vocoder and the stage1 pipeline; CPU baseline twice.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile_gpu.sh r03voc || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r03voc --json gpurun_out/prof_r03voc/pmc.json > gpurun_out/prof_r03voc/pmc.txt || exit 1
cat gpurun_out/prof_r03voc/pmc.txt
bash tools/profile_gpu.sh r03pipe --workload pipeline || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_r03pipe --json gpurun_out/prof_r03pipe/pmc.json > gpurun_out/prof_r03pipe/pmc.txt || exit 1
cat gpurun_out/prof_r03pipe/pmc.txt | head -40
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-extras > gpurun_out/r03v_cpu$i.json 2> gpurun_out/r03v_cpu$i.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r03v_cpu$i.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print(c['value'], c['median'], c['min'], c['spread'], c['inference_as_written']['value'])"
done
