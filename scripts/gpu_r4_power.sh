#!/bin/bash
# round 4: board power and shader clock (rocm-smi) sampled while the config-2 bench runs long
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 60 rocm-smi --showpower --showclocks > gpurun_out/r4/power_idle.txt 2>&1
timeout -k 10 400 python bench.py --steps ${STEPS:-300} --warmup 3 --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/pw.json 2> gpurun_out/pw.err &
bp=$!
sleep 25
for i in $(seq 1 ${SAMPLES:-8}); do
  timeout -k 5 20 rocm-smi --showpower --showclocks 2>&1 | grep -E "Power|sclk|fclk|mclk|socclk" | sed "s/^/s$i /" >> gpurun_out/r4/power_load.txt
  sleep 1
done
wait $bp; rc=$?
echo "bench rc=$rc"; cut -c1-200 gpurun_out/pw.json
python -c "import json; d=json.load(open('gpurun_out/pw.json')); r=d['roofline']; print(d['value'], r['kernel_ms_avg'], r['sclk_ghz'])"
cat gpurun_out/r4/power_idle.txt | grep -E "Power|sclk"; cat gpurun_out/r4/power_load.txt
