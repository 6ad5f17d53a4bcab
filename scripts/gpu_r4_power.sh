#!/bin/bash
# round 4: board power and shader clock (rocm-smi, about one sample a second) around a long
# config-2 bench run; each sample is stamped with the seconds since the script started
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py --steps ${STEPS:-1500} --warmup 3 --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/pw.json 2> gpurun_out/pw.err &
bp=$!
: > gpurun_out/r4/power_load.txt
while kill -0 $bp 2>/dev/null; do
  t=$(python3 -c "import time; print(f'{time.time()-$t0:.1f}')")
  timeout -k 5 20 rocm-smi --showpower --showclocks 2>&1 | grep -E "Graphics Package Power|sclk clock level" | tr -s ' \t' ' ' | sed "s/^/t=$t /" >> gpurun_out/r4/power_load.txt
done
wait $bp; rc=$?
echo "bench rc=$rc ended at $(python3 -c "import time; print(f'{time.time()-$t0:.1f}')") s"
python -c "import json; d=json.load(open('gpurun_out/pw.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['sclk_ghz'])"
cat gpurun_out/r4/power_load.txt
