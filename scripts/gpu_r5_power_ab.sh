#!/bin/bash
# round 5: the headline with and without the 10 ms amdsmi power sampler, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/pw
B="--steps 20 --warmup 3 --cpu-sample 0 --no-variants --dropin-frames 0"
for r in 1 2 3; do
  for v in "on:" "off:--no-power"; do
    timeout -k 10 300 python bench.py $B ${v#*:} > gpurun_out/pw/v.json 2> gpurun_out/pw/v.err || { echo "rc=$?"; tail -20 gpurun_out/pw/v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/pw/v.json')); print('round $r sampler ${v%%:*}', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], (d.get('power') or {}).get('socket_w_mean'))"
  done
done
