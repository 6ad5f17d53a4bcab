#!/bin/bash
# Does the workspace placement search still pay (round 6)?  Fresh bench processes, interleaved:
# TD_PLACEMENT_TRIALS=1 (a plain allocation) against the default search, config 2, ROUNDS rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-5}); do
  for t in 1 default; do
    if [ $t = default ]; then unset TD_PLACEMENT_TRIALS; else export TD_PLACEMENT_TRIALS=$t; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 2 --cpu-sample 0 --no-variants --dropin-frames 0 \
        > gpurun_out/pab.json 2> gpurun_out/pab.err || { echo "bench $r $t failed"; tail -20 gpurun_out/pab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/pab.json')); p=d['workspace_placement']; print('round $r trials $t', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['sclk_ghz'], d['power']['socket_w_mean'] if d.get('power') else None, p.get('kept_probe_ms'), p.get('launch_over_probe'), len(p.get('probe_ms') or []))"
  done
done
