#!/bin/bash
# GPU box job: the placement search over 8 fresh decoders in one process, then three bench lines
# (each a fresh process and a fresh search).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/spread_probe.py ${NINST:-8} 2 4 > gpurun_out/spread.log 2>&1 || { echo "spread failed rc=$?"; tail -20 gpurun_out/spread.log; exit 1; }
grep instance gpurun_out/spread.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-variants > gpurun_out/sp.json 2> gpurun_out/sp.err || { echo "bench failed"; tail -20 gpurun_out/sp.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sp.json')); print('run $r', d['value'], d['roofline']['kernel_ms_avg'], d['workspace_placement']['probe_ms'], d['workspace_placement']['kept'])"
done
