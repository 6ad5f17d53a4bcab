#!/bin/bash
# round 4: the GPU suite on the in-tree build, then N fresh bench processes (each with its own
# placement search) on one box: the run-to-run spread of the headline on a fixed kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r4/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4/pytest_gpu.log
for r in $(seq 1 ${RUNS:-4}); do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/sp.json 2> gpurun_out/sp.err || { echo "bench rc=$?"; tail -20 gpurun_out/sp.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sp.json')); r=d['roofline']; w=d['workspace_placement']; print('run $r', d['value'], r['kernel_ms_avg'], r['sclk_ghz'], w['kept_probe_ms'], w['launch_over_probe'])" | tee -a gpurun_out/r4/spread.txt
done
