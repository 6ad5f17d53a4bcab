#!/bin/bash
# round 4: stamps of the production kernel at a small batch (one group: the drop-in's latency) and in
# Max-Log-MAP (config 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
for args in "8 f64 logmap" "4096 f64 maxlog" "4096 f32 logmap"; do
  echo "== $args"
  timeout -k 10 300 python scripts/diag_stamps.py $args 2>&1 | grep -v amdgpu.ids | head -14 || exit 1
done 2>&1 | tee gpurun_out/r4/stamps_small_maxlog.txt
