#!/bin/bash
# GPU box job: the workspace-mode spread (scripts/spread_probe.py, plain allocations:
# TD_PLACEMENT_TRIALS=1) of each build variant turbo_decoder_cuda_amd/libvar_*.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in turbo_decoder_cuda_amd/libvar_*.so; do
  echo "== $lib"
  TD_PLACEMENT_TRIALS=${TRIALS:-1} TD_LIB_PATH=$PWD/$lib timeout -k 10 300 python scripts/spread_probe.py ${NINST:-6} 2 4 > gpurun_out/spread.log 2>&1 || { echo "$lib failed rc=$?"; tail -20 gpurun_out/spread.log; exit 1; }
  grep instance gpurun_out/spread.log
done
