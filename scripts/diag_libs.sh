#!/bin/bash
# GPU box job: the per-wave cycle split (diag_stamps.py) of each turbo_decoder_cuda_amd/libdiag_*.so
# (stamps builds of kernel variants, e.g. -DTD_DIAG=4 (TD_DIAG bits: td_kernels.hip "diagnostic builds")).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in turbo_decoder_cuda_amd/libdiag_*.so; do
  echo "== $lib"
  TD_STAMPS_LIB=$PWD/$lib timeout -k 10 300 python scripts/diag_stamps.py 4096 ${DIAG_PREC:-f64} ${DIAG_ALGO:-logmap} > gpurun_out/diag_v.log 2>&1 || { echo "$lib failed"; tail -20 gpurun_out/diag_v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/diag_v.log | head -${DIAG_LINES:-6}
done
