#!/bin/bash
# GPU box job: stamp diagnostics of TD_STAMPS variant libraries (DIAG_LIBS, names of libvar_*.so), then
# the interleaved A/B of the other libvar_*.so (scripts/variant_ab.sh, ROUNDS rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $DIAG_LIBS; do
  echo "== stamps $v"
  TD_STAMPS_LIB=$PWD/turbo_decoder_cuda_amd/libvar_$v.so timeout -k 10 200 python scripts/diag_stamps.py 4096 ${DIAG_PREC:-f64} ${DIAG_ALGO:-logmap} > gpurun_out/diag_$v.log 2>&1 || { echo "diag $v failed"; tail -20 gpurun_out/diag_$v.log; exit 1; }
  head -7 gpurun_out/diag_$v.log
  mv turbo_decoder_cuda_amd/libvar_$v.so gpurun_out/
done
ROUNDS=${ROUNDS:-2} bash scripts/variant_ab.sh
