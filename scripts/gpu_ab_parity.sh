#!/bin/bash
# GPU box job: parity of the variant library PARITY_LIB (GPU parity + decode tests), then an A/B of
# all turbo_decoder_cuda_amd/libvar_*.so (scripts/variant_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$PARITY_LIB" ]; then
  TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/$PARITY_LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parv.log 2>&1
  rc=$?
  grep -E "passed|failed|FAILED" gpurun_out/parv.log | tail -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
ROUNDS=${ROUNDS:-3} bash scripts/variant_ab.sh
