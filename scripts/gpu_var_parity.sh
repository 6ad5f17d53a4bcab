#!/bin/bash
# GPU box job: the parity tests (TESTS, default test_gpu_parity.py) against every libvar_*.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in turbo_decoder_cuda_amd/libvar_*.so; do
  TD_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/vp.log 2>&1
  rc=$?
  echo "$(basename $lib): rc=$rc $(tail -1 gpurun_out/vp.log)"
  [ $rc -eq 0 ] || exit 1   # a failed or faulted run ends the GPU work of this call
done
