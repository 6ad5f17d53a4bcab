#!/bin/bash
# GPU box job: parity (golden frames + oracle batches) of every libvar_*.so, then the interleaved
# A/B of scripts/variant_ab.sh.  Stops at the first failing variant.  TESTS overrides the test files.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in turbo_decoder_cuda_amd/libvar_*.so; do
  v=$(basename $lib .so)
  TD_LIB_PATH=$PWD/$lib timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_decode.py} -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pt_$v.log 2>&1 || { echo "parity $v failed rc=$?"; tail -30 gpurun_out/pt_$v.log; exit 1; }
  echo "== parity $v: $(tail -1 gpurun_out/pt_$v.log)"
done
bash scripts/variant_ab.sh
