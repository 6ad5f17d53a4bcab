#!/bin/bash
# Round 6: parity of one variant library (VARLIB) on the exact-kernel tests, then the interleaved A/B
# of all libvar_*.so (scripts/variant_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/${VARLIB} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_decode.py -k "not window and not compat" -x -q --timeout 300 --timeout-method thread > gpurun_out/var_parity.txt 2>&1
rc=$?; tail -3 gpurun_out/var_parity.txt; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-30} bash scripts/variant_ab.sh
