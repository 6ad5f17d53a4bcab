#!/bin/bash
# Parity of one variant library (VARLIB) on the windowed tests, then the interleaved config-5 A/B of all
# libvar_*.so (scripts/variant_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/${VARLIB} timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/var_parity.txt 2>&1
rc=$?; tail -3 gpurun_out/var_parity.txt; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-6} BENCH_SETS="--window 64 --overlap 30 --batch 32768 --dropin-frames 0" \
    bash scripts/variant_ab.sh
