#!/bin/bash
# GPU box job: parity tests of the default library (TESTS, default the decode/parity files), then
# the interleaved A/B of the libvar_*.so variants (scripts/variant_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_decode.py} -x -q -m gpu \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
ROUNDS=${ROUNDS:-3} bash scripts/variant_ab.sh
