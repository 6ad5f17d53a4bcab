#!/bin/bash
# round 4: parity subset on the in-tree build, an interleaved A/B of libvar_*.so and the stamps of libdiag_*.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
for v in ${PARITY_LIBS:-intree}; do
  if [ "$v" = intree ]; then unset TD_LIB_PATH; else export TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_$v.so; fi
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_decode.py > gpurun_out/r4/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc: $(tail -1 gpurun_out/r4/parity_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
unset TD_LIB_PATH
ROUNDS=${ROUNDS:-3} STEPS=${STEPS:-6} BENCH_SETS="${BENCH_SETS:-}" bash scripts/variant_ab.sh 2>&1 | tee gpurun_out/r4/ab2.txt || exit 1
for r in 1 2; do DIAG_LINES=14 bash scripts/diag_libs.sh 2>&1 | tee -a gpurun_out/r4/stamps.txt || exit 1; done
