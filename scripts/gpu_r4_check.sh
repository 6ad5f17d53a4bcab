# round 4: the full GPU suite on the in-tree build, then an interleaved A/B of turbo_decoder_cuda_amd/libvar_*.so
# (the A/B runs after test failures -- pytest rc 1 -- but not after a crash, a timeout or a hang)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/r4/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/r4/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; grep -E "FAILED|Error|assert" gpurun_out/r4/pytest_gpu.log | head -20; fi
  [ $rc -le 1 ] || exit $rc
fi
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-6} BENCH_SETS="${BENCH_SETS:-}" bash scripts/variant_ab.sh 2>&1 | tee gpurun_out/r4/ab.txt
