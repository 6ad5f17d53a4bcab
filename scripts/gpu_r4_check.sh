# round 4: the full GPU suite on the in-tree build, then an interleaved A/B of turbo_decoder_cuda_amd/libvar_*.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/r4/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/r4/pytest_gpu.log
fi
ROUNDS=${ROUNDS:-2} STEPS=${STEPS:-6} BENCH_SETS="${BENCH_SETS:-}" bash scripts/variant_ab.sh 2>&1 | tee gpurun_out/r4/ab.txt
