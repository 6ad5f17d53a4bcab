set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_b_kw15.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/par15.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" gpurun_out/par15.log | tail -15
exit $rc
