set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_handle.py -x -v --timeout 300 --timeout-method thread > gpurun_out/handle_pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/handle_pytest.txt; exit $rc
