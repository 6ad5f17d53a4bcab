cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/siso_edge_fit.py --rounds 3 > gpurun_out/siso_edge_fit.txt 2>&1; rc=$?; cat gpurun_out/siso_edge_fit.txt; exit $rc
