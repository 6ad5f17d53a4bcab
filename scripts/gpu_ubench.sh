set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_alpha > gpurun_out/ub_alpha.log 2>&1 && cat gpurun_out/ub_alpha.log && \
timeout -k 10 120 ./scripts/ubench_beta > gpurun_out/ub_beta.log 2>&1 && cat gpurun_out/ub_beta.log && \
timeout -k 10 300 python scripts/diag_stamps.py 4096 f64 logmap > gpurun_out/diag.log 2>&1 && cat gpurun_out/diag.log
