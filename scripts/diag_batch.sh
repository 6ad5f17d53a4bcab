set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for B in 2048 4096 8192; do timeout -k 10 200 python scripts/diag_stamps.py $B f64 maxlog || exit 1; done > gpurun_out/diag2.log 2>&1
cat gpurun_out/diag2.log | grep -v amdgpu.ids
