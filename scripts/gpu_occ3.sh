#!/bin/bash
# GPU box job: three workgroups per CU for large fp32 Max-Log-MAP batches (turbo_decode_kernel3).
# New parity test, then the kernel trace of one large decode, then an interleaved A/B of
# the libvar_*.so builds (OCC_SETS: the bench argument sets).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/occ3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v -m gpu --timeout 200 --timeout-method thread -k "three_workgroups or maxlog_vs_oracle or f32_logmap" > gpurun_out/occ3/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/occ3/pytest.log; exit 1; }
tail -3 gpurun_out/occ3/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/occ3/prof -o run -- python3 bench.py --precision f32 --algo maxlog --batch 32768 --steps 2 --warmup 1 --cpu-sample 0 --no-variants > gpurun_out/occ3/prof.json 2> gpurun_out/occ3/prof.err || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/occ3/prof.err; exit 1; }
find gpurun_out/occ3/prof -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -8
ROUNDS=2 BENCH_SETS="${OCC_SETS:---precision f32 --algo maxlog --batch 32768;--precision f32 --algo maxlog --batch 12288;--precision f32 --algo maxlog}" STEPS=4 bash scripts/variant_ab.sh
