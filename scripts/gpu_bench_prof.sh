#!/bin/bash
# GPU box job: parity tests, one bench line, rocprofv3 kernel-trace summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-variants > gpurun_out/prof.log 2>&1 || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python scripts/diag_stamps.py 4096 f64 logmap > gpurun_out/diag.log 2>&1 && \
  timeout -k 10 300 python scripts/diag_stamps.py 4096 f64 maxlog >> gpurun_out/diag.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/diag.log; exit 1; }
  cat gpurun_out/diag.log
fi
if [ -n "$UBENCH" ]; then
  timeout -k 10 120 ./scripts/ubench_latency > gpurun_out/ubench.log 2>&1; cat gpurun_out/ubench.log
fi
