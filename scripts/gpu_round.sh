#!/bin/bash
# GPU box job for a round's evidence: parity tests, smoke, the bench line, the rocprofv3
# kernel-trace summary and the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same bench.
# Outputs under gpurun_out/; copy what is judged into profiles/rNN/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
[ -n "$SKIP_BENCH" ] && exit 0
step bench
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
PB="--steps 8 --warmup 1 --cpu-sample 0 --no-variants"
step kernel-trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py $PB > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed rc=$?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
step pmc-fetch
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof -o fetch --output-format csv -- python3 bench.py $PB > gpurun_out/prof_fetch.log 2>&1 || { echo "rocprof fetch failed rc=$?"; tail -20 gpurun_out/prof_fetch.log; exit 1; }
step pmc-write
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof -o write --output-format csv -- python3 bench.py $PB > gpurun_out/prof_write.log 2>&1 || { echo "rocprof write failed rc=$?"; tail -20 gpurun_out/prof_write.log; exit 1; }
find gpurun_out/prof -name "*.csv" | sort
