#!/bin/bash
# round 4 evidence on one box: the full GPU suite, smoke, the full bench line (variants, cpu_baseline,
# dropin, clock), the rocprofv3 kernel trace and the FETCH / WRITE / SQ PMC passes of the same bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/r4/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4/pytest_gpu.log
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/r4/smoke.log; exit 1; }
cat gpurun_out/r4/smoke.log | tail -1
echo "== bench"
timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
PB="--steps 8 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0"
echo "== kernel-trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py $PB > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed rc=$?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
echo "== pmc-fetch"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof -o fetch --output-format csv -- python3 bench.py $PB > gpurun_out/prof_fetch.log 2>&1 || { echo "rocprof fetch failed rc=$?"; tail -20 gpurun_out/prof_fetch.log; exit 1; }
echo "== pmc-write"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof -o write --output-format csv -- python3 bench.py $PB > gpurun_out/prof_write.log 2>&1 || { echo "rocprof write failed rc=$?"; tail -20 gpurun_out/prof_write.log; exit 1; }
echo "== pmc-sq"
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/prof -o sq --output-format csv -- python3 bench.py $PB > gpurun_out/prof_sq.log 2>&1 || { echo "rocprof sq failed rc=$?"; tail -20 gpurun_out/prof_sq.log; exit 1; }
find gpurun_out/prof -name "*.csv" | sort
