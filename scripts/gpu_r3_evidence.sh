#!/bin/bash
# GPU box job (round 3 evidence): the bench line, the rocprofv3 kernel-trace summary and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE) of the same bench, one SQ pass (issue / dependency waits), and the
# placement spread of 8 fresh decoders WITH the placement search.  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
PB="--steps 8 --warmup 1 --cpu-sample 0 --no-variants"
echo "== kernel-trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py $PB > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed rc=$?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
echo "== pmc-fetch"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof -o fetch --output-format csv -- python3 bench.py $PB > gpurun_out/prof_fetch.log 2>&1 || { echo "rocprof fetch failed rc=$?"; tail -20 gpurun_out/prof_fetch.log; exit 1; }
echo "== pmc-write"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof -o write --output-format csv -- python3 bench.py $PB > gpurun_out/prof_write.log 2>&1 || { echo "rocprof write failed rc=$?"; tail -20 gpurun_out/prof_write.log; exit 1; }
echo "== pmc-sq"
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/prof -o sq --output-format csv -- python3 bench.py $PB > gpurun_out/prof_sq.log 2>&1 || { echo "rocprof sq failed rc=$?"; tail -20 gpurun_out/prof_sq.log; exit 1; }
echo "== spread with placement search"
timeout -k 10 400 python scripts/spread_probe.py 8 2 4 > gpurun_out/spread_probe8.log 2>&1 || { echo "spread failed rc=$?"; tail -20 gpurun_out/spread_probe8.log; exit 1; }
grep instance gpurun_out/spread_probe8.log
echo "== bench"
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
find gpurun_out/prof -name "*.csv" | sort
