#!/bin/bash
# round 4 evidence on one box: stamps of turbo_decoder_cuda_amd/libdiag_*.so (2 interleaved rounds), the full
# bench line (variants, cpu_baseline, dropin), the rocprofv3 kernel trace and the FETCH / WRITE PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
if [ -z "${SKIP_STAMPS:-}" ]; then
  for r in 1 2; do DIAG_LINES=14 bash scripts/diag_libs.sh 2>&1 | tee -a gpurun_out/r4/stamps.txt || exit 1; done
fi
echo "== bench"
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
[ -n "${SKIP_PROF:-}" ] && exit 0
PB="--steps 8 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0"
echo "== kernel-trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py $PB > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof kt failed rc=$?"; tail -20 gpurun_out/prof_kt.log; exit 1; }
echo "== pmc-fetch"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof -o fetch --output-format csv -- python3 bench.py $PB > gpurun_out/prof_fetch.log 2>&1 || { echo "rocprof fetch failed rc=$?"; tail -20 gpurun_out/prof_fetch.log; exit 1; }
echo "== pmc-write"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof -o write --output-format csv -- python3 bench.py $PB > gpurun_out/prof_write.log 2>&1 || { echo "rocprof write failed rc=$?"; tail -20 gpurun_out/prof_write.log; exit 1; }
find gpurun_out/prof -name "*.csv" | sort
