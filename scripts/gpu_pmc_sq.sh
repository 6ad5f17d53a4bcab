#!/bin/bash
# SQ counters of the turbo kernel (one PMC pass, kernel-trace only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"}
timeout -k 10 400 rocprofv3 --pmc $CTRS --kernel-trace -d gpurun_out/sq -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-variants ${BENCH_ARGS} > gpurun_out/sq.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/sq.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/sq/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if 'turbo_decode' in r['Kernel_Name']:
            print(r['Counter_Name'], r['Counter_Value'])
PY
