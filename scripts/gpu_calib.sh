#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calib -o fetch --output-format csv -- ./scripts/calib_fetch > gpurun_out/calib.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/calib -o write --output-format csv -- ./scripts/calib_fetch >> gpurun_out/calib.log 2>&1 || { echo "calib failed"; tail gpurun_out/calib.log; exit 1; }
grep -h "read8\|write8" gpurun_out/calib/*counter_collection.csv | awk -F'","' '{print $9, $16, $17}'
