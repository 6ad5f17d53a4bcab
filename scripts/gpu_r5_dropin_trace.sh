#!/bin/bash
# round 5: kernel trace of the drop-in's windowed single-frame path (td_dropin_latency with
# TD_WINDOW=64 TD_OVERLAP=30, 8 frames of K=6144, 15 iterations)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/dt
python3 -c "
import sys; sys.path.insert(0, 'oracle')
import pyoracle as O, numpy as np
_, flow = O.synth_batch(6144, 263, 480, 1.0, 7, 8)
np.ascontiguousarray(flow, dtype=np.float64).tofile('gpurun_out/dt/flows.bin')
"
TD_WINDOW=64 TD_OVERLAP=30 timeout -k 10 120 turbo_decoder_cuda_amd/td_dropin_latency 6144 263 480 8 gpurun_out/dt/flows.bin gpurun_out/dt/bits.bin || exit 1
TD_WINDOW=64 TD_OVERLAP=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dt/kt -o kt --output-format csv -- turbo_decoder_cuda_amd/td_dropin_latency 6144 263 480 8 gpurun_out/dt/flows.bin gpurun_out/dt/bits2.bin > gpurun_out/dt/kt.log 2>&1 || { tail -20 gpurun_out/dt/kt.log; exit 1; }
f=$(ls gpurun_out/dt/kt/*kernel_stats.csv gpurun_out/dt/kt/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:60].ljust(60), r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3), "total ms %.2f" % (float(r["TotalDurationNs"]) / 1e6))
PY
