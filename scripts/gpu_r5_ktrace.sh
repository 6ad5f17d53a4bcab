#!/bin/bash
# round 5: per-kernel times (rocprofv3 --kernel-trace --stats) of each libvar_*.so on one bench
# command (BENCH_ARGS), one process per library; prints the kernels' mean durations
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/kt
ARGS=${BENCH_ARGS:-"--window 64 --batch 32768 --steps 3 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0"}
for lib in turbo_decoder_cuda_amd/libvar_*.so; do
  n=$(basename $lib .so)
  TD_LIB_PATH=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$n -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/kt/$n.json 2> gpurun_out/kt/$n.err || { echo "$n rc=$?"; tail -20 gpurun_out/kt/$n.err; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/kt/{n}.json"))
print(n.ljust(22), "Mbit/s", d["value"], "decode ms", d["roofline"]["kernel_ms_avg"])
f = glob.glob(f"gpurun_out/kt/{n}/**/kt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r["TotalDurationNs"]) > 2e6:
        print("   ", r["Name"][:70].ljust(70), r["Calls"], "avg ms %.3f" % (float(r["AverageNs"]) / 1e6), "total ms %.1f" % (float(r["TotalDurationNs"]) / 1e6))
PY
done
