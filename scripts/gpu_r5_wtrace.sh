#!/bin/bash
# round 5: kernel trace (start/end of every dispatch) of config-5 decodes, to see how the two halves'
# alpha / beta launches overlap
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/wt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/wt/t -o kt --output-format csv -- python3 bench.py --window 64 --batch 32768 --steps 2 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power > gpurun_out/wt/b.json 2> gpurun_out/wt/b.err || { tail -20 gpurun_out/wt/b.err; exit 1; }
f=$(ls gpurun_out/wt/t/*kernel_trace.csv gpurun_out/wt/t/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sw_" in r["Kernel_Name"] or "bits_transpose" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last decode: from the last sw_demux
idx = max(i for i, r in enumerate(rows) if "sw_demux" in r["Kernel_Name"])
rows = rows[idx:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[:40]:
    k = r["Kernel_Name"]; k = "demux" if "demux" in k else "alpha" if "alpha" in k else "beta" if "beta" in k else "transpose"
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{k:9s} q{r.get('Queue_Id', r.get('Stream_Id','?'))} {s:10.1f} {e:10.1f} {e - s:8.1f} us")
PY
