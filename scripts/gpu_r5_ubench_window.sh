#!/bin/bash
# round 5: scripts/ubench_window (the windowed kernels' arithmetic at 1, 2, 3 waves per SIMD), timing run
# and one SQ_INSTS_VALU pass; prints the per-dispatch VALU issue fraction.  Build it first (see its header).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ubw
timeout -k 10 120 ./scripts/ubench_window > gpurun_out/ubw/run.jsonl 2>&1 || { cat gpurun_out/ubw/run.jsonl; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d gpurun_out/ubw/pmc -o pmc --output-format csv -- ./scripts/ubench_window > gpurun_out/ubw/pmc.log 2>&1 || { tail -5 gpurun_out/ubw/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, json, re, collections
runs = [json.loads(l) for l in open("gpurun_out/ubw/run.jsonl") if l.startswith("{")]
f = glob.glob("gpurun_out/ubw/pmc/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    m = re.search(r"ub<(\d+), (\d+)>", r["Kernel_Name"])
    if m:
        per[(int(m.group(1)), int(m.group(2)), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
for r in runs:
    ds = sorted(k for k in per if k[:2] == (r["mix"], r["waves_per_simd"]))
    d = per[ds[-1]]                                                   # the timed launch
    vi = d["SQ_INSTS_VALU"] / (d["SQ_WAVES"] * r["positions"])        # VALU a wave-position
    r["valu_per_wave_position"] = round(vi, 1)
    # issue fraction of all 1024 SIMDs over the launch, at the launch's measured clock
    r["simd_issue_frac"] = round(vi * r["waves"] * r["positions"] * 4 / (1024 * r["kernel_ms"] * 1e-3 * r["sclk_ghz"] * 1e9), 4)
    print(json.dumps(r))
PY
