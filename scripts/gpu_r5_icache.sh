#!/bin/bash
# round 5: instruction-cache / issue counters of the windowed kernels (config 5, one decode a pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/ic
P1="--window 64 --batch 32768 --steps 1 --warmup 0 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power"
n=0
for ctrs in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/ic/p$n -o pmc --output-format csv -- python3 bench.py $P1 > gpurun_out/ic/p$n.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/ic/p$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/ic/p*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "sw_" in k:
            kk = "alpha" if "alpha" in k else ("beta" if "beta" in k else "demux")
            per[(kk, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (kk, c, d), v in per.items():
        acc[kk][c].append(v)
for kk in acc:
    print(kk)
    for c, v in sorted(acc[kk].items()):
        print(f"   {c:28s} mean {sum(v)/len(v):.5g}")
PY
