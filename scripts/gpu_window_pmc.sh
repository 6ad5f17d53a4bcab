#!/bin/bash
# PMC of the windowed kernels (BASELINE config 5) for one library (LIB), one pass per counter group
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/wpmc
LIBP=$PWD/${LIB:-turbo_decoder_cuda_amd/libturbo_mi355x.so}
P1="--window 64 --batch 32768 --steps 1 --warmup 0 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power"
n=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  TD_LIB_PATH=$LIBP timeout -s KILL 200 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/wpmc/p$n -o pmc --output-format csv -- python3 bench.py $P1 > gpurun_out/wpmc/p$n.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/wpmc/p$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/wpmc/p*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "sw_" in k:
            kk = "alpha" if "alpha" in k else ("beta" if "beta" in k else "demux")
            per[(kk, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (kk, c, d), v in per.items():
        acc[kk][c].append(v)
for f in sorted(glob.glob("gpurun_out/wpmc/p1/**/*kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "sw_" in k:
            kk = "alpha" if "alpha" in k else ("beta" if "beta" in k else "demux")
            dur[kk].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for kk in acc:
    print(kk, "dispatches", len(dur[kk]), "mean ms %.3f" % (sum(dur[kk]) / max(1, len(dur[kk]))))
    for c, v in sorted(acc[kk].items()):
        print(f"   {c:24s} mean {sum(v)/len(v):.5g}")
PY
