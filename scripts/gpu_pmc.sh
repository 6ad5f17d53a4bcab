#!/bin/bash
# PMC counters of one kernel, one rocprofv3 pass per counter group (kernel-trace only):
#   KNAME=sw_siso BENCH_ARGS="--window 64 --batch 32768" CTR_GROUPS="FETCH_SIZE WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES" scripts/gpu_pmc.sh
# Prints, per counter, the mean over the kernel's dispatches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
KNAME=${KNAME:-turbo_decode}
CTR_GROUPS=${CTR_GROUPS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU;SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"}
n=0
IFS=';' read -ra G <<< "$CTR_GROUPS"
for ctrs in "${G[@]}"; do
  n=$((n+1))
  timeout -k 10 400 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc$n -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-variants ${BENCH_ARGS} > gpurun_out/pmc$n.log 2>&1 || { echo "rocprof pass $n failed"; tail -20 gpurun_out/pmc$n.log; exit 1; }
done
KNAME=$KNAME python3 - <<'PY'
import csv, glob, os, collections
k = os.environ["KNAME"]
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if k in r['Kernel_Name']:
            per[(r['Counter_Name'], r['Dispatch_Id'])] += float(r['Counter_Value'])
    for (c, d), v in per.items():
        acc[c].append(v)
for c, v in sorted(acc.items()):
    print(f"{c:28s} dispatches {len(v):4d}  mean {sum(v)/len(v):.6g}")
PY
