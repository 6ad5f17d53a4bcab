#!/bin/bash
# round 5: where the windowed kernel (config 5) spends its time.  Timing-only variants
# (libvar_*.so, TD_SW_DIAG: 1 = synthetic inputs, 2 = no checkpoint traffic; results wrong) in
# interleaved rounds, then FETCH / WRITE / SQ PMC of the product build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/w5
WB="--window 64 --batch 32768 --steps 3 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0"
for r in 1 2; do
  for lib in turbo_decoder_cuda_amd/libvar_*.so; do
    TD_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py $WB > gpurun_out/w5/v.json 2> gpurun_out/w5/v.err || { echo "$lib rc=$?"; tail -20 gpurun_out/w5/v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/w5/v.json')); print('round $r', '$lib'.split('/')[-1].ljust(24), d['value'], d['roofline']['kernel_ms_avg'], d['ber']['bit_errors'])"
  done
  TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_a_base.so timeout -k 10 200 python bench.py $WB --algo maxlog > gpurun_out/w5/v.json 2> gpurun_out/w5/v.err || { echo "maxlog rc=$?"; tail -20 gpurun_out/w5/v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/w5/v.json')); print('round $r', 'base maxlog'.ljust(24), d['value'], d['roofline']['kernel_ms_avg'], d['ber']['bit_errors'])"
done
P1="--window 64 --batch 32768 --steps 1 --warmup 0 --cpu-sample 0 --no-variants --dropin-frames 0"
n=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/w5/pmc$n -o pmc --output-format csv -- python3 bench.py $P1 > gpurun_out/w5/pmc$n.log 2>&1 || { echo "pmc $n failed"; tail -5 gpurun_out/w5/pmc$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/w5/pmc*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "sw_siso" in r["Kernel_Name"]:
            per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (c, d), v in per.items():
        acc[c].append(v)
for c, v in sorted(acc.items()):
    print(f"{c:28s} dispatches {len(v):4d}  mean {sum(v)/len(v):.6g}")
PY
