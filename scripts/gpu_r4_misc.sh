#!/bin/bash
# round 4: the bench's power record, stamps of the other modes, and SQ / LDS PMC of the windowed
# kernel (config 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/r4/pw5.json 2> gpurun_out/r4/pw5.err || { echo "bench rc=$?"; tail -20 gpurun_out/r4/pw5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4/pw5.json')); print(d['value'], d['roofline']['sclk_ghz'], d['power'])"
SL=$PWD/turbo_decoder_cuda_amd/libturbo_mi355x_stamps.so
TD_STAMPS_LIB=$SL timeout -k 10 300 python scripts/diag_stamps.py 4096 f64 maxlog > gpurun_out/r4/stamps_maxlog.txt 2>&1 || { echo "stamps maxlog rc=$?"; tail -5 gpurun_out/r4/stamps_maxlog.txt; exit 1; }
TD_STAMPS_LIB=$SL timeout -k 10 300 python scripts/diag_stamps.py 4096 f32 logmap > gpurun_out/r4/stamps_f32.txt 2>&1 || { echo "stamps f32 rc=$?"; tail -5 gpurun_out/r4/stamps_f32.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/stamps_maxlog.txt gpurun_out/r4/stamps_f32.txt | head -24
WB="--window 64 --batch 32768 --steps 1 --warmup 0 --cpu-sample 0 --no-variants --dropin-frames 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d gpurun_out/prof_w -o sq1 --output-format csv -- python3 bench.py $WB > gpurun_out/r4/wpmc1.log 2>&1 || { echo "pmc1 failed"; tail -5 gpurun_out/r4/wpmc1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/prof_w -o sq2 --output-format csv -- python3 bench.py $WB > gpurun_out/r4/wpmc2.log 2>&1 || { echo "pmc2 failed"; tail -5 gpurun_out/r4/wpmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("sq1", "sq2"):
    f = glob.glob(f"gpurun_out/prof_w/**/{tag}_counter_collection.csv", recursive=True)
    d = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "sw_siso_kernel" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(tag, {k: "%.4g" % v for k, v in d.items()}, dict(n))
PY
