#!/bin/bash
# Usage (GPU box): build turbo_decoder_cuda_amd/libdiag_nofold.so with -DTD_DIAG=4 (TD_DIAG bits: td_kernels.hip "diagnostic builds") first.
# LDS PMC of the default library and of diagnostic variants (turbo kernel only)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
run() { tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/ldsd_$tag -o lds --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-variants "$@" > gpurun_out/ldsd_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ldsd_$tag.log; exit 1; }; }
run base
TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libdiag_nofold.so run nofold
python3 - <<PY
import csv,glob,collections
for tag in ["base","nofold"]:
    f=glob.glob("gpurun_out/ldsd_%s/**/lds_counter_collection.csv"%tag,recursive=True)
    d=collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        if "turbo_decode" in r["Kernel_Name"]: d[r["Counter_Name"]]+=float(r["Counter_Value"])
    print(tag, {k:"%.4g"%v for k,v in d.items()}, "conflict/active %.3f"%(d["SQ_LDS_BANK_CONFLICT"]/d["SQ_LDS_IDX_ACTIVE"]))
PY
