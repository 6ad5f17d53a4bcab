#!/bin/bash
# round 5: the fp64 three-per-CU bound.  libvar_occ3.so is a timing-only
# build (-DTD_DIAG=16: beta rows and tile ring alias the alpha ring, 52.7 KB per workgroup, results
# WRONG, every DMA / store / instruction kept); TD_OCC3=0 runs it at two per CU, TD_OCC3=1 lets
# occupancy_pick take three.  Beside them the product library at two per CU.  Interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/occ3
for r in 1 2; do
  for B in 12288 32768; do
    for v in "prod 1 turbo_decoder_cuda_amd/libturbo_mi355x.so" "diag2 0 turbo_decoder_cuda_amd/libvar_occ3.so" "diag3 1 turbo_decoder_cuda_amd/libvar_occ3.so"; do
      set -- $v
      TD_OCC3=$2 TD_LIB_PATH=$PWD/$3 timeout -k 10 300 python bench.py --batch $B --steps 3 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power > gpurun_out/occ3/v.json 2> gpurun_out/occ3/v.err || { echo "$1 B=$B rc=$?"; tail -20 gpurun_out/occ3/v.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/occ3/v.json')); r=d['roofline']; print('round $r B=$B', '$1'.ljust(6), d['value'], 'kernel ms', r['kernel_ms_avg'], 'sclk', r.get('sclk_ghz'), 'errs', d['ber']['bit_errors'])"
    done
  done
done
for v in "prod 1 turbo_decoder_cuda_amd/libturbo_mi355x.so" "diag3 1 turbo_decoder_cuda_amd/libvar_occ3.so"; do
  set -- $v
  for c in FETCH_SIZE WRITE_SIZE; do
    TD_OCC3=$2 TD_LIB_PATH=$PWD/$3 timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/occ3/pmc_$1_$c -o pmc --output-format csv -- python3 bench.py --batch 32768 --steps 1 --warmup 0 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power > gpurun_out/occ3/pmc.log 2>&1 || { echo "pmc $1 $c failed"; tail -5 gpurun_out/occ3/pmc.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob
for tag in ("prod", "diag3"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/occ3/pmc_{tag}_{c}/**/*counter_collection.csv", recursive=True)[0]
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "turbo_decode_kernel" in r["Kernel_Name"]]
        print(tag, c, "KiB per launch", sum(v) / max(1, len(v)), "launches", len(v))
PY
