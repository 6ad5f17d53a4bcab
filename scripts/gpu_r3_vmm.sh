#!/bin/bash
# GPU box job: placement spread of the VMM-mapped workspace (chunk sizes) vs plain hipMalloc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TD_PLACEMENT_TRIALS=1 TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || echo "list-avail rc=$?"
for v in b_win v_vmm:0 v_vmm:2097152 v_vmm:67108864; do
  lib=${v%%:*}; ch=${v#*:}; [ "$ch" = "$v" ] && ch=0
  TD_VMM_CHUNK=$ch TD_LIB_PATH=$PWD/turbo_decoder_cuda_amd/libvar_$lib.so timeout -k 10 300 python scripts/spread_probe.py 6 2 4 > gpurun_out/vmm_$lib_$ch.log 2>&1 || { echo "$v failed rc=$?"; tail -20 gpurun_out/vmm_$lib_$ch.log; exit 1; }
  echo "== $v"; grep -E "instance|VMM" gpurun_out/vmm_$lib_$ch.log | sort | uniq -c | sort -rn | head -8
done
