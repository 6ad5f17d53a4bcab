#!/bin/bash
# round 5: the drop-in's windowed single-frame latency (TD_WINDOW=64 TD_OVERLAP=30) for each
# libvar_*.so, run through copies of td_dropin_latency + the compat library next to it ($ORIGIN)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/da
python3 -c "
import sys; sys.path.insert(0, 'oracle')
import pyoracle as O, numpy as np
_, flow = O.synth_batch(6144, 263, 480, 1.0, 7, 8)
np.ascontiguousarray(flow, dtype=np.float64).tofile('gpurun_out/da/flows.bin')
"
for r in 1 2; do
  for lib in turbo_decoder_cuda_amd/libvar_*.so; do
    n=$(basename $lib .so); d=gpurun_out/da/$n; mkdir -p $d
    cp turbo_decoder_cuda_amd/td_dropin_latency turbo_decoder_cuda_amd/libturbo_logmap_compat.so $d/
    cp $lib $d/libturbo_mi355x.so
    for env in "TD_WINDOW=64 TD_OVERLAP=30" "TD_WINDOW=0"; do
      out=$(env $env timeout -k 10 120 $d/td_dropin_latency 6144 263 480 8 gpurun_out/da/flows.bin $d/bits.bin) || { echo "$n rc=$?"; exit 1; }
      echo "round $r $n [$env] $out"
    done
  done
done
