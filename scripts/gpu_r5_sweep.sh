#!/bin/bash
# round 5: config-5 sweep -- each libvar_*.so at the default layout, then the product library at
# forced layouts, CFGS="P:M:MA ..." (P batch parts on P streams, beta run M, alpha run MA;
# TD_WINDOW_PARTS / TD_WINDOW_RUN / TD_WINDOW_RUN_A; 0 = default), interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/sw
WB="--window 64 --batch ${BATCH:-32768} --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 --no-power ${EXTRA:-}"
LIB=${LIB:-turbo_decoder_cuda_amd/libturbo_mi355x.so}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $(ls turbo_decoder_cuda_amd/libvar_*.so 2>/dev/null); do
    TD_LIB_PATH=$PWD/$lib timeout -k 10 200 python bench.py $WB > gpurun_out/sw/v.json 2> gpurun_out/sw/v.err || { echo "$lib rc=$?"; tail -20 gpurun_out/sw/v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sw/v.json')); print('round $r', '$lib'.split('/')[-1].ljust(24), d['value'], d['roofline']['kernel_ms_avg'])"
  done
  for c in ${CFGS:-0:0:0}; do
    IFS=: read P M MA <<< "$c"; TD_WINDOW_PARTS=$P TD_WINDOW_RUN=$M TD_WINDOW_RUN_A=$MA TD_LIB_PATH=$PWD/$LIB timeout -k 10 200 python bench.py $WB > gpurun_out/sw/v.json 2> gpurun_out/sw/v.err || { echo "cfg $c rc=$?"; tail -20 gpurun_out/sw/v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/sw/v.json')); print('round $r', 'run $c'.ljust(24), d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
