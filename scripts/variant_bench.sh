#!/bin/bash
# GPU box job: bench each turbo_decoder_cuda_amd/libvar_*.so (build variants) on the config-2 workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in turbo_decoder_cuda_amd/libvar_*.so; do
  TD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-variants ${BENCH_ARGS} > gpurun_out/var.json 2> gpurun_out/var.err || { echo "$lib failed rc=$?"; tail -20 gpurun_out/var.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/var.json')); print('$lib', d['value'], d['roofline']['kernel_ms_avg'], d['ber']['bit_errors'])"
done
