#!/bin/bash
# GPU box job: A/B of the build variants turbo_decoder_cuda_amd/libvar_*.so, ROUNDS interleaved
# rounds on one device (separate processes, same box), for each BENCH_SETS argument set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "${BENCH_SETS:-}"
[ ${#SETS[@]} -eq 0 ] && SETS=("")
for r in $(seq 1 ${ROUNDS:-2}); do
  for args in "${SETS[@]}"; do
    for lib in turbo_decoder_cuda_amd/libvar_*.so; do
      TD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 1 --cpu-sample 0 --no-variants $args > gpurun_out/var.json 2> gpurun_out/var.err || { echo "$lib failed rc=$?"; tail -20 gpurun_out/var.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/var.json')); print('round $r', '$args'.ljust(28), '$lib'.split('/')[-1].ljust(28), d['value'], d['roofline']['kernel_ms_avg'], d['roofline'].get('demux_ms_avg'), d['ber']['bit_errors'])"
    done
  done
done
