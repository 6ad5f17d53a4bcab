#!/bin/bash
# Round 6: what the exact kernel's HBM scratch costs in clock at the board's
# power cap.  Timing-only diagnostic builds (results wrong) of the same source, interleaved rounds, each
# bench process 100 config-2 steps with the amdsmi power / clock sampler over the timed region:
#   a_base      production
#   b_noastore  the F pass without its alpha scratch stores (-25.8 GB of writes a launch)
#   c_noadma    the B pass without the loader's alpha copies (-25.8 GB of reads)
#   d_noboth    neither (-51.6 GB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in turbo_decoder_cuda_amd/libvar_*.so; do
    TD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --cpu-sample 0 --no-variants \
        --dropin-frames 0 > gpurun_out/pw.json 2> gpurun_out/pw.err || { echo "$lib failed rc=$?"; tail -20 gpurun_out/pw.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/pw.json')); p=d.get('power') or {}; r=d['roofline']
print('round $r', '$lib'.split('/')[-1].ljust(26), 'Mbit/s', d['value'], 'kernel_ms', r['kernel_ms_avg'], 'sclk(td_clock)', r['sclk_ghz'],
      'W mean', p.get('socket_w_mean'), 'W max', p.get('socket_w_max'), 'sclk_mhz_mean', p.get('sclk_mhz_mean'), 'n', p.get('samples'))"
  done
done
