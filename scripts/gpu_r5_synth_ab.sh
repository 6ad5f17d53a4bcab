#!/bin/bash
# round 5: device frame generator (td_synth_frames) time for B = 4096 and 32768 frames of K = 6144, per
# library: libvar_a_head.so (before) and the product library (after), two interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for lib in turbo_decoder_cuda_amd/libvar_a_head.so turbo_decoder_cuda_amd/libturbo_mi355x.so; do
TD_LIB_PATH=$PWD/$lib timeout -k 10 120 python -c "
import torch
from turbo_decoder_cuda_amd import TurboCodec
res = {}
for B in (4096, 32768):
    with TurboCodec(6144, 263, 480, iterations=8) as c:
        c.synth_seed(20261015)
        u, x = c.synth(B, 1.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        u, x = c.synth(B, 1.0, info=u, llr=x)
        e1.record()
        torch.cuda.synchronize()
        res[B] = round(e0.elapsed_time(e1), 3)
print('$r', '$lib'.split('/')[-1], res)
" || exit 1
done; done
