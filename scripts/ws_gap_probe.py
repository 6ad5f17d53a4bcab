"""Layout probe on a physically contiguous workspace (build with -DTD_WS_EXPERIMENT
-DTD_WS_CONTIG, loaded via TD_LIB_PATH, GPU box): kernel time for gaps inserted before the extrinsic arrays, the alpha scratch and the
tempmax scratch (TD_WS_GAP_E / _A / _T).  A gap that moves the time points at conflicts between
the arrays' streams; none that does points elsewhere (pages, translation).
python scripts/ws_gap_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402

os.environ["TD_PLACEMENT_TRIALS"] = "1"
K, B = 6144, 4096
dev = torch.device("cuda", 0)
u, llr_h = synth.make_batch(B, K, 263, 480, 1.0, seed=20261015, dtype=np.float64)
llr = torch.from_numpy(llr_h).to(dev)
bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
cases = [(0, 0, 0), (0, 4096, 0), (0, 65536, 0), (0, 1 << 20, 0), (0, (2 << 20) + 4096, 0), (0, 0, 65536),
         (0, 0, (1 << 20) + 256), (65536, 0, 0), ((1 << 20) + 4096, 0, 0), (0, 3 << 20, 3 << 20), (0, 0, 0)]
keep = []
for ge, ga, gt in cases:
    os.environ["TD_WS_GAP_E"], os.environ["TD_WS_GAP_A"], os.environ["TD_WS_GAP_T"] = str(ge), str(ga), str(gt)
    codec = TurboCodec(K, 263, 480, iterations=8, algo="logmap", precision="f64", device=0)
    codec.reserve(B)
    codec.decode(llr, bits)
    torch.cuda.synchronize(dev)
    codec.profile(True)
    for _ in range(3):
        codec.decode(llr, bits)
    torch.cuda.synchronize(dev)
    _, kms, _ = codec.kernel_ms()
    ok = bool((bits != torch.from_numpy(u).to(dev)).sum().item() == 0)
    print(f"gap ext {ge >> 10:6d} KiB  alpha {ga >> 10:6d} KiB  tempmax {gt >> 10:6d} KiB: kernel {kms:.2f} ms  bits ok {ok}", flush=True)
    keep.append(codec)
