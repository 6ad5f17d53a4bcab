"""Workspace-placement probe (GPU box, a -DTD_WS_EXPERIMENT build via TD_LIB_PATH,
with TD_PLACEMENT_TRIALS=1): for several decoder
instances (fresh allocations), the kernel time with the workspace carve shifted by a list of
offsets inside the same allocation.  Offsets that change the time within an instance point at the
layout (channel / page mapping of the streams); a time set by the instance alone points at the
physical allocation.
python scripts/ws_offset_probe.py [instances] [steps]"""
import os
import sys
import time

import numpy as np
import torch

os.environ.setdefault("TD_PLACEMENT_TRIALS", "1")

sys.path.insert(0, ".")
from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402

K, B = 6144, 4096
ninst = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
offsets = [0, 4096, 65536, 1 << 20, 2 << 20, 3 << 20, 32 << 20, 128 << 20, 0]
dev = torch.device("cuda", 0)
u, llr_h = synth.make_batch(B, K, 263, 480, 1.0, seed=20261015, dtype=np.float64)
llr = torch.from_numpy(llr_h).to(dev)
bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
keep = []
for i in range(ninst):
    codec = TurboCodec(K, 263, 480, iterations=8, algo="logmap", precision="f64", device=0)
    codec.reserve(B)
    row = []
    for off in offsets:
        os.environ["TD_WS_OFFSET"] = str(off)
        codec.decode(llr, bits)
        torch.cuda.synchronize(dev)
        codec.profile(True)
        for _ in range(steps):
            codec.decode(llr, bits)
        torch.cuda.synchronize(dev)
        _, kms, _ = codec.kernel_ms()
        codec.profile(False)
        row.append("%d:%.2f" % (off >> 10, kms))
    print("instance", i, "offset KiB:kernel ms", " ".join(row), flush=True)
    keep.append(codec)
