"""Run-to-run spread probe (GPU box): several decoder instances in ONE process (each reserve() is a
fresh workspace allocation), several timed batches per instance.  Separates per-allocation effects
(spread between instances, stable within one) from dynamic ones (spread within an instance).
python scripts/spread_probe.py [instances] [batches] [steps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402

K, B = 6144, 4096
ninst = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nbat = int(sys.argv[2]) if len(sys.argv) > 2 else 4
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dev = torch.device("cuda", 0)
u, llr_h = synth.make_batch(B, K, 263, 480, 1.0, seed=20261015, dtype=np.float64)
llr = torch.from_numpy(llr_h).to(dev)
bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
keep = []
for i in range(ninst):
    codec = TurboCodec(K, 263, 480, iterations=8, algo="logmap", precision="f64", device=0)
    codec.reserve(B)
    codec.decode(llr, bits)
    torch.cuda.synchronize(dev)
    row = []
    for b in range(nbat):
        codec.profile(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            codec.decode(llr, bits)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        _, turbo_ms, _n = codec.kernel_ms()
        codec.profile(False)
        row.append("%.2f/%.0f" % (turbo_ms, B * K * steps / dt / 1e6))
    errs = int((bits.cpu().numpy() != u).sum())
    print("instance", i, "kernel_ms/Mbps per batch:", " ".join(row), "placement", codec.placement(), "bit errors", errs,
          flush=True)
    keep.append(codec)   # keep the workspace so the next instance gets another allocation
