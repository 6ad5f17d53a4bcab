"""The exact kernel's fixed cost per SISO (prologue, pipeline fill and drain, the inter-SISO barrier),
by fitting its launch time over block sizes at config 2's batch and iterations:
t(K) = 2·iters·(a·(K + 3) + b).  a is the cost of a trellis step (F + B pass), b the SISO edge.

    python scripts/siso_edge_fit.py [--rounds 3]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from turbo_decoder_cuda_amd import TurboCodec  # noqa: E402

SIZES = [(512, 31, 64), (1024, 31, 64), (2048, 31, 64), (3072, 47, 96), (4096, 31, 64), (6144, 263, 480)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    import torch

    iters, B = 8, a.batch
    best = {}
    codecs = []
    for K, f1, f2 in SIZES:
        c = TurboCodec(K, f1, f2, iterations=iters)
        c.synth_seed(20261018)
        _, llr = c.synth(B, 1.0)
        c.reserve(B)
        bits = torch.empty((B, K), dtype=torch.uint8, device=llr.device)
        codecs.append((K, c, llr, bits))
    for r in range(a.rounds):
        for K, c, llr, bits in codecs:
            c.decode(llr, bits)
            torch.cuda.synchronize()
            c.profile(True)
            for _ in range(a.steps):
                c.decode(llr, bits)
            torch.cuda.synchronize()
            _, m, n = c.kernel_ms()
            c.profile(False)
            assert n == a.steps, n
            best[K] = min(best.get(K, 1e9), m)
            ghz = c.clock()[0]
            print(f"round {r} K {K:5d}: kernel {m:8.3f} ms at {ghz:.3f} GHz", flush=True)
    Ks = np.array(sorted(best), dtype=float)
    t = np.array([best[int(k)] for k in Ks])
    S = 2 * iters
    A = np.stack([S * (Ks + 3), np.full_like(Ks, S)], 1)
    (ca, cb), *_ = np.linalg.lstsq(A, t, rcond=None)
    print(f"fit: {ca * 1e6:.2f} ns a trellis step, {cb * 1e3:.2f} us a SISO edge; "
          f"edges at K=6144: {S * cb / best[6144] * 100:.2f} % of the launch")
    for k in Ks:
        print(f"  K {int(k):5d}: measured {best[int(k)]:8.3f} ms, fit {S * (ca * (k + 3) + cb):8.3f} ms")
    for _, c, _, _ in codecs:
        c.close()


if __name__ == "__main__":
    main()
