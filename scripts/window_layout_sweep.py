"""Layout sweep of the windowed kernels at BASELINE config 5 (K=6144, 8 iterations, W=64, overlap 30,
batch 32768, fp64 log-MAP): sub-blocks per lane run of the beta and alpha kernels and batch parts
(td_debug_window_layout; results do not depend on them, speed does).  One process, one frame batch,
interleaved rounds; prints Mbit/s per layout.

    python scripts/window_layout_sweep.py [--exact-table] [--rounds 2]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from turbo_decoder_cuda_amd import TurboCodec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--exact-table", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--layouts", default="0:0:0,12:0:0,16:0:0,20:0:0,24:0:0,32:0:0,24:12:0,24:16:0,24:32:0,24:0:3")
    a = ap.parse_args()
    import torch

    K, B, iters = 6144, 32768, 8
    layouts = [tuple(int(v) for v in s.split(":")) for s in a.layouts.split(",")]
    with TurboCodec(K, 263, 480, iterations=iters) as c:
        c.synth_seed(20261015)
        info, llr = c.synth(B, 1.0)
        c.set_window_maxstar(a.exact_table)
        c.set_window(64, 30)
        c.reserve(B)
        bits = torch.empty((B, K), dtype=torch.uint8, device=llr.device)
        ref = None
        for r in range(a.rounds):
            for (run, run_a, parts) in layouts:
                c.debug_window_layout(run, run_a, parts)
                c.decode(llr, bits)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    c.decode(llr, bits)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.steps
                h = int(bits.sum().item())
                ref = h if ref is None else ref
                print(f"round {r} run {run:3d} run_a {run_a:3d} parts {parts}: {B * K / dt / 1e6:9.1f} Mbit/s "
                      f"({dt * 1e3:.2f} ms){'' if h == ref else '  BITS DIFFER'}", flush=True)


if __name__ == "__main__":
    main()
