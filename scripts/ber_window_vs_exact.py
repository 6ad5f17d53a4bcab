"""Config 5's BER gate (BASELINE north_star: "BER-vs-Eb/N0 within 0.05 dB of the CPU reference").

Paired Monte-Carlo on the GPU: at every Eb/N0 point the SAME frames of main.cpp's stream
(srand(seed + point), the device generator, bit-identical to the reference's frames) go through
the exact schedule (log_map.cpp's arithmetic, bit-exact against the compiled reference) and
through the windowed schedule (td_set_window), both fp64 table log-MAP, K=6144, 8 iterations.
A fixed frame count per point (no early stop) keeps the two sides on identical inputs, so the
difference in bit and block errors is the schedule's alone.  Writes one JSON record with the
per-point counts and the Eb/N0 where each curve crosses BER 1e-3 and 1e-4 (log-linear
interpolation between neighbouring points, as the reference's published curve is read).

    python scripts/ber_window_vs_exact.py --out gpurun_out/ber_window_vs_exact.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from turbo_decoder_cuda_amd.decoder import TurboCodec, stream_length  # noqa: E402


def crossing(ebn0, ber, target):
    """Eb/N0 where the curve first falls through `target` (log-linear between the two points)."""
    for i in range(1, len(ebn0)):
        a, b = ber[i - 1], ber[i]
        if a >= target > b:
            if b <= 0:
                return ebn0[i]
            t = (math.log(a) - math.log(target)) / (math.log(a) - math.log(b))
            return ebn0[i - 1] + t * (ebn0[i] - ebn0[i - 1])
    return None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--f1", type=int, default=263)
    ap.add_argument("--f2", type=int, default=480)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--window", type=int, default=64)
    ap.add_argument("--overlap", type=int, default=30)
    ap.add_argument("--nii", action="store_true")
    ap.add_argument("--ebn0", type=float, nargs="+",
                    default=[0.0, 0.1, 0.2, 0.25, 0.3, 0.325, 0.35, 0.375, 0.4, 0.425, 0.45, 0.5, 0.6])
    ap.add_argument("--frames", type=int, default=131072, help="frames per point")
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--seed", type=int, default=20261018)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)

    import torch

    dev = torch.device("cuda", 0)
    n = stream_length(a.K)
    B = min(a.batch, a.frames)
    info = torch.empty((B, a.K), dtype=torch.uint8, device=dev)
    llr = torch.empty((B, n), dtype=torch.float64, device=dev)
    bits = torch.empty((B, a.iters, a.K), dtype=torch.uint8, device=dev)
    rec = {"K": a.K, "iters": a.iters, "window": a.window, "overlap": a.overlap, "nii": a.nii,
           "algo": "logmap", "precision": "f64", "frames_per_point": a.frames, "seed": a.seed, "points": []}
    t0 = time.time()
    with TurboCodec(a.K, a.f1, a.f2, iterations=a.iters) as ex, \
            TurboCodec(a.K, a.f1, a.f2, iterations=a.iters) as win:
        win.set_window(a.window, a.overlap, nii=a.nii)
        for pi, e in enumerate(a.ebn0):
            ex.synth_seed(a.seed + pi)
            cnt = {s: {"bit": [0] * a.iters, "block": [0] * a.iters} for s in ("exact", "window")}
            differ = 0
            done = 0
            while done < a.frames:
                b = min(B, a.frames - done)
                ex.synth(b, e, info[:b], llr[:b])
                per = {}
                for name, c in (("exact", ex), ("window", win)):
                    c.decode(llr[:b], bits[:b], all_iters=True)
                    err = c.count_errors(bits[:b], info[:b]).cpu()
                    per[name] = err[:, -1].clone()
                    for it in range(a.iters):
                        cnt[name]["bit"][it] += int(err[:, it].sum())
                        cnt[name]["block"][it] += int((err[:, it] != 0).sum())
                differ += int(((per["exact"] != 0) != (per["window"] != 0)).sum())
                done += b
            bits_total = a.frames * a.K
            pt = {"ebn0_db": e, "frames": a.frames,
                  "exact": cnt["exact"], "window": cnt["window"],
                  "ber_exact": cnt["exact"]["bit"][-1] / bits_total,
                  "ber_window": cnt["window"]["bit"][-1] / bits_total,
                  "bler_exact": cnt["exact"]["block"][-1] / a.frames,
                  "bler_window": cnt["window"]["block"][-1] / a.frames,
                  "frames_error_state_differs": differ}
            rec["points"].append(pt)
            print(f"Eb/N0 {e:.3f}: BER exact {pt['ber_exact']:.3e} window {pt['ber_window']:.3e}  "
                  f"bits {cnt['exact']['bit'][-1]} / {cnt['window']['bit'][-1]}  "
                  f"blocks {cnt['exact']['block'][-1]} / {cnt['window']['block'][-1]}  "
                  f"({time.time() - t0:.0f} s)", flush=True)
    eb = [p["ebn0_db"] for p in rec["points"]]
    for tgt in (1e-3, 1e-4, 1e-5):
        ce = crossing(eb, [p["ber_exact"] for p in rec["points"]], tgt)
        cw = crossing(eb, [p["ber_window"] for p in rec["points"]], tgt)
        rec[f"crossing_{tgt:.0e}"] = {"exact_db": ce, "window_db": cw,
                                      "delta_db": (cw - ce) if ce is not None and cw is not None else None}
        print(f"BER {tgt:.0e}: exact {ce} dB, window {cw} dB", flush=True)
    rec["wall_s"] = round(time.time() - t0, 1)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
