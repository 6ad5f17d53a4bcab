"""Config 5's BER gate (BASELINE north_star: "BER-vs-Eb/N0 within 0.05 dB of the CPU reference").

Paired Monte-Carlo on the GPU: at every Eb/N0 point the SAME frames of main.cpp's stream
(srand(seed + point), the device generator, bit-identical to the reference's frames) go through
the exact schedule (log_map.cpp's arithmetic, bit-exact against the compiled reference) and
through the windowed schedule (td_set_window) with each max* form (td_set_window_maxstar: the
one-read table "window" and log_map.cpp's E_algorithm "window_exact_table"), all fp64 log-MAP,
K=6144, 8 iterations.
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
    names = ("exact", "window", "window_exact_table")
    with TurboCodec(a.K, a.f1, a.f2, iterations=a.iters) as ex, \
            TurboCodec(a.K, a.f1, a.f2, iterations=a.iters) as win, \
            TurboCodec(a.K, a.f1, a.f2, iterations=a.iters) as winx:
        win.set_window(a.window, a.overlap, nii=a.nii)
        winx.set_window_maxstar(True)
        winx.set_window(a.window, a.overlap, nii=a.nii)
        for pi, e in enumerate(a.ebn0):
            ex.synth_seed(a.seed + pi)
            cnt = {s: {"bit": [0] * a.iters, "block": [0] * a.iters} for s in names}
            differ = 0
            done = 0
            while done < a.frames:
                b = min(B, a.frames - done)
                ex.synth(b, e, info[:b], llr[:b])
                per = {}
                for name, c in zip(names, (ex, win, winx)):
                    c.decode(llr[:b], bits[:b], all_iters=True)
                    err = c.count_errors(bits[:b], info[:b]).cpu()
                    per[name] = err[:, -1].clone()
                    for it in range(a.iters):
                        cnt[name]["bit"][it] += int(err[:, it].sum())
                        cnt[name]["block"][it] += int((err[:, it] != 0).sum())
                differ += int(((per["exact"] != 0) != (per["window"] != 0)).sum())
                done += b
            bits_total = a.frames * a.K
            pt = {"ebn0_db": e, "frames": a.frames, "frames_error_state_differs": differ}
            for n_ in names:
                pt[n_] = cnt[n_]
                pt[f"ber_{n_}"] = cnt[n_]["bit"][-1] / bits_total
                pt[f"bler_{n_}"] = cnt[n_]["block"][-1] / a.frames
            rec["points"].append(pt)
            print(f"Eb/N0 {e:.3f}: BER " + "  ".join(f"{n_} {pt['ber_' + n_]:.3e}" for n_ in names) +
                  "  bits " + " / ".join(str(cnt[n_]["bit"][-1]) for n_ in names) +
                  "  blocks " + " / ".join(str(cnt[n_]["block"][-1]) for n_ in names) +
                  f"  ({time.time() - t0:.0f} s)", flush=True)
    eb = [p["ebn0_db"] for p in rec["points"]]
    for tgt in (1e-3, 1e-4, 1e-5):
        cr = {n_: crossing(eb, [p["ber_" + n_] for p in rec["points"]], tgt) for n_ in names}
        r = {f"{n_}_db": cr[n_] for n_ in names}
        for n_ in names[1:]:
            r[f"delta_{n_}_db"] = (cr[n_] - cr["exact"]) if cr[n_] is not None and cr["exact"] is not None else None
        rec[f"crossing_{tgt:.0e}"] = r
        print(f"BER {tgt:.0e}: " + ", ".join(f"{n_} {cr[n_]} dB" for n_ in names), flush=True)
    rec["wall_s"] = round(time.time() - t0, 1)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
