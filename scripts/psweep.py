"""Reproduce the reference's published P sweep on the GPU.

The reference GPU decoder (ITTC/CUDA/turboDecoderBianJieZhi.cu: Max-Log-MAP fp32, P sub-blocks of
6144/P steps, NII boundaries, concurrent SISOs, extrinsic x0.77) was run for P = 32..128 at
Eb/N0 0..1 dB, 10000 frames per point, 25 iterations (tests/golden/psweep_published.json).  This
runs the same schedule through td_set_window on main.cpp's frames (device generator, srand(seed))
and reports, per P and iteration, both BER curves and the Eb/N0 where each crosses 1e-3 / 1e-4
(log-linear interpolation).

    python scripts/psweep.py --frames 10000 --out gpurun_out/psweep.json
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def crossing(ebn0, ber, target):
    """Eb/N0 where the BER curve first falls to `target` (log-linear), or None."""
    for i in range(1, len(ber)):
        a, b = ber[i - 1], ber[i]
        if a > target >= b:
            if b <= 0:
                return ebn0[i]
            t = (math.log10(a) - math.log10(target)) / (math.log10(a) - math.log10(b))
            return ebn0[i - 1] + t * (ebn0[i] - ebn0[i - 1])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, nargs="+", default=[32, 48, 64, 96, 128])
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=25)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--batch", type=int, default=5000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from turbo_decoder_cuda_amd import TurboCodec
    from turbo_decoder_cuda_amd.ber import ber_sweep

    pub = json.load(open(os.path.join(REPO, "tests", "golden", "psweep_published.json")))
    ebn0, e = [], 0.0
    while e <= 1.0:   # main's loop accumulates the Eb/N0 this way
        ebn0.append(e)
        e += 0.1
    res = {"frames_per_point": a.frames, "iterations": a.iters, "seed": a.seed, "ebn0_db": ebn0, "P": {}}
    for P in a.P:
        t0 = time.time()
        with TurboCodec(6144, 263, 480, iterations=a.iters, algo="maxlog", precision="f32") as c:
            c.set_window(6144 // P, 0, 0.77, nii=True, concurrent=True)
            pts = ber_sweep(c, ebn0, a.seed, a.frames, min_block_errors=0, batch=a.batch)
        ours = [[p.ber[it] for p in pts] for it in range(a.iters)]
        theirs = [[p["ber"][it] for p in pub["P"][str(P)]] for it in range(a.iters)]
        rows = {}
        for it in range(a.iters):
            rows[it + 1] = {"ber": ours[it], "published": theirs[it],
                            "x1e-3": [crossing(ebn0, ours[it], 1e-3), crossing(ebn0, theirs[it], 1e-3)],
                            "x1e-4": [crossing(ebn0, ours[it], 1e-4), crossing(ebn0, theirs[it], 1e-4)]}
        res["P"][P] = {"window": 6144 // P, "seconds": round(time.time() - t0, 2), "iters": rows}
        r = rows
        print(f"P={P:4d} W={6144 // P:4d}  " + "  ".join(
            f"it{it}: 1e-4 at {r[it]['x1e-4'][0] or float('nan'):.3f} vs {r[it]['x1e-4'][1] or float('nan'):.3f} dB"
            for it in (6, 8, 10, 15, 25) if it <= a.iters), flush=True)
    if a.out:
        with open(a.out, "w") as fp:
            json.dump(res, fp)


if __name__ == "__main__":
    main()
