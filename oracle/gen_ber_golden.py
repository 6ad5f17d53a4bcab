#!/usr/bin/env python3
"""BER/BLER fixtures from the COMPILED REFERENCE (oracle/_ref/ref_harness `ber` mode).

TEST INFRASTRUCTURE.  Run in the build container (needs /root/reference):
    make -C oracle ref && python oracle/gen_ber_golden.py
Each point: srand(seed); frames of main.cpp's generator decoded by the reference TurboDecoding
until the chosen iteration has `minerr` block errors or `maxframes` frames (main.cpp:172-243).
Writes tests/golden/ber_K{K}.json: per point the frame count and per-iteration (bit, block)
error counts of the reference's 15 iterations.
"""
from __future__ import annotations

import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")

# (K, f1, f2, iters, ebn0 list, maxframes, minerr, seed)
CASES = [
    (1024, 31, 64, 8, [0.0, 0.2, 0.4, 0.6, 0.8], 3000, 50, 2026),
    (6144, 263, 480, 8, [0.2, 0.3, 0.4], 400, 30, 7),
]


def run_point(K, f1, f2, iters, e, maxf, minerr, seed):
    out = subprocess.run([HARNESS, "ber", str(K), str(f1), str(f2), str(iters), repr(e), str(maxf), str(minerr),
                          str(seed)], check=True, capture_output=True, text=True).stdout.split()
    # "ebn0 <e> frames <n> b0:k0 b1:k1 ..."
    frames = int(out[3])
    pairs = [tuple(int(v) for v in t.split(":")) for t in out[4:]]
    return {"ebn0": e, "frames": frames, "bit_errors": [p[0] for p in pairs], "block_errors": [p[1] for p in pairs]}


def main():
    with ThreadPoolExecutor(max_workers=os.cpu_count() or 4) as ex:
        jobs = {}
        for (K, f1, f2, iters, pts, maxf, minerr, seed) in CASES:
            for e in pts:
                jobs[(K, e)] = ex.submit(run_point, K, f1, f2, iters, e, maxf, minerr, seed)
        for (K, f1, f2, iters, pts, maxf, minerr, seed) in CASES:
            res = {"K": K, "f1": f1, "f2": f2, "iters": iters, "maxframes": maxf, "minerr": minerr, "seed": seed,
                   "reseed_each_point": True, "points": [jobs[(K, e)].result() for e in pts]}
            with open(os.path.join(GOLD, f"ber_K{K}.json"), "w") as f:
                json.dump(res, f, indent=1)
            print(K, [(p["ebn0"], p["frames"], p["block_errors"][iters - 1]) for p in res["points"]])


if __name__ == "__main__":
    main()
