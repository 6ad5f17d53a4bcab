#!/usr/bin/env python3
"""Golden vectors for the modulators / demodulators from the COMPILED
REFERENCE (oracle/_ref/ref_harness: ITTC/modanddem.cpp + log_map.cpp, unmodified).

TEST INFRASTRUCTURE.  Run in the build container (needs /root/reference):
    make -C oracle ref && python oracle/gen_demod_golden.py
Fixtures (data only):
  demod.npz            : per M in {1,2,3,4,6}: yi, yq (every constellation point, decision-boundary
                         points, uniform [-2,2]^2) and demodule()'s LLRs (Kf = 1.7), modanddem.cpp:674
  modframes_K1024.npz : per M in {2,3,4,6}: main.cpp frames with MODULATION = M (SYMBOL_NUM =
                         (3K+12)/M), srand(5), Eb/N0 = 1.5 dB: src, flow (TurboDecoding's input)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(os.path.dirname(HERE), "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")


def run(args):
    subprocess.run([HARNESS] + [str(a) for a in args], check=True, capture_output=True, text=True)


def main():
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    d, nsym = {}, 600
    with tempfile.TemporaryDirectory() as td:
        for M in (1, 2, 3, 4, 6):
            p = os.path.join(td, f"d{M}.bin")
            run(["demod", M, nsym, 40 + M, p])
            v = np.fromfile(p, dtype="<f8")
            d[f"yi_{M}"], d[f"yq_{M}"], d[f"llr_{M}"] = v[:nsym], v[nsym:2 * nsym], v[2 * nsym:]
        np.savez_compressed(os.path.join(GOLD, "demod.npz"), Kf=1.7, **d)
        K, f1, f2, nf, n = 1024, 31, 64, 3, 3 * 1024 + 12
        fm = {}
        for M in (2, 3, 4, 6):
            p = os.path.join(td, f"f{M}.bin")
            run(["framesmod", K, f1, f2, M, 1.5, 5, nf, p])
            rec = np.dtype([("src", "<i4", K), ("flow", "<f8", n)])
            arr = np.fromfile(p, dtype=rec, count=nf)
            fm[f"src_{M}"] = arr["src"].astype(np.uint8)
            fm[f"flow_{M}"] = arr["flow"].copy()
        np.savez_compressed(os.path.join(GOLD, "modframes_K1024.npz"), K=K, f1=f1, f2=f2, ebn0=1.5, seed=5, **fm)
    for m in ("demod.npz", "modframes_K1024.npz"):
        print(m, os.path.getsize(os.path.join(GOLD, m)))


if __name__ == "__main__":
    sys.exit(main())
