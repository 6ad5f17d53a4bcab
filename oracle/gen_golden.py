#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the COMPILED REFERENCE (oracle/_ref/ref_harness).

TEST INFRASTRUCTURE.  Run in the build container (needs /root/reference):
    make -C oracle ref && python oracle/gen_golden.py
Each fixture holds inputs and the reference's outputs only (data, no reference source).

Fixtures
  frames_K{K}_e{ebn0}_s{seed}.npz : src, flow (channel LLR fed to TurboDecoding), le[iters,2,L]
                                    (extrinsic after SISO1/SISO2, log_map.cpp:1234-1238,1255-1259),
                                    bits[iters,K] (flow_decoded rows) -- main.cpp frames, srand(seed)
  siso_L{L}_t{term}.npz           : recs, La, LLR of one Log_MAP_decoder call (log_map.cpp:898)
  maxstar.npz                     : x, y, E_algorithm(x, y) incl. threshold edges (log_map.cpp:779)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
HARNESS = os.path.join(HERE, "_ref", "ref_harness")

# (K, f1, f2, ebn0, seed, nframes, iters, le_dtype)
FRAME_CASES = [
    (1024, 31, 64, 0.0, 11, 1, 8, np.float64),
    (1024, 31, 64, 0.5, 11, 1, 8, np.float64),
    (1024, 31, 64, 1.0, 11, 1, 8, np.float64),
    (1024, 31, 64, 0.0, 12, 1, 8, np.float64),
    (1024, 31, 64, 0.5, 12, 1, 8, np.float64),
    (1024, 31, 64, 1.0, 12, 1, 8, np.float64),
    (6144, 263, 480, 0.3, 21, 1, 8, np.float32),
    (6144, 263, 480, 1.0, 21, 1, 8, np.float32),
    (40, 3, 10, 0.0, 31, 4, 8, np.float64),      # smallest LTE QPP size (36.212 Table 5.1.3-3)
    # round 3: trellis lengths below one kernel window (L = 11) and at the reference's capacity
    # (MAX_FRAME_LENGTH 10000, log_map.h:31), with QPP parameters that give permutations there
    (8, 1, 2, 0.5, 41, 2, 4, np.float64),
    (24, 1, 6, 0.5, 42, 2, 4, np.float64),
    (10000, 1, 10, 0.8, 43, 1, 4, np.float32),
    # round 4: trellis lengths L = K+3 at the 15-step window's edge residues -- L = 0 mod 15 (a full
    # last window, no partial-window loop: K = 72, 432) and L = 1 mod 15 (a one-step last window:
    # K = 88) -- with their 36.212 Table 5.1.3-3 parameters
    (72, 7, 18, 0.5, 44, 3, 4, np.float64),
    (88, 5, 22, 0.5, 45, 3, 4, np.float64),
    (432, 47, 72, 0.8, 46, 2, 4, np.float64),
    # round 5: more K = 6144 frames (the benchmark size had two frames of one seed): two seeds, two
    # frames each, below and above the waterfall
    (6144, 263, 480, 0.0, 22, 2, 8, np.float32),
    (6144, 263, 480, 0.6, 23, 2, 8, np.float32),
]


def run(args):
    out = subprocess.run([HARNESS] + [str(a) for a in args], check=True, capture_output=True, text=True)
    return out.stdout


def gen_frames(K, f1, f2, ebn0, seed, nf, iters, le_dtype):
    L, n = K + 3, 3 * K + 12
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "f.bin")
        log = run(["frames", K, f1, f2, ebn0, seed, nf, iters, path])
        assert "mismatching_rows 0" in log, log
        raw = open(path, "rb").read()
    rec = np.dtype([("src", "<i4", K), ("flow", "<f8", n), ("le", "<f8", (iters, 2, L)), ("bits", "<i4", (iters, K))])
    arr = np.frombuffer(raw, dtype=rec, count=nf)
    name = f"frames_K{K}_e{ebn0:.1f}_s{seed}.npz"
    np.savez_compressed(
        os.path.join(GOLD, name),
        K=K, f1=f1, f2=f2, ebn0=ebn0, seed=seed, iters=iters,
        src=arr["src"].astype(np.uint8),
        flow=arr["flow"].copy(),
        le=arr["le"].astype(le_dtype),
        bits=arr["bits"].astype(np.uint8),
    )
    return name


def gen_siso(L, term, seed):
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "s.bin")
        run(["siso", L, term, seed, path])
        raw = np.fromfile(path, dtype="<f8")
    recs, La, LLR = raw[: 2 * L], raw[2 * L: 3 * L], raw[3 * L:]
    name = f"siso_L{L}_t{term}.npz"
    np.savez_compressed(os.path.join(GOLD, name), L=L, terminated=term, recs=recs, La=La, LLR=LLR)
    return name


def gen_maxstar(n, seed):
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "m.bin")
        run(["maxstar", n, seed, path])
        raw = open(path, "rb").read()
    m = np.frombuffer(raw[:4], dtype="<i4")[0]
    v = np.frombuffer(raw[4:], dtype="<f8")
    np.savez_compressed(os.path.join(GOLD, "maxstar.npz"), x=v[:m], y=v[m: 2 * m], r=v[2 * m:])
    return "maxstar.npz"


def main():
    """All fixtures; with arguments `frames K:seed ...`, only those frame fixtures (the others keep
    their bytes)."""
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
    os.makedirs(GOLD, exist_ok=True)
    if len(sys.argv) > 2 and sys.argv[1] == "frames":
        want = {tuple(int(v) for v in a.split(":")) for a in sys.argv[2:]}
        made = [gen_frames(*c) for c in FRAME_CASES if (c[0], c[4]) in want]
    else:
        made = [gen_maxstar(2000, 7), gen_siso(1027, 1, 5), gen_siso(1027, 0, 6), gen_siso(43, 1, 8)]
        for case in FRAME_CASES:
            made.append(gen_frames(*case))
    for m in made:
        print(m, os.path.getsize(os.path.join(GOLD, m)))


if __name__ == "__main__":
    sys.exit(main())
