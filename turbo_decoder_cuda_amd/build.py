"""Build the native libraries in-tree (hipcc, gfx950).  No torch extension machinery: the
product is a plain C-ABI shared library (include/turbo_mi355x.h)."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(REPO, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB = os.path.join(PKG, "libturbo_mi355x.so")
COMPAT = os.path.join(PKG, "libturbo_logmap_compat.so")

# -ffp-contract=off: the parity mode reproduces the reference's operation order exactly.
# -fno-honor-nans: the decoder never produces a NaN from finite channel LLRs; without it hipcc
# canonicalises every DPP-moved operand (an extra v_max_f64 x,x) before each fmax.
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-honor-nans", f"-I{INC}", f"-I{CSRC}"]


def _newer(out: str, srcs) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force: bool = False, verbose: bool = False) -> None:
    srcs = [os.path.join(CSRC, f) for f in ("td_kernels.hip", "td_synth.hip", "td_api.cpp")]
    deps = srcs + [os.path.join(CSRC, f) for f in ("td_kernels.h", "td_tables.h")] + [os.path.join(INC, "turbo_mi355x.h")]
    if force or _newer(LIB, deps):
        extra = ["-Rpass-analysis=kernel-resource-usage"] if verbose else []
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, *extra, "-shared", "-o", LIB, *srcs])
    stamps = os.path.join(PKG, "libturbo_mi355x_stamps.so")   # diagnostic build (phase cycle stamps)
    if force or _newer(stamps, deps):
        _run([HIPCC, f"--offload-arch={ARCH}", *COMMON, "-DTD_STAMPS", "-shared", "-o", stamps, *srcs])
    csrc = os.path.join(CSRC, "log_map_compat.cpp")
    if os.path.exists(csrc) and (force or _newer(COMPAT, [csrc, LIB, os.path.join(INC, "turbo_mi355x.h")])):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", f"-I{INC}", "-shared", "-o", COMPAT, csrc,
              f"-L{PKG}", "-lturbo_mi355x", "-Wl,-rpath,$ORIGIN"])


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose="-v" in sys.argv)
