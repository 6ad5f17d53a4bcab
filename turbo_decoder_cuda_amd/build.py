"""Build the native libraries in-tree (hipcc, gfx950).  No torch extension machinery: the
product is a plain C-ABI shared library (include/turbo_mi355x.h)."""
from __future__ import annotations

import concurrent.futures
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
DROPIN = os.path.join(PKG, "td_dropin_latency")   # examples/dropin_latency.cpp

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


def _run_hip(cmd, verbose):
    """hipcc with the kernel resource report: a kernel that uses scratch is a build error.
    The turbo kernel's loader counts its vector-memory operations by hand (s_waitcnt vmcnt(N)),
    and a runtime-indexed array the compiler moved to scratch has also faulted it on the GPU."""
    cmd = cmd + ["-Rpass-analysis=kernel-resource-usage"]
    print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
    if verbose or r.returncode:
        sys.stderr.write(r.stderr)
    if r.returncode:
        raise subprocess.CalledProcessError(r.returncode, cmd)
    name, bad = None, []
    for line in r.stderr.splitlines():
        if "Function Name:" in line:
            name = line.split("Function Name:")[1].split("[")[0].strip()
        elif "ScratchSize [bytes/lane]:" in line:
            n = int(line.split("ScratchSize [bytes/lane]:")[1].split("[")[0])
            if n:
                bad.append(f"{name} ({n} B/lane)")
    if bad:
        raise RuntimeError("kernels use scratch: " + ", ".join(bad))


def _workers(n: int) -> int:
    """Parallel hipcc jobs: each whole-kernel compile takes a few GB; keep to the memory at hand."""
    try:
        avail = os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE") / 2**30
    except (ValueError, OSError):
        avail = 8.0
    return max(1, min(n, int(avail // 6)))


# td_kernels_win.hip (the sub-block schedule) under the max-ILP machine scheduler: +1.4 % at BASELINE
# config 5; the exact kernels (td_kernels.hip) lose 1 % under it and keep the default.
WIN_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
SRCS = ("td_kernels.hip", "td_kernels_w12.hip", "td_kernels_win.hip", "td_synth.hip", "td_api.cpp")
FILE_FLAGS = {"td_kernels_win.hip": WIN_FLAGS}


def lib_jobs(out: str, flags, verbose: bool = False):
    """The compile commands of one library build (one object per source, each with its own flags)
    and its link command.  Objects go to <out>.objs/ (git- and gpurun-ignored)."""
    odir = out + ".objs"
    os.makedirs(odir, exist_ok=True)
    objs, comp = [], []
    for f in SRCS:
        o = os.path.join(odir, f.rsplit(".", 1)[0] + ".o")
        objs.append(o)
        comp.append(([HIPCC, f"--offload-arch={ARCH}", *COMMON, *flags, *FILE_FLAGS.get(f, []), "-c", "-o", o,
                      os.path.join(CSRC, f)], verbose and f == "td_kernels.hip"))
    link = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", out, *objs]
    return comp, link


def build_lib(out: str, flags, verbose: bool = False) -> None:
    """One library from the sources with extra flags (scripts/build_variants.sh)."""
    comp, link = lib_jobs(out, flags, verbose)
    with concurrent.futures.ThreadPoolExecutor(max_workers=_workers(len(comp))) as ex:
        for f in [ex.submit(_run_hip, cmd, v) for cmd, v in comp]:
            f.result()
    _run(link)


def build(force: bool = False, verbose: bool = False, extra: bool = True) -> None:
    """The product library, the compat layer and the drop-in driver.  extra: also the two test /
    diagnostic builds of the same sources (libturbo_mi355x_redo.so, which every log-MAP alpha window
    takes the speculation's exact redo in, for test_alpha_speculation_redo_path_is_exact; and the
    stamps build for scripts/diag_stamps.py).  __graft_entry__.build() asks for them, as the GPU
    tests load the redo build."""
    srcs = [os.path.join(CSRC, f) for f in SRCS]
    deps = srcs + [os.path.join(CSRC, f) for f in ("td_kernels.h", "td_tables.h")] + [os.path.join(INC, "turbo_mi355x.h"),
                                                                                       __file__]
    stamps = os.path.join(PKG, "libturbo_mi355x_stamps.so")   # diagnostic build (phase cycle stamps)
    redo = os.path.join(PKG, "libturbo_mi355x_redo.so")       # test build: every log-MAP alpha window takes
    comp, links = [], []                                       # the speculation's exact redo (test_gpu_decode)
    for out, flags in ((LIB, []), (stamps, ["-DTD_STAMPS"]), (redo, ["-DTD_ASPEC_REDO"])):
        if out != LIB and not extra:
            continue
        if force or _newer(out, deps):
            c, l = lib_jobs(out, flags, verbose and out == LIB)
            comp += c
            links.append(l)
    # the compiles are independent: run them side by side, as memory allows
    with concurrent.futures.ThreadPoolExecutor(max_workers=_workers(len(comp) or 1)) as ex:
        for f in [ex.submit(_run_hip, cmd, v) for cmd, v in comp]:
            f.result()
    for l in links:
        _run(l)
    csrc = os.path.join(CSRC, "log_map_compat.cpp")
    if os.path.exists(csrc) and (force or _newer(COMPAT, [csrc, LIB, os.path.join(INC, "turbo_mi355x.h")])):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", f"-I{INC}", "-shared", "-o", COMPAT, csrc,
              f"-L{PKG}", "-lturbo_mi355x", "-Wl,-rpath,$ORIGIN"])
    # the unchanged caller's per-frame latency through the drop-in (bench.py `dropin`)
    drv = os.path.join(REPO, "examples", "dropin_latency.cpp")
    if os.path.exists(drv) and (force or _newer(DROPIN, [drv, COMPAT])):
        _run(["g++", "-O2", "-std=c++17", "-o", DROPIN, drv, f"-L{PKG}", "-lturbo_logmap_compat", "-lturbo_mi355x",
              "-Wl,-rpath,$ORIGIN"])


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose="-v" in sys.argv, extra="--no-extra" not in sys.argv)
