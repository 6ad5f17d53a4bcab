"""Heuristic check of the loader's hand-counted vector-memory waits (td_kernels.hip, TileRegs/TmRegs).

The loader issues its global loads through inline asm, so the compiler believes each destination
register holds its value at issue, while the hardware writes it when the load returns.  A
compiler-generated instruction that names such a register before the asm `s_waitcnt vmcnt(N)`
that retires the load (a register-allocation copy, a reuse as a temporary) reads garbage or is
overwritten; a garbage extrinsic write position then faults the GPU.

This scans each kernel's assembly in program order (branches not followed): for every asm
`global_load_*` it tracks the destination registers until a following vmcnt wait retires the
load, and counts every other instruction in between that names one of them.  Program order
crosses the loader's loop edges, so a correct build has a baseline of such counts (v11: 52, 52,
58, 54 for turbo_decode_kernel<f64|f32, log-MAP|max-log>); a build that faulted on the GPU
(a two-window loader pipeline, since reverted) showed 192 for the fp32 max-log kernel.  Compare
a changed kernel's counts with the baseline before running it.
Usage: python scripts/check_asm_loads.py file.s [kernel-name-substring ...]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def retire(inflight, s):
    m = re.search(r"vmcnt\((\d+)\)", s)
    if not m:
        return inflight
    n = int(m.group(1))
    return inflight[len(inflight) - n:] if 0 < n < len(inflight) else ([] if n == 0 else inflight)


def check(lines):
    issues, inflight, in_asm = [], [], False
    for ln, raw in enumerate(lines):
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(";") or s.endswith(":") or s.startswith("."):
            continue
        op = s.split()[0]
        if in_asm:
            if op.startswith("global_load_lds"):
                inflight.append((set(), ln))
            elif op.startswith("global_load"):
                inflight.append((regs(s.split(None, 1)[1].split(",")[0]), ln))
            elif op == "s_waitcnt":
                inflight = retire(inflight, s)
            continue
        if op == "s_waitcnt":
            inflight = retire(inflight, s)
            continue
        if op.startswith("s_endpgm"):
            break
        named = regs(s)
        for dst, iln in inflight:
            if named & dst:
                issues.append(f"line {ln + 1}: '{s}' names v{sorted(named & dst)} of the asm load at line {iln + 1}")
    return issues


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    text = open(path).read().splitlines()
    starts = [(i, l[:-1].split()[0]) for i, l in enumerate(text) if re.match(r"^_Z\w+:", l)]
    for k, (i, name) in enumerate(starts):
        if subs and not any(x in name for x in subs):
            continue
        end = starts[k + 1][0] if k + 1 < len(starts) else len(text)
        print(f"{len(check(text[i:end])):5d}  {name}")


if __name__ == "__main__":
    main()
