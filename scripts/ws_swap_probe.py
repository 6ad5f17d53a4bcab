"""Which workspace array carries the placement mode?  (GPU box, a -DTD_WS_EXPERIMENT build via
TD_LIB_PATH, TD_PLACEMENT_TRIALS=1.)  Creates decoders until it has one in the slow and one in the
fast mode, then swaps one array (or handle table) at a time between them and times both: the array
whose swap moves the slowness from one decoder to the other is the one whose physical pages matter.
python scripts/ws_swap_probe.py [max_instances] [steps]"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

os.environ.setdefault("TD_PLACEMENT_TRIALS", "1")
sys.path.insert(0, ".")
from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402
from turbo_decoder_cuda_amd import _native as N  # noqa: E402

K, B = 6144, 4096
nmax = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
u, llr_h = synth.make_batch(B, K, 263, 480, 1.0, seed=20261015, dtype=np.float64)
llr = torch.from_numpy(llr_h).to(dev)
bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
L = N.lib()
L.td_debug_swap_arrays.argtypes = [C.c_void_p, C.c_void_p, C.c_int]


def kms(c):
    c.decode(llr, bits)
    torch.cuda.synchronize(dev)
    c.profile(True)
    for _ in range(steps):
        c.decode(llr, bits)
    torch.cuda.synchronize(dev)
    _, t, _ = c.kernel_ms()
    c.profile(False)
    return t


codecs, times = [], []
for i in range(nmax):
    c = TurboCodec(K, 263, 480, iterations=8, device=0)
    c.reserve(B)
    codecs.append(c)
    times.append(kms(c))
    print("instance", i, "%.2f ms" % times[-1], flush=True)
    if max(times) > 1.04 * min(times):
        break
if max(times) <= 1.04 * min(times):
    print("no two modes among", len(times), "instances")
    sys.exit(0)
S, F = codecs[int(np.argmax(times))], codecs[int(np.argmin(times))]
names = ["sys1", "par1", "sys2", "par2", "ext12", "ext21", "astore", "tmstore", "pi+pinv", "lut+lane+slots"]
print("slow %.2f fast %.2f" % (kms(S), kms(F)), flush=True)
for i, nm in enumerate(names):
    N.check(L.td_debug_swap_arrays(S._h, F._h, 1 << i))
    a, b = kms(S), kms(F)
    N.check(L.td_debug_swap_arrays(S._h, F._h, 1 << i))
    print("swap %-15s slow-handle %.2f fast-handle %.2f" % (nm, a, b), flush=True)
N.check(L.td_debug_swap_arrays(S._h, F._h, 0xFF))
print("swap %-15s slow-handle %.2f fast-handle %.2f" % ("all arrays", kms(S), kms(F)), flush=True)
N.check(L.td_debug_swap_arrays(S._h, F._h, 0xFF))
errs = int((bits.cpu().numpy() != u).sum())
print("bit errors after the swaps", errs)
