"""Are the placement modes a property of the memory itself or of the decode's access pattern?
(GPU box, a -DTD_WS_EXPERIMENT build via TD_LIB_PATH, TD_PLACEMENT_TRIALS=1.)  For several fresh
decoders: the decode's kernel time (its mode) and the bandwidth of a plain device-to-device copy
between the two halves of the same workspace allocation (hipMemcpyAsync, streaming).  If the slow
decoders also copy slower, the slow allocations reach fewer HBM channels; if not, the mode belongs
to the decode's strided access pattern on those pages.
python scripts/ws_copy_probe.py [instances]"""
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
ninst = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
u, llr_h = synth.make_batch(B, K, 263, 480, 1.0, seed=20261015, dtype=np.float64)
llr = torch.from_numpy(llr_h).to(dev)
bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
L = N.lib()
L.td_debug_ws.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]


def copy_gbs(ptr, off, nbytes, reps=5):
    stream = torch.cuda.current_stream(dev).cuda_stream
    half = nbytes // 2
    src, dst = ptr + off, ptr + off + half
    hip.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), half, 3, C.c_void_p(stream))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        hip.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), half, 3, C.c_void_p(stream))
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / reps
    return 2 * half / dt / 1e9   # read + write


keep = []
for i in range(ninst):
    c = TurboCodec(K, 263, 480, iterations=8, device=0)
    c.reserve(B)
    c.decode(llr, bits)
    torch.cuda.synchronize(dev)
    c.profile(True)
    for _ in range(3):
        c.decode(llr, bits)
    torch.cuda.synchronize(dev)
    _, kms, _ = c.kernel_ms()
    c.profile(False)
    p, nb, aoff = C.c_void_p(), C.c_size_t(), C.c_size_t()
    N.check(L.td_debug_ws(c._h, C.byref(p), C.byref(nb), C.byref(aoff)))
    whole = copy_gbs(p.value, 0, nb.value)
    astore_bytes = nb.value - aoff.value
    alpha = copy_gbs(p.value, aoff.value, astore_bytes)
    print(f"instance {i}: decode {kms:.2f} ms   copy whole workspace {whole:7.0f} GB/s   copy alpha+tm region {alpha:7.0f} GB/s",
          flush=True)
    keep.append(c)
