"""Which pass slows down in the slow placement mode?  (GPU box; the TD_STAMPS library, plain
allocations.)  For several fresh decoders of one process: kernel ms and the per-role cycles per
SISO-step of the F and B passes (work / barrier wait), as scripts/diag_stamps.py prints them.
python scripts/stamps_modes.py [instances]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TD_LIB_PATH"] = os.path.join(REPO, "turbo_decoder_cuda_amd", "libturbo_mi355x_stamps.so")
os.environ.setdefault("TD_PLACEMENT_TRIALS", "1")
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402
from turbo_decoder_cuda_amd import _native as N  # noqa: E402

K, B, iters = 6144, 4096, 8
ninst = int(sys.argv[1]) if len(sys.argv) > 1 else 6
u, llr = synth.make_batch(B, K, 263, 480, 1.0, dtype=np.float64)
x = torch.from_numpy(llr).cuda()
slots = N.lib().td_debug_stamp_slots()
G = (B + 7) // 8
steps = 2 * iters * (K + 3)
keep = []
for i in range(ninst):
    c = TurboCodec(K, 263, 480, iterations=iters)
    c.reserve(B)
    st = torch.zeros((G, slots), dtype=torch.int64, device="cuda")
    N.check(N.lib().td_debug_set_stamps(c._h, C.c_void_p(st.data_ptr())))
    c.decode(x)
    torch.cuda.synchronize()
    c.profile(True)
    c.decode(x)
    _, kms, _ = c.kernel_ms()
    s = st.cpu().numpy().reshape(G, 4, slots // 4).astype(np.float64)
    row = " ".join(f"{nm}: F {s[:, w, 0].mean() / steps:5.1f}+{s[:, w, 1].mean() / steps:5.1f} "
                   f"B {s[:, w, 2].mean() / steps:5.1f}+{s[:, w, 3].mean() / steps:5.1f}"
                   for w, nm in enumerate(("A", "B", "F0", "F1")))
    print(f"instance {i}: {kms:.2f} ms  {row}  chains: alpha {s[:, 0, 4].mean() / steps:5.1f} beta {s[:, 1, 4].mean() / steps:5.1f}",
          flush=True)
    keep.append((c, st))
