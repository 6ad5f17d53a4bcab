"""Diagnostic: per-wave cycle split of the turbo kernel (TD_STAMPS build).
Usage on the GPU box: python scripts/diag_stamps.py [B] [precision] [algo]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TD_LIB_PATH"] = os.environ.get("TD_STAMPS_LIB") or os.path.join(REPO, "turbo_decoder_cuda_amd",
                                                                             "libturbo_mi355x_stamps.so")
sys.path.insert(0, REPO)
import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from turbo_decoder_cuda_amd import TurboCodec, synth  # noqa: E402
from turbo_decoder_cuda_amd import _native as N  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
prec = sys.argv[2] if len(sys.argv) > 2 else "f64"
algo = sys.argv[3] if len(sys.argv) > 3 else "logmap"
K, iters = 6144, 8
u, llr = synth.make_batch(B, K, 263, 480, 1.0, dtype=np.float64 if prec == "f64" else np.float32)
x = torch.from_numpy(llr).cuda()
c = TurboCodec(K, 263, 480, iterations=iters, precision=prec, algo=algo)
slots = N.lib().td_debug_stamp_slots()
G = (B + 7) // 8
st = torch.zeros((G, slots), dtype=torch.int64, device="cuda")
N.check(N.lib().td_debug_set_stamps(c._h, C.c_void_p(st.data_ptr())))
bits = c.decode(x)
torch.cuda.synchronize()
c.profile(True)
bits = c.decode(x)
_, kms, _ = c.kernel_ms()
NW = 4                  # waves per group
NS = slots // NW        # td_kernels.hip kStampSlots: 16 (14 before round 4)
s = st.cpu().numpy().reshape(G, NW, NS).astype(np.float64)
L = K + 3
steps = 2 * iters * L
print(f"B={B} {prec} {algo} kernel_ms={kms:.3f} errs={int((bits.cpu().numpy() != u).sum())}")
roles = ["A alpha|fold", "B beta", "F0 loader", "F1 fold", "R arec"][:NW]
for w in range(NW):
    fw, fwait, bw, bwait = (s[:, w, i].mean() / steps for i in range(4))
    print(f"  {roles[w]:14s} per SISO-step: F work {fw:7.1f}  F wait {fwait:7.1f}  B work {bw:7.1f}  B wait {bwait:7.1f}"
          f"  (slot4 {s[:, w, 4].mean() / steps:6.1f})")
kc, kr = s[:, :, 7], s[:, :, 8]
clk = kc.sum() / kr.sum() * 0.1   # GHz (realtime ticks at 100 MHz)
acc = s[:, :, 0:4].sum(axis=2)
print(f"  clock {clk:.3f} GHz; kernel {kc.mean() / steps:.1f} cycles per SISO-step, of which the pass stamps cover "
      f"{acc.mean() / steps:.1f} (unstamped: SISO prologues / epilogues, {(kc.mean() - acc.mean()) / steps:.1f})")
for w in range(NW):
    print(f"  {roles[w]:14s} per SISO-step: SISO calls {s[:, w, 9].mean() / steps:7.1f}  SISO-end barrier "
          f"{s[:, w, 10].mean() / steps:6.1f}  in-SISO unstamped {(s[:, w, 9] - s[:, w, 0:4].sum(axis=1)).mean() / steps:6.1f}"
          + (f"  F prologue {s[:, w, 11].mean() / steps:6.1f}" if NS > 11 else "")
          + (f"  B prologue {s[:, w, 12].mean() / steps:6.1f}  first tile {s[:, w, 13].mean() / steps:6.1f}" if NS > 13 and w == 2 else "")
          + (f"  B convert {s[:, w, 14].mean() / steps:6.1f}  DMA wait {s[:, w, 4].mean() / steps:6.1f}  tm_from_alpha "
             f"{s[:, w, 15].mean() / steps:6.1f}" if NS > 15 and w in (2, 3) else ""))
hw = st.cpu().numpy().reshape(G, NW, NS)[:, :, 6].astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
distinct = np.array([len(set(simd[g])) for g in range(G)])
print("  waves of a group on distinct SIMDs: " + ", ".join(f"{k}:{int((distinct == k).sum())}" for k in (1, 2, 3, 4)))
if NW == 5:
    print(f"  R shares its SIMD with A in {int((simd[:, 4] == simd[:, 0]).sum())} groups, B {int((simd[:, 4] == simd[:, 1]).sum())}, F0 {int((simd[:, 4] == simd[:, 2]).sum())}, F1 {int((simd[:, 4] == simd[:, 3]).sum())}")
same = lambda a, b: int((simd[:, a] == simd[:, b]).sum())
print(f"  A/B share SIMD in {same(0, 1)} groups, A/F0 {same(0, 2)}, A/F1 {same(0, 3)}, B/F0 {same(1, 2)}, B/F1 {same(1, 3)}")
# workgroups resident on the same CU (XCC, SE, SH, CU): which roles of the two share a SIMD
xcc = st.cpu().numpy().reshape(G, NW, NS)[:, 0, 5].astype(np.int64) & 0xF
sh = (hw >> 12) & 1
key = [(int(xcc[g]), int(se[g, 0]), int(sh[g, 0]), int(cu[g, 0])) for g in range(G)]
from collections import Counter, defaultdict  # noqa: E402
by = defaultdict(list)
for g, k in enumerate(key):
    by[k].append(g)
print("  groups per CU: " + str(sorted(Counter(len(v) for v in by.values()).items())))
pairs = Counter()
for v in by.values():
    for i in range(len(v)):
        for j in range(i + 1, len(v)):
            a, b = v[i], v[j]
            for ra in range(NW):
                for rb in range(NW):
                    if simd[a, ra] == simd[b, rb]:
                        pairs[(roles[ra].split()[0], roles[rb].split()[0])] += 1
    if len(v) == 2 and len(pairs) < 0:
        pass
print("  cross-group SIMD sharing (role pairs): " + ", ".join(f"{a}/{b}:{n}" for (a, b), n in sorted(pairs.items())))
ex = [v for v in by.values() if len(v) == 2][:4]
print("  example co-resident groups: " + "; ".join(f"{v[0]}&{v[1]}" for v in ex))
