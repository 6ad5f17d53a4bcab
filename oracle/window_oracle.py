"""Windowed Max-Log-MAP turbo decoder restatement -- TEST INFRASTRUCTURE ONLY.

The checker for the sliding-window schedule (td_set_window, SURVEY.md 8f row 3, BASELINE
config 5) in Max-Log-MAP, where the arithmetic is order-free, so the HIP kernel must agree to
rounding.  Imported only by tests/.  It restates the reference's sub-block GPU decoder,
generalised with an overlap warm-up:

  * sub-block s of a decoder's trellis covers [sW, (s+1)W), the last one up to L
    (ITTC/CUDA/turboDecoderBianJieZhi.cu:238, 321-376: the last sub-block also runs the 3 tail
    steps);
  * its alpha starts at sW - g from the initial state (sub-block 0), from the metric the
    neighbouring chain saved in the previous iteration (NII, :248 read, :302-304 write), or from
    equal metrics (first iteration, :495-500); its beta starts at the sub-block's end + g from the
    terminated state (last sub-block, :502-507), NII (:312 read, :397-400 write) or equal metrics;
  * Max-Log-MAP recursions with max normalisation (:265-300, :356-376), LLR = max - max over the
    8 (from-state, input) transitions (:383-393);
  * the extrinsic Le = scale * (LLR - La - 2 ys) (:423-434, scale 0.77 there);
  * schedule: serial (SISO1 then SISO2 on SISO1's fresh extrinsic, as ITTC/log_map.cpp:1207-1265)
    or concurrent (both SISOs on the other's extrinsic of the previous iteration, the reference
    GPU decoder's loop :642-690); hard decisions from SISO2's LLR (>= 0 -> 1, log_map.cpp:862-879).
"""
from __future__ import annotations

import numpy as np

import pyoracle as O

NEG = -1e20   # INFTY of ITTC/log_map.h:30


def _tables():
    t = O.trellis()
    ns = np.array(t.nextstat).reshape(8, 2)
    ls = np.array(t.laststat).reshape(8, 2)
    no = np.array(t.nextout).reshape(8, 4)
    return ns, ls, no[:, 1].astype(float), no[:, 3].astype(float)


def _init():
    v = np.full(8, NEG)
    v[0] = 0.0
    return v


def siso_window(ys, yp, La, W, g, nii_a, nii_b, use_nii):
    """One SISO over all sub-blocks.  nii_a / nii_b [nS][8]: the previous iteration's boundary
    metrics (read when use_nii).  Returns (LLR[L], new nii_a, new nii_b)."""
    ns, ls, o0, o1 = _tables()
    L = len(ys)
    nS = max(1, L // W)
    g0 = lambda i: -ys[i] + yp[i] * o0 - La[i] / 2   # gamma[s][i][0], per from-state s
    g1 = lambda i: ys[i] + yp[i] * o1 + La[i] / 2
    LLR = np.zeros(L)
    new_a = np.zeros((nS, 8))
    new_b = np.zeros((nS, 8))
    for s in range(nS):
        start = s * W
        end = L if s == nS - 1 else (s + 1) * W
        i0 = start - g
        if i0 <= 0:
            a = _init()
        elif use_nii:
            a = nii_a[s].copy()
        else:
            a = np.zeros(8)
        A = {}
        if s < nS - 1 and i0 + W < 0:
            new_a[s + 1] = _init()
        for p in range(max(i0, 0), end + 1):
            if start <= p < end:
                A[p] = a
            if s < nS - 1 and p == i0 + W:
                new_a[s + 1] = a
            if p < end:
                c0, c1 = g0(p), g1(p)
                nxt = np.maximum(a[ls[:, 0]] + c0[ls[:, 0]], a[ls[:, 1]] + c1[ls[:, 1]])
                a = nxt - nxt.max()
        e = end + g
        if e >= L:
            b = _init()
        elif use_nii:
            b = nii_b[s].copy()
        else:
            b = np.zeros(8)
        if s > 0 and start + g >= L:
            new_b[s - 1] = _init()
        for p in range(min(e, L) - 1, start - 1, -1):
            c0, c1 = g0(p), g1(p)
            if p < end:
                LLR[p] = (A[p] + c1 + b[ns[:, 1]]).max() - (A[p] + c0 + b[ns[:, 0]]).max()
            nb = np.maximum(c0 + b[ns[:, 0]], c1 + b[ns[:, 1]])
            b = nb - nb.max()
            if s > 0 and p == start + g:
                new_b[s - 1] = b
    return LLR, new_a, new_b


def turbo_decode_window(flow, K, f1, f2, iters, W, g, nii=False, concurrent=False, scale=1.0):
    """One codeword (flow [3K+12] f64, the main.cpp layout).  Returns (bits[iters, K] uint8,
    le[iters, 2, L]) like pyoracle.turbo_decode."""
    pi = O.qpp(K, f1, f2)
    L = K + 3
    f = np.asarray(flow, dtype=np.float64) * 0.5          # log_map.cpp:1202-1205
    ys1 = np.concatenate([f[0:3 * K:3], f[3 * K:3 * K + 6:2]])
    yp1 = np.concatenate([f[1:3 * K:3], f[3 * K + 1:3 * K + 6:2]])
    ys2 = np.concatenate([f[0:3 * K:3][pi], f[3 * K + 6:3 * K + 12:2]])
    yp2 = np.concatenate([f[2:3 * K:3], f[3 * K + 7:3 * K + 12:2]])
    nS = max(1, L // W)
    na = [np.zeros((nS, 8)), np.zeros((nS, 8))]
    nb = [np.zeros((nS, 8)), np.zeros((nS, 8))]
    Le1 = np.zeros(K)   # natural order
    Le2 = np.zeros(K)   # interleaved order
    bits = np.zeros((iters, K), dtype=np.uint8)
    le = np.zeros((iters, 2, L))
    for it in range(iters):
        use = nii and it > 0
        La1 = np.zeros(L)
        La1[pi] = Le2                                       # deinterleave
        if concurrent:
            La2 = np.zeros(L)
            La2[:K] = Le1[pi]
        LLR1, a1, b1 = siso_window(ys1, yp1, La1, W, g, na[0], nb[0], use)
        e1 = scale * (LLR1 - La1 - 2 * ys1)
        if not concurrent:
            La2 = np.zeros(L)
            La2[:K] = e1[:K][pi]                            # interleave SISO1's fresh Le
        LLR2, a2, b2 = siso_window(ys2, yp2, La2, W, g, na[1], nb[1], use)
        e2 = scale * (LLR2 - La2 - 2 * ys2)
        na, nb = [a1, a2], [b1, b2]
        Le1, Le2 = e1[:K], e2[:K]
        le[it, 0], le[it, 1] = e1, e2
        bits[it, pi] = (LLR2[:K] >= 0).astype(np.uint8)
    return bits, le
