"""Sliding-window schedule (td_set_window; BASELINE config 5).

Windowed decoding changes the arithmetic, so its gate is the BER curve.  Two exact anchors
pin the kernel's indexing first:
  * with an overlap that reaches both ends of the trellis from every sub-block, the windowed
    Max-Log-MAP decoder IS the exact one (max is order-free): bits equal the oracle's, Le
    within 1e-9;
  * the single-sub-block case (L <= 64) likewise, at overlap 0.
and every schedule option (sub-block length, overlap, NII boundaries, concurrent SISOs, extrinsic
scale) is checked in Max-Log-MAP against oracle/window_oracle.py, a restatement of the
reference's sub-block GPU decoder (ITTC/CUDA/turboDecoderBianJieZhi.cu).
Since round 5 every schedule, in log-MAP and Max-Log-MAP, fp64 and fp32, in both lane layouts
(one sub-block per lane; runs of consecutive sub-blocks per lane, forced by td_debug_window_layout), is
compared bit for bit with oracle/turbo_oracle_window.inc (pyoracle.turbo_decode_window), the C
restatement of the windowed kernels' arithmetic, which tests/test_window_oracle.py pins to the
numpy restatement above and to the exact oracle.
Then the BER of the windowed log-MAP decoder at K=6144 is compared with the exact schedule on
the same generator frames."""
import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu

# the windowed schedule's max* forms: "logmap" = the one-read table (td_set_window_maxstar default,
# the C restatement's TDO_ALGO_LOGMAP_Q), "logmap-exact" = log_map.cpp's E_algorithm, "maxlog"
ALGOS = ["logmap", "logmap-exact", "maxlog"]


def _oalgo(algo):
    return {"logmap": O.ALGO_LOGMAP_Q, "logmap-exact": O.ALGO_LOGMAP, "maxlog": O.ALGO_MAXLOG}[algo]


def _decode(K, f1, f2, iters, flow, algo, window, overlap, precision="f64", ext_scale=1.0, nii=False,
            concurrent=False, run=0):
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    dt = torch.float64 if precision == "f64" else torch.float32
    x = torch.from_numpy(flow).to("cuda:0").to(dt).contiguous()
    B = flow.shape[0]
    with TurboCodec(K, f1, f2, iterations=iters, algo=algo.split("-")[0], precision=precision) as c:
        c.debug_window_layout(run)
        c.set_window_maxstar(algo == "logmap-exact")
        c.set_window(window, overlap, ext_scale, nii=nii, concurrent=concurrent)
        bits = torch.empty((B, iters, K), dtype=torch.uint8, device=x.device)
        le = torch.empty((B, iters, 2, K + 3), dtype=dt, device=x.device)
        c.decode(x, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
    return bits.cpu().numpy(), le.cpu().numpy()


@pytest.mark.parametrize("K,f1,f2,B,overlap", [(40, 3, 10, 5, 0), (40, 3, 10, 9, 9), (160, 21, 120, 11, 192),
                                               (120, 103, 90, 16, 120)])
def test_window_maxlog_full_overlap_is_exact(K, f1, f2, B, overlap):
    _, flow = O.synth_batch(K, f1, f2, 0.0, 300 + K, B)
    iters = 4
    bits, le = _decode(K, f1, f2, iters, flow, "maxlog", 64, overlap)
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=O.ALGO_MAXLOG)
        assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"


@pytest.mark.parametrize("K,f1,f2,W,g,nii,conc,scale", [
    (200, 13, 50, 48, 0, True, True, 0.77),      # the reference GPU decoder's schedule
    (200, 13, 50, 64, 0, True, False, 1.0),
    (200, 13, 50, 48, 6, False, True, 1.0),
    (200, 13, 50, 50, 9, True, True, 0.77),      # W not a multiple of 3, overlap with NII
    (512, 31, 64, 96, 30, True, False, 0.77),
    (160, 21, 120, 64, 192, True, True, 1.0),    # overlap beyond both ends
    (40, 3, 10, 16, 0, True, True, 0.5),
])
def test_window_schedules_vs_restatement(K, f1, f2, W, g, nii, conc, scale):
    import window_oracle as WO
    B, iters = 9, 5
    _, flow = O.synth_batch(K, f1, f2, 0.3, 11 + W + g, B)
    bits, le = _decode(K, f1, f2, iters, flow, "maxlog", W, g, ext_scale=scale, nii=nii, concurrent=conc)
    for b in range(B):
        ob, ol = WO.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, nii=nii, concurrent=conc, scale=scale)
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"
        assert np.array_equal(bits[b], ob), f"codeword {b}"


# (K, f1, f2, W, g, nii, concurrent, scale, run): run 0 = the layout's own choice (one
# sub-block per lane at these batches); runs need g <= W and W a multiple of the checkpoint spacing
WIN_CASES = [
    (1024, 31, 64, 64, 30, False, False, 1.0, 0),
    (1024, 31, 64, 64, 30, False, False, 1.0, 2),
    (1024, 31, 64, 64, 30, True, False, 1.0, 5),      # 16 sub-blocks in runs of 5 (the last run 1)
    (512, 31, 64, 48, 48, True, True, 0.77, 3),       # overlap = window
    (200, 13, 50, 48, 0, True, True, 0.77, 2),        # the reference GPU decoder's schedule, in runs
    (200, 13, 50, 64, 0, True, False, 1.0, 3),
    (200, 13, 50, 50, 9, True, True, 0.77, 2),        # W not a multiple of 4: one sub-block per lane
    (160, 21, 120, 64, 192, True, True, 1.0, 2),      # overlap beyond both ends: one per lane
    (40, 3, 10, 16, 0, True, True, 0.5, 2),
    (6144, 263, 480, 64, 30, False, False, 1.0, 7),   # config 5's schedule, 96 sub-blocks in runs of 7
]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("K,f1,f2,W,g,nii,conc,scale,run", WIN_CASES)
def test_window_vs_c_restatement(K, f1, f2, W, g, nii, conc, scale, run, algo):
    """Every schedule option, both algorithms, both lane layouts: bits identical to the C
    restatement, Le within 1e-9 (the same fp64 operations in the same order)."""
    B, iters = (3, 3) if K > 2048 else (9, 5)
    _, flow = O.synth_batch(K, f1, f2, 0.3, 11 + W + g, B)
    bits, le = _decode(K, f1, f2, iters, flow, algo, W, g, ext_scale=scale, nii=nii, concurrent=conc, run=run)
    oalgo = _oalgo(algo)
    for b in range(B):
        ob, ol = O.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, algo=oalgo, nii=nii, concurrent=conc,
                                       scale=scale)
        assert np.array_equal(bits[b], ob), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("K,f1,f2,W,g,nii,conc,scale", [
    (1024, 31, 64, 64, 30, False, False, 1.0),
    (512, 31, 64, 48, 48, True, True, 0.77),
    (200, 13, 50, 50, 9, True, True, 0.77),       # W not a multiple of the segment
    (160, 21, 120, 64, 192, True, True, 1.0),     # overlap beyond both ends
    (6144, 263, 480, 64, 30, False, False, 1.0),  # the drop-in's opt-in schedule at config 5's K
    (1024, 31, 64, 64, 30, True, True, 0.77),     # beta warm-up in the alpha kernel, with NII, concurrent
    (1024, 31, 64, 64, 20, True, False, 1.0),     # the same, serial, another overlap
])
def test_window_single_frame_vs_c_restatement(K, f1, f2, W, g, nii, conc, scale, algo, precision):
    """A batch of one codeword (the drop-in's frame) takes the beta kernel's lane-fold variant (the S
    LLRs of a segment folded side by side, one per lane): bits identical to the C restatement, Le
    within 1e-9 (fp64) / relative 1e-4 (fp32), every iteration, for two frames decoded one at a time."""
    iters = 3 if K > 2048 else 5
    _, flow = O.synth_batch(K, f1, f2, 0.3, 5 + W + g, 2)
    if precision == "f32":
        flow = flow.astype(np.float32)
    oalgo = _oalgo(algo)
    for b in range(2):
        bits, le = _decode(K, f1, f2, iters, flow[b:b + 1], algo, W, g, precision=precision, ext_scale=scale,
                           nii=nii, concurrent=conc)
        ob, ol = O.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, algo=oalgo, nii=nii, concurrent=conc,
                                       scale=scale)
        assert np.array_equal(bits[0], ob), f"frame {b}"
        tol = 1e-9 if precision == "f64" else 1e-4 * max(1.0, np.abs(ol).max())
        assert np.abs(le[0] - ol).max() <= tol, f"frame {b}"


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("run", [0, 3])
def test_window_f32_vs_c_restatement(algo, run):
    """fp32 (checkpoints and normalisation every 8 positions) against the fp32 restatement."""
    K, f1, f2, B, iters, W, g = 1024, 31, 64, 9, 4, 64, 30
    _, flow = O.synth_batch(K, f1, f2, 0.5, 77, B)
    flow = flow.astype(np.float32)
    bits, le = _decode(K, f1, f2, iters, flow, algo, W, g, precision="f32", run=run)
    oalgo = _oalgo(algo)
    for b in range(B):
        ob, ol = O.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, algo=oalgo)
        assert np.array_equal(bits[b], ob), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-4 * max(1.0, np.abs(ol).max()), f"codeword {b}"


@pytest.mark.parametrize("nii,conc,scale,precision,algo", [(False, False, 1.0, "f64", "logmap"),
                                                         (True, True, 0.77, "f64", "logmap"),
                                                         (False, False, 1.0, "f64", "logmap-exact"),
                                                         (False, False, 1.0, "f32", "logmap"),
                                                         (True, True, 0.77, "f32", "maxlog")])
def test_window_batch_parts_and_runs_do_not_change_results(nii, conc, scale, precision, algo):
    """Large batches run in parts on several streams (one part's alpha beside another's beta), with
    lane runs sized on the whole batch and the alpha kernel's own run length: none of it may change a
    bit.  A ragged batch big enough for four parts, decoded with 1, 2, 3 and 4 parts and two alpha
    run lengths, gives the one-part bits and Le; sampled codewords of every part equal the C
    restatement."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, iters, W, g = 512, 31, 64, 3, 64, 30
    B = 4 * 64 * 64 + 37                      # 257 waves of 64 codewords
    _, flow = O.synth_batch(K, f1, f2, 0.4, 5, 64)
    flow = np.tile(flow, (B // 64 + 1, 1))[:B]
    if precision == "f32":
        flow = flow.astype(np.float32)
    dt = torch.float64 if precision == "f64" else torch.float32
    x = torch.from_numpy(np.ascontiguousarray(flow)).to("cuda:0")
    outs = {}
    for parts, run_a in ((1, 0), (2, 0), (3, 0), (4, 0), (2, 1), (4, 3)):
        with TurboCodec(K, f1, f2, iterations=iters, algo=algo.split("-")[0], precision=precision) as c:
            c.set_window_maxstar(algo == "logmap-exact")
            c.set_window(W, g, scale, nii=nii, concurrent=conc)
            c.debug_window_layout(0, run_a, parts)   # after set_window: applies to the current schedule too
            bits = torch.empty((B, K), dtype=torch.uint8, device=x.device)
            le = torch.empty((B, iters, 2, K + 3), dtype=dt, device=x.device)
            c.decode(x, bits, le=le)
            torch.cuda.synchronize()
        outs[(parts, run_a)] = (bits.cpu().numpy(), le.cpu().numpy())
    b1, l1 = outs[(1, 0)]
    for key, (bk, lk) in outs.items():
        assert np.array_equal(bk, b1), key
        assert np.array_equal(lk, l1), key
    oalgo = _oalgo(algo)
    for b in (0, 64 * 64 + 5, 2 * 64 * 64 + 11, B - 1):   # one codeword in each of the four parts
        ob, ol = O.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, algo=oalgo, nii=nii, concurrent=conc,
                                       scale=scale)
        assert np.array_equal(b1[b], ob[-1]), b
        tol = 1e-9 if precision == "f64" else 1e-4 * max(1.0, np.abs(ol).max())
        assert np.abs(l1[b] - ol).max() <= tol, b


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("algo", ALGOS)
def test_window_high_snr_ragged_batch_error_free(algo, precision):
    """Ragged batch (B = 13) at 3 dB: every codeword decodes without error by the last iteration."""
    K, f1, f2, B = 6144, 263, 480, 13
    info, flow = O.synth_batch(K, f1, f2, 3.0, 5, B)
    if precision == "f32":
        flow = flow.astype(np.float32)
    bits, _ = _decode(K, f1, f2, 4, flow, algo, 64, 30, precision)
    assert np.array_equal(bits[:, -1, :], info.astype(np.uint8))


@pytest.mark.parametrize("table", ["fast", "exact"])
def test_window_ber_close_to_exact(table):
    """north_star's gate for config 5 ("BER-vs-Eb/N0 within 0.05 dB of the CPU reference"), on the
    waterfall: K=6144, 8 iterations, the same 32768 generator frames at 0.35 and 0.40 dB through the
    exact schedule (bit-exact against the reference) and the windowed one (W = 64, overlap 30).
    Bit and block errors of the window within 1.1x the exact decoder's at both points, and the
    window's BER shift, read through the exact curve's local slope, within 0.02 dB.  The full paired
    curve (262144 frames a point, profiles/r06/ber_window_vs_exact.json): 1e-4 crossed at 0.3819 dB
    against 0.3806 dB, a 0.0013 dB shift; window / exact bits 1.036 at 0.35 dB, 1.060 at 0.40 dB."""
    import math

    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, B, iters = 6144, 263, 480, 32768, 8
    res = {}
    with TurboCodec(K, f1, f2, iterations=iters) as ex, TurboCodec(K, f1, f2, iterations=iters) as win:
        win.set_window_maxstar(table == "exact")
        win.set_window(64, 30, 1.0)
        for k, e in enumerate((0.35, 0.40)):
            ex.synth_seed(100 + k)
            info, llr = ex.synth(B, e)
            bits = torch.empty((B, iters, K), dtype=torch.uint8, device=llr.device)
            for name, c in (("exact", ex), ("window", win)):
                c.decode(llr, bits, all_iters=True)
                err = c.count_errors(bits, info)[:, -1]
                res[(name, e)] = (int(err.sum()), int((err != 0).sum()))
            del bits, llr, info
    print(res)
    for e in (0.35, 0.40):
        (be, ke), (bw, kw) = res[("exact", e)], res[("window", e)]
        assert be > 1000 and ke > 50, (e, be, ke)
        assert bw <= 1.1 * be and kw <= 1.1 * ke, (e, res)
    slope = math.log(res[("exact", 0.35)][0] / res[("exact", 0.40)][0]) / 0.05   # ln(BER) per dB
    for e in (0.35, 0.40):
        shift_db = math.log(res[("window", e)][0] / res[("exact", e)][0]) / slope
        assert shift_db <= 0.02, (e, shift_db)


def test_set_window_rejects_bad_arguments():
    from turbo_decoder_cuda_amd import TurboCodec
    from turbo_decoder_cuda_amd import _native as N
    with TurboCodec(1024, 31, 64, iterations=2) as c:
        for w, g, s in ((2, 0, 1.0), (64, -3, 1.0), (64, 195, 1.0), (64, 30, 0.0), (64, 30, 5.0)):
            with pytest.raises(N.TurboError):
                c.set_window(w, g, s)
        c.set_window(0, 0, 1.0)


@pytest.mark.parametrize("conc", [False, True])
def test_window_launch_clock(conc):
    """td_clock_read after a windowed decode (round 5): the first workgroup of the last SISO2 beta
    launch samples the clock, so the config-5 roofline prices VALU issue at the launch's own clock."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2 = 1024, 31, 64
    _, flow = O.synth_batch(K, f1, f2, 0.4, 91, 300)
    with TurboCodec(K, f1, f2, iterations=2) as c:
        c.set_window(64, 30, concurrent=conc)
        c.decode(torch.from_numpy(flow).to("cuda:0"))
        ghz, span = c.clock()
        assert 0.5 < ghz < 3.0 and span > 0, (ghz, span)


def test_reference_gpu_decoder_ber_matches_published():
    """The reference GPU decoder's schedule (P = 64 sub-blocks, NII, concurrent SISOs, Le x0.77,
    Max-Log-MAP fp32) at 10 iterations on 2000 of main.cpp's frames per point: BER and FER
    within 25% of the published 10000-frame values (tests/golden/psweep_published.json) at
    0.4-0.6 dB, where both have thousands of bit errors.  The full sweep (all P, 25 iterations,
    10000 frames) is scripts/psweep.py: profiles/r01/psweep_summary.txt."""
    import json
    import os

    from conftest import GOLD
    from turbo_decoder_cuda_amd import TurboCodec
    from turbo_decoder_cuda_amd.ber import ber_point
    pub = json.load(open(os.path.join(GOLD, "psweep_published.json")))["P"]["64"]
    with TurboCodec(6144, 263, 480, iterations=10, algo="maxlog", precision="f32") as c:
        c.set_window(96, 0, 0.77, nii=True, concurrent=True)
        c.synth_seed(3)
        for k in (4, 5, 6):
            pt = ber_point(c, pub[k]["ebn0_db"], 2000, min_block_errors=0, batch=2000)
            ber, fer = pt.ber[9], pt.bler[9]
            print(pub[k]["ebn0_db"], ber, pub[k]["ber"][9], fer, pub[k]["fer"][9])
            assert abs(ber / pub[k]["ber"][9] - 1) < 0.25
            assert abs(fer / pub[k]["fer"][9] - 1) < 0.25


@pytest.mark.timeout(300)
def test_config5_full_batch():
    """BASELINE config 5 at its stated size: K=6144, sliding window 64 with overlap 30, batch
    32768 of main.cpp's frames (device generator) at 1.0 dB, 8 iterations.
      * fp64 log-MAP (the bench's config-5 line): residual bit errors no more than the exact
        schedule's on the same frames;
      * fp64 Max-Log-MAP on the same batch: two seeded codewords equal to oracle/window_oracle.py
        (the restatement of the reference's sub-block decoder, turboDecoderBianJieZhi.cu:248,
        302-304, 397-400) -- every iteration's bits, Le within 1e-9."""
    import torch

    import window_oracle as WO
    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, B, iters = 6144, 263, 480, 32768, 8
    errs = {}
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        c.synth_seed(20261015)
        info, llr = c.synth(B, 1.0)
        for mode in ("exact", "window"):
            c.set_window(64 if mode == "window" else 0, 30, 1.0)
            c.reserve(B)
            bits = c.decode(llr)
            torch.cuda.synchronize()
            errs[mode] = int((bits != info).sum().item())
            del bits
    print(errs)
    assert errs["window"] <= errs["exact"]   # no escape margin: both 0 on these frames
    sample = np.random.default_rng(5).choice(B, 2, replace=False)
    with TurboCodec(K, f1, f2, iterations=iters, algo="maxlog") as c:
        c.set_window(64, 30, 1.0)
        c.reserve(B)
        bits = torch.empty((B, iters, K), dtype=torch.uint8, device=llr.device)
        le = torch.empty((B, iters, 2, K + 3), dtype=torch.float64, device=llr.device)
        c.decode(llr, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
        idx = torch.from_numpy(sample).to(llr.device)
        bs, ls, fs = bits[idx].cpu().numpy(), le[idx].cpu().numpy(), llr[idx].cpu().numpy()
    del bits, le, llr, info
    for k in range(len(sample)):
        ob, ol = WO.turbo_decode_window(fs[k], K, f1, f2, iters, 64, 30)
        assert np.array_equal(bs[k], ob), f"codeword {sample[k]}"
        assert np.abs(ls[k] - ol).max() <= 1e-9, f"codeword {sample[k]}"
    # the bench's config-5 line itself (fp64 log-MAP, the run layout this batch selects): two seeded
    # codewords equal to the C restatement in every iteration's bits, Le within 1e-9
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        c.synth_seed(20261015)
        _, llr = c.synth(B, 1.0)
        c.set_window(64, 30, 1.0)
        c.reserve(B)
        bits = torch.empty((B, iters, K), dtype=torch.uint8, device=llr.device)
        le = torch.empty((B, iters, 2, K + 3), dtype=torch.float64, device=llr.device)
        c.decode(llr, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
        bs, ls, fs = bits[idx].cpu().numpy(), le[idx].cpu().numpy(), llr[idx].cpu().numpy()
    del bits, le, llr
    for k in range(len(sample)):
        ob, ol = O.turbo_decode_window(fs[k], K, f1, f2, iters, 64, 30, algo=O.ALGO_LOGMAP_Q)
        assert np.array_equal(bs[k], ob), f"codeword {sample[k]} (log-MAP)"
        assert np.abs(ls[k] - ol).max() <= 1e-9, f"codeword {sample[k]} (log-MAP)"
