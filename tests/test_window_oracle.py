"""Pins oracle/window_oracle.py (the windowed Max-Log-MAP restatement that checks the
sliding-window kernel) to the exact restatement: with one sub-block, or an overlap reaching both
ends of the trellis from every sub-block, the windowed serial decoder is the exact Max-Log-MAP
decoder of log_map.cpp (max is order-free), whatever the NII setting."""
import numpy as np
import pytest

import pyoracle as O
import window_oracle as WO


@pytest.mark.parametrize("K,f1,f2,W,g,nii", [(40, 3, 10, 64, 0, False), (40, 3, 10, 43, 0, True),
                                             (160, 21, 120, 48, 170, True), (200, 13, 50, 64, 203, False)])
def test_window_restatement_reduces_to_exact(K, f1, f2, W, g, nii):
    _, flow = O.synth_batch(K, f1, f2, 0.2, 7 + K, 3)
    for b in range(3):
        wb, wl = WO.turbo_decode_window(flow[b], K, f1, f2, 4, W, g, nii=nii)
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, 4, algo=O.ALGO_MAXLOG)
        assert np.array_equal(wb, ob.astype(np.uint8))
        assert np.abs(wl - ol).max() <= 1e-9


def test_window_restatement_nii_recovers_short_subblocks():
    """32-step sub-blocks without warm-up: equal-metric boundaries leave errors at 1.5 dB that
    NII boundaries (the reference GPU decoder's scheme) remove."""
    K, f1, f2 = 512, 31, 64
    src, flow = O.synth_batch(K, f1, f2, 1.5, 5, 6)
    errs = {}
    for nii in (False, True):
        errs[nii] = sum(int((WO.turbo_decode_window(flow[b], K, f1, f2, 6, 32, 0, nii=nii, concurrent=True,
                                                    scale=0.77)[0][-1] != src[b]).sum()) for b in range(6))
    assert errs[True] == 0 and errs[False] > 0


# ---------------------------------------------------------------- the C restatement (round 5)
# pyoracle.turbo_decode_window (oracle/turbo_oracle_window.inc) restates the windowed kernels'
# arithmetic on log_map.cpp's operations, log-MAP included; the GPU tests compare the kernels with
# it bit for bit.  Here it is pinned to the two independent restatements.

@pytest.mark.parametrize("K,f1,f2,W,g,nii,conc,scale", [
    (200, 13, 50, 48, 0, True, True, 0.77), (200, 13, 50, 64, 0, True, False, 1.0),
    (200, 13, 50, 48, 6, False, True, 1.0), (200, 13, 50, 50, 9, True, True, 0.77),
    (512, 31, 64, 96, 30, True, False, 0.77), (160, 21, 120, 64, 192, True, True, 1.0),
    (40, 3, 10, 16, 0, True, True, 0.5), (1024, 31, 64, 64, 30, False, False, 1.0),
    (1024, 31, 64, 64, 64, True, False, 1.0)])
def test_c_window_restatement_matches_numpy_maxlog(K, f1, f2, W, g, nii, conc, scale):
    """Max-Log-MAP (max is order-free, so the normalisation spacing changes only rounding): the C
    restatement equals window_oracle.py in bits, Le within 1e-9, for every schedule option."""
    _, flow = O.synth_batch(K, f1, f2, 0.3, 11 + W + g, 3)
    for b in range(3):
        wb, wl = WO.turbo_decode_window(flow[b], K, f1, f2, 5, W, g, nii=nii, concurrent=conc, scale=scale)
        cb, cl = O.turbo_decode_window(flow[b], K, f1, f2, 5, W, g, algo=O.ALGO_MAXLOG, nii=nii, concurrent=conc,
                                       scale=scale)
        assert np.array_equal(wb, cb)
        assert np.abs(wl - cl).max() <= 1e-9


@pytest.mark.parametrize("algo", [O.ALGO_LOGMAP, O.ALGO_MAXLOG])
@pytest.mark.parametrize("K,f1,f2,W,g", [(40, 3, 10, 64, 0), (160, 21, 120, 64, 192), (120, 103, 90, 64, 120),
                                         (200, 13, 50, 64, 203)])
def test_c_window_restatement_reduces_to_exact(K, f1, f2, W, g, algo):
    """One sub-block, or an overlap reaching both trellis ends from every sub-block: the windowed
    decoder is log_map.cpp's own (exact oracle) up to the normalisation's rounding, in log-MAP too
    (table max* included): bits identical, Le within 1e-9 on these frames."""
    _, flow = O.synth_batch(K, f1, f2, 0.0, 300 + K, 4)
    for b in range(4):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, 4, algo=algo)
        cb, cl = O.turbo_decode_window(flow[b], K, f1, f2, 4, W, g, algo=algo)
        assert np.array_equal(cb, ob.astype(np.uint8))
        assert np.abs(cl - ol).max() <= 1e-9


def test_c_window_restatement_f32_tracks_f64():
    """fp32 restatement (normalised every 8 positions) against fp64 (every 4): bits of the last
    iteration identical on converged frames."""
    K, f1, f2 = 1024, 31, 64
    _, flow = O.synth_batch(K, f1, f2, 1.0, 3, 3)
    for b in range(3):
        b64, _ = O.turbo_decode_window(flow[b], K, f1, f2, 6, 64, 30)
        b32, _ = O.turbo_decode_window(flow[b].astype(np.float32), K, f1, f2, 6, 64, 30)
        assert np.array_equal(b64[-1], b32[-1])
