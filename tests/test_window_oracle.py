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
