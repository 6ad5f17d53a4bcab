"""GPU parity: the HIP decoder against the golden vectors of the compiled reference and
against the CPU restatement (oracle/), through the C ABI.

Gates (BASELINE.json north_star): hard bits bit-exact; per-iteration extrinsic Le within
1e-4 of ITTC/log_map.cpp on identical channel input (fp64 parity mode).  Against the oracle
(same operation order) the fp64 kernel is expected to be bit-identical; the test allows 1e-9.
"""
import glob
import os

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD

pytestmark = pytest.mark.gpu

LE_TOL_REF = 1e-4      # north_star: per-iteration extrinsic LLR vs log_map.cpp
LE_TOL_ORACLE = 1e-9   # same op order as the restatement


def codec(K, f1, f2, iters, algo="logmap", precision="f64"):
    from turbo_decoder_cuda_amd import TurboCodec
    return TurboCodec(K, f1, f2, iterations=iters, algo=algo, precision=precision)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "siso_*.npz"))))
def test_siso_vs_reference(path):
    d = np.load(path)
    L = int(d["L"])
    c = codec(max(L - 3, 1), 1, 0, 1)
    llr = c.Log_MAP_decoder(d["recs"], d["La"], int(d["terminated"]))
    assert np.abs(llr - d["LLR"]).max() <= 1e-9


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "frames_*.npz"))))
def test_turbo_vs_reference(path):
    d = np.load(path)
    K, it = int(d["K"]), int(d["iters"])
    c = codec(K, int(d["f1"]), int(d["f2"]), it)
    out, le = c.TurboDecoding(d["flow"], return_le=True)
    assert np.array_equal(out.astype(np.uint8), d["bits"]), "hard bits differ from log_map.cpp"
    assert np.abs(le - d["le"]).max() <= LE_TOL_REF
    for fr in range(d["flow"].shape[0]):
        ob, ol = O.turbo_decode(d["flow"][fr], K, int(d["f1"]), int(d["f2"]), it)
        assert np.array_equal(out[fr], ob)
        assert np.abs(le[fr] - ol).max() <= LE_TOL_ORACLE


@pytest.mark.parametrize("terminated", [1, 0])
@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_siso_maxlog_vs_oracle(terminated, precision):
    """The standalone SISO (Log_MAP_decoder) in Max-Log-MAP, whose folds recompute alpha between
    the stored rows: LLRs against the oracle's max-log SISO on random channel values and a-priori,
    several windows long and ragged (L = 1027)."""
    rng = np.random.default_rng(11 + terminated)
    L = 1027
    recs = rng.normal(0.0, 2.0, 2 * L)
    La = rng.normal(0.0, 3.0, L)
    c = codec(L - 3, 1, 0, 1, algo="maxlog", precision=precision)
    llr = c.Log_MAP_decoder(recs.astype(c.dtype), La.astype(c.dtype), terminated)
    ref = O.siso(recs.astype(c.dtype).astype(np.float64), La.astype(c.dtype).astype(np.float64), terminated,
                 algo=O.ALGO_MAXLOG)
    tol = 1e-9 if precision == "f64" else 1e-3 * max(1.0, float(np.abs(ref).max()))
    assert np.abs(llr - ref).max() <= tol
