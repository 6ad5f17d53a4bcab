"""The oracle (oracle/liboracle.so, CPU restatement of ITTC/log_map.cpp) pinned against the
golden vectors produced by the compiled reference (oracle/gen_golden.py), plus the
known-answer tables of SURVEY.md 8(c).  CPU only."""
import glob
import os

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD

FRAMES = sorted(glob.glob(os.path.join(GOLD, "frames_*.npz")))
SISOS = sorted(glob.glob(os.path.join(GOLD, "siso_*.npz")))


def test_golden_present():
    assert len(FRAMES) >= 9 and len(SISOS) >= 3
    assert os.path.exists(os.path.join(GOLD, "maxstar.npz"))


def test_trellis_known_answer():
    """nextstat u=0 {0,4,5,1,2,6,7,3}, u=1 {4,0,1,5,6,2,3,7}; parity outputs."""
    t = O.trellis()
    ns = np.array(t.nextstat).reshape(8, 2)
    assert ns[:, 0].tolist() == [0, 4, 5, 1, 2, 6, 7, 3]
    assert ns[:, 1].tolist() == [4, 0, 1, 5, 6, 2, 3, 7]
    no = np.array(t.nextout).reshape(8, 4)
    for s in range(8):
        assert no[s, 0] == -1 and no[s, 2] == 1                 # systematic = 2u-1
        if s in (0, 1, 6, 7):
            assert (no[s, 1], no[s, 3]) == (-1, 1)
        else:
            assert (no[s, 1], no[s, 3]) == (1, -1)
    ls = np.array(t.laststat).reshape(8, 2)
    for s in range(8):
        for u in range(2):
            assert ls[ns[s, u], u] == s


def test_qpp_known_answer():
    pi = O.qpp(6144, 263, 480)
    assert pi[:5].tolist() == [0, 743, 2446, 5109, 2588]          # also TurboDecoder.cu:60
    assert O.qpp(1024, 31, 64)[1] == 95
    for K, f1, f2 in ((40, 3, 10), (1024, 31, 64), (6144, 263, 480)):
        assert np.array_equal(np.sort(O.qpp(K, f1, f2)), np.arange(K))


def test_maxstar_vs_reference():
    d = np.load(os.path.join(GOLD, "maxstar.npz"))
    got = np.array([O.maxstar(x, y) for x, y in zip(d["x"], d["y"])])
    assert np.array_equal(got, d["r"])


@pytest.mark.parametrize("path", SISOS, ids=os.path.basename)
def test_siso_vs_reference(path):
    d = np.load(path)
    llr = O.siso(d["recs"], d["La"], int(d["terminated"]))
    assert np.array_equal(llr, d["LLR"])


@pytest.mark.parametrize("path", FRAMES, ids=os.path.basename)
def test_channel_vs_reference(path):
    """main.cpp's frame generator (srand, rand, TurboEnCoding, BPSK, AWGN/mgrns, demod)
    restated bit-exactly: same info bits and the same channel LLRs."""
    d = np.load(path)
    K, nf = int(d["K"]), d["flow"].shape[0]
    src, flow = O.make_frames(K, int(d["f1"]), int(d["f2"]), float(d["ebn0"]), int(d["seed"]), nf)
    assert np.array_equal(src.astype(np.uint8), d["src"])
    assert np.array_equal(flow, d["flow"])


@pytest.mark.parametrize("path", FRAMES, ids=os.path.basename)
def test_turbo_vs_reference(path):
    """TurboDecoding restatement: hard bits identical every iteration, Le within 1e-4
    (BASELINE north_star).  The reference leaves tempmax uninitialised (log_map.cpp:925);
    the restatement defines it, which moves Le by <1e-9 in converged frames."""
    d = np.load(path)
    K, it = int(d["K"]), int(d["iters"])
    for fr in range(d["flow"].shape[0]):
        bits, le = O.turbo_decode(d["flow"][fr], K, int(d["f1"]), int(d["f2"]), it)
        assert np.array_equal(bits.astype(np.uint8), d["bits"][fr])
        tol = 1e-4 if d["le"].dtype == np.float64 else 1e-4 + 1e-6 * np.abs(d["le"][fr]).max()
        assert np.abs(le - d["le"][fr]).max() <= tol


def test_encoder_matches_synth():
    """The numpy encoder used by bench.py / synth equals the restated TurboEnCoding."""
    from turbo_decoder_cuda_amd import synth
    rng = np.random.default_rng(5)
    for K, f1, f2 in ((40, 3, 10), (1024, 31, 64), (6144, 263, 480)):
        u = rng.integers(0, 2, size=(3, K), dtype=np.uint8)
        got = synth.turbo_encode(u, f1, f2)
        for b in range(3):
            ref = O.encode(u[b].astype(np.int32), f1, f2)
            assert np.array_equal(got[b], ref.astype(np.uint8))


def test_decode_batch_threads_agree():
    """The threaded CPU baseline (bench.py cpu_baseline) equals the single-frame path."""
    src, flow = O.synth_batch(1024, 31, 64, 0.5, 3, 6)
    bits = O.decode_batch(flow, 1024, 31, 64, 4, nthreads=3)
    for b in range(6):
        ob, _ = O.turbo_decode(flow[b], 1024, 31, 64, 4)
        assert np.array_equal(bits[b], ob[-1].astype(np.uint8))


# ------------------------------------------------------------ modulators / demodulators (row 4)
@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
def test_demodulate_matches_reference(M):
    """demodule() restatement == the compiled reference's output, bit for bit, on every
    constellation point, decision-boundary points and random symbols (tests/golden/demod.npz)."""
    d = np.load(os.path.join(GOLD, "demod.npz"))
    got = O.demodulate(d[f"yi_{M}"], d[f"yq_{M}"], M, float(d["Kf"]))
    assert np.array_equal(got, d[f"llr_{M}"])


@pytest.mark.parametrize("M", [2, 3, 4, 6])
def test_frames_with_modulation_match_reference(M):
    """main.cpp's frames with MODULATION = M (module, AWGN I/Q, demodule) bit for bit."""
    d = np.load(os.path.join(GOLD, "modframes_K1024.npz"))
    src, flow = O.make_frames_mod(int(d["K"]), int(d["f1"]), int(d["f2"]), float(d["ebn0"]), M, int(d["seed"]),
                                  d[f"src_{M}"].shape[0])
    assert np.array_equal(src.astype(np.uint8), d[f"src_{M}"])
    assert np.array_equal(flow, d[f"flow_{M}"])


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
def test_modulate_demodulate_round_trip(M):
    """Noise-free symbols demodulate to LLRs whose signs are the transmitted bits."""
    bits = np.random.default_rng(M).integers(0, 2, 60 * M)
    si, sq = O.modulate(bits, M)
    llr = O.demodulate(si, sq, M, 1.0)
    assert np.array_equal((llr > 0).astype(int), bits)


REF_HARNESS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "ref_harness")


@pytest.mark.skipif(not os.access(REF_HARNESS, os.X_OK), reason="compiled reference not built here (make -C oracle ref)")
def test_reference_decode_mode_matches_oracle(tmp_path):
    """bench.py's CPU baseline runs the compiled reference's `decode` mode (TurboDecoding's loop
    through log_map.cpp's own functions, frames over threads): its bits equal the restatement's."""
    import subprocess

    from turbo_decoder_cuda_amd import synth

    u, llr = synth.make_batch(6, 1024, 31, 64, 0.5, seed=3, dtype=np.float64)
    fin, fout = str(tmp_path / "flows.bin"), str(tmp_path / "bits.bin")
    llr.tofile(fin)
    r = subprocess.run([REF_HARNESS, "decode", "1024", "31", "64", "4", "3", fin, fout], capture_output=True,
                       text=True, check=True)
    assert r.stdout.startswith("seconds ") and " frames 6 " in r.stdout
    rb = np.fromfile(fout, dtype=np.uint8).reshape(6, 1024)
    ob = O.decode_batch(np.ascontiguousarray(llr), 1024, 31, 64, 4, O.ALGO_LOGMAP, nthreads=2)
    assert np.array_equal(rb, ob)
