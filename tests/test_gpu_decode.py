"""GPU decode through the C ABI beyond the golden frames: batched device-resident decode
against the oracle on seeded synthetic codewords (ragged batches, every iteration's bits and
Le), Max-Log-MAP and fp32 against the oracle's same-order arithmetic, the compat layer
(the reference's C++ entry points), and full-size properties at BASELINE config 2."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD, REPO

pytestmark = pytest.mark.gpu

PKG = os.path.join(REPO, "turbo_decoder_cuda_amd")


def _dev():
    import torch
    return torch.device("cuda", 0)


def _decode_all(K, f1, f2, iters, flow, algo="logmap", precision="f64"):
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    dt = torch.float64 if precision == "f64" else torch.float32
    x = torch.from_numpy(flow).to(_dev()).to(dt).contiguous()
    B = flow.shape[0]
    with TurboCodec(K, f1, f2, iterations=iters, algo=algo, precision=precision) as c:
        bits = torch.empty((B, iters, K), dtype=torch.uint8, device=x.device)
        le = torch.empty((B, iters, 2, K + 3), dtype=dt, device=x.device)
        c.decode(x, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
    return bits.cpu().numpy(), le.cpu().numpy()


@pytest.mark.parametrize("K,f1,f2,B,ebn0", [(40, 3, 10, 1, 0.0), (40, 3, 10, 13, -1.0), (1024, 31, 64, 9, 0.3),
                                            (6144, 263, 480, 3, 0.6), (104, 7, 26, 17, 0.5)])
def test_batch_vs_oracle_every_iteration(K, f1, f2, B, ebn0):
    """Ragged batches (B not a multiple of 8): every iteration's hard bits identical to the
    oracle, Le within 1e-9 (same fp64 operation order)."""
    _, flow = O.synth_batch(K, f1, f2, ebn0, 100 + B, B)
    iters = 5
    bits, le = _decode_all(K, f1, f2, iters, flow)
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters)
        assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"


# LTE sizes with their 36.212 Table 5.1.3-3 parameters: 4 to 137 windows of the kernel's 15-step
# windows, L = K+3 mod 15 = 6, 14, 3, 4, 5, 11 (the edge residues have their own test below), ragged
# batches
@pytest.mark.parametrize("K,f1,f2", [(48, 7, 12), (56, 19, 42), (120, 103, 90), (136, 9, 34),
                                     (512, 31, 64), (2048, 31, 64)])
@pytest.mark.parametrize("algo", ["logmap", "maxlog"])
def test_lte_sizes_vs_oracle(K, f1, f2, algo):
    B, iters = 11, 3
    _, flow = O.synth_batch(K, f1, f2, 0.4, 900 + K, B)
    bits, le = _decode_all(K, f1, f2, iters, flow, algo=algo)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=oalgo)
        assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"


# The 15-step window's edge residues (round 4): L = K+3 = 0 mod 15 -- the last window is full, so
# the B pass has no partial window (K = 72, 192, 432) -- L = 1 mod 15 -- a one-step last window
# (K = 88) -- and L = 9, 10 mod 15 (K = 216, 352).  LTE sizes, 36.212 Table 5.1.3-3 parameters.
WINDOW_EDGE_SIZES = [(72, 7, 18), (88, 5, 22), (192, 23, 48), (216, 11, 36), (352, 21, 44), (432, 47, 72)]


@pytest.mark.parametrize("K,f1,f2", WINDOW_EDGE_SIZES)
@pytest.mark.parametrize("algo", ["logmap", "maxlog"])
@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_window_edge_residues_vs_oracle(K, f1, f2, algo, precision):
    """Every iteration's bits and Le against the oracle at the window residues L mod 15 = 0, 1, 9, 10,
    ragged B = 13 (one padded codeword group).  fp64: bits identical, Le within 1e-9 (the oracle's
    operation order); fp32: the oracle's fp32 restatement, Max-Log-MAP bits identical and log-MAP
    bits identical at the last iteration (converged frames at 1.5 dB), Le within 1e-3 relative."""
    B, iters = 13, 4
    ebn0 = 0.4 if precision == "f64" else 1.5
    _, flow = O.synth_batch(K, f1, f2, ebn0, 1300 + K, B)
    if precision == "f32":
        flow = flow.astype(np.float32)
    bits, le = _decode_all(K, f1, f2, iters, flow, algo=algo, precision=precision)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=oalgo)
        if precision == "f64":
            assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
            assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"
            continue
        if algo == "maxlog":
            assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
        else:
            assert np.array_equal(bits[b, -1], ob[-1].astype(np.uint8)), f"codeword {b}"
        tol = 2e-3 if algo == "maxlog" else 1e-3
        assert np.abs(le[b] - ol).max() <= tol * max(1.0, np.abs(ol).max()), f"codeword {b}"


@pytest.mark.parametrize("K,f1,f2", [(9, 2, 3), (10, 3, 10), (20, 3, 10), (117, 2, 39)])
@pytest.mark.parametrize("algo", ["logmap", "maxlog"])
def test_four_per_cu_w12_residues(monkeypatch, K, f1, f2, algo):
    """fp32 at four workgroups per CU runs the 12-step-window build (launch_turbo4_w12): B = 6150
    (769 groups) at L = K+3 = 0, 1, 11, 0 mod 12 (K = 9, 10, 20, 117; LTE sizes only take 3, 7, 11).
    Bits and Le equal the two-per-CU 15-step kernel's (TD_OCC3=0) exactly, and a sample of codewords
    matches the oracle's fp32 restatement (Max-Log-MAP bits identical, log-MAP bits identical at the
    last iteration on converged frames at 2.5 dB, Le within 1e-3 / 2e-3 relative)."""
    B, iters = 6150, 3
    _, flow = O.synth_batch(K, f1, f2, 2.5, 4100 + K, B)
    flow = flow.astype(np.float32)
    monkeypatch.setenv("TD_OCC3", "0")
    bits2, le2 = _decode_all(K, f1, f2, iters, flow, algo=algo, precision="f32")
    monkeypatch.setenv("TD_OCC3", "1")
    bits4, le4 = _decode_all(K, f1, f2, iters, flow, algo=algo, precision="f32")
    fast4 = _decode_bits(K, f1, f2, iters, flow, algo=algo, precision="f32")
    assert np.array_equal(bits2, bits4)
    assert np.array_equal(le2.view(np.uint8), le4.view(np.uint8))
    assert np.array_equal(fast4, bits4)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    for b in range(0, B, 409):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=oalgo)
        if algo == "maxlog":
            assert np.array_equal(bits4[b], ob.astype(np.uint8)), f"codeword {b}"
        else:
            assert np.array_equal(bits4[b, -1], ob[-1].astype(np.uint8)), f"codeword {b}"
        tol = 2e-3 if algo == "maxlog" else 1e-3
        assert np.abs(le4[b] - ol).max() <= tol * max(1.0, np.abs(ol).max()), f"codeword {b}"


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_maxlog_vs_oracle(precision):
    K, f1, f2, B, iters = 1024, 31, 64, 8, 4
    _, flow = O.synth_batch(K, f1, f2, 0.2, 7, B)
    if precision == "f32":
        flow = flow.astype(np.float32)
    bits, le = _decode_all(K, f1, f2, iters, flow, algo="maxlog", precision=precision)
    tol = 1e-9 if precision == "f64" else 2e-3
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=O.ALGO_MAXLOG)
        assert np.array_equal(bits[b], ob.astype(np.uint8))
        assert np.abs(le[b] - ol).max() <= tol * max(1.0, np.abs(ol).max() if precision == "f32" else 1.0)


def _decode_bits(K, f1, f2, iters, flow, algo="logmap", precision="f64"):
    """Every iteration's bits without an Le dump: the folds' fast path (siso_wg, TD_FOLD_FAST)."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    dt = torch.float64 if precision == "f64" else torch.float32
    x = torch.from_numpy(flow).to(_dev()).to(dt).contiguous()
    with TurboCodec(K, f1, f2, iterations=iters, algo=algo, precision=precision) as c:
        bits = torch.empty((flow.shape[0], iters, K), dtype=torch.uint8, device=x.device)
        c.decode(x, bits, all_iters=True)
        torch.cuda.synchronize()
    return bits.cpu().numpy()


@pytest.mark.parametrize("precision,algo,K,f1,f2,B", [("f32", "maxlog", 40, 3, 10, 5000), ("f32", "logmap", 40, 3, 10, 5000),
                                                      ("f32", "maxlog", 40, 3, 10, 6150), ("f32", "logmap", 40, 3, 10, 6150),
                                                      ("f64", "maxlog", 40, 3, 10, 6150), ("f64", "logmap", 40, 3, 10, 6150),
                                                      ("f64", "logmap", 1024, 31, 64, 6150)])
def test_three_workgroups_per_cu(monkeypatch, precision, algo, K, f1, f2, B):
    """More codeword groups than two per CU (B = 5000: 625 groups; 6150: 769, more than three per
    CU on 256 CUs) run turbo_decode_kernel3 / turbo_decode_kernel4 (three / four workgroups per CU)
    where the build has them (fp32).  Bits and Le equal the two-workgroup kernel's (TD_OCC3=0)
    exactly -- with an Le dump (the generic fold) and without (the fast fold) -- and a sample of
    codewords matches the oracle: fp64 bit for bit (Le to 1e-9); fp32 as test_maxlog_vs_oracle /
    test_f32_logmap_vs_oracle_f32 (log-MAP: the last iteration's bits on converged frames at 1.0 dB)."""
    iters = 3
    _, flow = O.synth_batch(K, f1, f2, 0.3 if (algo == "maxlog" or precision == "f64") else 1.0, 31, B)
    if precision == "f32":
        flow = flow.astype(np.float32)
    monkeypatch.setenv("TD_OCC3", "0")
    bits2, le2 = _decode_all(K, f1, f2, iters, flow, algo=algo, precision=precision)
    fast2 = _decode_bits(K, f1, f2, iters, flow, algo=algo, precision=precision)
    monkeypatch.setenv("TD_OCC3", "1")
    bits3, le3 = _decode_all(K, f1, f2, iters, flow, algo=algo, precision=precision)
    fast3 = _decode_bits(K, f1, f2, iters, flow, algo=algo, precision=precision)
    assert np.array_equal(bits2, bits3)
    assert np.array_equal(le2.view(np.uint8), le3.view(np.uint8))
    assert np.array_equal(fast2, fast3) and np.array_equal(fast3, bits3)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    # the oracle sample: every 41st (K = 40) / 193rd (K = 1024) codeword and the last one, so every
    # dispatch round and the partial last group are covered (122-151 / 33 codewords)
    for b in list(range(0, B, 41 if K == 40 else 193)) + [B - 1]:
        ob, ol = O.turbo_decode(np.ascontiguousarray(flow[b]), K, f1, f2, iters, algo=oalgo)   # fp32: its restatement
        if precision == "f64":
            assert np.array_equal(bits3[b], ob.astype(np.uint8)), f"codeword {b}"
            assert np.abs(le3[b] - ol).max() <= 1e-9, f"codeword {b}"
            continue
        if algo == "maxlog":
            assert np.array_equal(bits3[b], ob.astype(np.uint8)), f"codeword {b}"
        else:
            assert np.array_equal(bits3[b, -1], ob[-1].astype(np.uint8)), f"codeword {b}"
        tol = 2e-3 if algo == "maxlog" else 1e-3
        assert np.abs(le3[b] - ol).max() <= tol * max(1.0, np.abs(ol).max()), f"codeword {b}"


def test_f32_logmap_vs_oracle_f32():
    """fp32 throughput mode against the oracle's fp32 restatement (same op order): bits identical
    on converged frames, Le close relative to its magnitude."""
    K, f1, f2, B, iters = 1024, 31, 64, 8, 6
    _, flow = O.synth_batch(K, f1, f2, 1.0, 9, B)
    flow = flow.astype(np.float32)
    bits, le = _decode_all(K, f1, f2, iters, flow, precision="f32")
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters)
        assert np.array_equal(bits[b, -1], ob[-1].astype(np.uint8))
        assert np.abs(le[b] - ol).max() <= 1e-3 * max(1.0, np.abs(ol).max())


def test_decode_is_deterministic_and_batch_invariant():
    """Same codeword alone or inside a batch, and decoded twice: identical bits and Le."""
    K, f1, f2 = 1024, 31, 64
    _, flow = O.synth_batch(K, f1, f2, 0.4, 55, 24)
    b1, l1 = _decode_all(K, f1, f2, 3, flow)
    b2, l2 = _decode_all(K, f1, f2, 3, flow)
    assert np.array_equal(b1, b2) and np.array_equal(l1, l2)
    b3, l3 = _decode_all(K, f1, f2, 3, flow[17:18])
    assert np.array_equal(b3[0], b1[17]) and np.array_equal(l3[0], l1[17])


def test_full_size_config2_round_trip():
    """BASELINE config 2 at full size (B=4096, K=6144, 8 iterations, 1.0 dB, fp64 log-MAP):
    encode -> AWGN -> decode recovers every info bit (the size-independent property), and a
    seeded sample of codewords matches the oracle bit for bit."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec, synth
    B, K, f1, f2 = 4096, 6144, 263, 480
    u, flow = synth.make_batch(B, K, f1, f2, 1.0, seed=20261015)
    x = torch.from_numpy(flow).to(_dev())
    with TurboCodec(K, f1, f2, iterations=8) as c:
        bits = c.decode(x)
        torch.cuda.synchronize()
    bits = bits.cpu().numpy()
    assert int((bits != u).sum()) == 0
    sample = np.random.default_rng(0).choice(B, 4, replace=False)
    ob = O.decode_batch(np.ascontiguousarray(flow[sample]), K, f1, f2, 8, nthreads=4)
    assert np.array_equal(ob, bits[sample])
    # the other arithmetic modes at full size (both dispatch rounds of workgroups, whose roles are
    # rotated): every info bit recovered at 1.0 dB
    u_d = torch.from_numpy(u).to(_dev())
    for algo, prec in (("logmap", "f32"), ("maxlog", "f64"), ("maxlog", "f32")):
        xx = x if prec == "f64" else x.float()
        with TurboCodec(K, f1, f2, iterations=8, algo=algo, precision=prec) as c:
            b2 = c.decode(xx)
            torch.cuda.synchronize()
        assert int((b2 != u_d).sum().item()) == 0, (algo, prec)


def test_full_size_f32_large_batch(monkeypatch):
    """Config 4's per-GPU shard size in fp32 (B = 32768, K = 6144, 8 iterations, 1.0 dB, the
    device generator's frames of srand(20261015)): the occupancy pick runs four workgroups per CU
    (turbo_decode_kernel4); its hard bits equal the two-per-CU kernel's (TD_OCC3=0) and recover
    every info bit, in log-MAP and Max-Log-MAP; six codewords across its dispatch rounds equal the
    oracle's fp32 restatement."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    B, K, f1, f2 = 32768, 6144, 263, 480
    with TurboCodec(K, f1, f2, iterations=8) as g:
        g.synth_seed(20261015)
        u, llr = g.synth(B, 1.0)
        torch.cuda.synchronize()
    x = llr.float()
    del llr
    for algo in ("logmap", "maxlog"):
        out = {}
        for occ in ("1", "0"):
            monkeypatch.setenv("TD_OCC3", occ)
            with TurboCodec(K, f1, f2, iterations=8, algo=algo, precision="f32") as c:
                out[occ] = c.decode(x)
                torch.cuda.synchronize()
        assert torch.equal(out["1"], out["0"]), algo
        assert int((out["1"] != u).sum().item()) == 0, algo
        # parity, not only self-consistency: a sample spread over the four-per-CU kernel's dispatch
        # rounds against the oracle's fp32 restatement (converged frames: equal bits)
        sample = [0, 4097, 12345, 20000, 28671, 32767]
        xs = np.ascontiguousarray(x[sample].cpu().numpy())
        ob = O.decode_batch(xs, K, f1, f2, 8, algo=O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP,
                            nthreads=6)
        assert np.array_equal(ob, out["1"][sample].cpu().numpy()), algo


def test_le_dump_layout_against_golden():
    """td_decode_device's Le dump ([B][iters][2][K+3]) and all-iteration bits on a golden frame."""
    d = np.load(os.path.join(GOLD, "frames_K1024_e0.5_s11.npz"))
    bits, le = _decode_all(int(d["K"]), int(d["f1"]), int(d["f2"]), int(d["iters"]), d["flow"])
    assert np.array_equal(bits, d["bits"])
    assert np.abs(le - d["le"]).max() <= 1e-4


# ---------------------------------------------------------------- compat layer on the GPU
@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("compat") / "compat_driver")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(REPO, "tests", "compat_driver.cpp"),
                           f"-L{PKG}", "-lturbo_logmap_compat", "-lturbo_mi355x", f"-Wl,-rpath,{PKG}"])
    return out


@pytest.mark.parametrize("name", ["frames_K1024_e0.0_s11.npz", "frames_K40_e0.0_s31.npz"])
def test_compat_turbo_decoding(driver, tmp_path, name):
    """The reference's TurboDecoding(flow, out, 3K+12) entry point: out[15][K] rows equal the
    reference's first 8 rows (golden), flow is scaled by 0.5 in place (log_map.cpp:1202-1205)."""
    d = np.load(os.path.join(GOLD, name))
    K, nf = int(d["K"]), d["flow"].shape[0]
    d["flow"].astype(np.float64).tofile(tmp_path / "flow.bin")
    subprocess.check_call([driver, "decode", str(K), str(int(d["f1"])), str(int(d["f2"])), str(nf),
                           str(tmp_path / "flow.bin"), str(tmp_path / "out.bin")], timeout=300)
    out = np.fromfile(tmp_path / "out.bin", dtype=np.int32).reshape(nf, 15, K)
    it = int(d["iters"])
    assert np.array_equal(out[:, :it].astype(np.uint8), d["bits"])
    flow2 = np.fromfile(str(tmp_path / "out.bin") + ".flow", dtype=np.float64).reshape(nf, -1)
    assert np.array_equal(flow2, d["flow"] * 0.5)


@pytest.mark.parametrize("algo,W,g,table", [("maxlog", 16, 48, ""), ("logmap", 64, 30, ""), ("logmap", 32, 30, ""),
                                            ("logmap", 64, 30, "exact")])
def test_compat_window_schedule(driver, tmp_path, algo, W, g, table):
    """The compat layer's opt-in sub-block schedule (TD_WINDOW / TD_OVERLAP, read at
    TurboCodingInit): the unchanged caller's TurboDecoding then runs the windowed kernels.  Its rows
    equal the windowed restatement (oracle/turbo_oracle_window.inc) bit for bit; with Max-Log-MAP
    and an overlap reaching both trellis ends (K = 40: L = 43 <= 48) they also equal the exact
    decoder's (the exact anchor of test_gpu_window.py).  Without TD_WINDOW the same driver is the
    exact schedule (test_compat_turbo_decoding)."""
    K, f1, f2, nf, it = (40, 3, 10, 4, 4) if algo == "maxlog" else (1024, 31, 64, 3, 4)
    _, flow = O.synth_batch(K, f1, f2, 0.3, 51 + W, nf)
    flow.astype(np.float64).tofile(tmp_path / "flow.bin")
    env = dict(os.environ, TD_ITERATIONS=str(it), TD_WINDOW=str(W), TD_OVERLAP=str(g), TD_ALGO=algo,
               TD_WINDOW_MAXSTAR=table)
    subprocess.run([driver, "decode", str(K), str(f1), str(f2), str(nf), str(tmp_path / "flow.bin"),
                    str(tmp_path / "out.bin")], env=env, timeout=300, check=True)
    out = np.fromfile(tmp_path / "out.bin", dtype=np.int32).reshape(nf, 15, K)[:, :it].astype(np.uint8)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else (O.ALGO_LOGMAP if table == "exact" else O.ALGO_LOGMAP_Q)
    for b in range(nf):
        wb, _ = O.turbo_decode_window(flow[b], K, f1, f2, it, W, g, algo=oalgo)
        assert np.array_equal(out[b], wb), f"frame {b}"
        if algo == "maxlog":
            ob, _ = O.turbo_decode(flow[b], K, f1, f2, it, algo=oalgo)
            assert np.array_equal(out[b], ob.astype(np.uint8)), f"frame {b}"
    flow2 = np.fromfile(str(tmp_path / "out.bin") + ".flow", dtype=np.float64).reshape(nf, -1)
    assert np.array_equal(flow2, flow * 0.5)


def test_decode_rejects_bad_buffers():
    """Shape / dtype / device checks of TurboCodec.decode (the kernels would write past a short
    buffer): wrong stream length, all_iters bits of the final-only shape, Le of the other dtype."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, B, iters = 40, 4, 2
    dev = _dev()
    with TurboCodec(K, 3, 10, iterations=iters) as c:
        good = torch.zeros((B, 3 * K + 12), dtype=torch.float64, device=dev)
        with pytest.raises(ValueError):
            c.decode(torch.zeros((B, 3 * K + 11), dtype=torch.float64, device=dev))
        with pytest.raises(ValueError):
            c.decode(good, torch.empty((B, K), dtype=torch.uint8, device=dev), all_iters=True)
        with pytest.raises(ValueError):
            c.decode(good, le=torch.empty((B, iters, 2, K + 3), dtype=torch.float32, device=dev))
        with pytest.raises(ValueError):
            c.decode(good, le=torch.empty((B, iters, 2, K + 2), dtype=torch.float64, device=dev))
        c.decode(good, torch.empty((B, iters, K), dtype=torch.uint8, device=dev), all_iters=True,
                 le=torch.empty((B, iters, 2, K + 3), dtype=torch.float64, device=dev))
        torch.cuda.synchronize()


def test_one_handle_two_streams():
    """One handle, decodes issued alternately on two streams with no host synchronisation: the
    handle orders them on its workspace (td_decode_device waits on the previous decode's event),
    so every batch decodes to the oracle's bits."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, B, iters = 1024, 31, 64, 16, 3
    dev = _dev()
    flows = [O.synth_batch(K, f1, f2, 0.3 + 0.1 * k, 300 + k, B)[1] for k in range(4)]
    xs = [torch.from_numpy(f).to(dev) for f in flows]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        outs = []
        for k, x in enumerate(xs):
            s = streams[k % 2]
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                outs.append(c.decode(x, stream=s))
        torch.cuda.synchronize()
    for f, b in zip(flows, outs):
        ob = O.decode_batch(np.ascontiguousarray(f), K, f1, f2, iters, nthreads=4)
        assert np.array_equal(b.cpu().numpy(), ob)


@pytest.mark.parametrize("K,f1,f2", [(1, 1, 2), (5, 1, 10), (16, 1, 4)])
@pytest.mark.parametrize("algo", ["logmap", "maxlog"])
def test_tiny_K_vs_oracle(K, f1, f2, algo):
    """Trellises shorter than one 15-step kernel window (L = 4, 8) and one window and a third
    (L = 19): every iteration's bits equal the oracle's, Le within 1e-9 (the reference's own
    frames at K = 8, 24 and 10000 are in tests/golden and run through test_turbo_vs_reference)."""
    B, iters = 9, 3
    _, flow = O.synth_batch(K, f1, f2, 0.3, 700 + K, B)
    bits, le = _decode_all(K, f1, f2, iters, flow, algo=algo)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=oalgo)
        assert np.array_equal(bits[b], ob.astype(np.uint8)), f"codeword {b}"
        assert np.abs(le[b] - ol).max() <= 1e-9, f"codeword {b}"


@pytest.mark.parametrize("name", ["frames_K40_e0.0_s31.npz", "frames_K72_e0.5_s44.npz"])
def test_dropin_latency_driver_matches_reference(tmp_path, name):
    """examples/dropin_latency.cpp (bench.py's `dropin`): the unchanged caller's one-frame-per-call
    TurboDecoding through libturbo_logmap_compat.so.  With TD_ITERATIONS = the golden frames' iteration
    count, each frame's last-iteration row equals the compiled reference's (tests/golden), and the
    driver reports a positive warm per-frame time."""
    import json

    d = np.load(os.path.join(GOLD, name))
    K, nf, it = int(d["K"]), d["flow"].shape[0], int(d["iters"])
    d["flow"].astype(np.float64).tofile(tmp_path / "flow.bin")
    env = dict(os.environ, TD_ITERATIONS=str(it))
    r = subprocess.run([os.path.join(PKG, "td_dropin_latency"), str(K), str(int(d["f1"])), str(int(d["f2"])), str(nf),
                        str(tmp_path / "flow.bin"), str(tmp_path / "bits.bin")], capture_output=True, text=True,
                       env=env, timeout=300, check=True)
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["frames"] == nf and rec["ms_per_frame"] > 0
    bits = np.fromfile(tmp_path / "bits.bin", dtype=np.uint8).reshape(nf, K)
    assert np.array_equal(bits, d["bits"][:, it - 1])


_REDO_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from turbo_decoder_cuda_amd import TurboCodec
d = np.load(sys.argv[2])
out = {}
for prec, dt in (("f64", torch.float64), ("f32", torch.float32)):
    x = torch.from_numpy(d["flow"]).to("cuda").to(dt).contiguous()
    K, B, it = int(d["K"]), x.shape[0], int(d["iters"])
    with TurboCodec(K, int(d["f1"]), int(d["f2"]), iterations=it, precision=prec) as c:
        bits = torch.empty((B, it, K), dtype=torch.uint8, device=x.device)
        le = torch.empty((B, it, 2, K + 3), dtype=dt, device=x.device)
        c.decode(x, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
    out["bits_" + prec], out["le_" + prec] = bits.cpu().numpy(), le.cpu().numpy()
np.savez(sys.argv[3], **out)
"""


def test_alpha_speculation_redo_path_is_exact(tmp_path):
    """The log-MAP alpha window reads its max* rows speculatively and recomputes a window in the
    committed order when a bucket check fails (td_kernels.hip kASpec), which practically never
    happens on real data.  libturbo_mi355x_redo.so (build.py, -DTD_ASPEC_REDO) takes the redo on
    every window: its bits and Le equal the production library's bit for bit, fp64 and fp32, on
    the reference's K = 1024 frames and a K = 6144 batch (and the fp64 bits the reference's)."""
    redo = os.path.join(PKG, "libturbo_mi355x_redo.so")
    assert os.path.exists(redo), "build() makes the redo-forced library"
    K, f1, f2 = 6144, 263, 480
    _, flow = O.synth_batch(K, f1, f2, 0.6, 4242, 11)
    cases = [("gold", dict(np.load(os.path.join(GOLD, "frames_K1024_e0.5_s11.npz")))),
             ("k6144", dict(K=K, f1=f1, f2=f2, iters=3, flow=flow))]
    for tag, d in cases:
        np.savez(tmp_path / f"{tag}_in.npz", **{k: d[k] for k in ("K", "f1", "f2", "iters", "flow")})
        env = dict(os.environ, TD_LIB_PATH=redo)
        subprocess.run(["python", "-c", _REDO_CHILD, REPO, str(tmp_path / f"{tag}_in.npz"), str(tmp_path / f"{tag}_out.npz")],
                       env=env, check=True, timeout=300)
        r = np.load(tmp_path / f"{tag}_out.npz")
        K_, it = int(d["K"]), int(d["iters"])
        for prec in ("f64", "f32"):
            bits, le = _decode_all(K_, int(d["f1"]), int(d["f2"]), it, d["flow"].astype(np.float64), precision=prec)
            assert np.array_equal(r["bits_" + prec], bits), (tag, prec)
            assert np.array_equal(r["le_" + prec], le), (tag, prec)
        if tag == "gold":
            assert np.array_equal(r["bits_f64"], d["bits"])
