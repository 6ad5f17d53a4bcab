"""Device frame generator and BER harness against the compiled
reference's own frames and BER counts (tests/golden, oracle/gen_golden.py, gen_ber_golden.py)."""
import glob
import json
import os

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD

pytestmark = pytest.mark.gpu


def _codec(K, f1, f2, iters=8):
    from turbo_decoder_cuda_amd import TurboCodec
    return TurboCodec(K, f1, f2, iterations=iters)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "frames_*.npz"))), ids=os.path.basename)
def test_synth_reproduces_reference_frames(path):
    """srand(seed) + main.cpp's frames (source, TurboEnCoding, BPSK, AWGN x2, demod) on the GPU:
    the same source bits and bit-identical channel LLRs as the compiled reference."""
    import torch
    d = np.load(path)
    K, nf = int(d["K"]), d["flow"].shape[0]
    with _codec(K, int(d["f1"]), int(d["f2"])) as c:
        c.synth_seed(int(d["seed"]))
        info, llr = c.synth(nf, float(d["ebn0"]))
        torch.cuda.synchronize()
    assert np.array_equal(info.cpu().numpy(), d["src"])
    assert np.array_equal(llr.cpu().numpy(), d["flow"])


def test_synth_long_stream_and_seek():
    """Frames deep into the stream (jump-ahead) equal the restated generator run sequentially;
    seek repositions the stream."""
    import torch
    K, f1, f2, seed = 1024, 31, 64, 99
    src, flow = O.make_frames(K, f1, f2, 0.7, seed, 40)
    with _codec(K, f1, f2) as c:
        c.synth_seed(seed)
        i1, l1 = c.synth(25, 0.7)
        i2, l2 = c.synth(15, 0.7)
        c.synth_seek(33)
        i3, l3 = c.synth(2, 0.7)
        torch.cuda.synchronize()
    info = np.concatenate([i1.cpu().numpy(), i2.cpu().numpy()])
    llr = np.concatenate([l1.cpu().numpy(), l2.cpu().numpy()])
    assert np.array_equal(info, src.astype(np.uint8))
    assert np.array_equal(llr, flow)
    assert np.array_equal(l3.cpu().numpy(), flow[33:35])


def test_count_errors_matches_numpy():
    import torch
    K, B, it = 1024, 13, 3
    rng = np.random.default_rng(4)
    info = rng.integers(0, 2, (B, K), dtype=np.uint8)
    bits = np.repeat(info[:, None, :], it, axis=1).copy()
    flip = rng.random((B, it, K)) < 0.01
    bits[flip] ^= 1
    with _codec(K, 31, 64, it) as c:
        err = c.count_errors(torch.from_numpy(bits).cuda(), torch.from_numpy(info).cuda()).cpu().numpy()
    assert np.array_equal(err, flip.sum(axis=2))


def _oracle_point(K, f1, f2, iters, ebn0, seed, maxf, minerr):
    """main.cpp's loop with the CPU restatement (oracle): srand(seed), frames in order."""
    src, flow = O.make_frames(K, f1, f2, ebn0, seed, maxf)
    bit, blk, nf = [0] * iters, [0] * iters, 0
    for fr in range(maxf):
        bits, _ = O.turbo_decode(flow[fr], K, f1, f2, iters)
        nf += 1
        for it in range(iters):
            e = int((bits[it] != src[fr]).sum())
            bit[it] += e
            blk[it] += e != 0
        if blk[iters - 1] >= minerr:
            break
    return nf, bit, blk


def test_ber_matches_oracle_exactly():
    """GPU harness (device frames + GPU decode + device error counts + main.cpp's stopping rule)
    equals the same loop run with the CPU restatement, count for count."""
    from turbo_decoder_cuda_amd.ber import ber_sweep
    K, f1, f2, it, seed, maxf, minerr = 1024, 31, 64, 8, 2026, 400, 30
    pts_e = [0.0, 0.3, 0.5]
    with _codec(K, f1, f2, it) as c:
        pts = ber_sweep(c, pts_e, seed, maxf, minerr, batch=256, reseed_each_point=True)
    for e, got in zip(pts_e, pts):
        nf, bit, blk = _oracle_point(K, f1, f2, it, e, seed, maxf, minerr)
        assert (got.frames, got.bit_errors, got.block_errors) == (nf, bit, blk), e


@pytest.mark.parametrize("K", [1024, 6144])
def test_ber_matches_reference(K):
    """Against the compiled reference's own BER runs (same srand stream, same stopping rule): the
    same frame counts, block errors within one frame and bit errors within 0.5 % (far inside the
    0.05 dB BER gate of BASELINE.json).  Exact equality is not defined: the reference normalises
    with an uninitialised tempmax (log_map.cpp:925,989), which moves a non-converged frame's LLRs
    near zero.  Observed (the oracle, equal to the GPU count for count): identical counts at
    every point but 0.0/0.2 dB K=1024, whose iterations 7-8 differ by at most 9 of ~4000 bits."""
    from turbo_decoder_cuda_amd.ber import ber_sweep
    g = json.load(open(os.path.join(GOLD, f"ber_K{K}.json")))
    it = g["iters"]
    with _codec(K, g["f1"], g["f2"], it) as c:
        pts = ber_sweep(c, [p["ebn0"] for p in g["points"]], g["seed"], g["maxframes"], g["minerr"], batch=1024,
                        reseed_each_point=True)
    for ref, got in zip(g["points"], pts):
        assert got.frames == ref["frames"], ref["ebn0"]
        for a, b in zip(got.block_errors, ref["block_errors"][:it]):
            assert abs(a - b) <= 1, ref["ebn0"]
        for a, b in zip(got.bit_errors, ref["bit_errors"][:it]):
            assert abs(a - b) <= max(2, 5e-3 * b), ref["ebn0"]


def test_config4_shard_reference_frames():
    """BASELINE config 4's per-GPU shard at full size: 32768 K=6144 frames of main.cpp's own stream
    (device generator, bit-identical to the reference's frames) at 1.0 dB through the exact fp64
    decoder -- eight dispatch rounds of workgroups.  The BER is at the reference's level at 1.0 dB
    (ITTC/result.txt:18, :92: 0 and below 1e-8), and every frame with a residual error, plus a seeded
    sample, equals the oracle bit for bit (the errors are the code's, not the decoder's)."""
    import torch
    K, f1, f2, B, seed = 6144, 263, 480, 32768, 20261016
    with _codec(K, f1, f2) as c:
        c.synth_seed(seed)
        info, llr = c.synth(B, 1.0)
        bits = c.decode(llr)
        err = c.count_errors(bits.view(B, 1, K), info)[:, 0]
        torch.cuda.synchronize()
        bad = torch.nonzero(err).flatten().cpu().numpy()
        pick = np.unique(np.concatenate([bad, np.random.default_rng(1).choice(B, 3, replace=False)]))
        idx = torch.from_numpy(pick).cuda()
        flows, got = llr[idx].cpu().numpy(), bits[idx].cpu().numpy()
        nerr = int(err.sum().item())
    assert nerr / (B * K) < 1e-6 and len(bad) <= 8
    ob = O.decode_batch(np.ascontiguousarray(flows), K, f1, f2, 8, nthreads=4)
    assert np.array_equal(ob, got)
