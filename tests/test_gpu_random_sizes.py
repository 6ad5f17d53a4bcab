"""Seeded random block sizes through the C ABI against the oracle (a property sweep beside the fixed
LTE sizes of test_gpu_decode.py / test_gpu_window.py).

The reference takes K, f1 and f2 from its command line (ITTC/main.cpp:18-19) with K up to
MAX_FRAME_LENGTH (main.h), so any K in [1, 10000] whose (f1, f2) gives a QPP permutation is a valid
input.  Each case draws K (LTE-like multiples of 8 and arbitrary K, up to 10000 > 6144), a valid
(f1, f2), a ragged batch, an Eb/N0 and an algorithm from one seeded generator, and checks:
  * the exact schedule: every iteration's hard bits equal the oracle's TurboDecoding restatement and
    Le within 1e-9 (log_map.cpp:1146-1280; the same fp64 operation order);
  * the windowed schedule (W a multiple of the checkpoint spacing, overlaps 0..3W): bits equal
    and Le within 1e-9 of the C restatement of the windowed kernels (turbo_oracle_window.inc).
The draws are fixed by the seed, so a failure names a reproducible case."""
import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu


def _qpp_ok(K, f1, f2):
    return np.unique(O.qpp(K, f1, f2)).size == K


def _draw(rng, n, kmax=10000):
    cases = []
    while len(cases) < n:
        K = int(rng.integers(5, 1251)) * 8 if len(cases) % 2 == 0 else int(rng.integers(9, kmax + 1))
        if K > kmax:
            continue
        for _ in range(200):   # a random valid (f1, f2): f1 < K coprime-ish, f2 < K, permutation checked
            f1 = int(rng.integers(1, K))
            f2 = int(rng.integers(0, K))
            if _qpp_ok(K, f1, f2):
                break
        else:
            continue
        B = int(rng.integers(1, 20))
        ebn0 = float(np.round(rng.uniform(-0.5, 1.0), 2))
        cases.append((K, f1, f2, B, ebn0))
    return cases


EXACT_CASES = _draw(np.random.default_rng(20261018), 24)
WINDOW_CASES = _draw(np.random.default_rng(20261019), 16, kmax=6144)


def _decode(K, f1, f2, iters, flow, algo, window=0, overlap=0):
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    x = torch.from_numpy(flow).to("cuda:0").contiguous()
    B = flow.shape[0]
    with TurboCodec(K, f1, f2, iterations=iters, algo=algo) as c:
        if window:
            c.set_window(window, overlap)
        bits = torch.empty((B, iters, K), dtype=torch.uint8, device=x.device)
        le = torch.empty((B, iters, 2, K + 3), dtype=torch.float64, device=x.device)
        c.decode(x, bits, all_iters=True, le=le)
        torch.cuda.synchronize()
    return bits.cpu().numpy(), le.cpu().numpy()


@pytest.mark.parametrize("case", range(len(EXACT_CASES)))
def test_random_size_exact_vs_oracle(case):
    K, f1, f2, B, ebn0 = EXACT_CASES[case]
    algo = "maxlog" if case % 3 == 2 else "logmap"
    iters = 3
    _, flow = O.synth_batch(K, f1, f2, ebn0, 7000 + case, B)
    bits, le = _decode(K, f1, f2, iters, flow, algo)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP
    for b in range(B):
        ob, ol = O.turbo_decode(flow[b], K, f1, f2, iters, algo=oalgo)
        assert np.array_equal(bits[b], ob.astype(np.uint8)), (EXACT_CASES[case], algo, b)
        assert np.abs(le[b] - ol).max() <= 1e-9, (EXACT_CASES[case], algo, b)


@pytest.mark.parametrize("case", range(len(WINDOW_CASES)))
def test_random_size_window_vs_restatement(case):
    K, f1, f2, B, ebn0 = WINDOW_CASES[case]
    rng = np.random.default_rng(100 + case)
    W = int(rng.choice([16, 32, 48, 64, 96]))
    # every fourth case an overlap past the window (td_set_window allows up to 3 W)
    g = int(rng.integers(0, W + 1)) if case % 4 else W + int(rng.integers(1, 2 * W + 1))
    algo = "maxlog" if case % 3 == 2 else "logmap"
    iters = 3
    _, flow = O.synth_batch(K, f1, f2, ebn0, 8000 + case, B)
    bits, le = _decode(K, f1, f2, iters, flow, algo, W, g)
    oalgo = O.ALGO_MAXLOG if algo == "maxlog" else O.ALGO_LOGMAP_Q
    for b in range(B):
        ob, ol = O.turbo_decode_window(flow[b], K, f1, f2, iters, W, g, algo=oalgo)
        assert np.array_equal(bits[b], ob), (WINDOW_CASES[case], W, g, algo, b)
        assert np.abs(le[b] - ol).max() <= 1e-9, (WINDOW_CASES[case], W, g, algo, b)
