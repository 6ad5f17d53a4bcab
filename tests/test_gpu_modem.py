"""Modulators / demodulators on the GPU (td_modulate / td_demodulate /
td_synth_modulation) against the compiled reference's outputs (tests/golden/demod.npz,
modframes_K1024.npz, oracle/gen_demod_golden.py) and the oracle restatement: bit-exact."""
import os

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
def test_demodulate_matches_reference(M):
    import torch

    from turbo_decoder_cuda_amd import demodulate
    d = np.load(os.path.join(GOLD, "demod.npz"))
    yi = torch.from_numpy(d[f"yi_{M}"]).cuda()
    yq = torch.from_numpy(d[f"yq_{M}"]).cuda()
    got = demodulate(yi, yq, M, float(d["Kf"])).cpu().numpy()
    assert np.array_equal(got, d[f"llr_{M}"])


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
def test_demodulate_large_random_matches_oracle(M):
    import torch

    from turbo_decoder_cuda_amd import demodulate
    rng = np.random.default_rng(M)
    yi, yq = rng.normal(0, 1.2, 200_003), rng.normal(0, 1.2, 200_003)
    got = demodulate(torch.from_numpy(yi).cuda(), torch.from_numpy(yq).cuda(), M, 0.83).cpu().numpy()
    assert np.array_equal(got, O.demodulate(yi, yq, M, 0.83))


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1001])
def test_demodulate_ragged_and_unaligned(M, n):
    """Symbol counts around a wave (the staged stores' partial last wave, BPSK's odd count) and
    buffers 8 bytes off a 16-byte boundary (the 8-byte-access kernel): equal to the oracle."""
    import torch

    from turbo_decoder_cuda_amd import demodulate
    rng = np.random.default_rng(100 * M + n)
    yi, yq = rng.normal(0, 1.2, n), rng.normal(0, 1.2, n)
    want = O.demodulate(yi, yq, M, 0.83)
    got = demodulate(torch.from_numpy(yi).cuda(), torch.from_numpy(yq).cuda(), M, 0.83).cpu().numpy()
    assert np.array_equal(got, want)
    bi = torch.zeros(n + 1, dtype=torch.float64, device="cuda")
    bq = torch.zeros(n + 1, dtype=torch.float64, device="cuda")
    bi[1:] = torch.from_numpy(yi).cuda()
    bq[1:] = torch.from_numpy(yq).cuda()
    got = demodulate(bi[1:], bq[1:], M, 0.83).cpu().numpy()   # inputs at +8 bytes
    assert np.array_equal(got, want)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6])
def test_modulate_matches_oracle(M):
    import torch

    from turbo_decoder_cuda_amd import modulate
    bits = np.random.default_rng(10 + M).integers(0, 2, 3000 * M)
    si, sq = modulate(torch.from_numpy(bits.astype(np.uint8)).cuda(), M)
    oi, oq = O.modulate(bits, M)
    assert np.array_equal(si.cpu().numpy(), oi) and np.array_equal(sq.cpu().numpy(), oq)


@pytest.mark.parametrize("M", [2, 3, 4, 6])
def test_generator_with_modulation_reproduces_reference_frames(M):
    """td_synth_modulation(M): main.cpp's frames with MODULATION = M, bit for bit; decoding them
    gives the oracle's bits (same input, exact decoder)."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    d = np.load(os.path.join(GOLD, "modframes_K1024.npz"))
    K, f1, f2 = int(d["K"]), int(d["f1"]), int(d["f2"])
    nf = d[f"src_{M}"].shape[0]
    with TurboCodec(K, f1, f2, iterations=4) as c:
        c.synth_modulation(M)
        c.synth_seed(int(d["seed"]))
        info, llr = c.synth(nf, float(d["ebn0"]))
        assert np.array_equal(info.cpu().numpy(), d[f"src_{M}"])
        assert np.array_equal(llr.cpu().numpy(), d[f"flow_{M}"])
        bits = torch.empty((nf, K), dtype=torch.uint8, device=llr.device)
        c.decode(llr, bits)
        for b in range(nf):
            ob, _ = O.turbo_decode(d[f"flow_{M}"][b], K, f1, f2, 4)
            assert np.array_equal(bits[b].cpu().numpy(), ob[-1].astype(np.uint8))


def test_modulation_rejects_bad_arguments():
    """Only 1, 2, 3, 4, 6 bits per symbol (modanddem.cpp:674-685); 3K+12 = 3(K+4) is a whole number
    of symbols for every LTE K (K = 0 mod 8)."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec, demodulate
    from turbo_decoder_cuda_amd import _native as N
    with TurboCodec(40, 3, 10, iterations=2) as c:
        for M in (0, 5, 7, 8):
            with pytest.raises(N.TurboError):
                c.synth_modulation(M)
        for M in (1, 2, 3, 4, 6):
            c.synth_modulation(M)
    with pytest.raises(N.TurboError):
        demodulate(torch.zeros(4, dtype=torch.float64, device="cuda"), torch.zeros(4, dtype=torch.float64,
                                                                                   device="cuda"), 5, 1.0)
