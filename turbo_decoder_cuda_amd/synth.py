"""Synthetic channel input for the benchmark and the BER harness (host, numpy, batched).

Restates the producer side of the reference for BPSK/AWGN (the decode's input):
  rsc_encode / encoderm_turbo   ITTC/log_map.cpp:451-583   (RSC 13/15, trellis-terminated, QPP)
  _bpsk_module                  ITTC/modanddem.cpp:88-102  (bit 1 -> +1, bit 0 -> -1)
  sigma                         ITTC/main.cpp:47,174       (sigma = 10^(-EbN0/20) * sqrt(0.5/R))
  _bpsk_demodule                ITTC/modanddem.cpp:189-224 (LLR = 2y/sigma^2)
The noise comes from numpy's PCG64 normal generator (the reference's mgrns CLT-12 generator is
restated in oracle/ for bit-exact fixtures; it is not needed for throughput or BER curves).
"""
from __future__ import annotations

import numpy as np

G_FB = (1, 0, 1, 1)   # 13 octal (G_ROW_1, log_map.h:35)
G_FF = (1, 1, 0, 1)   # 15 octal (G_ROW_2, log_map.h:36)


def qpp(K: int, f1: int, f2: int) -> np.ndarray:
    """gen_qpp_index (log_map.cpp:616-624)."""
    i = np.arange(K, dtype=np.int64)
    return ((f1 * i + ((f2 * i) % K * i) % K) % K).astype(np.int64)


def rsc_encode(u: np.ndarray) -> np.ndarray:
    """Terminated RSC encoding of each row of u [B, K] -> [B, K+3, 2] (systematic, parity)."""
    B, K = u.shape
    out = np.zeros((B, K + 3, 2), dtype=np.uint8)
    s0 = np.zeros(B, dtype=np.uint8)
    s1 = np.zeros(B, dtype=np.uint8)
    s2 = np.zeros(B, dtype=np.uint8)
    for i in range(K + 3):
        fb = (G_FB[1] * s0 + G_FB[2] * s1 + G_FB[3] * s2) & 1
        dk = u[:, i] if i < K else fb            # termination drives the register to 0 (:483-491)
        ak = (G_FB[0] * dk + fb) & 1
        par = (G_FF[0] * ak + G_FF[1] * s0 + G_FF[2] * s1 + G_FF[3] * s2) & 1   # encode_bit (:247-269)
        s2, s1, s0 = s1, s0, ak
        out[:, i, 0] = dk
        out[:, i, 1] = par
    return out


def turbo_encode(u: np.ndarray, f1: int, f2: int) -> np.ndarray:
    """encoderm_turbo (log_map.cpp:530-583): [B, K] bits -> [B, 3K+12] coded stream."""
    B, K = u.shape
    pi = qpp(K, f1, f2)
    r1 = rsc_encode(u)
    r2 = rsc_encode(u[:, pi])
    coded = np.empty((B, 3 * K + 12), dtype=np.uint8)
    coded[:, 0:3 * K:3] = r1[:, :K, 0]
    coded[:, 1:3 * K:3] = r1[:, :K, 1]
    coded[:, 2:3 * K:3] = r2[:, :K, 1]
    coded[:, 3 * K:3 * K + 6] = r1[:, K:, :].reshape(B, 6)
    coded[:, 3 * K + 6:] = r2[:, K:, :].reshape(B, 6)
    return coded


def sigma_for(ebn0_db: float, K: int) -> float:
    rate = K / (3 * K + 12)
    return 10 ** (-ebn0_db / 20) * np.sqrt(0.5 / rate)


def make_batch(B: int, K: int, f1: int, f2: int, ebn0_db: float, seed: int = 20261015,
               dtype=np.float64):
    """Returns (info bits [B, K] uint8, channel LLR [B, 3K+12] dtype)."""
    rng = np.random.default_rng(seed)
    u = rng.integers(0, 2, size=(B, K), dtype=np.uint8)
    coded = turbo_encode(u, f1, f2)
    sigma = sigma_for(ebn0_db, K)
    y = (2.0 * coded.astype(np.float64) - 1.0) + sigma * rng.standard_normal(coded.shape)
    llr = (2.0 / sigma ** 2) * y
    return u, llr.astype(dtype)
