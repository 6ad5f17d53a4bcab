"""ctypes front-end of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
the checker or the reported CPU baseline.  The product package (turbo_decoder_cuda_amd)
never imports this module.  Every wrapped function restates a reference function; the
citations live in oracle/turbo_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

ALGO_LOGMAP = 0
ALGO_MAXLOG = 1
ALGO_LOGMAP_Q = 2   # the windowed schedule's one-read max* table (td_set_window_maxstar TD_WMAXSTAR_FAST)


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


class Trellis(C.Structure):
    _fields_ = [
        ("nextout", (C.c_int * 4) * 8),
        ("nextstat", (C.c_int * 2) * 8),
        ("lastout", (C.c_int * 4) * 8),
        ("laststat", (C.c_int * 2) * 8),
        ("g_fb", C.c_int * 4),
        ("g_ff", C.c_int * 4),
    ]


class GlibcRand(C.Structure):
    _fields_ = [("tbl", C.c_int32 * 31), ("f", C.c_int), ("b", C.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.tdo_build_trellis.argtypes = [C.c_int, C.c_int, C.POINTER(Trellis)]
        L.tdo_qpp.argtypes = [C.c_int, C.c_int, C.c_int, P]
        L.tdo_turbo_encode.argtypes = [C.POINTER(Trellis), P, P, C.c_int, P]
        L.tdo_maxstar.argtypes = [C.c_double, C.c_double]
        L.tdo_maxstar.restype = C.c_double
        L.tdo_maxstar_f32.argtypes = [C.c_float, C.c_float]
        L.tdo_maxstar_f32.restype = C.c_float
        L.tdo_maxstar_q.argtypes = [C.c_double, C.c_double]
        L.tdo_maxstar_q.restype = C.c_double
        L.tdo_maxstar_q_f32.argtypes = [C.c_float, C.c_float]
        L.tdo_maxstar_q_f32.restype = C.c_float
        L.tdo_maxstar_seq.argtypes = [P, C.c_int]
        L.tdo_maxstar_seq.restype = C.c_double
        L.tdo_demultiplex.argtypes = [P, C.c_int, P, P]
        L.tdo_siso_f64.argtypes = [C.POINTER(Trellis), P, P, C.c_int, P, C.c_int, C.c_int]
        L.tdo_siso_f32.argtypes = [C.POINTER(Trellis), P, P, C.c_int, P, C.c_int, C.c_int]
        L.tdo_turbo_decode_f64.argtypes = [C.POINTER(Trellis), P, P, C.c_int, C.c_int, C.c_int, P, P]
        L.tdo_turbo_decode_f32.argtypes = [C.POINTER(Trellis), P, P, C.c_int, C.c_int, C.c_int, P, P]
        for sfx in ("f64", "f32"):
            getattr(L, f"tdo_turbo_decode_window_{sfx}").argtypes = [C.POINTER(Trellis), P, P, C.c_int, C.c_int,
                                                                    C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                                    C.c_int, C.c_double, P, P]
        L.tdo_decode_batch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int, P, C.c_int]
        L.tdo_synth_batch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_uint64, C.c_int, P, P]
        L.tdo_glibc_srand.argtypes = [C.POINTER(GlibcRand), C.c_uint]
        L.tdo_glibc_rand_next.argtypes = [C.POINTER(GlibcRand)]
        L.tdo_glibc_rand_next.restype = C.c_int
        L.tdo_make_frame.argtypes = [C.POINTER(Trellis), P, C.c_int, C.c_double, C.POINTER(GlibcRand), P, P]
        L.tdo_mgrns.argtypes = [C.c_double, C.c_double, C.c_double, C.c_int, P]
        L.tdo_modulate.argtypes = [P, C.c_int, C.c_int, P, P]
        L.tdo_demodulate.argtypes = [P, P, C.c_int, C.c_int, C.c_double, P]
        L.tdo_make_frame_mod.argtypes = [C.POINTER(Trellis), P, C.c_int, C.c_double, C.c_int, C.POINTER(GlibcRand),
                                         P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def trellis() -> Trellis:
    t = Trellis()
    assert lib().tdo_build_trellis(13, 15, C.byref(t)) == 1
    return t


def qpp(K: int, f1: int, f2: int) -> np.ndarray:
    pi = np.zeros(K, dtype=np.int32)
    lib().tdo_qpp(K, f1, f2, _p(pi))
    return pi


def encode(src: np.ndarray, f1: int, f2: int) -> np.ndarray:
    src = np.ascontiguousarray(src, dtype=np.int32)
    K = src.size
    coded = np.zeros(3 * K + 12, dtype=np.int32)
    t = trellis()
    pi = qpp(K, f1, f2)
    lib().tdo_turbo_encode(C.byref(t), _p(pi), _p(src), K, _p(coded))
    return coded


def maxstar(x: float, y: float) -> float:
    return lib().tdo_maxstar(x, y)


def maxstar_f32(x: float, y: float) -> float:
    return lib().tdo_maxstar_f32(x, y)


def maxstar_q(x: float, y: float) -> float:
    return lib().tdo_maxstar_q(x, y)


def maxstar_q_f32(x: float, y: float) -> float:
    return lib().tdo_maxstar_q_f32(x, y)


def siso(recs: np.ndarray, La: np.ndarray, terminated: int = 1, algo: int = ALGO_LOGMAP) -> np.ndarray:
    f32 = recs.dtype == np.float32
    recs = np.ascontiguousarray(recs)
    La = np.ascontiguousarray(La, dtype=recs.dtype)
    L = La.size
    out = np.zeros(L, dtype=recs.dtype)
    t = trellis()
    fn = lib().tdo_siso_f32 if f32 else lib().tdo_siso_f64
    fn(C.byref(t), _p(recs), _p(La), terminated, _p(out), L, algo)
    return out


def turbo_decode(flow: np.ndarray, K: int, f1: int, f2: int, iters: int, algo: int = ALGO_LOGMAP):
    """One codeword through the TurboDecoding restatement. Returns (bits[iters,K] int32, le[iters,2,L])."""
    f32 = flow.dtype == np.float32
    flow = np.ascontiguousarray(flow)
    L = K + 3
    bits = np.zeros((iters, K), dtype=np.int32)
    le = np.zeros((iters, 2, L), dtype=flow.dtype)
    t = trellis()
    pi = qpp(K, f1, f2)
    fn = lib().tdo_turbo_decode_f32 if f32 else lib().tdo_turbo_decode_f64
    fn(C.byref(t), _p(pi), _p(flow), K, iters, algo, _p(bits), _p(le))
    return bits, le


def turbo_decode_window(flow: np.ndarray, K: int, f1: int, f2: int, iters: int, W: int, g: int,
                       algo: int = ALGO_LOGMAP, nii: bool = False, concurrent: bool = False, scale: float = 1.0,
                       nrm: int | None = None):
    """One codeword through the sub-block schedule restatement (turbo_oracle_window.inc): the
    arithmetic of the HIP windowed kernel, normalised every nrm positions of a sub-block (default:
    the kernel's checkpoint spacing, 4 in fp64, 8 in fp32).  Returns (bits[iters,K] uint8, le[iters,2,L])."""
    f32 = flow.dtype == np.float32
    flow = np.ascontiguousarray(flow)
    L = K + 3
    bits = np.zeros((iters, K), dtype=np.int32)
    le = np.zeros((iters, 2, L), dtype=flow.dtype)
    t = trellis()
    pi = qpp(K, f1, f2)
    nrm = nrm or (8 if f32 else 4)
    fn = lib().tdo_turbo_decode_window_f32 if f32 else lib().tdo_turbo_decode_window_f64
    fn(C.byref(t), _p(pi), _p(flow), K, iters, algo, W, g, nrm, int(nii), int(concurrent), scale, _p(bits), _p(le))
    return bits.astype(np.uint8), le


def decode_batch(flow: np.ndarray, K: int, f1: int, f2: int, iters: int, algo: int = ALGO_LOGMAP,
                 nthreads: int = 1) -> np.ndarray:
    """B codewords (flow[B, 3K+12], f64 or f32); returns final-iteration bits[B, K] uint8."""
    flow = np.ascontiguousarray(flow)
    B = flow.shape[0]
    bits = np.zeros((B, K), dtype=np.uint8)
    lib().tdo_decode_batch(K, f1, f2, iters, algo, int(flow.dtype == np.float32), _p(flow), B, _p(bits), nthreads)
    return bits


def synth_batch(K: int, f1: int, f2: int, ebn0_db: float, seed: int, B: int):
    """Synthetic codewords (DESIGN.md 'Synthetic input'): returns (src[B,K] int32, flow[B,3K+12] f64)."""
    src = np.zeros((B, K), dtype=np.int32)
    flow = np.zeros((B, 3 * K + 12), dtype=np.float64)
    lib().tdo_synth_batch(K, f1, f2, ebn0_db, seed, B, _p(src), _p(flow))
    return src, flow


def make_frames(K: int, f1: int, f2: int, ebn0_db: float, seed: int, nframes: int):
    """main.cpp's frame generator with a glibc-rand stream seeded by srand(seed)."""
    g = GlibcRand()
    lib().tdo_glibc_srand(C.byref(g), seed)
    t = trellis()
    pi = qpp(K, f1, f2)
    srcs = np.zeros((nframes, K), dtype=np.int32)
    flows = np.zeros((nframes, 3 * K + 12), dtype=np.float64)
    for i in range(nframes):
        lib().tdo_make_frame(C.byref(t), _p(pi), K, ebn0_db, C.byref(g), _p(srcs[i]), _p(flows[i]))
    return srcs, flows


def modulate(bits: np.ndarray, M: int):
    """module() (modanddem.cpp:175): bits -> (symbols_i, symbols_q)."""
    bits = np.ascontiguousarray(bits, dtype=np.int32)
    n = bits.size // M
    si, sq = np.zeros(n), np.zeros(n)
    assert lib().tdo_modulate(_p(bits), bits.size, M, _p(si), _p(sq)) == 0
    return si, sq


def demodulate(yi: np.ndarray, yq: np.ndarray, M: int, Kf: float) -> np.ndarray:
    """demodule() (modanddem.cpp:674): max-log bit LLRs [M * nsym]."""
    yi = np.ascontiguousarray(yi, dtype=np.float64)
    yq = np.ascontiguousarray(yq, dtype=np.float64)
    out = np.zeros(yi.size * M)
    assert lib().tdo_demodulate(_p(yi), _p(yq), yi.size, M, Kf, _p(out)) == 0
    return out


def make_frames_mod(K: int, f1: int, f2: int, ebn0_db: float, M: int, seed: int, nframes: int):
    """main.cpp's frames with MODULATION = M (SYMBOL_NUM = (3K+12)/M), srand(seed)."""
    g = GlibcRand()
    lib().tdo_glibc_srand(C.byref(g), seed)
    t = trellis()
    pi = qpp(K, f1, f2)
    srcs = np.zeros((nframes, K), dtype=np.int32)
    flows = np.zeros((nframes, 3 * K + 12), dtype=np.float64)
    for i in range(nframes):
        lib().tdo_make_frame_mod(C.byref(t), _p(pi), K, ebn0_db, M, C.byref(g), _p(srcs[i]), _p(flows[i]))
    return srcs, flows


def glibc_rand_stream(seed: int, n: int) -> np.ndarray:
    g = GlibcRand()
    lib().tdo_glibc_srand(C.byref(g), seed)
    return np.array([lib().tdo_glibc_rand_next(C.byref(g)) for _ in range(n)], dtype=np.int64)
