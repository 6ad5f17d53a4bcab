"""Host-side mirror of the reference codec interface (ITTC/log_map.cpp), over the C ABI.

Reference                                   here
  TurboCodingInit()          :349-434   ->  TurboCodec(K, f1, f2, iterations, algo, precision, device)
  TurboDecoding(flow,out,n)  :1146-1280 ->  TurboCodec.TurboDecoding(flow)  (host arrays, batched)
                                            TurboCodec.decode(llr_tensor)   (device-resident, batched)
  Log_MAP_decoder(...)       :898-1047  ->  TurboCodec.Log_MAP_decoder(recs, La, terminated)
  TurboCodingRelease()       :1330-1345 ->  TurboCodec.close()
  N_ITERATION (log_map.h:30)            ->  `iterations` (runtime, default 15 like the macro)
  TYPE_DECODER (log_map.h:26)           ->  `algo` ("logmap" = table max*, "maxlog")

Every decode runs on the MI355X through libturbo_mi355x.so; nothing here computes on the CPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N

N_ITERATION = 15   # log_map.h:30
TERMINATED = 1     # log_map.h:24

_ALGOS = {"logmap": N.TD_ALGO_LOGMAP, "maxlog": N.TD_ALGO_MAXLOG}
_PRECS = {"f64": N.TD_F64, "f32": N.TD_F32}


def stream_length(K: int) -> int:
    """3K+12: the coded stream length TurboDecoding takes (main.cpp:221)."""
    return 3 * K + 12


class TurboCodec:
    def __init__(self, K: int, f1: int, f2: int, iterations: int = N_ITERATION, algo: str = "logmap",
                 precision: str = "f64", device: int = 0):
        self.K, self.f1, self.f2 = int(K), int(f1), int(f2)
        self.L = self.K + 3
        self.iterations = int(iterations)
        self.algo, self.precision = algo, precision
        self.dtype = np.float64 if precision == "f64" else np.float32
        p = N.TdParams(self.K, self.f1, self.f2, self.iterations, _ALGOS[algo], _PRECS[precision], int(device))
        h = C.c_void_p()
        N.check(N.lib().td_create(C.byref(h), C.byref(p)))
        self._h = h
        self.device = int(device)

    # -- lifetime (TurboCodingRelease) -------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            N.lib().td_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reserve(self, B: int) -> None:
        N.check(N.lib().td_reserve(self._h, int(B)))

    def placement(self):
        """(probe ms of each candidate workspace, index kept) of the last reserve that allocated
        (td_debug_placement; ([], -1) for a plain allocation)."""
        pick = C.c_int(-1)
        n = N.lib().td_debug_placement(self._h, None, 0, C.byref(pick))   # the count first
        if n < 0:
            N.check(n)
        ms = (C.c_float * max(n, 1))()
        n = N.lib().td_debug_placement(self._h, ms, n, C.byref(pick))
        return [round(ms[i], 4) for i in range(n)], pick.value

    def placement_cost(self):
        """(wall ms, peak bytes of candidate workspaces held) of that search (td_debug_placement_cost)."""
        if not hasattr(N.lib(), "td_debug_placement_cost"):
            return None, None
        w, b = C.c_double(0), C.c_double(0)
        N.check(N.lib().td_debug_placement_cost(self._h, C.byref(w), C.byref(b)))
        return w.value, b.value

    def workspace_bytes(self) -> int:
        """Bytes of the decode workspace (td_debug_workspace_bytes)."""
        v = C.c_ulonglong(0)
        N.check(N.lib().td_debug_workspace_bytes(self._h, C.byref(v)))
        return int(v.value)

    def set_window_maxstar(self, exact: bool) -> None:
        """max* of the windowed log-MAP schedule (td_set_window_maxstar): exact=False the one-read
        table (default), exact=True log_map.cpp's E_algorithm exactly."""
        N.check(N.lib().td_set_window_maxstar(self._h, N.TD_WMAXSTAR_EXACT if exact else N.TD_WMAXSTAR_FAST))

    def set_window(self, window: int = 64, overlap: int = 30, ext_scale: float = 1.0, nii: bool = False,
                   concurrent: bool = False) -> None:
        """Windowed schedule (td_set_window; BASELINE config 5); window=0: exact.
        The reference GPU decoder with P sub-blocks (turboDecoderBianJieZhi.cu) is
        set_window(6144 // P, 0, 0.77, nii=True, concurrent=True) on a maxlog / f32 codec."""
        w = N.TdWindowParams(int(window), int(overlap), int(bool(nii)), int(bool(concurrent)), float(ext_scale))
        N.check(N.lib().td_set_window(self._h, C.byref(w)))
        self.window = int(window)

    def debug_window_layout(self, run: int = 0, run_a: int = 0, parts: int = 0) -> None:
        """Windowed kernels' layout for tests and measurements (td_debug_window_layout): sub-blocks
        per lane run (beta and alpha kernels) and batch parts; 0 = the layout's own choice."""
        N.check(N.lib().td_debug_window_layout(self._h, int(run), int(run_a), int(parts)))

    # -- TurboDecoding, host arrays ------------------------------------------------------
    def TurboDecoding(self, flow: np.ndarray, return_le: bool = False):
        """flow [B, 3K+12] (or one row) -> out int32 [B, iterations, K] (the reference's
        flow_decoded rows); with return_le also Le [B, iterations, 2, K+3]."""
        flow = np.ascontiguousarray(flow, dtype=self.dtype)
        one = flow.ndim == 1
        flow = flow.reshape(-1, stream_length(self.K))
        B = flow.shape[0]
        out = np.zeros((B, self.iterations, self.K), dtype=np.int32)
        le = np.zeros((B, self.iterations, 2, self.L), dtype=self.dtype) if return_le else None
        N.check(N.lib().td_decode_host(self._h, flow.ctypes.data_as(C.c_void_p), B,
                                       out.ctypes.data_as(C.c_void_p),
                                       le.ctypes.data_as(C.c_void_p) if return_le else None))
        if one:
            out, le = out[0], (le[0] if return_le else None)
        return (out, le) if return_le else out

    # -- device-resident decode (torch tensors as HBM buffers) ---------------------------
    def decode(self, llr, bits=None, all_iters: bool = False, le=None, stream=None):
        """llr: torch tensor [B, 3K+12] on this codec's device (float64 for f64, float32 for f32).
        Returns uint8 bits [B, K] (or [B, iterations, K] with all_iters).  Asynchronous on
        `stream` (default: torch's current stream)."""
        import torch

        want = torch.float64 if self.precision == "f64" else torch.float32
        if llr.dtype != want or not llr.is_cuda or not llr.is_contiguous():
            raise ValueError(f"llr must be a contiguous {want} CUDA tensor")
        if llr.ndim != 2 or llr.shape[1] != stream_length(self.K):
            raise ValueError(f"llr must be [B, {stream_length(self.K)}] (3K+12), got {tuple(llr.shape)}")
        if llr.device.index != self.device:
            raise ValueError(f"llr is on {llr.device}, the codec on cuda:{self.device}")
        B = llr.shape[0]
        shape = (B, self.iterations, self.K) if all_iters else (B, self.K)
        if bits is None:
            bits = torch.empty(shape, dtype=torch.uint8, device=llr.device)
        else:
            self._check_out("bits", bits, torch.uint8, shape, llr.device)
        if le is not None:
            self._check_out("le", le, want, (B, self.iterations, 2, self.L), llr.device)
        if stream is None:
            stream = torch.cuda.current_stream(llr.device)
        N.check(N.lib().td_decode_device(self._h, C.c_void_p(llr.data_ptr()), B, C.c_void_p(bits.data_ptr()),
                                         int(all_iters), C.c_void_p(le.data_ptr()) if le is not None else None,
                                         C.c_void_p(stream.cuda_stream)))
        return bits

    @staticmethod
    def _check_out(name, t, dtype, shape, device) -> None:
        """An output buffer the kernels write B*... elements into: its dtype, shape, device and
        layout must be exactly what they assume, or they write past its end."""
        if t.dtype != dtype or tuple(t.shape) != tuple(shape) or t.device != device or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)} on {device}, "
                             f"got {t.dtype} {tuple(t.shape)} on {t.device}")

    def decode_raw(self, llr_ptr: int, B: int, bits_ptr: int, all_iters: bool = False, le_ptr: int = 0,
                   stream_ptr: int = 0) -> None:
        """td_decode_device on raw device pointers (no checks possible here: the caller owns the
        sizes -- llr B*(3K+12), bits B*K or B*iterations*K bytes, le B*iterations*2*(K+3))."""
        if B < 0 or not llr_ptr or not bits_ptr:
            raise ValueError("decode_raw: B >= 0 and non-null llr / bits pointers")
        N.check(N.lib().td_decode_device(self._h, C.c_void_p(llr_ptr), int(B), C.c_void_p(bits_ptr),
                                         int(all_iters), C.c_void_p(le_ptr) if le_ptr else None,
                                         C.c_void_p(stream_ptr) if stream_ptr else None))

    # -- measurement ---------------------------------------------------------------------
    def profile(self, on: bool = True) -> None:
        """Bracket the next decodes' kernels with hipEvents (see td_profile_enable)."""
        N.check(N.lib().td_profile_enable(self._h, int(on)))

    def kernel_ms(self):
        """(demux_ms, turbo_ms, launches): average kernel durations over the decodes since the
        last call (synchronises on their events)."""
        a, b, n = C.c_float(), C.c_float(), C.c_int()
        N.check(N.lib().td_profile_read(self._h, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value

    def clock(self):
        """(sustained shader clock GHz, workgroup span ms) of the last decode: the exact schedule's
        turbo launch, or a windowed decode's last SISO2 beta workgroup (td_clock_read; waits for
        this handle's last decode)."""
        g, s = C.c_double(), C.c_double()
        N.check(N.lib().td_clock_read(self._h, C.byref(g), C.byref(s)))
        return g.value, s.value

    # -- frame generator and error counts (main.cpp's channel, on the device) -------------
    def synth_seed(self, seed: int) -> None:
        """srand(seed) for the handle's frame stream (main.cpp:170)."""
        N.check(N.lib().td_synth_seed(self._h, int(seed) & 0xFFFFFFFF))

    def synth_modulation(self, modulation: int) -> None:
        """MODULATION of the generator's frames: 1 BPSK, 2 QPSK, 3 8PSK, 4 16QAM, 6 64QAM."""
        N.check(N.lib().td_synth_modulation(self._h, int(modulation)))

    def synth_seek(self, frame: int) -> None:
        N.check(N.lib().td_synth_seek(self._h, int(frame)))

    def synth(self, B: int, ebn0_db: float, info=None, llr=None, stream=None):
        """The next B frames of the stream: (info uint8 [B, K], llr float64 [B, 3K+12]) tensors
        on this codec's device, bit-identical to main.cpp's frames of the same srand seed."""
        import torch

        dev = torch.device("cuda", self.device)
        if info is None:
            info = torch.empty((B, self.K), dtype=torch.uint8, device=dev)
        if llr is None:
            llr = torch.empty((B, stream_length(self.K)), dtype=torch.float64, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        N.check(N.lib().td_synth_frames(self._h, float(ebn0_db), int(B), C.c_void_p(info.data_ptr()),
                                        C.c_void_p(llr.data_ptr()), C.c_void_p(stream.cuda_stream)))
        return info, llr

    def count_errors(self, bits, info, stream=None):
        """bits uint8 [B, iters, K], info uint8 [B, K] -> int32 [B, iters] bit-error counts."""
        import torch

        B, iters = int(bits.shape[0]), int(bits.shape[1])
        err = torch.empty((B, iters), dtype=torch.int32, device=bits.device)
        if stream is None:
            stream = torch.cuda.current_stream(bits.device)
        N.check(N.lib().td_count_errors(self._h, C.c_void_p(bits.data_ptr()), iters, C.c_void_p(info.data_ptr()), B,
                                        C.c_void_p(err.data_ptr()), C.c_void_p(stream.cuda_stream)))
        return err

    # -- Log_MAP_decoder -----------------------------------------------------------------
    def Log_MAP_decoder(self, recs: np.ndarray, La: np.ndarray, terminated: int = TERMINATED) -> np.ndarray:
        """recs [B, 2L] (ys, yp pairs), La [B, L] -> LLR [B, L] (or 1-D for one codeword)."""
        recs = np.ascontiguousarray(recs, dtype=self.dtype)
        La = np.ascontiguousarray(La, dtype=self.dtype)
        one = La.ndim == 1
        La2 = La.reshape(1, -1) if one else La
        L = La2.shape[1]
        recs2 = recs.reshape(-1, 2 * L)
        B = La2.shape[0]
        out = np.zeros((B, L), dtype=self.dtype)
        N.check(N.lib().td_siso_host(self._h, recs2.ctypes.data_as(C.c_void_p), La2.ctypes.data_as(C.c_void_p),
                                     int(terminated), out.ctypes.data_as(C.c_void_p), L, B))
        return out[0] if one else out


def modulate(bits, modulation: int, stream=None):
    """module (modanddem.cpp:175) on the GPU: uint8 bits [nsym * M] (cuda) -> (si, sq) float64."""
    import torch

    bits = bits.contiguous()
    nsym = bits.numel() // modulation
    si = torch.empty(nsym, dtype=torch.float64, device=bits.device)
    sq = torch.empty_like(si)
    if stream is None:
        stream = torch.cuda.current_stream(bits.device)
    N.check(N.lib().td_modulate(C.c_void_p(bits.data_ptr()), nsym, int(modulation), C.c_void_p(si.data_ptr()),
                                C.c_void_p(sq.data_ptr()), C.c_void_p(stream.cuda_stream)))
    return si, sq


def demodulate(yi, yq, modulation: int, Kf: float, stream=None):
    """demodule (modanddem.cpp:674) on the GPU: float64 symbols [nsym] (cuda) -> LLRs [nsym * M]."""
    import torch

    yi, yq = yi.contiguous(), yq.contiguous()
    out = torch.empty(yi.numel() * modulation, dtype=torch.float64, device=yi.device)
    if stream is None:
        stream = torch.cuda.current_stream(yi.device)
    N.check(N.lib().td_demodulate(C.c_void_p(yi.data_ptr()), C.c_void_p(yq.data_ptr()), yi.numel(), int(modulation),
                                  float(Kf), C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream)))
    return out


def TurboCodingInit(K: int, f1: int, f2: int, **kw) -> TurboCodec:
    """Reference-named constructor (log_map.cpp:349): parameters explicit instead of globals."""
    return TurboCodec(K, f1, f2, **kw)


def device_count() -> int:
    return N.lib().td_device_count()
