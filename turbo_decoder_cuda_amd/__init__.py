"""turbo_decoder_cuda_amd -- MI355X-native LTE turbo decoder (log-MAP BCJR, QPP, 8-state RSC).

The product is libturbo_mi355x.so (C ABI: include/turbo_mi355x.h, HIP kernels for gfx950 in
csrc/).  This package holds its build script and a thin host-side mirror of the reference
codec interface (decoder.py).  See DESIGN.md.
"""
from .decoder import (N_ITERATION, TERMINATED, TurboCodec, TurboCodingInit, demodulate, device_count, modulate,
                      stream_length)

__all__ = ["TurboCodec", "TurboCodingInit", "N_ITERATION", "TERMINATED", "device_count", "stream_length",
           "modulate", "demodulate"]
