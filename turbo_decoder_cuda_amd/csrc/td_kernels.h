// td_kernels.h -- launch interface between the C ABI (td_api.cpp) and td_kernels.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "td_tables.h"

namespace td {

// Kernel parameter block (passed by value).  Device arrays are batch-interleaved:
// group g = codewords 8g..8g+7, element [g][step][c].
template <typename T>
struct DecodeParams {
    T* sys1;   // [G][L][8] systematic of decoder 1 (x0.5)
    T* par1;   // [G][L][8] parity 1
    T* sys2;   // [G][L][8] interleaved systematic (decoder 2)
    T* par2;   // [G][L][8] parity 2
    T* ext12;  // [G][K][8] Le of decoder 1, natural order
    T* ext21;  // [G][K][8] Le of decoder 2 scattered to natural order (= La of decoder 1)
    T* ckpt;   // [G][nT+1][64] alpha checkpoints
    T* llr_out;                 // bare SISO: [G][L][8]
    const int* pi;              // [K]
    const LutEntry<T>* lut;     // [kLutSize]
    uint8_t* bits;              // decisions (see td_decode_device)
    T* le_dump;                 // nullable
    int K, L, nT, G, B, iters, all_iters, algo;
    int nextstat[kStates][2];
    int laststat[kStates][2];
    int nextout[kStates][4];
};

// demultiplex + x0.5 of the stream into the batch-interleaved arrays
template <typename T>
hipError_t launch_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st);
// the turbo iterations (one wave per 8 codewords)
template <typename T>
hipError_t launch_turbo(const DecodeParams<T>& p, hipStream_t st);

template <typename T>
hipError_t launch_siso(const DecodeParams<T>& p, const T* recs, const T* la, T* la_ws, int terminated, T* llr,
                       hipStream_t st);

int window_steps();

}  // namespace td
