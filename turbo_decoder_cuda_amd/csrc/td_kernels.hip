// td_kernels.hip -- gfx950 kernels of the MI355X turbo decoder.
//
// Mapping (DESIGN.md "Kernel"): one wave64 decodes 8 codewords; lane = 8*c + s holds trellis
// state s of codeword c.  The whole turbo loop (all iterations, both SISOs) runs inside one
// launch per wave: codewords never interact, so there is no inter-workgroup traffic.
//
// SISO = Log_MAP_decoder (ITTC/log_map.cpp:898-1047), serial schedule of TurboDecoding
// (:1217-1265).  Per SISO:
//   F pass  alpha forward over all L = K+3 steps, checkpointing alpha every W steps (HBM scratch);
//   B pass  windows last..first: recompute alpha of the window from its checkpoint (keeps the
//           reference's tempmax and the per-state sums gamma+alpha), then beta backward with
//           the reference's normalisation (beta -= tempmax[i+1]), then the LLR folds
//           E_seq(temp1) - E_seq(temp0) in state order 0..7 and the extrinsic update.
// Every floating-point operation is the reference's, in the reference's order; gamma uses
// fma(yp, +-1, -+ys), which rounds identically because yp*(+-1) is exact.  Build with
// -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "td_kernels.h"
#include "td_tables.h"

namespace td {

constexpr int kW = 32;           // steps per window / tile
constexpr int kCw = 8;           // codewords per wave
constexpr int kLanes = 64;
constexpr int kTileElems = kW * kCw;   // 256 values of one array per tile
constexpr int kPerLane = kTileElems / kLanes;   // 4

template <typename T>
__device__ __forceinline__ T shfl_any(T v, int src)
{
    return __shfl(v, src, kLanes);
}

template <typename T>
__device__ __forceinline__ T group_max8(T v)
{
    // max over the 8 lanes of one codeword (exact in any order)
    T o = __shfl_xor(v, 1, kLanes);
    v = v > o ? v : o;
    o = __shfl_xor(v, 2, kLanes);
    v = v > o ? v : o;
    o = __shfl_xor(v, 4, kLanes);
    v = v > o ? v : o;
    return v;
}

template <typename T, int ALGO>
__device__ __forceinline__ T mstar(T x, T y, const LutEntry<T>* lut)
{
    if constexpr (ALGO == 1) {
        return x > y ? x : y;
    } else {
        return maxstar_lut<T>(x, y, lut);
    }
}

// Per-lane constants of the trellis for state s (lane & 7).
struct LaneTrellis {
    int srcA, srcB;   // lanes holding alpha of the two predecessors (u = 0, u = 1)
    int srcN0, srcN1; // lanes holding beta of the two successors
    int s;
};

template <typename T>
struct LaneSigns {
    T sA, sB;   // parity sign of the transition predecessor(u) -> s  (alpha / LLR)
    T sC, sD;   // parity sign of the transitions s -> next(u)        (beta)
};

template <typename T>
struct SisoLds {
    LutEntry<T> lut[kLutSize];
    T ys[2][kTileElems];
    T yp[2][kTileElems];
    T la[2][kTileElems];
    T X[kW][kLanes];   // temp0 = (gamma + alpha) + beta, per step and lane
    T Y[kW][kLanes];   // temp1
    T tm[kW][kCw];     // tempmax[i+1] of the window
};

template <typename T>
struct TileRegs {
    T ys[kPerLane], yp[kPerLane], la[kPerLane];
};

// Source of one SISO's inputs.  Arrays are batch-interleaved [group][step][8].
template <typename T>
struct SisoSrc {
    const T* sys;   // [G][L][8]
    const T* par;   // [G][L][8]
    const T* la;    // a-priori source (see la_mode)
    int la_mode;    // 0: none (zeros), 1: direct la[g][i][c] for i < la_len, 2: gathered la[g][pi[i]][c]
    int la_len;     // number of steps that carry a-priori (K for the turbo loop; L for bare SISO)
    int terminated;
};

template <typename T>
struct SisoDst {
    T* ext;          // extrinsic out (ext_mode)
    int ext_mode;    // 0: none, 1: direct ext[g][i][c] (i < ext_len), 2: scattered ext[g][pi[i]][c]
    int ext_len;
    T* llr;          // optional raw LLR out, [G][L][8]
    T* le_dump;      // optional [B][iters][2][L]
    uint8_t* bits;   // optional decisions, natural order via pi
    int bits_row;    // row offset (in units of K) inside a codeword's bits block
    int bits_stride; // codeword stride of bits (in bytes)
    int dump_slot;   // it*2 + dec
    int dump_stride; // codeword stride of le_dump (elements)
};

struct Geom {
    int K, L, nT, B, g;
    const int* pi;
};

template <typename T>
__device__ __forceinline__ void load_tile(TileRegs<T>& r, const SisoSrc<T>& src, const Geom& gm, int t, int lane)
{
#pragma unroll
    for (int q = 0; q < kPerLane; ++q) {
        const int e = lane + kLanes * q;
        const int k = e >> 3, c = e & 7;
        const int i = t * kW + k;
        T ys = 0, yp = 0, la = 0;
        if (i < gm.L) {
            const size_t off = ((size_t)gm.g * gm.L + i) * kCw + c;
            ys = src.sys[off];
            yp = src.par[off];
            if (i < src.la_len) {
                if (src.la_mode == 1)
                    la = src.la[((size_t)gm.g * src.la_len + i) * kCw + c];
                else if (src.la_mode == 2)
                    la = src.la[((size_t)gm.g * src.la_len + gm.pi[i]) * kCw + c];
            }
        }
        r.ys[q] = ys;
        r.yp[q] = yp;
        r.la[q] = la;
    }
}

template <typename T>
__device__ __forceinline__ void store_tile(const TileRegs<T>& r, SisoLds<T>& sm, int buf, int lane)
{
#pragma unroll
    for (int q = 0; q < kPerLane; ++q) {
        const int e = lane + kLanes * q;
        sm.ys[buf][e] = r.ys[q];
        sm.yp[buf][e] = r.yp[q];
        sm.la[buf][e] = r.la[q];
    }
}

// One alpha step i -> i+1 (log_map.cpp:975-1001).  Returns normalised alpha[s][i+1];
// x/y = the sums gamma+alpha entering the max* (reused by the LLR, :1028-1034); m = tempmax[i+1].
template <typename T, int ALGO>
__device__ __forceinline__ T alpha_step(T alpha, T ys, T yp, T la, const LaneTrellis& lt, const LaneSigns<T>& sg,
                                        const LutEntry<T>* lut, T& x, T& y, T& m)
{
    const T hla = la / (T)2;
    const T gx = fma(yp, sg.sA, -ys) - hla;   // gamma[p0][i][0] = ((-ys) + yp*o) - La/2  (:967-968)
    const T gy = fma(yp, sg.sB, ys) + hla;    // gamma[p1][i][1] = (ys + yp*o) + La/2     (:969-970)
    const T aA = shfl_any(alpha, lt.srcA);
    const T aB = shfl_any(alpha, lt.srcB);
    x = gx + aA;
    y = gy + aB;
    const T a = mstar<T, ALGO>(x, y, lut);
    m = group_max8(a);
    return a - m;
}

// One beta step i+1 -> i (log_map.cpp:1004-1021): beta[s][i] = E(g0 + b[n0], g1 + b[n1]) - tempmax[i+1].
template <typename T, int ALGO>
__device__ __forceinline__ T beta_step(T beta, T ys, T yp, T la, T tmax, const LaneTrellis& lt,
                                       const LaneSigns<T>& sg, const LutEntry<T>* lut)
{
    const T hla = la / (T)2;
    const T gx = fma(yp, sg.sC, -ys) - hla;
    const T gy = fma(yp, sg.sD, ys) + hla;
    const T bA = shfl_any(beta, lt.srcN0);
    const T bB = shfl_any(beta, lt.srcN1);
    const T b = mstar<T, ALGO>(gx + bA, gy + bB, lut);
    return b - tmax;
}

// E_algorithm_seq over 8 values in state order (log_map.cpp:817-829).
template <typename T, int ALGO>
__device__ __forceinline__ T fold8(const T* v, const LutEntry<T>* lut)
{
    T t = mstar<T, ALGO>(v[0], v[1], lut);
#pragma unroll
    for (int j = 2; j < 8; ++j) t = mstar<T, ALGO>(t, v[j], lut);
    return t;
}

// One SISO over the wave's 8 codewords.
template <typename T, int ALGO>
__device__ void siso_wave(SisoLds<T>& sm, const SisoSrc<T>& src, const SisoDst<T>& dst, const Geom& gm,
                          T* ckpt, const LaneTrellis& lt, const LaneSigns<T>& sg, int lane)
{
    const int c = lane >> 3;
    const int s = lane & 7;
    const int nT = gm.nT;
    T* my_ckpt = ckpt + (size_t)gm.g * (nT + 1) * kLanes + lane;
    TileRegs<T> pre;

    // ------------------------------------------------------------- F pass (alpha forward)
    T alpha = (s == 0) ? (T)0 : (T)-kInfty;   // :943,948
    my_ckpt[0] = alpha;
    load_tile(pre, src, gm, 0, lane);
    store_tile(pre, sm, 0, lane);
    __syncthreads();
    for (int t = 0; t < nT; ++t) {
        const int buf = t & 1;
        if (t + 1 < nT) load_tile(pre, src, gm, t + 1, lane);
        const int n = min(kW, gm.L - t * kW);
        for (int k = 0; k < n; ++k) {
            const int e = k * kCw + c;
            T x, y, m;
            alpha = alpha_step<T, ALGO>(alpha, sm.ys[buf][e], sm.yp[buf][e], sm.la[buf][e], lt, sg, sm.lut, x, y, m);
        }
        my_ckpt[(size_t)(t + 1) * kLanes] = alpha;
        if (t + 1 < nT) store_tile(pre, sm, buf ^ 1, lane);
        __syncthreads();
    }

    // ------------------------------------------------------------- B pass (windows backward)
    T beta = (src.terminated && s != 0) ? (T)-kInfty : (T)0;   // :944,951-959
    {
        const int t = nT - 1;
        load_tile(pre, src, gm, t, lane);
        store_tile(pre, sm, t & 1, lane);
        __syncthreads();
    }
    for (int t = nT - 1; t >= 0; --t) {
        const int buf = t & 1;
        if (t > 0) load_tile(pre, src, gm, t - 1, lane);
        const int n = min(kW, gm.L - t * kW);
        // alpha recompute of this window from its checkpoint (bit-identical to the F pass)
        T a = my_ckpt[(size_t)t * kLanes];
        for (int k = 0; k < n; ++k) {
            const int e = k * kCw + c;
            T x, y, m;
            a = alpha_step<T, ALGO>(a, sm.ys[buf][e], sm.yp[buf][e], sm.la[buf][e], lt, sg, sm.lut, x, y, m);
            sm.X[k][lane] = x;
            sm.Y[k][lane] = y;
            if (s == 0) sm.tm[k][c] = m;
        }
        __syncthreads();
        // beta backward; temp_u[j] = (gamma + alpha) + beta[j][i+1]  (:1028-1034)
        for (int k = n - 1; k >= 0; --k) {
            const int e = k * kCw + c;
            sm.X[k][lane] = sm.X[k][lane] + beta;
            sm.Y[k][lane] = sm.Y[k][lane] + beta;
            beta = beta_step<T, ALGO>(beta, sm.ys[buf][e], sm.yp[buf][e], sm.la[buf][e], sm.tm[k][c], lt, sg,
                                      sm.lut);
        }
        __syncthreads();
        // LLR = E_seq(temp1) - E_seq(temp0) (:1038); extrinsic Le = LLR - La - 2*ys (:1237,1258)
#pragma unroll
        for (int q = 0; q < kPerLane; ++q) {
            const int e = lane + kLanes * q;
            const int k = e >> 3, cc = e & 7;
            if (k < n) {
                const int i = t * kW + k;
                const T llr = fold8<T, ALGO>(&sm.Y[k][cc * 8], sm.lut) - fold8<T, ALGO>(&sm.X[k][cc * 8], sm.lut);
                const T la = sm.la[buf][e];
                const T le = llr - la - (T)2 * sm.ys[buf][e];
                const int b = gm.g * kCw + cc;
                if (dst.llr) dst.llr[((size_t)gm.g * gm.L + i) * kCw + cc] = llr;
                if (i < dst.ext_len) {
                    if (dst.ext_mode == 1)
                        dst.ext[((size_t)gm.g * dst.ext_len + i) * kCw + cc] = le;
                    else if (dst.ext_mode == 2)
                        dst.ext[((size_t)gm.g * dst.ext_len + gm.pi[i]) * kCw + cc] = le;
                }
                if (b < gm.B) {
                    if (dst.le_dump) dst.le_dump[(size_t)b * dst.dump_stride + (size_t)dst.dump_slot * gm.L + i] = le;
                    if (dst.bits && i < gm.K)   // decision (:862-879) + random_deinterlvr_int (:1264)
                        dst.bits[(size_t)b * dst.bits_stride + (size_t)dst.bits_row * gm.K + gm.pi[i]] =
                            (llr < (T)0) ? 0 : 1;
                }
            }
        }
        if (t > 0) store_tile(pre, sm, buf ^ 1, lane);
        __syncthreads();
    }
}

template <typename T>
__device__ __forceinline__ void lane_setup(const DecodeParams<T>& p, int lane, LaneTrellis& lt, LaneSigns<T>& sg)
{
    const int s = lane & 7, base = lane & ~7;
    lt.s = s;
    lt.srcA = base | p.laststat[s][0];
    lt.srcB = base | p.laststat[s][1];
    lt.srcN0 = base | p.nextstat[s][0];
    lt.srcN1 = base | p.nextstat[s][1];
    sg.sA = (T)p.nextout[p.laststat[s][0]][1];   // parity of p0 -(u=0)-> s  (mx_nextout[p0*4+1])
    sg.sB = (T)p.nextout[p.laststat[s][1]][3];   // parity of p1 -(u=1)-> s  (mx_nextout[p1*4+3])
    sg.sC = (T)p.nextout[s][1];
    sg.sD = (T)p.nextout[s][3];
}

template <typename T>
__device__ __forceinline__ void lut_to_lds(const DecodeParams<T>& p, SisoLds<T>& sm, int lane)
{
    for (int q = lane; q < kLutSize; q += kLanes) sm.lut[q] = p.lut[q];
}

// The whole turbo decode of 8 codewords per workgroup (TurboDecoding, log_map.cpp:1146-1280).
template <typename T, int ALGO>
__global__ __launch_bounds__(64) void turbo_decode_kernel(DecodeParams<T> p)
{
    __shared__ SisoLds<T> sm;
    const int lane = threadIdx.x;
    LaneTrellis lt;
    LaneSigns<T> sg;
    lane_setup(p, lane, lt, sg);
    lut_to_lds(p, sm, lane);
    __syncthreads();

    Geom gm{p.K, p.L, p.nT, p.B, (int)blockIdx.x, p.pi};
    for (int it = 0; it < p.iters; ++it) {
        // decoder 1: La = deinterleaved Le of decoder 2 (:1221); zero before the first iteration (:1212-1215)
        SisoSrc<T> s1{p.sys1, p.par1, p.ext21, it == 0 ? 0 : 1, p.K, 1};
        SisoDst<T> d1{p.ext12, 1, p.K, nullptr, p.le_dump, nullptr, 0, 0, it * 2 + 0, p.iters * 2 * p.L};
        siso_wave<T, ALGO>(sm, s1, d1, gm, p.ckpt, lt, sg, lane);
        __syncthreads();
        // decoder 2: La = interleaved Le of decoder 1 (:1242); its Le goes back deinterleaved
        SisoSrc<T> s2{p.sys2, p.par2, p.ext12, 2, p.K, 1};
        const bool want_bits = p.all_iters || it == p.iters - 1;
        SisoDst<T> d2{p.ext21, 2, p.K, nullptr, p.le_dump, want_bits ? p.bits : nullptr,
                      p.all_iters ? it : 0, p.all_iters ? p.iters * p.K : p.K, it * 2 + 1, p.iters * 2 * p.L};
        siso_wave<T, ALGO>(sm, s2, d2, gm, p.ckpt, lt, sg, lane);
        __syncthreads();
    }
}

// Standalone SISO (Log_MAP_decoder) over interleaved [G][L][8] inputs.
template <typename T, int ALGO>
__global__ __launch_bounds__(64) void siso_kernel(DecodeParams<T> p, const T* la, int terminated)
{
    __shared__ SisoLds<T> sm;
    const int lane = threadIdx.x;
    LaneTrellis lt;
    LaneSigns<T> sg;
    lane_setup(p, lane, lt, sg);
    lut_to_lds(p, sm, lane);
    __syncthreads();
    Geom gm{p.K, p.L, p.nT, p.B, (int)blockIdx.x, p.pi};
    SisoSrc<T> s{p.sys1, p.par1, la, 1, p.L, terminated};
    SisoDst<T> d{nullptr, 0, 0, p.llr_out, nullptr, nullptr, 0, 0, 0, 0};
    siso_wave<T, ALGO>(sm, s, d, gm, p.ckpt, lt, sg, lane);
}

// Demultiplex + x0.5 (log_map.cpp:1202-1205, 1083-1127) of the reference stream layout into the
// batch-interleaved arrays.  One thread per (group, step, codeword).
template <typename T>
__global__ __launch_bounds__(256) void demux_kernel(DecodeParams<T> p, const T* __restrict__ flow)
{
    const int K = p.K, L = p.L, n = 3 * K + 4 * kMemory;
    const size_t total = (size_t)p.G * L * kCw;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e & 7);
        const size_t gi = e >> 3;
        const int i = (int)(gi % L);
        const int g = (int)(gi / L);
        const int b = g * kCw + c;
        T ys1 = 0, yp1 = 0, ys2 = 0, yp2 = 0;
        if (b < p.B) {
            const T* r = flow + (size_t)b * n;
            const T h = (T)0.5;
            if (i < K) {
                ys1 = r[3 * i] * h;
                yp1 = r[3 * i + 1] * h;
                yp2 = r[3 * i + 2] * h;
                ys2 = r[3 * p.pi[i]] * h;
            } else {
                const int j = i - K;
                ys1 = r[3 * K + 2 * j] * h;
                yp1 = r[3 * K + 2 * j + 1] * h;
                ys2 = r[3 * K + 2 * kMemory + 2 * j] * h;
                yp2 = r[3 * K + 2 * kMemory + 2 * j + 1] * h;
            }
        }
        p.sys1[e] = ys1;
        p.par1[e] = yp1;
        p.sys2[e] = ys2;
        p.par2[e] = yp2;
    }
}

// Bare-SISO input transpose: recs[B][2L] / La[B][L] -> [G][L][8]
template <typename T>
__global__ __launch_bounds__(256) void siso_in_kernel(DecodeParams<T> p, const T* recs, const T* la, T* la_out)
{
    const int L = p.L;
    const size_t total = (size_t)p.G * L * kCw;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(e & 7);
        const size_t gi = e >> 3;
        const int i = (int)(gi % L);
        const int b = (int)(gi / L) * kCw + c;
        T ys = 0, yp = 0, a = 0;
        if (b < p.B) {
            ys = recs[(size_t)b * 2 * L + 2 * i];
            yp = recs[(size_t)b * 2 * L + 2 * i + 1];
            a = la[(size_t)b * L + i];
        }
        p.sys1[e] = ys;
        p.par1[e] = yp;
        la_out[e] = a;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void siso_out_kernel(DecodeParams<T> p, T* llr)
{
    const int L = p.L;
    const size_t total = (size_t)p.B * L;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / L), i = (int)(e % L);
        llr[e] = p.llr_out[((size_t)(b / kCw) * L + i) * kCw + (b % kCw)];
    }
}

// ------------------------------------------------------------------ launchers
template <typename T>
hipError_t launch_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st)
{
    const size_t total = (size_t)p.G * p.L * kCw;
    int gblocks = (int)((total + 255) / 256);
    if (gblocks > 8192) gblocks = 8192;
    hipLaunchKernelGGL(demux_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, flow);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_turbo(const DecodeParams<T>& p, hipStream_t st)
{
    if (p.algo == 1)
        hipLaunchKernelGGL((turbo_decode_kernel<T, 1>), dim3(p.G), dim3(kLanes), 0, st, p);
    else
        hipLaunchKernelGGL((turbo_decode_kernel<T, 0>), dim3(p.G), dim3(kLanes), 0, st, p);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_siso(const DecodeParams<T>& p, const T* recs, const T* la, T* la_ws, int terminated, T* llr,
                       hipStream_t st)
{
    const size_t total = (size_t)p.G * p.L * kCw;
    int gblocks = (int)((total + 255) / 256);
    if (gblocks > 8192) gblocks = 8192;
    hipLaunchKernelGGL(siso_in_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, recs, la, la_ws);
    if (p.algo == 1)
        hipLaunchKernelGGL((siso_kernel<T, 1>), dim3(p.G), dim3(kLanes), 0, st, p, (const T*)la_ws, terminated);
    else
        hipLaunchKernelGGL((siso_kernel<T, 0>), dim3(p.G), dim3(kLanes), 0, st, p, (const T*)la_ws, terminated);
    hipLaunchKernelGGL(siso_out_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, llr);
    return hipGetLastError();
}

template hipError_t launch_demux<double>(const DecodeParams<double>&, const double*, hipStream_t);
template hipError_t launch_demux<float>(const DecodeParams<float>&, const float*, hipStream_t);
template hipError_t launch_turbo<double>(const DecodeParams<double>&, hipStream_t);
template hipError_t launch_turbo<float>(const DecodeParams<float>&, hipStream_t);
template hipError_t launch_siso<double>(const DecodeParams<double>&, const double*, const double*, double*, int,
                                        double*, hipStream_t);
template hipError_t launch_siso<float>(const DecodeParams<float>&, const float*, const float*, float*, int, float*,
                                       hipStream_t);

int window_steps() { return kW; }

}  // namespace td
