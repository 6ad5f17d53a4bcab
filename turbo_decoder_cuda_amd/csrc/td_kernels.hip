// td_kernels.hip -- gfx950 kernels of the MI355X turbo decoder.
//
// Mapping (DESIGN.md "Kernel"): one workgroup (4 waves) decodes 8 codewords; in the recursion
// waves, lane 8*c + l holds one trellis state of codeword c.  The whole turbo loop (all
// iterations, both SISOs) runs inside one launch: codewords never interact, so there is no
// inter-workgroup traffic at all.
//
// Rotating state labels.  At trellis step i the slot l of a codeword holds state
//     state(l, i) = rotr^(i mod 3)(A(l)),     A = GF(2)-linear map 1->1, 2->2, 4->7.
// With this labeling both recursions of the 8-state RSC (predecessors of j = {rotl(j), rotl(j)^1},
// successors = {rotr(j), rotr(j)^4}) need exactly ONE cross-lane value per step: the partner
// lane l ^ m, m = 1, 2, 7 for i mod 3 = 0, 1, 2 -- DPP quad_perm / quad_perm / row_half_mirror.
// The normalising max over the 8 lanes is three DPP levels.  No LDS round trip sits on the
// alpha/beta critical path except the max* table (one ds_read per max*).
//
// SISO = Log_MAP_decoder (ITTC/log_map.cpp:898-1047) in the serial schedule of TurboDecoding
// (:1217-1265).  Per SISO:
//   F pass  alpha forward over the L = K+3 steps, alpha checkpoint every W steps (HBM scratch);
//   B pass  windows last..first.  beta of window t runs fused with the alpha recompute of
//           window t-1 (two independent chains per step); the recompute stores per step and
//           state the sums (gamma + alpha) entering the max* (= the LLR terms, :1028-1034) and
//           the reference's tempmax, beta subtracts tempmax[i+1] (:1019) and adds itself into
//           the stored sums; then the LLR folds E_seq(temp1) - E_seq(temp0) run over
//           (step, codeword) items in state order 0..7 (:1038) and the extrinsic update
//           Le = LLR - La - 2*ys (:1237, :1258) is written out.
// Every floating-point operation is the reference's, in the reference's order (max* is
// symmetric, so the two operands may arrive in either order).  Build with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "td_kernels.h"
#include "td_tables.h"

namespace td {

constexpr int kW = 12;                          // steps per window (multiple of 3)
constexpr int kCw = 8;                          // codewords per workgroup
constexpr int kLanes = 64;
constexpr int kTile = kW * kCw;                 // (step, codeword) elements per window
static_assert(kW % 3 == 0, "window must be a multiple of the label period");

// ------------------------------------------------------------------ DPP helpers
constexpr int kDppXor1 = 0xB1;    // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;    // quad_perm [2,3,0,1]
constexpr int kDppMir8 = 0x141;   // row_half_mirror: l -> 7-l inside 8 lanes (= l ^ 7)

template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// partner exchange mask of phase PH (i mod 3)
template <int PH>
struct PhaseDpp {
    static constexpr int ctrl = PH == 0 ? kDppXor1 : (PH == 1 ? kDppXor2 : kDppMir8);
};

// fmax -> v_max_f64 / v_max_f32.  Equal to the reference's `x > y ? x : y` / running
// `if (m < a) m = a` for every non-NaN pair (they can differ only in the sign of a zero,
// which never changes a later non-zero value or a hard decision).
__device__ __forceinline__ double vmax(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ float vmax(float a, float b) { return fmaxf(a, b); }

// max over the 8 lanes of one codeword (exact in any order)
template <typename T>
__device__ __forceinline__ T group_max8(T v)
{
    v = vmax(v, dpp<kDppXor1>(v));
    v = vmax(v, dpp<kDppXor2>(v));
    v = vmax(v, dpp<kDppMir8>(v));
    return v;
}

// ------------------------------------------------------------------ max*
// Exact bucket form of E_algorithm (td_tables.h, build_lut): the bucket index is a bit field of
// d (exponent + 3 mantissa bits; the sign bit is outside the field, so d need not be |d|).
template <typename T>
__device__ __forceinline__ int bucket_dev(T d);
template <>
__device__ __forceinline__ int bucket_dev<double>(double d)
{
    const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
    const int q = (int)__builtin_amdgcn_ubfe(hi, BucketBits<double>::shift, BucketBits<double>::width);
    return min(max(q, BucketBits<double>::base), BucketBits<double>::base + kLutSize - 1) - BucketBits<double>::base;
}
template <>
__device__ __forceinline__ int bucket_dev<float>(float d)
{
    const unsigned b = (unsigned)__float_as_int(d);
    const int q = (int)__builtin_amdgcn_ubfe(b, BucketBits<float>::shift, BucketBits<float>::width);
    return min(max(q, BucketBits<float>::base), BucketBits<float>::base + kLutSize - 1) - BucketBits<float>::base;
}

// The table lives in LDS as three arrays (thr | vlo | vhi, kLutPad entries each): one 8-byte read
// per field spreads the buckets over 32 bank pairs (a 32-byte AoS entry would leave only 8 bank
// groups for the 64 lanes' random buckets).
constexpr int kLutPad = 64;
static_assert(kLutSize <= kLutPad, "LUT padding");

template <typename T, int ALGO>
__device__ __forceinline__ T mstar(T x, T y, const T* lut)
{
    if constexpr (ALGO == 1) {
        return vmax(x, y);   // Max-Log-MAP
    } else {
        const T d = y - x;
        const int q = bucket_dev<T>(d);
        const T thr = lut[q], lo = lut[kLutPad + q], hi = lut[2 * kLutPad + q];
        return vmax(x, y) + (fabs(d) >= thr ? hi : lo);
    }
}

// ------------------------------------------------------------------ gamma
// The reference's branch metrics (log_map.cpp:967-970) of one step take only four values:
//   gamma(u=0, o=+1) = ((-ys) + yp) - La/2 = -Q      gamma(u=1, o=+1) = (ys + yp) + La/2 = P
//   gamma(u=0, o=-1) = ((-ys) - yp) - La/2 = -P      gamma(u=1, o=-1) = (ys - yp) + La/2 = Q
// with P = (ys + yp) + La/2 and Q = (ys - yp) + La/2, exactly (IEEE addition is sign-symmetric).
// The tile loader computes P, Q once per (step, codeword); a lane reads the one it needs through
// a per-lane offset and applies the sign in the fma that adds the state metric:
//   gamma + metric = fma(sg, G, metric)   (sg*G is exact).
template <typename T>
struct LaneConst {
    T a_sg[3], a_pg[3];    // alpha step i -> i+1 (i mod 3 = PH): signs of the self / partner gamma
    int a_sel[3], a_psel[3];
    T b_sg[3], b_pg[3];    // beta step i+1 -> i
    int b_sel[3], b_psel[3];
    int a_offS[3], a_offP[3];   // LDS offsets of the self / partner LLR term: u*(W*64) + 8c + state
    int bv_off[3];              // LDS offset of beta[.][i+1] for the LLR terms: 8c + state
    int a_init0;                // alpha[.][0]: this lane holds state 0 at phase 0
    int b_init0;                // bit PH: this lane holds state 0 at phase PH (beta[.][L])
};

template <typename T>
__device__ __forceinline__ void lane_setup(const DecodeParams<T>& p, int lane, LaneConst<T>& lc)
{
    const int slot = lane & 7, c8 = lane & ~7;
#pragma unroll
    for (int ph = 0; ph < 3; ++ph) {
        lc.a_sg[ph] = (T)p.lane->a_sg[ph][slot];
        lc.a_pg[ph] = (T)p.lane->a_pg[ph][slot];
        lc.a_sel[ph] = p.lane->a_sel[ph][slot];
        lc.a_psel[ph] = p.lane->a_psel[ph][slot];
        lc.b_sg[ph] = (T)p.lane->b_sg[ph][slot];
        lc.b_pg[ph] = (T)p.lane->b_pg[ph][slot];
        lc.b_sel[ph] = p.lane->b_sel[ph][slot];
        lc.b_psel[ph] = p.lane->b_psel[ph][slot];
        const int j = p.lane->a_j[ph][slot], sw = p.lane->a_swap[ph][slot];
        lc.a_offS[ph] = sw * (kW * kLanes) + c8 + j;
        lc.a_offP[ph] = (1 - sw) * (kW * kLanes) + c8 + j;
        lc.bv_off[ph] = c8 + j;
    }
    lc.a_init0 = p.lane->state[0][slot] == 0;
    lc.b_init0 = (p.lane->state[0][slot] == 0) | ((p.lane->state[1][slot] == 0) << 1) |
                 ((p.lane->state[2][slot] == 0) << 2);
}

// ------------------------------------------------------------------ workgroup roles
// One workgroup = 4 waves = 8 codewords.  A SISO runs as a pipeline over windows of kW steps:
//   wave 0 (A)  alpha: F pass (forward, checkpoints) then the window-by-window recompute;
//   wave 1 (B)  beta, one window behind the recompute;
//   wave 2 (F0) LLR folds of the window beta finished last iteration (first half of the
//               items) + the tile loader (global -> registers -> (P, Q) in LDS, two windows ahead);
//   wave 3 (F1) the other half of the folds.
// The iterations end at a raw s_barrier that waits only for LDS (lgkmcnt), so global loads stay
// in flight across it.  Chain waves run at s_setprio 2 so folds and loads fill their bubbles.
constexpr int kWaves = 4;
constexpr int kFoldWaves = 3;                        // waves 1..3 fold (B has slack beside beta)
constexpr int kFoldPerWave = kTile / kFoldWaves;     // items (step, codeword) per fold wave per window
static_assert(kTile % kFoldWaves == 0 && 2 * kFoldPerWave <= kLanes, "one fold item per lane pair");

template <typename T>
struct Smem {
    T lut[3 * kLutPad];        // max* table: thr[64] | vlo[64] | vhi[64]
    T G[3][kW][kCw][2];        // (P, Q) per step and codeword, ring by window index mod 3
    T XY[3][2][kW][kLanes];    // [window mod 3][u] LLR terms (gamma + alpha) by state slot 8c + j
    T Bv[2][kW][kLanes];       // [window parity] beta[.][i+1] by state slot (LLR terms of step i)
    T tm[2][kW][kCw];          // [window parity] tempmax[i+1] per step and codeword
};

// raw barrier: waits for this wave's LDS traffic only, so prefetched global loads stay in flight
__device__ __forceinline__ void wg_sync_lds()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Inputs of one SISO.  Arrays are batch-interleaved [group][step][8].
template <typename T>
struct SisoSrc {
    const T* sys;
    const T* par;
    const T* la;      // a-priori la[g][i][c] (i < la_len), already in this decoder's order; null = zeros
    int la_len;
    int terminated;
};

template <typename T>
struct SisoDst {
    T* ext;           // extrinsic out (ext_mode), written in the OTHER decoder's order
    int ext_mode;     // 0: none, 1: ext[g][i][c], 2: ext[g][pi[i]][c], 3: ext[g][pinv[i]][c]  (i < ext_len)
    int ext_len;
    T* llr;           // optional raw LLR out, [G][L][8]
    T* le_dump;       // optional [B][iters][2][L]
    uint8_t* bits;    // optional decisions, written at pi[i] (random_deinterlvr_int, :1264)
    int bits_row;
    int bits_stride;
    int dump_slot;
    int dump_stride;
};

struct Geom {
    int K, L, nT, B, g;
    const int* pi;     // QPP pi[i]
    const int* pinv;   // its inverse
};

__device__ __forceinline__ int window_len(const Geom& gm, int t) { return min(kW, gm.L - t * kW); }

// channel values and a-priori of tile element e = k*8 + c of window t.  Every read is sequential:
// the interleaver permutations are applied when the extrinsic is WRITTEN (fold), so no load
// address depends on another load.
template <typename T>
__device__ __forceinline__ void load_elem(const SisoSrc<T>& src, const Geom& gm, int t, int e, T& ys, T& yp, T& la,
                                          bool want_yp)
{
    const int k = e >> 3, c = e & 7;
    const int i = t * kW + k;
    ys = 0;
    yp = 0;
    la = 0;
    if (i < gm.L) {
        const size_t off = ((size_t)gm.g * gm.L + i) * kCw + c;
        ys = src.sys[off];
        if (want_yp) yp = src.par[off];
        if (src.la && i < src.la_len) la = src.la[((size_t)gm.g * src.la_len + i) * kCw + c];
    }
}

// ---- tile loader (wave F0): element e = lane and e = lane + 64 (< kTile) of a window
constexpr int kLoadPerLane = (kTile + kLanes - 1) / kLanes;   // 2

template <typename T>
struct TileRegs {
    T ys[kLoadPerLane], yp[kLoadPerLane], la[kLoadPerLane];
};

template <typename T>
__device__ __forceinline__ void tile_issue(TileRegs<T>& r, const SisoSrc<T>& src, const Geom& gm, int t, int lane)
{
#pragma unroll
    for (int q = 0; q < kLoadPerLane; ++q) {
        const int e = lane + kLanes * q;
        if (e < kTile) load_elem(src, gm, t, e, r.ys[q], r.yp[q], r.la[q], true);
    }
}

// (P, Q) of the four branch metrics (see "gamma") into the LDS ring slot of window t
template <typename T>
__device__ __forceinline__ void tile_store(const TileRegs<T>& r, Smem<T>& sm, int t, int lane)
{
    T* g = &sm.G[t % 3][0][0][0];
#pragma unroll
    for (int q = 0; q < kLoadPerLane; ++q) {
        const int e = lane + kLanes * q;
        if (e < kTile) {
            const T hla = r.la[q] / (T)2;
            g[2 * e] = (r.ys[q] + r.yp[q]) + hla;
            g[2 * e + 1] = (r.ys[q] - r.yp[q]) + hla;
        }
    }
}

// ---- fold inputs (waves F0/F1): one item (k, c) per lane
template <typename T>
struct FoldRegs {
    T ys, la;
    int wext;   // extrinsic write position (per ext_mode)
    int wbit;   // decision write position pi[i]
};

template <typename T>
__device__ __forceinline__ void fold_issue(FoldRegs<T>& r, const SisoSrc<T>& src, const SisoDst<T>& dst,
                                           const Geom& gm, int t, int e)
{
    T yp;
    load_elem(src, gm, t, e, r.ys, yp, r.la, false);
    const int i = t * kW + (e >> 3);
    const bool in_k = i < gm.K;
    r.wext = i;
    if (dst.ext_mode == 2 && in_k) r.wext = gm.pi[i];
    if (dst.ext_mode == 3 && in_k) r.wext = gm.pinv[i];
    r.wbit = (dst.bits && in_k) ? gm.pi[i] : 0;
}

// ---- recursion steps
// Operands of one step are read from LDS ahead of the step group that uses them (the compiler
// cannot prove the LLR-term stores do not alias these reads).
template <typename T>
struct StepIn {
    T gs, gp;   // gamma magnitudes (P or Q) of the self / partner transition
    T tm;       // beta steps: tempmax[i+1]
};

template <typename T, int PH>
__device__ __forceinline__ StepIn<T> alpha_in(const Smem<T>& sm, int tb, int k, int c, const LaneConst<T>& lc)
{
    const T* g = &sm.G[tb][k][c][0];
    return StepIn<T>{g[lc.a_sel[PH]], g[lc.a_psel[PH]], (T)0};
}

template <typename T, int PH>
__device__ __forceinline__ StepIn<T> beta_in(const Smem<T>& sm, int tb, int k, int c, const LaneConst<T>& lc,
                                             const T* tmw)
{
    const T* g = &sm.G[tb][k][c][0];
    return StepIn<T>{g[lc.b_sel[PH]], g[lc.b_psel[PH]], tmw[k * kCw + c]};
}

// alpha step i -> i+1 with i mod 3 = PH (log_map.cpp:975-1001).  STORE: keep the LLR terms
// (by state and input u) and tempmax of the step for beta and the folds.
template <typename T, int ALGO, int PH, bool STORE>
__device__ __forceinline__ T alpha_step(T alpha, const StepIn<T>& in, const T* lut, int k, int c,
                                        const LaneConst<T>& lc, T* XYw, T* tmw)
{
    const T ap = dpp<PhaseDpp<PH>::ctrl>(alpha);
    const T xs = fma(lc.a_sg[PH], in.gs, alpha);   // gamma + alpha, predecessor in this lane
    const T xp = fma(lc.a_pg[PH], in.gp, ap);      // ... predecessor in the partner lane
    const T a = mstar<T, ALGO>(xs, xp, lut);
    const T m = group_max8(a);
    if constexpr (STORE) {
        XYw[k * kLanes + lc.a_offS[PH]] = xs;
        XYw[k * kLanes + lc.a_offP[PH]] = xp;
        tmw[k * kCw + c] = m;   // the 8 lanes of a codeword hold the same m
    }
    return a - m;
}

// beta step i+1 -> i with i mod 3 = PH (log_map.cpp:1004-1021).  Publishes beta[.][i+1] for the
// LLR terms of step i first.
template <typename T, int ALGO, int PH>
__device__ __forceinline__ T beta_step(T beta, const StepIn<T>& in, const T* lut, int k,
                                       const LaneConst<T>& lc, T* Bvw)
{
    Bvw[k * kLanes + lc.bv_off[PH]] = beta;
    const T bp = dpp<PhaseDpp<PH>::ctrl>(beta);
    const T b = mstar<T, ALGO>(fma(lc.b_sg[PH], in.gs, beta), fma(lc.b_pg[PH], in.gp, bp), lut);
    return b - in.tm;
}

template <typename T, int ALGO>
__device__ __forceinline__ T beta_step_rt(int ph, T beta, const Smem<T>& sm, int tb, int k, int c,
                                          const LaneConst<T>& lc, T* Bvw, const T* tmw)
{
    if (ph == 0) return beta_step<T, ALGO, 0>(beta, beta_in<T, 0>(sm, tb, k, c, lc, tmw), sm.lut, k, lc, Bvw);
    if (ph == 1) return beta_step<T, ALGO, 1>(beta, beta_in<T, 1>(sm, tb, k, c, lc, tmw), sm.lut, k, lc, Bvw);
    return beta_step<T, ALGO, 2>(beta, beta_in<T, 2>(sm, tb, k, c, lc, tmw), sm.lut, k, lc, Bvw);
}

// alpha over the n steps of window t (window starts are = 0 mod 3)
template <typename T, int ALGO, bool STORE>
__device__ __forceinline__ T alpha_window(T alpha, int t, int n, const Smem<T>& sm, int c, const LaneConst<T>& lc,
                                          T* XYw, T* tmw)
{
    const int tb = t % 3;
    int k = 0;
    for (; k + 3 <= n; k += 3) {
        const StepIn<T> i0 = alpha_in<T, 0>(sm, tb, k, c, lc);
        const StepIn<T> i1 = alpha_in<T, 1>(sm, tb, k + 1, c, lc);
        const StepIn<T> i2 = alpha_in<T, 2>(sm, tb, k + 2, c, lc);
        alpha = alpha_step<T, ALGO, 0, STORE>(alpha, i0, sm.lut, k, c, lc, XYw, tmw);
        alpha = alpha_step<T, ALGO, 1, STORE>(alpha, i1, sm.lut, k + 1, c, lc, XYw, tmw);
        alpha = alpha_step<T, ALGO, 2, STORE>(alpha, i2, sm.lut, k + 2, c, lc, XYw, tmw);
    }
    if (k < n)
        alpha = alpha_step<T, ALGO, 0, STORE>(alpha, alpha_in<T, 0>(sm, tb, k, c, lc), sm.lut, k, c, lc, XYw, tmw);
    if (k + 1 < n)
        alpha = alpha_step<T, ALGO, 1, STORE>(alpha, alpha_in<T, 1>(sm, tb, k + 1, c, lc), sm.lut, k + 1, c, lc, XYw,
                                              tmw);
    return alpha;
}

// beta over the n steps of window t, downwards (full windows: static phases; else runtime)
template <typename T, int ALGO>
__device__ __forceinline__ T beta_window(T beta, int t, int n, Smem<T>& sm, int c, const LaneConst<T>& lc)
{
    const int tb = t % 3, xb = t & 1;
    T* Bvw = &sm.Bv[xb][0][0];
    const T* tmw = &sm.tm[xb][0][0];
    if (n == kW) {
        for (int k = kW - 1; k >= 0; k -= 3) {   // phases 2, 1, 0 (kW = 0 mod 3)
            const StepIn<T> b2 = beta_in<T, 2>(sm, tb, k, c, lc, tmw);
            const StepIn<T> b1 = beta_in<T, 1>(sm, tb, k - 1, c, lc, tmw);
            const StepIn<T> b0 = beta_in<T, 0>(sm, tb, k - 2, c, lc, tmw);
            beta = beta_step<T, ALGO, 2>(beta, b2, sm.lut, k, lc, Bvw);
            beta = beta_step<T, ALGO, 1>(beta, b1, sm.lut, k - 1, lc, Bvw);
            beta = beta_step<T, ALGO, 0>(beta, b0, sm.lut, k - 2, lc, Bvw);
        }
    } else {
        for (int k = n - 1; k >= 0; --k) beta = beta_step_rt<T, ALGO>(k % 3, beta, sm, tb, k, c, lc, Bvw, tmw);
    }
    return beta;
}

// E_algorithm_seq over 8 values in state order (log_map.cpp:817-829)
template <typename T, int ALGO>
__device__ __forceinline__ T fold8(const T* v, const T* lut)
{
    T t = mstar<T, ALGO>(v[0], v[1], lut);
#pragma unroll
    for (int j = 2; j < 8; ++j) t = mstar<T, ALGO>(t, v[j], lut);
    return t;
}

// LLR fold + extrinsic + outputs of item e = k*8 + c of window t (:1024-1039, :1234-1264), on a
// lane pair: the odd lane folds temp1 (u = 1), the even lane temp0 (u = 0); the even lane
// combines LLR = E_seq(temp1) - E_seq(temp0) and writes the outputs.  All lanes of the wave
// must call this (DPP exchange); `live` masks the lanes whose item is outside the window.
template <typename T, int ALGO>
__device__ __forceinline__ void fold_item(const Smem<T>& sm, const FoldRegs<T>& fr, int t, int e, bool live,
                                          const SisoDst<T>& dst, const Geom& gm, int lane)
{
    const int k = e >> 3, c = e & 7, u = lane & 1;
    const int xs = t % 3, bs = t & 1;
    const int i = t * kW + k;
    T r = (T)0;
    if (live) {
        T tv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)   // temp_u[j] = (gamma + alpha) + beta[j][i+1]
            tv[j] = sm.XY[xs][u][k][c * 8 + j] + sm.Bv[bs][k][c * 8 + j];
        r = fold8<T, ALGO>(tv, sm.lut);
    }
    const T r1 = dpp<kDppXor1>(r);   // the odd partner's E_seq(temp1)
    if (!live || u) return;
    const T llr = r1 - r;
    const T le = llr - fr.la - (T)2 * fr.ys;
    const int b = gm.g * kCw + c;
    if (dst.llr) dst.llr[((size_t)gm.g * gm.L + i) * kCw + c] = llr;
    if (dst.ext_mode && i < dst.ext_len) dst.ext[((size_t)gm.g * dst.ext_len + fr.wext) * kCw + c] = le;
    if (b < gm.B) {
        if (dst.le_dump) dst.le_dump[(size_t)b * dst.dump_stride + (size_t)dst.dump_slot * gm.L + i] = le;
        if (dst.bits && i < gm.K)   // decision (:862-879: LLR < 0 -> 0, else 1) at pi[i] (:1264)
            dst.bits[(size_t)b * dst.bits_stride + (size_t)dst.bits_row * gm.K + fr.wbit] = (llr < (T)0) ? 0 : 1;
    }
}

#ifdef TD_STAMPS
// diagnostic build only: per-wave cycle totals (s_memtime, shader clock)
#define TD_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TD_ACC(slot, a, b) (st[slot] += (b) - (a))
#else
#define TD_STAMP(v)
#define TD_ACC(slot, a, b)
#endif
constexpr int kStampSlots = 7;   // per wave: F pass, F wait, B work, B wait, -, -, HW_ID (see diag)

// Register sets for data in flight are indexed by window parity through explicit branches and
// always consumed before they are re-issued: selecting or copying a register whose load is still
// in flight would force a vmcnt wait (or push the set to scratch).

// loader step: store tile `ws` (< 0: none) from its parity set, then re-issue that parity set
// with tile `wi` (< 0: none).  When both are given they have the same parity.
template <typename T>
__device__ __forceinline__ void loader_step(TileRegs<T>& even, TileRegs<T>& odd, Smem<T>& sm, const SisoSrc<T>& src,
                                            const Geom& gm, int ws, int wi, int lane)
{
    const int par = (ws >= 0 ? ws : wi) & 1;
    if (par) {
        if (ws >= 0) tile_store(odd, sm, ws, lane);
        if (wi >= 0) tile_issue(odd, src, gm, wi, lane);
    } else {
        if (ws >= 0) tile_store(even, sm, ws, lane);
        if (wi >= 0) tile_issue(even, src, gm, wi, lane);
    }
}

// One SISO over the workgroup's 8 codewords.  Each role runs its own loops (so only that role's
// state is live in its code); every role executes the same sequence of wg_sync_lds barriers:
// 1 (F prologue) + nT (F iterations) + nT + 2 (B iterations).
template <typename T, int ALGO>
__device__ void siso_wg(Smem<T>& sm, const SisoSrc<T>& src, const SisoDst<T>& dst, const Geom& gm, T* ckpt,
                        const LaneConst<T>& lc, int wave, int lane, unsigned long long* st)
{
    (void)st;
    const int nT = gm.nT;
    const int tl = nT - 1;
    const int nB = nT + 2;   // B-pass iterations: j = 0 .. nT+1 (wa = tl - j, wb = wa + 1, wf = wa + 2)

    if (wave == 0) {
        // ===================================== A: alpha
        const int c = lane >> 3;
        T* my_ckpt = ckpt + (size_t)gm.g * (nT + 1) * kLanes + lane;
        T alpha = lc.a_init0 ? (T)0 : (T)-kInfty;   // :943,948
        wg_sync_lds();
        for (int t = 0; t < nT; ++t) {   // F pass: window t, checkpoint at its start
            TD_STAMP(f0);
            my_ckpt[(size_t)t * kLanes] = alpha;
            alpha = alpha_window<T, ALGO, false>(alpha, t, window_len(gm, t), sm, c, lc, nullptr, nullptr);
            TD_STAMP(f1);
            wg_sync_lds();
            TD_STAMP(f2);
            TD_ACC(0, f0, f1);
            TD_ACC(1, f1, f2);
        }
        // B pass: recompute window wa from its checkpoint (prefetched two windows ahead)
        T ck_even = (T)0, ck_odd = (T)0;
        {
            const T c0 = my_ckpt[(size_t)tl * kLanes];
            const T c1 = tl > 0 ? my_ckpt[(size_t)(tl - 1) * kLanes] : (T)0;
            if (tl & 1) {
                ck_odd = c0;
                ck_even = c1;
            } else {
                ck_even = c0;
                ck_odd = c1;
            }
        }
        for (int j = 0; j < nB; ++j) {
            TD_STAMP(b0);
            const int wa = tl - j;
            if (wa >= 0) {
                T a0;
                if (wa & 1) {
                    a0 = ck_odd;
                    if (wa >= 2) ck_odd = my_ckpt[(size_t)(wa - 2) * kLanes];
                } else {
                    a0 = ck_even;
                    if (wa >= 2) ck_even = my_ckpt[(size_t)(wa - 2) * kLanes];
                }
                alpha_window<T, ALGO, true>(a0, wa, window_len(gm, wa), sm, c, lc, &sm.XY[wa % 3][0][0][0],
                                            &sm.tm[wa & 1][0][0]);
            }
            TD_STAMP(b1);
            wg_sync_lds();
            TD_STAMP(b2);
            TD_ACC(2, b0, b1);
            TD_ACC(3, b1, b2);
        }
        return;
    }

    // ===================================== waves 1..3
    // F pass: wave 2 loads tiles (tile t+1, issued at t-2, into ring slot (t+1) % 3; then issue
    // tile t+3); waves 1 and 3 only keep the barrier count.
    TileRegs<T> t_even, t_odd;   // wave 2: tiles in flight by window parity
    if (wave == 2) {
        tile_issue(t_even, src, gm, 0, lane);
        tile_store(t_even, sm, 0, lane);
        if (nT > 1) tile_issue(t_odd, src, gm, 1, lane);
        if (nT > 2) tile_issue(t_even, src, gm, 2, lane);
    }
    wg_sync_lds();
    for (int t = 0; t < nT; ++t) {
        TD_STAMP(f0);
        if (wave == 2 && t + 1 < nT) loader_step(t_even, t_odd, sm, src, gm, t + 1, t + 3 < nT ? t + 3 : -1, lane);
        TD_STAMP(f1);
        wg_sync_lds();
        TD_STAMP(f2);
        TD_ACC(0, f0, f1);
        TD_ACC(1, f1, f2);
    }

    // B pass: wave 1 runs beta over wb; wave 2 stores tile wa-1 (issued at j-2 as "wa-3"; tiles
    // tl-2..tl never left the ring) into the slot nobody reads this iteration; waves 1..3 fold
    // window wf, one item per lane, with inputs prefetched two windows ahead.
    const int fe = (wave - 1) * kFoldPerWave + (lane >> 1);   // item of this lane pair
    const bool folder = (lane >> 1) < kFoldPerWave;
    FoldRegs<T> f_even{}, f_odd{};
    T beta = (T)0;
    if (wave == 1) {
        const int phL = gm.L % 3;   // beta[.][L] lives in the labeling of phase L mod 3
        beta = (src.terminated && !((lc.b_init0 >> phL) & 1)) ? (T)-kInfty : (T)0;   // :944,951-959
    }
    if (folder) {
        if (tl & 1) {
            fold_issue(f_odd, src, dst, gm, tl, fe);
            if (tl > 0) fold_issue(f_even, src, dst, gm, tl - 1, fe);
        } else {
            fold_issue(f_even, src, dst, gm, tl, fe);
            if (tl > 0) fold_issue(f_odd, src, dst, gm, tl - 1, fe);
        }
    }
    for (int j = 0; j < nB; ++j) {
        TD_STAMP(b0);
        const int wa = tl - j, wb = wa + 1, wf = wa + 2;
        if (wave == 1 && wb >= 0 && wb <= tl) beta = beta_window<T, ALGO>(beta, wb, window_len(gm, wb), sm, lane >> 3, lc);
        if (wave == 2) {
            const int ws = (wa - 1 >= 0 && wa - 1 <= tl - 3) ? wa - 1 : -1;   // issued at j-2 as "wa-3"
            const int wi = (wa - 3 >= 0 && wa - 3 <= tl - 3) ? wa - 3 : -1;
            if (ws >= 0 || wi >= 0) loader_step(t_even, t_odd, sm, src, gm, ws, wi, lane);
        }
        if (wf >= 0 && wf <= tl) {
            const bool live = folder && (fe >> 3) < window_len(gm, wf);
            if (wf & 1) {
                fold_item<T, ALGO>(sm, f_odd, wf, fe, live, dst, gm, lane);
                if (folder && wf - 2 >= 0) fold_issue(f_odd, src, dst, gm, wf - 2, fe);
            } else {
                fold_item<T, ALGO>(sm, f_even, wf, fe, live, dst, gm, lane);
                if (folder && wf - 2 >= 0) fold_issue(f_even, src, dst, gm, wf - 2, fe);
            }
        }
        TD_STAMP(b1);
        wg_sync_lds();
        TD_STAMP(b2);
        TD_ACC(2, b0, b1);
        TD_ACC(3, b1, b2);
    }
}

template <typename T>
__device__ __forceinline__ void lut_to_lds(const DecodeParams<T>& p, Smem<T>& sm, int tid)
{
    for (int q = tid; q < kLutPad; q += kWaves * kLanes) {
        const bool ok = q < kLutSize;
        sm.lut[q] = ok ? p.lut[q].thr : (T)INFINITY;
        sm.lut[kLutPad + q] = ok ? p.lut[q].vlo : (T)0;
        sm.lut[2 * kLutPad + q] = ok ? p.lut[q].vhi : (T)0;
    }
}

template <typename T>
__device__ __forceinline__ Smem<T>& smem()
{
    extern __shared__ __attribute__((aligned(16))) unsigned char td_smem[];
    return *reinterpret_cast<Smem<T>*>(td_smem);
}

// The whole turbo decode of 8 codewords per workgroup (TurboDecoding, log_map.cpp:1146-1280).
template <typename T, int ALGO>
__global__ __launch_bounds__(256, 2) void turbo_decode_kernel(DecodeParams<T> p)
{
    Smem<T>& sm = smem<T>();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    LaneConst<T> lc;
    lane_setup(p, lane, lc);
    lut_to_lds(p, sm, threadIdx.x);
    if (wave < 2) __builtin_amdgcn_s_setprio(2);   // the recursions first; folds and loads fill in
    __syncthreads();

    Geom gm{p.K, p.L, p.nT, p.B, (int)blockIdx.x, p.pi, p.pinv};
    unsigned long long st[kStampSlots] = {};
    // SISO pass s = 2*it + dec
    for (int s = 0; s < 2 * p.iters; ++s) {
        const int it = s >> 1, dec = s & 1;
        const bool want_bits = dec == 1 && (p.all_iters || it == p.iters - 1);
        // decoder 1: La = deinterleaved Le of decoder 2 (:1221), zero before the first
        //            iteration (:1212-1215); its Le is written interleaved (ext12[pinv[i]]),
        //            i.e. already as decoder 2's La (:1242).
        // decoder 2: La read in order; its Le is written deinterleaved (ext21[pi[i]], = the
        //            next La of decoder 1); decisions deinterleaved (:1261-1264).
        SisoSrc<T> src{dec ? p.sys2 : p.sys1, dec ? p.par2 : p.par1,
                       dec ? p.ext12 : (it == 0 ? nullptr : p.ext21), p.K, 1};
        SisoDst<T> dst{dec ? p.ext21 : p.ext12, dec ? 2 : 3, p.K, nullptr, p.le_dump,
                       want_bits ? p.bits : nullptr, p.all_iters ? it : 0, p.all_iters ? p.iters * p.K : p.K,
                       s, p.iters * 2 * p.L};
        siso_wg<T, ALGO>(sm, src, dst, gm, p.ckpt, lc, wave, lane, st);
        __syncthreads();   // extrinsic stores of this SISO visible to the next one's loads
    }
#ifdef TD_STAMPS
    st[6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    if (p.stamps && lane == 0)
        for (int q = 0; q < kStampSlots; ++q)
            p.stamps[((size_t)blockIdx.x * kWaves + wave) * kStampSlots + q] = st[q];
#endif
}

// Standalone SISO (Log_MAP_decoder) over interleaved [G][L][8] inputs.
template <typename T, int ALGO>
__global__ __launch_bounds__(256, 2) void siso_kernel(DecodeParams<T> p, const T* la, int terminated)
{
    Smem<T>& sm = smem<T>();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    LaneConst<T> lc;
    lane_setup(p, lane, lc);
    lut_to_lds(p, sm, threadIdx.x);
    if (wave < 2) __builtin_amdgcn_s_setprio(2);
    __syncthreads();
    Geom gm{p.K, p.L, p.nT, p.B, (int)blockIdx.x, p.pi, p.pinv};
    SisoSrc<T> s{p.sys1, p.par1, la, p.L, terminated};
    SisoDst<T> d{nullptr, 0, 0, p.llr_out, nullptr, nullptr, 0, 0, 0, 0};
    siso_wg<T, ALGO>(sm, s, d, gm, p.ckpt, lc, wave, lane, nullptr);
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
// Dynamic LDS above 64 KiB must be allowed per kernel (once per device and kernel).
inline hipError_t allow_smem(const void* fn, size_t bytes)
{
    static thread_local const void* done_fn[32] = {};
    static thread_local int done_dev[32] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 32; ++i)
        if (done_fn[i] == fn && done_dev[i] == dev) return hipSuccess;
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 32; ++i)
        if (!done_fn[i]) {
            done_fn[i] = fn;
            done_dev[i] = dev;
            break;
        }
    return hipSuccess;
}

template <typename T, int ALGO>
hipError_t launch_turbo_algo(const DecodeParams<T>& p, hipStream_t st)
{
    hipError_t e = allow_smem(reinterpret_cast<const void*>(&turbo_decode_kernel<T, ALGO>), sizeof(Smem<T>));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((turbo_decode_kernel<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), sizeof(Smem<T>), st, p);
    return hipGetLastError();
}

template <typename T, int ALGO>
hipError_t launch_siso_algo(const DecodeParams<T>& p, const T* la, int terminated, hipStream_t st)
{
    hipError_t e = allow_smem(reinterpret_cast<const void*>(&siso_kernel<T, ALGO>), sizeof(Smem<T>));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((siso_kernel<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), sizeof(Smem<T>), st, p, la, terminated);
    return hipGetLastError();
}

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
    return p.algo == 1 ? launch_turbo_algo<T, 1>(p, st) : launch_turbo_algo<T, 0>(p, st);
}

template <typename T>
hipError_t launch_siso(const DecodeParams<T>& p, const T* recs, const T* la, T* la_ws, int terminated, T* llr,
                       hipStream_t st)
{
    const size_t total = (size_t)p.G * p.L * kCw;
    int gblocks = (int)((total + 255) / 256);
    if (gblocks > 8192) gblocks = 8192;
    hipLaunchKernelGGL(siso_in_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, recs, la, la_ws);
    hipError_t e = p.algo == 1 ? launch_siso_algo<T, 1>(p, la_ws, terminated, st)
                               : launch_siso_algo<T, 0>(p, la_ws, terminated, st);
    if (e != hipSuccess) return e;
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
