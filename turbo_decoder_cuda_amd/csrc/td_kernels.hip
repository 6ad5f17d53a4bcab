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
// (:1217-1265).  Per SISO, over windows of kW = 15 trellis steps (12 in the td_kernels_w12.hip build):
//   F pass  wave A runs alpha forward over the L = K+3 steps.  Log-MAP streams the UNNORMALISED
//           alpha_raw of every step (by state, 512 B per group and step in fp64) and row L to an HBM
//           scratch (astore [G][L+1][64]); tempmax (:986-993) is the max of such a row, formed on
//           chip where it is needed.  Max-Log-MAP stores the normalised alpha one step in three and
//           tempmax (tmstore); its folds recompute the steps in between.  No alpha is recomputed in
//           log-MAP.
//   B pass  windows last..first in a three-stage pipeline: wave B runs beta of window t
//           (subtracting tempmax[i+1], :1019, staged in LDS) and publishes beta by state; the
//           loader DMAs the alpha rows of window t-1 from the scratch into an LDS ring; the two
//           fold waves run the LLR folds E_seq(temp1) - E_seq(temp0) of window t+1 over
//           (step, codeword) items in state order 0..7 (:1038) and write the extrinsic update
//           Le = LLR - La - 2*ys (:1237, :1258) at the interleaved position.
// The scratch stream is ~70 % of the kernel's HBM traffic (bench.py traffic_model).
// Every floating-point operation is the reference's, in the reference's order (max* is
// symmetric, so the two operands may arrive in either order).  Build with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "td_kernels.h"
#include "td_tables.h"

// td_kernels_w12.hip compiles this file a second time with 12-step windows (TD_W12_TU) into its own
// namespace, for the one launch that needs them: fp32 at four workgroups per CU (launch_turbo4_w12).
#ifdef TD_W12_TU
namespace td_w12 {
using namespace ::td;
#else
namespace td {
#endif

#ifndef TD_KW
#define TD_KW 15   // td_kernels_w12.hip: 12
#endif
constexpr int kW = TD_KW;                       // steps per window (multiple of 3; td_kernels.h kWindowStepsMax)
static_assert(kW == 12 || kW == 15, "windows of 12 or 15 steps");
static_assert(kW <= kWindowStepsMax, "the host sizes the alpha scratch's DMA tail for the longest window");
constexpr int kArow0 = kW / 2;                  // scheduled alpha stores: rows addressed from row kArow0 (immediates)
constexpr int kCw = 8;                          // codewords per workgroup
constexpr int kLanes = 64;
constexpr int kTile = kW * kCw;                 // (step, codeword) elements per window
static_assert(kW % 3 == 0, "window must be a multiple of the label period");

// ------------------------------------------------------------------ diagnostic builds
// TD_DIAG, a bit mask (0, the product, unless a diagnostic library is built with -DTD_DIAG=n):
// timing-only builds whose decoded results are WRONG, used to attribute the kernel's time
// (DESIGN.md 3.2).  No test, smoke() or bench.py run loads them.
#ifndef TD_DIAG
#define TD_DIAG 0
#endif
constexpr unsigned kDiagNoAdma = 1;       // the B pass without the loader's alpha copies
constexpr unsigned kDiagNoBConvert = 2;   // the B pass without the loader's tile / tempmax converts
constexpr unsigned kDiagNoFold = 4;       // the B pass without its folds
constexpr unsigned kDiagNoBeta = 8;       // the B pass without the beta chain
constexpr unsigned kDiagOcc3Alias = 16;   // beta rows and tile ring alias the alpha ring: fp64 three per CU (Smem)
constexpr unsigned kDiagNoAStore = 32;    // the F pass without its alpha scratch stores (power / clock attribution)
constexpr unsigned kDiagFoldNoLut = 64;   // the B pass's folds with a table-free max* (no LDS reads; LDS contention test)
constexpr unsigned kDiagSwNoCk = 128;     // windowed kernels: no alpha checkpoint stores / loads (HBM share test)
template <unsigned D>
constexpr bool kDiag = (TD_DIAG & D) != 0;

// Alpha rows kept in the F pass -> B pass scratch, by phase i mod 3 (bit p: steps i = p mod 3).
// Log-MAP keeps every row; Max-Log-MAP only the rows of phase 0, and its folds recompute the two
// steps in between (alpha_recompute).  Log-MAP keeping a subset measured 16 % (phases {0, 1}) and 40 %
// (phase 0) slower in round 3: eight table max* per recomputed step cost the fold waves more than
// the scratch traffic costs the kernel; Max-Log-MAP keeping two phases in three
// measured slower than one (1635 vs 1860 Mbit/s).
template <int ALGO>
constexpr int kCkPh = ALGO == 1 ? 1 : 7;                                      // stored phases of this algorithm
template <int ALGO>
constexpr bool kCkAll = kCkPh<ALGO> == 7;                                    // every row stored
// the phase whose steps sit furthest from a kept row (recomputed through the most steps)
constexpr int ck_depth(int ph, int p)
{
    int d = 0;
    while (!((ph >> p) & 1)) --p, ++d;
    return d;
}
template <int ALGO>
constexpr int kCkDeepest = ck_depth(kCkPh<ALGO>, 2) >= ck_depth(kCkPh<ALGO>, 1) ? 2 : 1;

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

// fp32: bound_ctrl set (every pattern here permutes within a row, so no lane reads out of bounds and
// the values are the same) lets the compiler fold the move into its consumer (v_max_f32_dpp): 148 of
// the fp32 log-MAP kernel's 258 moves go, fp32 log-MAP +2.5 %, Max-Log-MAP +4.4 %, at 32768 +0.6 /
// +2.4 % (profiles/r04/ab_v32_f32_dpp_combine.txt).  fp64 has no 64-bit DPP operand to fold into.
template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// partner exchange mask of phase PH (i mod 3)
template <int PH>
struct PhaseDpp {
    static constexpr int ctrl = PH == 0 ? kDppXor1 : (PH == 1 ? kDppXor2 : kDppMir8);
};

// x + s*g for a sign s = +-1 and a DPP-moved x: fma(s, g, x), exact.  fp32 writes it as a multiply
// (off the chain) and an add whose DPP operand the compiler folds into v_add_f32_dpp, so the move
// leaves the chain; fp64 has no 64-bit DPP operand and keeps the fma (its code is unchanged).
// fp32 log-MAP +2.0 %, Max-Log-MAP and the 32768 batch level (profiles/r04/ab_v33_f32_partner_add_dpp.txt).
__device__ __forceinline__ double fma_pm(double s, double g, double x) { return fma(s, g, x); }
__device__ __forceinline__ float fma_pm(float s, float g, float x) { return x + s * g; }

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

// The alpha step's tempmax (the max over the codeword's 8 lanes) and the partner's metric an: three
// (DPP, max) levels, the first one the partner exchange of this phase.  (A quad tree -- the three
// quad mates in one DPP level, then one row_half_mirror -- measured 0.4-1.7 % slower in round 3: in
// fp64 the DPP pairs' issue, not their hazard, is the cost.)
template <typename T, int PH>
__device__ __forceinline__ T alpha_tempmax(T a, T& an)
{
    an = dpp<PhaseDpp<PH>::ctrl>(a);
    T m = vmax(a, an);
    m = vmax(m, dpp<PhaseDpp<(PH + 1) % 3>::ctrl>(m));
    return vmax(m, dpp<PhaseDpp<(PH + 2) % 3>::ctrl>(m));
}

// ------------------------------------------------------------------ max*
// Exact bucket form of E_algorithm (td_tables.h, build_lut): the bucket index is a bit field of
// d (exponent + 2 mantissa bits; the sign bit is outside the field, so d need not be |d|).
template <typename T>
__device__ __forceinline__ int bucket_dev(T d);
template <>
__device__ __forceinline__ int bucket_dev<double>(double d)
{
    const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
    const int q = (int)__builtin_amdgcn_ubfe(hi, BucketBits<double>::shift, BucketBits<double>::width);
    return min(max(q, BucketBits<double>::base), BucketBits<double>::base + kLutSize - 1);
}
template <>
__device__ __forceinline__ int bucket_dev<float>(float d)
{
    const unsigned b = (unsigned)__float_as_int(d);
    const int q = (int)__builtin_amdgcn_ubfe(b, BucketBits<float>::shift, BucketBits<float>::width);
    return min(max(q, BucketBits<float>::base), BucketBits<float>::base + kLutSize - 1);
}

// The table lives in LDS as rows of two fields per bucket, thr[q] and v[q] (= vlo[q]; vhi[q] =
// vlo[q+1], see build_lut), each field replicated in 16 columns: lane l reads column l % 16, so
// the 16 lanes an LDS cycle serves always hit 16 distinct bank pairs whatever their buckets (the
// random buckets of a single shared copy cost ~40% extra LDS cycles in bank conflicts).  Element
// (q, field f, column) sits at (2q + f) * 16 + column.  A lane's pointer is its column shifted
// down by the first bucket's bit-field value (lut_origin), so the row address is one lshl_add of
// the clamped bit field and thr, vlo, vhi are ds_read offsets 0, 128, 384 B of it (one
// ds_read2 + one ds_read, no address add on the chain).
constexpr int kLutRows = kLutSize + 1;   // + a pad row: v[q+1] for the last bucket
// fp32: 32 columns.  Its 4-byte reads are served 32 lanes per LDS cycle on 32 banks, so with 16
// columns lanes l and l+16 shared a bank whenever their buckets differed (SQ_LDS_BANK_CONFLICT
// was 28 % of the fp32 kernel's LDS cycles).  fp64 keeps 16: 8-byte elements in 16 columns
// already cover the 32 banks that ds_read2_b64 serves per cycle (32 columns measured level, and a
// row read as three ds_read_b64 from them 2-6 % slower: DESIGN.md 3.2).
template <typename T>
constexpr int kLutCols = sizeof(T) == 4 ? 32 : 16;
template <typename T>
constexpr int kLutElems = 2 * kLutRows * kLutCols<T>;

template <typename T>
__device__ __forceinline__ const T* lut_origin(const T* col)
{
    return col - 2 * BucketBits<T>::base * kLutCols<T>;
}

// fill a table copy: element e of the 2 * kLutRows * 16 (one thread per element)
template <typename T>
__device__ __forceinline__ T lut_elem(const LutEntry<T>* lut, int e)
{
    const int q = e / (2 * kLutCols<T>), f = (e / kLutCols<T>) & 1;
    if (q >= kLutSize) return f ? (T)lut[kLutSize - 1].vhi : (T)INFINITY;
    return f ? (T)lut[q].vlo : (T)lut[q].thr;
}

struct LutRow {
    int o;   // element offset of the bucket's row from the lane's origin
};
template <typename T>
__device__ __forceinline__ LutRow lut_row(T d)
{
    return LutRow{bucket_dev<T>(d) * 2 * kLutCols<T>};
}
// the row's threshold and its two values
template <typename T>
__device__ __forceinline__ void lut_fields(const T* lut, int o, T& thr, T& lo, T& hi)
{
    thr = lut[o];
    lo = lut[o + kLutCols<T>];
    hi = lut[o + 3 * kLutCols<T>];
}
template <typename T>
__device__ __forceinline__ T lut_pick(const T* lut, LutRow r, T d)
{
    T thr, lo, hi;
    lut_fields<T>(lut, r.o, thr, lo, hi);
    return fabs(d) >= thr ? hi : lo;
}

template <typename T, int ALGO>
__device__ __forceinline__ T mstar(T x, T y, const T* lut)
{
    if constexpr (ALGO == 1) {
        return vmax(x, y);   // Max-Log-MAP
    } else {
        const T d = y - x;
        return vmax(x, y) + lut_pick(lut, lut_row(d), d);
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
    int st_off[3];         // 8c + state held by this lane at phase PH: alpha / beta stored by state
    int tm_writer;         // one lane per codeword stores tempmax
    int a_init0;           // alpha[.][0]: this lane holds state 0 at phase 0
    int b_init0;           // bit PH: this lane holds state 0 at phase PH (beta[.][L])
};

// (re)loaded per SISO by the two recursion waves only, so the other roles keep no copy live
template <typename T>
__device__ __forceinline__ void lane_setup(const LaneTables* lt, int lane, LaneConst<T>& lc)
{
    const int slot = lane & 7, c8 = lane & ~7;
#pragma unroll
    for (int ph = 0; ph < 3; ++ph) {
        lc.a_sg[ph] = (T)lt->a_sg[ph][slot];
        lc.a_pg[ph] = (T)lt->a_pg[ph][slot];
        lc.a_sel[ph] = lt->a_sel[ph][slot];
        lc.a_psel[ph] = lt->a_psel[ph][slot];
        lc.b_sg[ph] = (T)lt->b_sg[ph][slot];
        lc.b_pg[ph] = (T)lt->b_pg[ph][slot];
        lc.b_sel[ph] = lt->b_sel[ph][slot];
        lc.b_psel[ph] = lt->b_psel[ph][slot];
        lc.st_off[ph] = c8 + lt->state[ph][slot];
    }
    lc.tm_writer = slot == 0;
    lc.a_init0 = lt->state[0][slot] == 0;
    lc.b_init0 = (lt->state[0][slot] == 0) | ((lt->state[1][slot] == 0) << 1) |
                 ((lt->state[2][slot] == 0) << 2);
}

// ------------------------------------------------------------------ workgroup roles
// One workgroup = 4 waves = 8 codewords.  A SISO is two passes over windows of kW steps:
//   F pass   wave 0 (A) runs alpha forward and streams alpha (by state) and tempmax of every
//            step to HBM scratch; wave 2 (F0) stages the window inputs by LDS DMA and converts
//            them into the (P, Q) tiles one window ahead.
//   B pass   windows last..first, a three-stage pipeline per iteration j (wa = tl - j):
//            wave 1 (B)   beta over window wa+1 (tempmax from LDS), publishing beta by state;
//            wave 2 (F0)  converts the staged tiles and tempmax of window wa, stages window wa-3
//                         and copies alpha of wa-1, all HBM -> LDS by DMA;
//            waves 0, 3   LLR folds of window wa+2 (beta finished last iteration), one (step,
//                         codeword) item per lane, both input bits in the same lane.
// Only the two recursions are serial chains; nothing else waits on them but the barriers.  The
// barriers are raw `s_waitcnt lgkmcnt(0); s_barrier`, so prefetched global loads stay in flight.
// (Measured and retired in round 3, numbers in DESIGN.md 3.2 / 6: a fifth wave recomputing alpha in
// the B pass from one checkpoint per window, -10 % at B = 4096; the fold lanes loading their alpha
// blocks from HBM instead of the Av ring, -9 %; F1 folding with one E_seq chain per lane, level.)
constexpr int kWaves = kGroupWaves;                  // waves per codeword group
// items of fold wave A (beside the other workgroup's loader) per window; F1 (beside its beta) the
// rest.  64 / 56 measured level with 60 / 60 (round 4), as 40/56 .. 56/40 against 48/48 did with
// 12-step windows (round 3).
constexpr int kFoldA = kTile / 2;
static_assert(kFoldA <= kLanes && kTile - kFoldA <= kLanes, "one fold item per lane");
// fp64 Max-Log-MAP, whose B pass the two fold waves (A and F0) bound: A takes 64 items (8 whole
// steps), F0 the other 56 (profiles/r04/ab_v32_maxlog_foldsplit.txt: config 3 +1.2 %, its 32768
// batch +1.5 %; 56/64 the same; fp32 Max-Log-MAP lost 1.5 % either way and keeps 60/60).
constexpr int kFoldAMaxLog64 = 64;
template <typename T, int ALGO>
constexpr int kFoldAOf = (ALGO == 1 && sizeof(T) == 8) ? kFoldAMaxLog64 : kFoldA;   // items of fold wave A
static_assert(kFoldAOf<double, 1> <= kLanes && kTile - kFoldAOf<double, 1> <= kLanes, "one fold item per lane");
constexpr int kAvSlots = 4;   // alpha ring: copied 3 iterations before its fold (loader depth 3)
// every alpha row of a window is in the Av ring for the folds (no fold-side recompute)
template <int ALGO>
constexpr bool kFoldRows = kCkAll<ALGO>;

// Loader staging.  Window inputs travel HBM -> LDS by DMA (global_load_lds_dwordx4: no VGPR
// destination, completion counted by vmcnt; LDS target = wave-uniform base + 16 * lane) and the
// loader then converts a landed slot into the ring.  A staged window is 16-byte chunks: ys, yp, La
// ([kW][8] each), then the write positions pi-or-pinv[kW] and pi[kW]; spare lanes land past them.
constexpr int kDmaBytes = kLanes * 16;   // one DMA instruction

template <typename T>
constexpr int kStreamChunks = kTile * (int)sizeof(T) / 16;   // chunks of one [kW][8] stream
// write positions: a window's kW ints of each table from the 16-byte-aligned chunk at or below its
// first step (kW = 12: always aligned, 3 chunks; 15: start offset (15 t) mod 4, 5 chunks)
constexpr int kWpChunks = kW % 4 == 0 ? kW / 4 : (kW + 3 + 3) / 4;
constexpr int kWpInts = 4 * kWpChunks;   // staged ints per table
static_assert(kW % 4 == 0 || kWpInts >= kW + 3, "a window's write positions lie within its staged chunks");
// Lane-aligned staging (round 4): each stream occupies a power-of-two run of P lanes of a DMA (fp64:
// 64, one stream per DMA; fp32: 32, two per DMA), so a lane's stream and chunk are a shift and a
// mask of its lane index -- no per-lane division by the chunk count in the loader's address math
// (it had been recomputed in every B-pass iteration).  The write-position chunks take the spare
// lanes: fp64 the P - nc lanes at the end of each stream run, fp32 the fourth run of 32.
template <typename T>
constexpr int kStreamLanes = kStreamChunks<T> > 32 ? 64 : 32;                // P
template <typename T>
constexpr int kStreamsPerDma = kLanes / kStreamLanes<T>;
static_assert(kStreamChunks<double> <= 64 && kStreamChunks<float> <= 32, "a stream fits its lane run");
template <typename T>
constexpr bool kWpInSpare = kStreamsPerDma<T> == 1;   // fp64: write positions in the stream runs' spare lanes
template <typename T>
constexpr int kWpPerRun = kStreamLanes<T> - kStreamChunks<T>;   // fp64: spare lanes per stream run
static_assert(!kWpInSpare<double> || 3 * kWpPerRun<double> >= 2 * kWpChunks, "the write positions fit the spare lanes");
static_assert(kStreamsPerDma<float> != 2 || 2 * kWpChunks <= 32, "the write positions fit the fourth lane run");
template <typename T>
constexpr int kTileDma = kWpInSpare<T> ? 3 : 2;   // DMA instructions per staged window
// lanes of the last DMA that carry a chunk (the slot ends there)
template <typename T>
constexpr int kLastDmaLanes = kWpInSpare<T> ? kLanes : 32 + 2 * kWpChunks;
template <typename T>
constexpr int kStageBytes = (kTileDma<T> - 1) * kDmaBytes + kLastDmaLanes<T> * 16;
// byte offset in a staging slot of stream s (0 ys, 1 yp, 2 La; element e at + e * sizeof(T)) ...
template <typename T>
constexpr int stage_stream_off(int s)
{
    return ((s / kStreamsPerDma<T>) * kLanes + (s % kStreamsPerDma<T>) * kStreamLanes<T>) * 16;
}
// ... and of write-position int n (n < kWpInts: pi-or-pinv from the window's aligned chunk, then pi)
template <typename T>
__device__ __forceinline__ int stage_wp_off(int n)
{
    if constexpr (kWpInSpare<T>) {
        constexpr unsigned per = 4 * kWpPerRun<T>;   // ints per stream run's spare lanes
        return (int)(((unsigned)n / per) * kDmaBytes + kStreamChunks<T> * 16 + ((unsigned)n % per) * 4);
    } else {
        return kDmaBytes + 32 * 16 + n * 4;
    }
}
template <typename T>
constexpr int kTmStageBytes = kStreamChunks<T> * 16;
static_assert(3 * kTmStageBytes<double> <= kStageBytes<double> && 3 * kTmStageBytes<float> <= kStageBytes<float>,
              "Max-Log-MAP's three tempmax stagings fit staging slot 3");
static_assert(kStageBytes<double> % 16 == 0 && kStageBytes<float> % 16 == 0, "16-byte staging slots");

template <typename T>
struct Smem {
    T lut[kLutElems<T>];   // max* table: [bucket][thr | v][kLutCols columns] (see lut_origin)
#if (TD_DIAG & 16) != 0
    // timing-only build (kDiagOcc3Alias, results WRONG): the beta rows and the tile ring alias the
    // alpha ring, so an fp64 workgroup fits three per CU (52.7 KB) with every DMA, store and
    // instruction of the product kept -- the upper bound of a three-per-CU fp64 kernel.
    // The write positions (Wp) and the staging slots stay apart, so every global store stays in range.
    union {
        alignas(16) T Av[kAvSlots][kW][kLanes];
        struct {
            alignas(16) T Bv[2][kW][kLanes];
            T G[3][kW][kCw][4];
        };
    };
    alignas(8) int Wp[3][kW][2];
#else
    T G[3][kW][kCw][4];        // (P, Q, ys, La) per step and codeword, ring by window index mod 3
    alignas(8) int Wp[3][kW][2];   // extrinsic / decision write positions (pi or pinv, pi) per step, same ring
    alignas(16) T Av[kAvSlots][kW][kLanes];   // [window mod 4] alpha[.][i] by 8c + state (fold input, DMA from HBM)
    alignas(16) T Bv[2][kW][kLanes];       // [window parity] beta[.][i+1] by 8c + state (fold input)
#endif
    alignas(16) T tm[2][kW][kCw];          // [window parity] tempmax[i+1] per step and codeword (beta input)
    // loader: staged window inputs, slots 0-2 (window t in slot t % 3); Max-Log-MAP keeps its three
    // staged tempmax windows in slot 3
    alignas(16) unsigned char stage[4][kStageBytes<T>];
};

// Fold-input rows (Av, Bv): a (row, codeword) block holds the 8 states, 64 B in fp64 (4 chunks of
// 16 B), 32 B in fp32 (2 chunks).  A fold lane reads its whole block one 16-B chunk per
// ds_read_b128; with the blocks unrotated, the 16 lanes of a read group hit only 4 (fp64) or 8
// (fp32) distinct bank slots, a 4- or 2-way conflict.  Chunk p of the block in row r is stored at
// chunk (p + r) mod (chunks per block): the lane of row r then reads chunk p at slot
// 4c + ((p + r) & 3) (fp64), and the read groups of ds_read_b128 ({0-3,12-15,20-27}, ...) pair
// every codeword c with four different rows -- conflict-free.  The alpha copy pre-rotates its
// per-lane source addresses (the DMA's LDS side stays linear); beta publishes to rotated offsets.
// A/B on one box: fp64 log-MAP 1180 -> 1211 Mbit/s, fp64 max-log 1900 -> 1928; fp32 lost 2 %
// (1403 -> 1378, 2389 -> 2344), so fp32 keeps plain blocks.
template <typename T>
constexpr bool kFoldSwz = sizeof(T) == 8;
template <typename T>
constexpr int kBlkChunks = 8 * (int)sizeof(T) / 16;   // 16-B chunks per (row, codeword) block
// element offset of state s (0..7) inside the block of row r
template <typename T>
__device__ __forceinline__ int blk_off(int s, int r)
{
    if (!kFoldSwz<T>) return s;
    constexpr int E = 16 / (int)sizeof(T);   // states per chunk
    return (((s / E) + r) & (kBlkChunks<T> - 1)) * E + (s & (E - 1));
}
// the 8 states of the block at blk (row r) in state order: one 16-B read per chunk
template <typename T>
__device__ __forceinline__ void load_block(const T* blk, int r, T (&v)[8])
{
    constexpr int E = 16 / (int)sizeof(T);
    using V = typename std::conditional<sizeof(T) == 8, double2, float4>::type;
    if constexpr (kFoldSwz<T>) {
#pragma unroll
        for (int p = 0; p < kBlkChunks<T>; ++p) {
            const V x = *reinterpret_cast<const V*>(blk + ((p + r) & (kBlkChunks<T> - 1)) * E);
            __builtin_memcpy(&v[p * E], &x, 16);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = blk[j];
    }
}
// Rotation of alpha block (row r, codeword c).  Log-MAP: r (rows are the fold lanes' steps k).
// Max-Log-MAP rows are checkpoints, r = k / 3, so the read groups hold up to three lanes of one
// row; rotating by r + 2 (c >> 2) keeps their blocks' slots apart as well (+0.6 %, config 3).
template <int ALGO>
__device__ __forceinline__ int av_rot(int r, int c)
{
    return !kCkAll<ALGO> ? r + 2 * (c >> 2) : r;
}
// row offset 8c + s (st_off) -> rotated
template <typename T>
__device__ __forceinline__ int rot_off(int off, int r)
{
    if (!kFoldSwz<T>) return off;
    return (off & ~7) + blk_off<T>(off & 7, r);
}

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
    const T* la;      // a-priori la[g][i][c], i < la_cap, already in this decoder's order (always valid memory)
    int la_cap;       // rows of the la array
    int la_len;       // steps with a non-zero a-priori (0 = none: the first SISO of the first iteration)
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
    T* sys2_out;      // first SISO only (sys2_in_turbo): sys2[g][i][c] = sys[g][pi[i]][c], i < K
};

struct Geom {
    int K, L, nT, B, g, G;
    const int* pi;     // QPP pi[i]
    const int* pinv;   // its inverse
};

__device__ __forceinline__ int window_len(const Geom& gm, int t) { return min(kW, gm.L - t * kW); }

// channel values and a-priori of tile element e = k*8 + c of window t.  Every read is sequential:
// the interleaver permutations are applied when the extrinsic is WRITTEN (fold), so no load
// address depends on another load.  Prefetch loads are unconditional (rows clamped into range)
// and their values are masked only where they are consumed: a load under a lane-dependent branch
// makes the compiler drain the whole vector-memory queue at the join.
template <typename T>
__device__ __forceinline__ void load_elem(const SisoSrc<T>& src, const Geom& gm, int t, int e, T& ys, T& yp, T& la,
                                          bool want_yp)
{
    const int k = e >> 3, c = e & 7;
    const int i = min(t * kW + k, gm.L - 1);
    const size_t off = ((size_t)gm.g * gm.L + i) * kCw + c;
    ys = src.sys[off];
    yp = want_yp ? src.par[off] : (T)0;
    la = src.la[((size_t)gm.g * src.la_cap + min(i, src.la_cap - 1)) * kCw + c];   // masked at use (la_at)
}

// a-priori of step i as the reference sees it: zero for the tail steps (:1224-1227, 1245-1248)
template <typename T>
__device__ __forceinline__ T la_at(const SisoSrc<T>& src, int i, T raw)
{
    return i < src.la_len ? raw : (T)0;
}

// ---- loader helpers
template <int N>
__device__ __forceinline__ void vm_wait()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <typename V>
__device__ __forceinline__ void touch(V& v)
{
    asm volatile("" : "+v"(v));
}
// fire-and-forget store pinned in program order against the wave's other memory operations (the
// scheduler otherwise hoists it onto the recursion's critical path)
__device__ __forceinline__ void gstore(double* p, double v)
{
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void gstore(float* p, float v)
{
    asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
}

// the same with a wave-uniform base in SGPRs, a per-lane 32-bit byte offset and an immediate (the
// scheduled alpha windows: no per-step 64-bit address arithmetic).  The fp64 stores carry nt (v29:
// with the alpha copy at sc0 sc1 nt, 16.84 / 16.87 / 17.01 ms without, 16.72 / 16.73 / 16.81 with; one
// box, 3 rounds); the fp32 stores are plain (never measured with nt).
template <int IMM>
__device__ __forceinline__ void gstore_s(double* base, unsigned voff, double v)
{
    asm volatile("global_store_dwordx2 %0, %1, %2 offset:%3 nt" ::"v"(voff), "v"(v), "s"(base), "n"(IMM) : "memory");
}
template <int IMM>
__device__ __forceinline__ void gstore_s(float* base, unsigned voff, float v)
{
    asm volatile("global_store_dword %0, %1, %2 offset:%3" ::"v"(voff), "v"(v), "s"(base), "n"(IMM) : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p)
{
    return (unsigned)(size_t)(__attribute__((address_space(3))) const char*)(reinterpret_cast<const char*>(p));
}
// One 16-byte chunk per lane, HBM -> LDS at lds + 16 * lane.  Issued through inline asm (M0 saved
// and restored around it): with the builtin the compiler guards every later LDS access of this
// wave with vmcnt(0), as it cannot tell the DMA's LDS target from the other LDS arrays, which would
// serialise the loader on each copy.  The loader waits for completion with vm_wait<N>() before the
// barrier that publishes the slot (or before reading the slot itself).
__device__ __forceinline__ void dma16(unsigned lds, const void* src)
{
    unsigned save;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(save)
                 : "s"(lds), "v"(src)
                 : "memory");
}

// One 4-byte element per lane, HBM -> LDS at lds + 4 * lane (as dma16)
__device__ __forceinline__ void dma4(unsigned lds, const void* src)
{
    unsigned save;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(save)
                 : "s"(lds), "v"(src)
                 : "memory");
}

// dma16 with sc0 sc1 nt on the load: the alpha copies, whose lines are read once -- not keeping them
// in L2 / MALL leaves those to the other streams.  Measured (config 2, one box, 2 rounds): nt 16.95 /
// 16.91 ms, sc0 sc1 nt 16.94 / 16.88, sc1 17.15 / 17.22, against 17.14 / 17.21 without.  The same bits
// on the tile stagings (read twice) measured level or slower, so those stay plain.
__device__ __forceinline__ void dma16_stream(unsigned lds, const void* src)
{
    unsigned save;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off sc0 sc1 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(save) : "s"(lds), "v"(src) : "memory");
}

// Stage window t (rows clamped into range, so the count of DMA instructions never varies; values
// are masked where they are converted).  Every read is sequential: the interleaver permutations
// are applied when the extrinsic is WRITTEN (fold), so no load address depends on another load.
// The write-position chunks read up to kMemory + kWpInts - 1 ints past K - 1: the permutation tables
// carry kPermPad spare ints.
template <typename T>
__device__ __forceinline__ void tile_dma(Smem<T>& sm, int slot, const SisoSrc<T>& src, const SisoDst<T>& dst,
                                         const Geom& gm, int t, int lane)
{
    constexpr int E = 16 / (int)sizeof(T);   // elements per chunk (a chunk never crosses a step row)
    constexpr int nc = kStreamChunks<T>, P = kStreamLanes<T>;
    const int* pperm = dst.ext_mode == 3 ? gm.pinv : gm.pi;
    const unsigned base = lds_addr(&sm.stage[slot][0]);
    const int tc = max(t, 0);
    const int u = lane & (P - 1);            // chunk within the lane's stream run
#pragma unroll
    for (int q = 0; q < kTileDma<T>; ++q) {
        const int sg = q * kStreamsPerDma<T> + lane / P;   // the lane's run: 0 ys, 1 yp, 2 La, 3 (fp32) positions
        const int s = min(sg, 2);
        const int e0 = min(u, nc - 1) * E;
        const int i = min(tc * kW + (e0 >> 3), gm.L - 1);
        // base of stream s by arithmetic (a select chain over the three pointers becomes a
        // runtime-indexed private array, i.e. scratch)
        const size_t a0 = (size_t)src.sys, a1 = (size_t)src.par, a2 = (size_t)src.la;
        const size_t sb = a0 + (size_t)(s == 1) * (a1 - a0) + (size_t)(s == 2) * (a2 - a0);
        const size_t row = s == 2 ? (size_t)gm.g * src.la_cap + min(i, src.la_cap - 1) : (size_t)gm.g * gm.L + i;
        const char* ps = reinterpret_cast<const char*>(sb + (row * kCw + (e0 & 7)) * sizeof(T));
        // write-position chunk r (r < kWpChunks pi-or-pinv, else pi) from the aligned chunk at or below
        // the window's first step: fp64 in the spare lanes u >= nc of each run, fp32 in run 3
        const int rr = kWpInSpare<T> ? sg * kWpPerRun<T> + (u - nc) : u;
        const int r = min(max(rr, 0), 2 * kWpChunks - 1);
        const int* pb = r < kWpChunks ? pperm : gm.pi;
        const char* pw = reinterpret_cast<const char*>(pb + ((tc * kW) & ~3) + (r % kWpChunks) * 4);
        const bool stream = sg < 3 && u < nc;
        const bool wp = kWpInSpare<T> ? (u >= nc && rr < 2 * kWpChunks) : (sg == 3 && u < 2 * kWpChunks);
        if ((q + 1 < kTileDma<T> && kWpInSpare<T>) || stream || wp)   // the lanes with a chunk only
            dma16(base + q * kDmaBytes, stream ? ps : pw);
    }
}

// tempmax of window t ([kW][8], rows clamped) -> staging slot; one DMA instruction
template <typename T>
__device__ __forceinline__ void tm_dma(Smem<T>& sm, int slot, const T* tmstore, const Geom& gm, int t, int lane)
{
    constexpr int E = 16 / (int)sizeof(T);
    const int e0 = min(lane, kStreamChunks<T> - 1) * E;
    const int i = min(max(t * kW + (e0 >> 3), 0), gm.L - 1);
    if (lane < kStreamChunks<T>)   // the lanes with a chunk only (kTmStageBytes)
        dma16(lds_addr(&sm.stage[3][slot * kTmStageBytes<T>]), tmstore + ((size_t)gm.g * gm.L + i) * kCw + (e0 & 7));
}

// staged tempmax of window t -> its LDS slot (beta input; Max-Log-MAP's B-pass loader).  Batched
// reads (TD_TM_CONVERT_BATCH, fp64): config 3 2380-2389 -> 2399-2404 Mbit/s (+0.8 %, 3 rounds); fp32
// Max-Log-MAP lost 1.3 % with it and keeps the masked form (profiles/r06/ab_maxlog_tm_convert.txt)
#ifndef TD_TM_CONVERT_BATCH
#define TD_TM_CONVERT_BATCH 1
#endif
template <typename T>
__device__ __forceinline__ void tm_convert(Smem<T>& sm, int slot, int t, int lane)
{
    const T* sv = reinterpret_cast<const T*>(&sm.stage[3][slot * kTmStageBytes<T>]);
    T* d = &sm.tm[t & 1][0][0];
    if constexpr (TD_TM_CONVERT_BATCH != 0 && kW == 15 && sizeof(T) == 8) {
        // both reads before the first write and no lane masked (as tile_convert): lanes past the window
        // repeat its last element, the same value to the same address.  (The 12-step build is left as
        // it was: with this form its TU hits an instruction-selection error in the compiler.)
        const int e0 = lane, e1 = min(lane + kLanes, kTile - 1);
        const T v0 = sv[e0], v1 = sv[e1];
        d[e0] = v0;
        d[e1] = v1;
    } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = lane + kLanes * q;
            if (e < kTile) d[e] = sv[e];
        }
    }
}

// (P, Q) of the four branch metrics (see "gamma"), ys and La for the extrinsic, and the write
// positions of staged window t, into the LDS ring slot of window t
template <typename T>
__device__ __forceinline__ void tile_convert(Smem<T>& sm, int slot, const SisoSrc<T>& src, int t, int lane)
{
    // Every LDS read is issued before the first write, and no lane is masked: the compiler cannot tell
    // the staging slot from the rings, so a write between two reads made it wait for the write, and a
    // lane-masked write put a branch around it -- written per pass and per write position, the
    // conversion was six serial LDS round trips a window (87 cycles a step of the loader's 182 at
    // B = 8, round 4 stamps).  Lanes past the window (second pass) and past its steps (positions)
    // repeat the last item: the same values to the same address.
    const unsigned char* sb = &sm.stage[slot][0];
    const T* sy = reinterpret_cast<const T*>(sb + stage_stream_off<T>(0));
    const T* sp = reinterpret_cast<const T*>(sb + stage_stream_off<T>(1));
    const T* sl = reinterpret_cast<const T*>(sb + stage_stream_off<T>(2));
    const int wo = (t * kW) & 3;   // the window's first position within its aligned chunk
    const int e[2] = {lane, min(lane + kLanes, kTile - 1)};
    const int kp = min(lane, kW - 1);   // this lane's step for the write positions
    T ys[2], yp[2], lr[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        ys[q] = sy[e[q]];
        yp[q] = sp[e[q]];
        lr[q] = sl[e[q]];
    }
    const int w0 = *reinterpret_cast<const int*>(sb + stage_wp_off<T>(wo + kp));
    const int w1 = *reinterpret_cast<const int*>(sb + stage_wp_off<T>(kWpInts + wo + kp));
    T* g = &sm.G[t % 3][0][0][0];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const T la = la_at(src, t * kW + (e[q] >> 3), lr[q]);
        const T hla = la / (T)2;
        g[4 * e[q]] = (ys[q] + yp[q]) + hla;
        g[4 * e[q] + 1] = (ys[q] - yp[q]) + hla;
        g[4 * e[q] + 2] = ys[q];
        g[4 * e[q] + 3] = la;
    }
    // one entry per step (every codeword has the same positions), both tables as one 8-byte write
    *reinterpret_cast<int2*>(&sm.Wp[t % 3][kp][0]) = make_int2(w0, w1);
}
static_assert(kTile <= 2 * kLanes, "tile_convert covers a window in two passes");

// the last window starts at most at step L-1 = K+kMemory-1 and stages kW write positions from there
static_assert(kMemory + kWpInts - 1 <= kPermPad, "write-position chunks stay within the padded tables");

// ---- alpha of a window, HBM scratch -> LDS (wave F0, B pass).
// Scratch layout: alpha by 8c + state, group-major [G][L][64] (td_kernels.h astore_elems), tempmax
// [g][L][8].
// alpha of window t: HBM scratch -> LDS slot t % 4 directly (global_load_lds_dwordx4, no
// registers): the window's kW rows are one contiguous block on both sides.  Completion is tracked
// by vmcnt; the loader waits for it before the barrier that publishes the slot.
// Max-Log-MAP stores alpha only at the steps of phase 0 (kCkPh) and the folds recompute the steps in
// between from the last stored one (alpha_recompute): less alpha traffic, which otherwise bounds its
// forward pass (HBM writes).  The copy gathers the window's stored rows into consecutive LDS rows.
// element offset of row 0 of window t of group g in the alpha scratch
__device__ __forceinline__ size_t astore_window_off(int g, int t, int L)
{
    return (size_t)g * astore_group_elems(L) + (size_t)t * kW * 64;
}
template <int ALGO>
constexpr int kCkPerGroup = (kCkPh<ALGO> & 1) + ((kCkPh<ALGO> >> 1) & 1) + ((kCkPh<ALGO> >> 2) & 1);
template <int ALGO>
constexpr int kCkRows = kW / 3 * kCkPerGroup<ALGO>;   // stored rows per window
// window-relative step of stored row r, and the stored row at or before step k (with its step)
template <int ALGO>
__host__ __device__ constexpr int ck_step(int r)
{
    int m = r % kCkPerGroup<ALGO>, p = 0;
    for (; p < 3; ++p)
        if ((kCkPh<ALGO> >> p) & 1) {
            if (m == 0) break;
            --m;
        }
    return 3 * (r / kCkPerGroup<ALGO>) + p;
}
template <int ALGO>
__device__ __forceinline__ int ck_row_of(int k, int& ks)
{
    int p = k % 3;
    while (!((kCkPh<ALGO> >> p) & 1)) --p;   // phase 0 is always stored
    ks = k - (k % 3) + p;
    int m = 0;
    for (int q = 0; q < p; ++q) m += (kCkPh<ALGO> >> q) & 1;
    return (k / 3) * kCkPerGroup<ALGO> + m;
}
template <typename T, int ALGO>
constexpr int alpha_dma_count()
{
    return (kCkRows<ALGO> * kLanes * (int)sizeof(T) + kDmaBytes - 1) / kDmaBytes;
}
// bytes of a window's stored alpha rows (the last DMA covers the lanes below it only)
template <typename T, int ALGO>
constexpr int alpha_dma_bytes()
{
    return kCkRows<ALGO> * kLanes * (int)sizeof(T);
}
static_assert(kW % 3 == 0, "stored rows repeat every 3 window-relative steps");

// A 64-bit per-lane source pointer per DMA.  (The saddr form -- an SGPR base and 32-bit per-lane
// offsets -- saves 17 VGPRs but measured 0.9 % slower, round 3.)  LDS row r holds the window's step r
// (max-log: ck_step(r)); chunk pc of codeword block cb holds the block's chunk (pc - av_rot) mod
// kBlkChunks (blk_off).
template <typename T, int ALGO>
__device__ __forceinline__ void alpha_dma(Smem<T>& sm, const T* astore, const Geom& gm, int t, int lane)
{
    const int slot = ((t % kAvSlots) + kAvSlots) % kAvSlots;
    const int tc = max(t, 0);
    const char* src = reinterpret_cast<const char*>(astore + astore_window_off(gm.g, tc, gm.L));
    const unsigned lds = lds_addr(&sm.Av[slot][0][0]);
    constexpr int n = alpha_dma_count<T, ALGO>();
    constexpr int row_bytes = kLanes * (int)sizeof(T);   // one step of the window
#pragma unroll
    for (int q = 0; q < n; ++q) {
        const int b = q * kDmaBytes + lane * 16;
        int off = ck_step<ALGO>(b / row_bytes) * row_bytes + b % row_bytes;
        if constexpr (kFoldSwz<T>) {
            const int r = b / row_bytes, w = b % row_bytes;
            constexpr int blk = 8 * (int)sizeof(T);
            const int pc = ((w % blk) / 16 - av_rot<ALGO>(r, w / blk)) & (kBlkChunks<T> - 1);
            off = ck_step<ALGO>(r) * row_bytes + (w / blk) * blk + pc * 16;
        }
        if (q + 1 < n || b < alpha_dma_bytes<T, ALGO>()) dma16_stream(lds + q * kDmaBytes, src + off);
    }
}

// Log-MAP: the first DMA of alpha_dma for window t alone (its first kDmaBytes / (64 sizeof(T)) rows):
// row 0 of the window after the last, i.e. alpha_raw[.][L] when the last window is full (L = 0 mod
// kW), for tm_from_alpha of the last window.  One DMA instruction.
template <typename T>
__device__ __forceinline__ void alpha_dma_head(Smem<T>& sm, const T* astore, const Geom& gm, int t, int lane)
{
    const int slot = t % kAvSlots;
    const char* src = reinterpret_cast<const char*>(astore + astore_window_off(gm.g, t, gm.L));
    constexpr int row_bytes = kLanes * (int)sizeof(T);
    const int b = lane * 16;
    int off = b;
    if constexpr (kFoldSwz<T>) {   // the same chunk placement as alpha_dma (the max reads a block in any order)
        const int r = b / row_bytes, w = b % row_bytes;
        constexpr int blk = 8 * (int)sizeof(T);
        const int pc = ((w % blk) / 16 - av_rot<0>(r, w / blk)) & (kBlkChunks<T> - 1);
        off = r * row_bytes + (w / blk) * blk + pc * 16;
    }
    dma16_stream(lds_addr(&sm.Av[slot][0][0]), src + off);
}

// max of the 8 states of one (row, codeword) block of the Av / Bv rings, read in any chunk order
template <typename T>
__device__ __forceinline__ T block_max(const T* blk)
{
    constexpr int E = 16 / (int)sizeof(T);
    using V = typename std::conditional<sizeof(T) == 8, double2, float4>::type;
    T v[8];
#pragma unroll
    for (int p = 0; p < kBlkChunks<T>; ++p) {
        const V x = *reinterpret_cast<const V*>(blk + p * E);
        __builtin_memcpy(&v[p * E], &x, 16);
    }
    return vmax(vmax(vmax(v[0], v[1]), vmax(v[2], v[3])), vmax(vmax(v[4], v[5]), vmax(v[6], v[7])));
}

// Log-MAP, loader, B pass: beta's input tempmax[i+1] (:1019) of window t, for the window's steps
// i = t kW + k: the reference's tempmax[i+1] = max_j alpha_raw[j][i+1] (:986-993, exact in any
// order) over the alpha_raw rows the loader copied -- rows k+1 < kW from window t's Av slot, row kW
// (= row 0 of window t+1) from the next window's slot (the last window: alpha_raw[.][L], row L of the
// scratch, copied with window t or by alpha_dma_head).  Replaces the tempmax scratch stream.
template <typename T>
__device__ __forceinline__ void tm_from_alpha(Smem<T>& sm, int t, int lane)
{
    const T* a0 = &sm.Av[t % kAvSlots][0][0];
    const T* a1 = &sm.Av[(t + 1) % kAvSlots][0][0];
    T* d = &sm.tm[t & 1][0][0];
    T m[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {   // lanes past the window (second pass) repeat the last item
        const int e = min(lane + kLanes * q, kTile - 1);
        const int k = e >> 3, c = e & 7;
        m[q] = block_max<T>((k + 1 < kW ? a0 + (k + 1) * kLanes : a1) + c * 8);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) d[min(lane + kLanes * q, kTile - 1)] = m[q];
}

// Log-MAP folds: alpha[.][i] = alpha_raw[.][i] - tempmax[i] (:995-1000), the alpha wave's own
// subtraction of the same exact max
template <typename T>
__device__ __forceinline__ void normalise8(T (&a)[8])
{
    const T m = vmax(vmax(vmax(a[0], a[1]), vmax(a[2], a[3])), vmax(vmax(a[4], a[5]), vmax(a[6], a[7])));
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = a[j] - m;
}

// ---- recursion steps
// Operands of one step are read from LDS ahead of the step group that uses them.
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

// alpha step i -> i+1 with i mod 3 = PH (log_map.cpp:975-1001).  `a` carries the UNnormalised
// metric alpha_raw[.][i] of this lane's state; the step takes the reference's tempmax[i] =
// max_j alpha_raw[j][i] (three DPP levels, the first one the partner exchange of this phase),
// normalises (:986-1000) and returns alpha_raw[.][i+1].  fl(an - m) is exactly the partner's
// normalised alpha, so the exchange is taken on the raw metric, ahead of the max.
// Scratch (round 4): log-MAP streams alpha_RAW[.][i] (by state, to `pa`) and nothing else -- the B
// pass takes tempmax[i] = max_j alpha_raw[j][i] from the copied rows (beta: the loader's
// tm_from_alpha; the folds: normalise8), the same exact max and the same subtraction, so the values
// are bit-identical to streaming alpha[.][i] and tempmax; Max-Log-MAP, which keeps one row in three,
// streams the normalised checkpoint rows and tempmax[i] (to `ptm`).
// The table row read ahead of the max from the unnormalised difference, with an exact redo of the
// window on a bucket mismatch, is the kASpec path below (round 1's first form of it measured 1098 vs
// 1203 Mbit/s; round 4's, with the mismatch flag in a VGPR, +1.3 %: DESIGN.md 3.2).
template <typename T>
struct StepHalf {   // a recursion step split at its max* table read (see beta_issue)
    T xs, xp, d, thr, lo, hi;
};

template <typename T, int ALGO, int PH>
__device__ __forceinline__ StepHalf<T> alpha_issue(T a, const StepIn<T>& in, const T* lut, const LaneConst<T>& lc,
                                                   T* pa, T* ptm)
{
    T an;                                         // partner's alpha_raw
    const T m = alpha_tempmax<T, PH>(a, an);       // tempmax[i] (:986-993)
    const T alpha = a - m, ap = an - m;             // alpha[.][i] of this lane and of the partner
    StepHalf<T> h;
    h.xs = fma(lc.a_sg[PH], in.gs, alpha);   // gamma + alpha, predecessor in this lane
    h.xp = fma(lc.a_pg[PH], in.gp, ap);      // ... predecessor in the partner lane
    if constexpr (ALGO == 0) {
        h.d = h.xp - h.xs;
        const LutRow r = lut_row(h.d);
        lut_fields<T>(lut, r.o, h.thr, h.lo, h.hi);
    }
    if constexpr (ALGO == 0) {
        gstore(pa, a);   // in the table read's shadow
    } else {
        if ((kCkPh<ALGO> >> PH) & 1) gstore(pa, alpha);   // only the kept phases (kCkPh)
        gstore(ptm, m);
    }
    return h;
}

template <typename T, int ALGO>
__device__ __forceinline__ T step_done(const StepHalf<T>& h)
{
    if constexpr (ALGO == 1) return vmax(h.xs, h.xp);
    return vmax(h.xs, h.xp) + (fabs(h.d) >= h.thr ? h.hi : h.lo);   // = mstar(xs, xp)
}

template <typename T, int ALGO, int PH>
__device__ __forceinline__ T alpha_step(T a, const StepIn<T>& in, const T* lut, const LaneConst<T>& lc, T* pa, T* ptm)
{
    return step_done<T, ALGO>(alpha_issue<T, ALGO, PH>(a, in, lut, lc, pa, ptm));
}

// beta step i+1 -> i with i mod 3 = PH (log_map.cpp:1004-1021).  beta[.][i+1] (the incoming
// metric) is published (by state) for the LLR terms of step i by the caller: an LDS store on the
// chain costs ~45 cycles a step in isolation (ubench_beta), so a full window stores its kW values
// behind the steps' table reads (BetaSched) or at its end (beta_window).
template <typename T, int ALGO, int PH>
__device__ __forceinline__ T beta_step(T beta, const StepIn<T>& in, const T* lut, const LaneConst<T>& lc)
{
    const T bp = dpp<PhaseDpp<PH>::ctrl>(beta);
    const T b = mstar<T, ALGO>(fma(lc.b_sg[PH], in.gs, beta), fma_pm(lc.b_pg[PH], in.gp, bp), lut);
    return b - in.tm;
}

// The same step split at its table read, so that other LDS reads can be issued in its shadow:
// beta_issue returns once the max* row read is in flight; step_done(h) - tempmax completes it.
template <typename T, int ALGO, int PH>
__device__ __forceinline__ StepHalf<T> beta_issue(T beta, const StepIn<T>& in, const T* lut, const LaneConst<T>& lc)
{
    const T bp = dpp<PhaseDpp<PH>::ctrl>(beta);
    StepHalf<T> h;
    h.xs = fma(lc.b_sg[PH], in.gs, beta);
    h.xp = fma_pm(lc.b_pg[PH], in.gp, bp);
    if constexpr (ALGO == 0) {
        h.d = h.xp - h.xs;
        const LutRow r = lut_row(h.d);
        lut_fields<T>(lut, r.o, h.thr, h.lo, h.hi);
    }
    return h;
}

template <typename T, int ALGO>
__device__ __forceinline__ T beta_step_rt(int ph, T beta, const Smem<T>& sm, const T* lut, int tb, int k, int c,
                                          const LaneConst<T>& lc, const T* tmw)
{
    if (ph == 0) return beta_step<T, ALGO, 0>(beta, beta_in<T, 0>(sm, tb, k, c, lc, tmw), lut, lc);
    if (ph == 1) return beta_step<T, ALGO, 1>(beta, beta_in<T, 1>(sm, tb, k, c, lc, tmw), lut, lc);
    return beta_step<T, ALGO, 2>(beta, beta_in<T, 2>(sm, tb, k, c, lc, tmw), lut, lc);
}

// Diagnostic build (TD_STAMPS) only: shader-clock reads around the 12 chain steps of a scheduled
// window, summed into the wave's stamp slot 4 (the recursion's chain alone, without the window's
// operand prologue, publish and barrier).
#ifdef TD_STAMPS
#define TD_CHAIN_T0(v)                              \
    __builtin_amdgcn_sched_barrier(0);              \
    const unsigned long long v = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0)
#define TD_CHAIN_ACC(v)                                                       \
    do {                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                    \
        if (chain_st) *chain_st += __builtin_amdgcn_s_memtime() - (v);        \
        __builtin_amdgcn_sched_barrier(0);                                    \
    } while (0)
#else
#define TD_CHAIN_T0(v)
#define TD_CHAIN_ACC(v)
#endif

// ------------------------------------------------------------------ scheduled windows (log-MAP)
// A full window of either recursion as 12 unrolled steps with one fixed schedule per step:
//   [chain up to the max* row address] [the row's three reads] [operand reads of a step two
//   away] [HBM stores] [select + add]
// as separate scheduling regions.  LDS returns a wave's reads in order, so any read issued
// before the row read delays the chain by its LDS time.  Left to itself, the compiler sank the
// next steps' operand reads in front of the row read, or split the row (ds_read2, operand reads,
// then the row's third read), in every step group.  Reads issued right behind the row read
// complete in its shadow, long before the next step's row read.

// max(xs, xp) + (|d| >= thr ? hi : lo), the max* of a scheduled step.  (Forming both candidate sums
// and selecting measured 0.5 % slower: one dependent op less on the chain, one VALU more.)
template <typename T>
__device__ __forceinline__ T sched_finish(T xs, T xp, T d, T thr, T lo, T hi)
{
    return vmax(xs, xp) + (fabs(d) >= thr ? hi : lo);
}

template <typename T, int K>
struct AlphaSched {
    // alpha step K (phase K mod 3) of a full log-MAP window: a = alpha_raw[.][i] in, alpha_raw[.][i+1]
    // out; op[K % 3] holds this step's operands, op[(K + 2) % 3] receives step K+2's
    static __device__ __forceinline__ void run(T& a, StepIn<T> (&op)[3], const Smem<T>& sm, int tb, const T* lut,
                                               int c, const LaneConst<T>& lc, T* ga)
    {
        constexpr int PH = K % 3;
        const StepIn<T> in = op[K % 3];
        T an;                                         // partner's alpha_raw
        const T m = alpha_tempmax<T, PH>(a, an);       // tempmax[i] (:986-993)
        const T alpha = a - m, ap = an - m;                   // :995-1000
        const T xs = fma(lc.a_sg[PH], in.gs, alpha);
        const T xp = fma(lc.a_pg[PH], in.gp, ap);
        const T d = xp - xs;
        const LutRow r = lut_row(d);
        __builtin_amdgcn_sched_barrier(0);
        T thr, lo, hi;
        lut_fields<T>(lut, r.o, thr, lo, hi);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K + 2 < kW) op[(K + 2) % 3] = alpha_in<T, (K + 2) % 3>(sm, tb, K + 2, c, lc);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!kDiag<kDiagNoAStore>) gstore(ga + K * kLanes + lc.st_off[PH], a);   // alpha_raw[.][i]
        __builtin_amdgcn_sched_barrier(0);
        a = sched_finish(xs, xp, d, thr, lo, hi);
        AlphaSched<T, K + 1>::run(a, op, sm, tb, lut, c, lc, ga);
    }
};
template <typename T>
struct AlphaSched<T, kW> {
    static __device__ __forceinline__ void run(T&, StepIn<T> (&)[3], const Smem<T>&, int, const T*, int,
                                               const LaneConst<T>&, T*)
    {
    }
};

// AlphaSched for a full window t >= 1 with its scratch stores addressed off wave-uniform bases:
// sa = alpha rows of the window + kArow0 rows, stm = tempmax rows of the window; va[PH] = this
// lane's byte offset of its state in a row of phase PH.  Step K stores alpha at sa + va + (K -
// kArow0) rows.  Log-MAP and fp64 Max-Log-MAP take this path (fp64 Max-Log-MAP 1930 -> 2050 Mbit/s
// with it; fp32 Max-Log-MAP lost 23 %, so it keeps alpha_window's pinned step groups).
template <typename T, int ALGO>
constexpr bool kAlphaSchedS = ALGO == 0 || sizeof(T) == 8;
// The 8 lanes of a codeword hold the same tempmax, so instead of a store per step each lane keeps
// the tempmax of one step (lane slot l: steps l and 8 + tm2_slot(l) of the window) and the window
// writes them with two stores (steps 0-7, then 8..kW-1; lanes whose slots map to one step write the
// same value twice in the second): 2 scratch stores a window instead of kW.
static_assert(kW > 8 && kW <= 16, "the tempmax batches cover a window of 8 + (kW - 8) steps");
// the second batch's step (minus 8) kept by lane slot l
__host__ __device__ constexpr int tm2_slot(int l) { return kW - 8 == 4 ? (l & 3) : (l < kW - 8 ? l : kW - 9); }
template <typename T>
struct TmBatch {
    T buf;
    int slot;          // lane & 7
    unsigned v1, v2;   // byte offsets of this lane's entry in the first / second batch
};
template <typename T, int K>
__device__ __forceinline__ void tm_keep(TmBatch<T>& tbh, T m, T* stm)
{
    if constexpr (K < 8)
        tbh.buf = tbh.slot == K ? m : tbh.buf;
    else
        tbh.buf = tm2_slot(tbh.slot) == K - 8 ? m : tbh.buf;
    if constexpr (K == 7) gstore_s<-kCw * (int)sizeof(T)>(stm, tbh.v1, tbh.buf);           // steps 0-7 at i - 1
    if constexpr (K == kW - 1) gstore_s<7 * kCw * (int)sizeof(T)>(stm, tbh.v2, tbh.buf);   // steps 8..kW-1
}

// alpha row K of a full window: wave-uniform base sa (row kArow0 of the window) in SGPRs, per-lane
// byte offset voff, the row an immediate offset (no per-step address arithmetic)
template <typename T, int K>
__device__ __forceinline__ void astore_row(T* sa, unsigned voff, T v)
{
    if constexpr (!kDiag<kDiagNoAStore>) gstore_s<(K - kArow0) * kLanes * (int)sizeof(T)>(sa, voff, v);
}

// Log-MAP, speculative table row (kASpec): the step's max* row is read from the bucket of the
// UNnormalised difference fl(fl(g_p + an) - fl(g_s + a)), which is known before the tempmax tree,
// so the table read (60-70 cycles) overlaps the tree's three (DPP, max) levels and the exact
// difference's sub / fma / sub instead of following them.  The exact difference d is formed as
// before and only its bucket is compared with the speculated one (OR-ed into `miss`); the
// threshold compare, the select and the add use d itself, so a step whose buckets agree is
// bit-identical to the committed order.  A window with any mismatch in any lane is recomputed in
// the committed order from its first alpha (alpha_window), stores included, before the barrier:
// the two differences differ by roundings of the normalisation only, so a mismatch needs d within
// a few ulps of a bucket edge and the redo practically never runs (TD_ASPEC_REDO forces it on
// every window: that build must and does decode bit-identically).  One box, 3 interleaved rounds
// (profiles/r04/ab_v31_aspec.txt): config 2 1502 -> 1521 Mbit/s (+1.3 %), fp32 log-MAP +0.4 %, the
// 32768 shard level; the fp32 four-per-CU kernel of the 12-step TU lost 3.4 %, so it keeps the
// committed order.  (With the flag left to the compiler, and with SLP packing the two buckets into
// 16-bit pairs, the same speculation measured 1.2 % slower.)
#ifndef TD_ASPEC
#define TD_ASPEC (TD_KW == 15)
#endif
template <typename T, int ALGO>
constexpr bool kASpec = ALGO == 0 && TD_ASPEC != 0;

template <typename T, int ALGO, int K>
struct AlphaSchedS {
    static __device__ __forceinline__ void run(T& a, StepIn<T> (&op)[3], const Smem<T>& sm, int tb, const T* lut,
                                               int c, const LaneConst<T>& lc, T* sa, T* stm, const unsigned (&va)[3],
                                               TmBatch<T>& tbh, unsigned& miss)
    {
        constexpr int PH = K % 3;
        const StepIn<T> in = op[K % 3];
        if constexpr (kASpec<T, ALGO>) {
            const T an = dpp<PhaseDpp<PH>::ctrl>(a);   // partner's alpha_raw
            const T dr = fma_pm(lc.a_pg[PH], in.gp, an) - fma(lc.a_sg[PH], in.gs, a);
            const int qr = bucket_dev<T>(dr);
            __builtin_amdgcn_sched_barrier(0);
            T thr, lo, hi;
            lut_fields<T>(lut, qr * 2 * kLutCols<T>, thr, lo, hi);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (K + 2 < kW) op[(K + 2) % 3] = alpha_in<T, (K + 2) % 3>(sm, tb, K + 2, c, lc);
            __builtin_amdgcn_sched_barrier(0);
            astore_row<T, K>(sa, va[PH], a);   // alpha_raw[.][i]
            __builtin_amdgcn_sched_barrier(0);
            T m = vmax(a, an);                                   // tempmax[i] (:986-993), alpha_tempmax's tree
            m = vmax(m, dpp<PhaseDpp<(PH + 1) % 3>::ctrl>(m));
            m = vmax(m, dpp<PhaseDpp<(PH + 2) % 3>::ctrl>(m));
            const T alpha = a - m, ap = an - m;                  // :995-1000
            const T xs = fma(lc.a_sg[PH], in.gs, alpha);
            const T xp = fma(lc.a_pg[PH], in.gp, ap);
            const T d = xp - xs;
            // per step, in a VGPR (left to itself the compiler turns the flag into 15 compares and
            // SALU ORs of VCC at the window's end, on the chain's tail)
            unsigned x = (unsigned)bucket_dev<T>(d);
            asm("v_xor_b32 %1, %1, %2\n\tv_or_b32 %0, %0, %1" : "+v"(miss), "+v"(x) : "v"(qr));
            a = sched_finish(xs, xp, d, thr, lo, hi);
            AlphaSchedS<T, ALGO, K + 1>::run(a, op, sm, tb, lut, c, lc, sa, stm, va, tbh, miss);
            return;
        }
        T an;                                         // partner's alpha_raw
        const T m = alpha_tempmax<T, PH>(a, an);       // tempmax[i] (:986-993)
        const T alpha = a - m, ap = an - m;                   // :995-1000
        const T xs = fma(lc.a_sg[PH], in.gs, alpha);
        const T xp = fma(lc.a_pg[PH], in.gp, ap);
        if constexpr (ALGO == 0) {
            const T d = xp - xs;
            const LutRow r = lut_row(d);
            __builtin_amdgcn_sched_barrier(0);
            T thr, lo, hi;
        lut_fields<T>(lut, r.o, thr, lo, hi);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (K + 2 < kW) op[(K + 2) % 3] = alpha_in<T, (K + 2) % 3>(sm, tb, K + 2, c, lc);
            __builtin_amdgcn_sched_barrier(0);
            astore_row<T, K>(sa, va[PH], a);   // alpha_raw[.][i]; no tempmax (alpha_issue)
            __builtin_amdgcn_sched_barrier(0);
            a = sched_finish(xs, xp, d, thr, lo, hi);
        } else {
            // Max-Log-MAP: no table; alpha stored at the checkpoint phases only (kCkPhases)
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (K + 2 < kW) op[(K + 2) % 3] = alpha_in<T, (K + 2) % 3>(sm, tb, K + 2, c, lc);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((kCkPh<ALGO> >> PH) & 1) astore_row<T, K>(sa, va[PH], alpha);
            tm_keep<T, K>(tbh, m, stm);
            __builtin_amdgcn_sched_barrier(0);
            a = vmax(xs, xp);
        }
        AlphaSchedS<T, ALGO, K + 1>::run(a, op, sm, tb, lut, c, lc, sa, stm, va, tbh, miss);
    }
};
template <typename T, int ALGO>
struct AlphaSchedS<T, ALGO, kW> {
    static __device__ __forceinline__ void run(T&, StepIn<T> (&)[3], const Smem<T>&, int, const T*, int,
                                               const LaneConst<T>&, T*, T*, const unsigned (&)[3], TmBatch<T>&, unsigned&)
    {
    }
};
static_assert(kArow0 * kLanes * 8 <= 4096 && (kW - 1 - kArow0) * kLanes * 8 < 4096, "scheduled alpha store offsets fit the immediate");

// Each beta step writes its incoming beta[.][i+1] (the fold input of step i) into the window's Bv
// rows behind its own row read, instead of the kW writes (and their rotated addresses) after the
// window, which the chain waited for at the window's barrier.

template <typename T, int K>
struct BetaSched {
    // beta step K (phase K mod 3, steps run K = kW-1 .. 0): beta[.][i+1] in, beta[.][i] out;
    // bs[K] keeps the incoming beta for the window's publish; op[(K + 1) % 3] receives step K-2's
    static __device__ __forceinline__ void run(T& beta, StepIn<T> (&op)[3], T (&bs)[kW], const Smem<T>& sm, int tb,
                                               const T* lut, int c, const LaneConst<T>& lc, const T* tmw, T* Bvw)
    {
        constexpr int PH = K % 3;
        const StepIn<T> in = op[K % 3];
        bs[K] = beta;
        const T bp = dpp<PhaseDpp<PH>::ctrl>(beta);
        const T xs = fma(lc.b_sg[PH], in.gs, beta);
        const T xp = fma_pm(lc.b_pg[PH], in.gp, bp);
        const T d = xp - xs;
        const LutRow r = lut_row(d);
        __builtin_amdgcn_sched_barrier(0);
        T thr, lo, hi;
        lut_fields<T>(lut, r.o, thr, lo, hi);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (K >= 2) op[(K + 1) % 3] = beta_in<T, (K - 2) % 3>(sm, tb, K - 2, c, lc, tmw);
        __builtin_amdgcn_sched_barrier(0);
        Bvw[K * kLanes + rot_off<T>(lc.st_off[(K + 1) % 3], K)] = bs[K];
        __builtin_amdgcn_sched_barrier(0);
        beta = sched_finish(xs, xp, d, thr, lo, hi) - in.tm;   // :1012-1019
        BetaSched<T, K - 1>::run(beta, op, bs, sm, tb, lut, c, lc, tmw, Bvw);
    }
};
template <typename T>
struct BetaSched<T, -1> {
    static __device__ __forceinline__ void run(T&, StepIn<T> (&)[3], T (&)[kW], const Smem<T>&, int, const T*, int,
                                               const LaneConst<T>&, const T*, T*)
    {
    }
};

// alpha over the n steps of window t (window starts are = 0 mod 3); ga / gtm point at step t*kW.
// Step k stores tempmax[i] at scratch index i - 1 (the B pass reads tempmax[i+1] at index i); at
// t = 0 the first store (tempmax[0]) lands on index 0, which step 1 then overwrites.  The caller
// stores tempmax[L] after the last window.
template <typename T, int ALGO>
__device__ __forceinline__ T alpha_window(T a, int t, int n, const Smem<T>& sm, const T* lut, int c,
                                          const LaneConst<T>& lc, T* ga, T* gtm,
                                          unsigned long long* chain_st = nullptr)
{
    (void)chain_st;
    constexpr size_t arow = kLanes;   // rows of a window, arow elements apart
    const int tb = t % 3;
    if constexpr (ALGO == 0) {
        if (n == kW) {
            StepIn<T> op[3];
            op[0] = alpha_in<T, 0>(sm, tb, 0, c, lc);
            op[1] = alpha_in<T, 1>(sm, tb, 1, c, lc);
            TD_CHAIN_T0(c0);
            AlphaSched<T, 0>::run(a, op, sm, tb, lut, c, lc, ga);
            TD_CHAIN_ACC(c0);
            return a;
        }
    }
    T* pa0 = ga + lc.st_off[0];
    T* pa1 = ga + arow + lc.st_off[1];
    T* pa2 = ga + 2 * arow + lc.st_off[2];
    T* ptm = gtm + c - (t > 0 ? kCw : 0);
    int k = 0;
    StepIn<T> i0 = alpha_in<T, 0>(sm, tb, 0, c, lc);   // operands read one step group ahead
    StepIn<T> i1 = alpha_in<T, 1>(sm, tb, 1, c, lc);
    if constexpr (ALGO == 1) {
        // Max-Log-MAP: the next group's reads pinned right behind the group's first step
        // (1324 -> 1494 Mbit/s); with the table the same placement measured slower (alpha 237 -> 248
        // cycles a step), so log-MAP keeps the compiler's placement below.
        StepIn<T> i2 = alpha_in<T, 2>(sm, tb, 2, c, lc);
        for (; k + 3 <= n; k += 3) {
            const StepIn<T> c1 = i1, c2 = i2;
            const int kn = min(k + 3, kW - 3);
            const StepHalf<T> h = alpha_issue<T, ALGO, 0>(a, i0, lut, lc, pa0 + k * arow, ptm);
            __builtin_amdgcn_sched_barrier(0);
            i0 = alpha_in<T, 0>(sm, tb, kn, c, lc);
            i1 = alpha_in<T, 1>(sm, tb, kn + 1, c, lc);
            i2 = alpha_in<T, 2>(sm, tb, kn + 2, c, lc);
            __builtin_amdgcn_sched_barrier(0);
            a = step_done<T, ALGO>(h);
            a = alpha_step<T, ALGO, 1>(a, c1, lut, lc, pa1 + k * arow, gtm + c + k * kCw);
            a = alpha_step<T, ALGO, 2>(a, c2, lut, lc, pa2 + k * arow, gtm + c + (k + 1) * kCw);
            ptm = gtm + c + (k + 2) * kCw;
        }
    } else {
        for (; k + 3 <= n; k += 3) {
            const StepIn<T> c1 = alpha_in<T, 1>(sm, tb, k + 1, c, lc);
            const StepIn<T> c2 = alpha_in<T, 2>(sm, tb, k + 2, c, lc);
            a = alpha_step<T, ALGO, 0>(a, i0, lut, lc, pa0 + k * arow, ptm);
            i0 = alpha_in<T, 0>(sm, tb, min(k + 3, kW - 1), c, lc);
            a = alpha_step<T, ALGO, 1>(a, c1, lut, lc, pa1 + k * arow, gtm + c + k * kCw);
            a = alpha_step<T, ALGO, 2>(a, c2, lut, lc, pa2 + k * arow, gtm + c + (k + 1) * kCw);
            ptm = gtm + c + (k + 2) * kCw;
        }
        i1 = alpha_in<T, 1>(sm, tb, min(k + 1, kW - 1), c, lc);
    }
    if (k < n) {
        a = alpha_step<T, ALGO, 0>(a, i0, lut, lc, pa0 + k * arow, ptm);
        ptm = gtm + c + k * kCw;
    }
    if (k + 1 < n) {
        a = alpha_step<T, ALGO, 1>(a, i1, lut, lc, pa1 + k * arow, ptm);
    }
    return a;
}

// operand prefetch pinned behind a table read (A/B on one box, config 2: fp64 1192 -> 1207
// Mbit/s).  fp32 log-MAP lost with it before its table went to 32 columns (1461 -> 1436) and gains
// with it since (with beta at priority 2: 1414 -> 1443); fp32 Max-Log-MAP still loses (-0.4 %).
template <typename T, int ALGO>
constexpr bool kBetaPin = sizeof(T) == 8 || ALGO == 0;

// beta over the n steps of window t, downwards (full windows: static phases; else runtime).
// FULL = false keeps only the rolled runtime-phase loop (the last window in the dedicated loop of
// the B pass, so that the unrolled full-window code exists once in the kernel)
template <typename T, int ALGO, bool FULL = true>
__device__ __forceinline__ T beta_window(T beta, int t, int n, Smem<T>& sm, const T* lut, int c, const LaneConst<T>& lc,
                                         unsigned long long* chain_st = nullptr)
{
    (void)chain_st;
    const int tb = t % 3, xb = t & 1;
    T* Bvw = &sm.Bv[xb][0][0];
    const T* tmw = &sm.tm[xb][0][0];
    if constexpr (!FULL) {
        for (int k = n - 1; k >= 0; --k) {
            const int ph1 = (k + 1) % 3;   // constant indices only: a runtime index into lc moves it to scratch
            Bvw[k * kLanes + rot_off<T>(ph1 == 0 ? lc.st_off[0] : ph1 == 1 ? lc.st_off[1] : lc.st_off[2], k)] = beta;
            beta = beta_step_rt<T, ALGO>(k % 3, beta, sm, lut, tb, k, c, lc, tmw);
        }
        return beta;
    }
    if (ALGO == 0 && n == kW) {
        T bs[kW];   // beta[.][i+1] of step k (BetaSched publishes it behind the step's row read)
        StepIn<T> op[3];
        op[(kW - 1) % 3] = beta_in<T, (kW - 1) % 3>(sm, tb, kW - 1, c, lc, tmw);
        op[(kW - 2) % 3] = beta_in<T, (kW - 2) % 3>(sm, tb, kW - 2, c, lc, tmw);
        TD_CHAIN_T0(c0);
        BetaSched<T, kW - 1>::run(beta, op, bs, sm, tb, lut, c, lc, tmw, Bvw);
        TD_CHAIN_ACC(c0);
        return beta;
    }
    if (n == kW) {
        T bs[kW];   // beta[.][i+1] of step k, stored by lane after the window (an LDS store per step on
                    // the chain costs ~45 cycles a step in isolation, ubench_beta)
        auto put = [&](int k, T v) { bs[k] = v; };
        // operands read one step group ahead (the next group's inputs load under this group's chain)
        StepIn<T> b2 = beta_in<T, 2>(sm, tb, kW - 1, c, lc, tmw);
        StepIn<T> b1 = beta_in<T, 1>(sm, tb, kW - 2, c, lc, tmw);
        StepIn<T> b0 = beta_in<T, 0>(sm, tb, kW - 3, c, lc, tmw);
#pragma unroll
        for (int k = kW - 1; k >= 0; k -= 3) {   // phases 2, 1, 0 (kW = 0 mod 3)
            const int kn = k >= 3 ? k - 3 : k;
            put(k, beta);
            const StepHalf<T> h = beta_issue<T, ALGO, 2>(beta, b2, lut, lc);
            // the next group's operands, issued right behind this step's table read (kBetaPin)
            if (kBetaPin<T, ALGO>) __builtin_amdgcn_sched_barrier(0);
            const StepIn<T> n2 = beta_in<T, 2>(sm, tb, kn, c, lc, tmw);
            const StepIn<T> n1 = beta_in<T, 1>(sm, tb, kn - 1, c, lc, tmw);
            const StepIn<T> n0 = beta_in<T, 0>(sm, tb, kn - 2, c, lc, tmw);
            if (kBetaPin<T, ALGO>) __builtin_amdgcn_sched_barrier(0);
            beta = step_done<T, ALGO>(h) - b2.tm;   // :1019
            put(k - 1, beta);
            beta = beta_step<T, ALGO, 1>(beta, b1, lut, lc);
            put(k - 2, beta);
            beta = beta_step<T, ALGO, 0>(beta, b0, lut, lc);
            b2 = n2;
            b1 = n1;
            b0 = n0;
        }
#pragma unroll
        for (int k = 0; k < kW; ++k) Bvw[k * kLanes + rot_off<T>(lc.st_off[(k + 1) % 3], k)] = bs[k];
    } else {
        for (int k = n - 1; k >= 0; --k) {
            const int ph1 = (k + 1) % 3;   // constant indices only: a runtime index into lc moves it to scratch
            Bvw[k * kLanes + rot_off<T>(ph1 == 0 ? lc.st_off[0] : ph1 == 1 ? lc.st_off[1] : lc.st_off[2], k)] = beta;
            beta = beta_step_rt<T, ALGO>(k % 3, beta, sm, lut, tb, k, c, lc, tmw);
        }
    }
    return beta;
}

// beta_window's scheduled path for a full window whose ring slots the caller keeps as running
// counters (tb = t % 3, xb = t & 1): no window-length test, no modular arithmetic
template <typename T, int ALGO>
__device__ __forceinline__ T beta_window_full(T beta, int tb, int xb, Smem<T>& sm, const T* lut, int c,
                                              const LaneConst<T>& lc, unsigned long long* chain_st = nullptr)
{
    (void)chain_st;
    T* Bvw = &sm.Bv[xb][0][0];
    const T* tmw = &sm.tm[xb][0][0];
    T bs[kW];
    StepIn<T> op[3];
    op[(kW - 1) % 3] = beta_in<T, (kW - 1) % 3>(sm, tb, kW - 1, c, lc, tmw);
    op[(kW - 2) % 3] = beta_in<T, (kW - 2) % 3>(sm, tb, kW - 2, c, lc, tmw);
    TD_CHAIN_T0(c0);
    BetaSched<T, kW - 1>::run(beta, op, bs, sm, tb, lut, c, lc, tmw, Bvw);
    TD_CHAIN_ACC(c0);
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

// Alpha step in one lane, all 8 states (:975-1001): the alpha wave's arithmetic exactly -- each
// state's two candidates alpha[p] -+ (P|Q) (fma(+-1, G, alpha) there), their max* (symmetric: the
// table reads |d|, so the operands may come in either order; Max-Log-MAP: the max), the max over
// the states (tempmax, exact in any order) and the subtraction.
template <typename T, int ALGO>
__device__ __forceinline__ void alpha_recompute(T (&a)[8], T P, T Q, const T* lut)
{
    T n[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        n[j] = mstar<T, ALGO>(a[p0] - (kTrellisQ[p0] ? Q : P), a[p1] + (kTrellisQ[p1] ? Q : P), lut);
    }
    const T m = vmax(vmax(vmax(n[0], n[1]), vmax(n[2], n[3])), vmax(vmax(n[4], n[5]), vmax(n[6], n[7])));
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = n[j] - m;
}

// LLR fold + extrinsic + outputs of item e = k*8 + c of window t (:1024-1039, :1234-1264):
//   temp_u[j] = (gamma[p][i][u] + alpha[p][i]) + beta[j][i+1],  p = laststat[j][u],
//   LLR = E_seq(temp1) - E_seq(temp0)
// with gamma[p][.][u] = +-P or +-Q (see "gamma"; kTrellisQ) -- the same two roundings as the
// reference's (gamma + alpha) + beta.  Both folds run in the same lane (independent chains).
template <typename T, int ALGO>
__device__ __forceinline__ void fold_item(const Smem<T>& sm, const T* lut, int t, int e, const SisoDst<T>& dst,
                                          const Geom& gm)
{
    const int k = e >> 3, c = e & 7;
    const int i = t * kW + k;
    const T* g = &sm.G[t % 3][k][c][0];
    const T P = g[0], Q = g[1], ys = g[2], la = g[3];
    const int wperm = sm.Wp[t % 3][k][0], wbit = sm.Wp[t % 3][k][1];
    T a[8], b[8], t0[8], t1[8];
    const T* bv = &sm.Bv[t & 1][k][c * 8];
    load_block<T>(bv, k, b);
    if constexpr (!kFoldRows<ALGO>) {
        // alpha[.][i] from the last stored step ks <= k, recomputed through the steps in between
        // exactly as the alpha wave computed them (:975-1001)
        int ks;
        const int r = ck_row_of<ALGO>(k, ks);
        const T* av = &sm.Av[t % kAvSlots][r][c * 8];
        load_block<T>(av, av_rot<ALGO>(r, c), a);
        for (int s = ks; s < k; ++s) {
            const T* gs = &sm.G[t % 3][s][c][0];
            alpha_recompute<T, ALGO>(a, gs[0], gs[1], lut);
        }
    } else {
        const T* av = &sm.Av[t % kAvSlots][k][c * 8];
        load_block<T>(av, k, a);
        if constexpr (ALGO == 0) normalise8(a);   // the rows are alpha_raw (alpha_issue)
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        t0[j] = (a[p0] - (kTrellisQ[p0] ? Q : P)) + b[j];   // u = 0: gamma = -(P|Q)
        t1[j] = (a[p1] + (kTrellisQ[p1] ? Q : P)) + b[j];   // u = 1: gamma = +(P|Q)
    }
    T r0, r1;
    if constexpr (ALGO == 1) {
        // Max-Log-MAP: E_seq is a plain max, exact in any order -- a tree of depth 3, not 7
        r0 = vmax(vmax(vmax(t0[0], t0[1]), vmax(t0[2], t0[3])), vmax(vmax(t0[4], t0[5]), vmax(t0[6], t0[7])));
        r1 = vmax(vmax(vmax(t1[0], t1[1]), vmax(t1[2], t1[3])), vmax(vmax(t1[4], t1[5]), vmax(t1[6], t1[7])));
    } else {
        // the two folds advanced in lock step (independent chains: twice the latency hidden)
        r0 = mstar<T, ALGO>(t0[0], t0[1], lut);
        r1 = mstar<T, ALGO>(t1[0], t1[1], lut);
#pragma unroll
        for (int j = 2; j < 8; ++j) {
            r0 = mstar<T, ALGO>(r0, t0[j], lut);
            r1 = mstar<T, ALGO>(r1, t1[j], lut);
        }
    }
    const T llr = r1 - r0;
    const T le = llr - la - (T)2 * ys;
    const int b_ = gm.g * kCw + c;
    if (dst.llr) dst.llr[((size_t)gm.g * gm.L + i) * kCw + c] = llr;
    if (dst.ext_mode && i < dst.ext_len) {
        const int w = dst.ext_mode == 1 ? i : wperm;
        dst.ext[((size_t)gm.g * dst.ext_len + w) * kCw + c] = le;
    }
    if (b_ < gm.B) {
        if (dst.le_dump) dst.le_dump[(size_t)b_ * dst.dump_stride + (size_t)dst.dump_slot * gm.L + i] = le;
        if (dst.bits && i < gm.K)   // decision (:862-879: LLR < 0 -> 0, else 1) at pi[i] (:1264)
            dst.bits[(size_t)b_ * dst.bits_stride + (size_t)dst.bits_row * gm.K + wbit] = (llr < (T)0) ? 0 : 1;
    }
}

// fold_item for the turbo decode's full windows: the lane's LDS rows and output bases are set up
// once per SISO, the window enters only as its ring slots (s3 = t % 3, s4 = t % kAvSlots, s2 = t &
// 1, kept as running counters by the caller) and its first step i0.  Extrinsic written permuted
// (ext_mode 2 / 3), no raw-LLR or Le dump (those take fold_item).
// the folds' extrinsic stores non-temporal (A/B switch; read a SISO later by the loader's tile DMA):
// config 2 level (1514-1516 against 1516-1522 Mbit/s, profiles/r06/ab_extrinsic_nt.txt), not kept
#ifndef TD_EXT_NT
#define TD_EXT_NT 0
#endif
template <typename T>
struct FoldLane {
    int k, c;
    const T* G;      // &sm.G[0][k][c][0]
    const int* Wp;   // &sm.Wp[0][k][0]
    const T* Bv;     // &sm.Bv[0][k][c * 8]
    const T* Av;     // &sm.Av[0][r][c * 8], r = the stored row of step k (or the one before it)
    int arot;        // the block rotation of that row (av_rot)
    int rec;         // steps recomputed from the stored row (0 when every row is kept)
    const T* Gr;     // &sm.G[0][k - rec][c][0]: the recomputed steps' (P, Q)
    T* ext;          // this codeword's extrinsic row base
    uint8_t* bits;   // this codeword's decision row (nullptr: none)
};
template <typename T, int ALGO>
__device__ __forceinline__ void fold_item_fast(const FoldLane<T>& fl, const T* lut, int s3, int s4, int s2, int i0,
                                               int ext_len, int K)
{
    const int k = fl.k;
    const T* g = fl.G + s3 * (kW * kCw * 4);
    const T P = g[0], Q = g[1], ys = g[2], la = g[3];
    const int* wp = fl.Wp + s3 * (kW * 2);
    const int wperm = wp[0], wbit = wp[1];
    T a[8], b[8], t0[8], t1[8];
    load_block<T>(fl.Bv + s2 * (kW * kLanes), k, b);
    load_block<T>(fl.Av + s4 * (kW * kLanes), kFoldRows<ALGO> ? k : fl.arot, a);
    if constexpr (ALGO == 0) normalise8(a);   // the rows are alpha_raw (alpha_issue)
    if constexpr (!kFoldRows<ALGO>) {   // alpha rows not kept: recomputed from the last kept one (fold_item)
        const T* gr = fl.Gr + s3 * (kW * kCw * 4);
        for (int q = 0; q < fl.rec; ++q) alpha_recompute<T, ALGO>(a, gr[q * kCw * 4], gr[q * kCw * 4 + 1], lut);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        t0[j] = (a[p0] - (kTrellisQ[p0] ? Q : P)) + b[j];   // u = 0: gamma = -(P|Q)
        t1[j] = (a[p1] + (kTrellisQ[p1] ? Q : P)) + b[j];   // u = 1: gamma = +(P|Q)
    }
    T r0, r1;
    if constexpr (ALGO == 1) {   // Max-Log-MAP: a max tree (exact in any order), as fold_item
        r0 = vmax(vmax(vmax(t0[0], t0[1]), vmax(t0[2], t0[3])), vmax(vmax(t0[4], t0[5]), vmax(t0[6], t0[7])));
        r1 = vmax(vmax(vmax(t1[0], t1[1]), vmax(t1[2], t1[3])), vmax(vmax(t1[4], t1[5]), vmax(t1[6], t1[7])));
    } else if constexpr (kDiag<kDiagFoldNoLut>) {
        // diagnostic (results wrong): the same dependent chain without its table reads
        auto ms = [](T x, T y) { const T d = y - x; return vmax(x, y) + (fabs(d) >= (T)0.5 ? (T)0.25 : (T)0.5); };
        r0 = ms(t0[0], t0[1]);
        r1 = ms(t1[0], t1[1]);
#pragma unroll
        for (int j = 2; j < 8; ++j) {
            r0 = ms(r0, t0[j]);
            r1 = ms(r1, t1[j]);
        }
    } else {
        r0 = mstar<T, ALGO>(t0[0], t0[1], lut);
        r1 = mstar<T, ALGO>(t1[0], t1[1], lut);
#pragma unroll
        for (int j = 2; j < 8; ++j) {
            r0 = mstar<T, ALGO>(r0, t0[j], lut);
            r1 = mstar<T, ALGO>(r1, t1[j], lut);
        }
    }
    const T llr = r1 - r0;
    const T le = llr - la - (T)2 * ys;
    const int i = i0 + k;
    if (i < ext_len) {
        if constexpr (TD_EXT_NT != 0)
            __builtin_nontemporal_store(le, &fl.ext[(size_t)wperm * kCw]);
        else
            fl.ext[(size_t)wperm * kCw] = le;
    }
    if (fl.bits && i < K) fl.bits[wbit] = (llr < (T)0) ? 0 : 1;   // :862-879 at pi[i] (:1264)
}

#ifdef TD_STAMPS
// diagnostic build only: per-wave cycle totals (s_memtime, shader clock)
#define TD_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define TD_ACC(slot, a, b) (st[slot] += (b) - (a))
#else
#define TD_STAMP(v)
#define TD_ACC(slot, a, b)
#endif
// Which wave loads in the B pass: 2 (F0, the F pass's loader) or 3 (F1, beside the other
// workgroup's beta; F0 then folds beside the other workgroup's fold wave A).  Log-MAP keeps F0
// (beta bounds its B pass; F1 measured 0.5 % slower, fp32 0.8 %); Max-Log-MAP, whose B pass the
// folds and the loader bound, moves it to F1 (+3.0 %, config 3).  The F pass then stages nothing
// past the last window (kFSkip), so no F-pass DMA is in flight when F1 starts staging.
template <int ALGO>
constexpr int kBLoaderWave = ALGO == 1 ? 3 : 2;
// Max-Log-MAP fold items sorted by recompute depth over the two fold waves (15-step windows; A/B
// switch TD_ML_DEPTH) and its full windows through fold_item_fast (TD_ML_FAST)
#ifndef TD_ML_DEPTH
#define TD_ML_DEPTH 1
#endif
#ifndef TD_ML_FAST
#define TD_ML_FAST 1
#endif
template <typename T, int ALGO>
constexpr bool kMlDepthSplit = TD_ML_DEPTH && ALGO == 1 && kCkPh<ALGO> == 1 && kW == 15 &&
                               kFoldAOf<T, ALGO> == 64 && kTile - kTile / 3 > kLanes;
template <typename T, int ALGO>
constexpr bool kMlFast = TD_ML_FAST && ALGO == 1;
template <int ALGO>
constexpr bool kFSkip = kBLoaderWave<ALGO> == 3;   // (on its own, with F0 loading both passes: level)
constexpr int kAlphaPrio = 2;   // VALU priority of the alpha wave in the F pass
// The lane index made opaque at the start of every SISO (role remat), so that the compiler cannot
// hoist the roles' lane-derived addresses (fold lanes, alpha store offsets, ...) out of the SISO loop,
// where they were all live at once, in every role: fp64 log-MAP 256 -> 95 VGPRs, fp32 log-MAP 191 ->
// 78, so that three workgroups fit a CU (turbo_decode_kernel3).  On for fp32, and for fp64 with
// 15-step windows (without it that build spills to scratch) -- with 12-step windows at two
// workgroups per CU it measured level in fp64 log-MAP (17.39 vs 17.40 ms) and 1.4 % slower in fp64
// Max-Log-MAP.
template <typename T>
constexpr bool kRoleRemat = sizeof(T) == 4 || kW != 12;
constexpr int kStampSlots = 16;  // per wave: F pass, F wait, B work, B wait, chain, XCC_ID, HW_ID, kernel
                                 // shader cycles, kernel realtime (100 MHz ticks), SISO calls, SISO-end
                                 // barriers, F prologue, loader B prologue, loader first tile (see diag)

// The loader wave keeps one register set per stream, issued one iteration ahead and consumed
// (stored to LDS) at the start of the next iteration before it is re-issued; it issues the same
// loads in every iteration (clamped addresses), so the compiler's vmcnt bookkeeping stays exact.
// The other waves issue no global loads inside the passes (the folds only store).

// The loader's B pass (wave kBLoaderWave<ALGO>).
template <typename T, int ALGO>
__device__ void bpass_loader(Smem<T>& sm, const SisoSrc<T>& src, const SisoDst<T>& dst, const Geom& gm, T* astore,
                             T* tmstore, int lane, int tl, int nB, unsigned long long* st)
{
    (void)st;
    (void)tmstore;
    constexpr int kF = kTileDma<T>;
    // B pass iteration j (wa = tl - j) converts the tiles of wa (tiles tl-2..tl never left the
    // ring) and tempmax of wa (beta, next iteration) from staging slot j % 3 into the LDS slots
    // nobody reads this iteration, stages the same streams three windows lower into the slot it
    // just read, and copies alpha of wa-1 (folded at j+3) straight into LDS slot (wa-1) % 4
    // (last read at j-1).  All DMAs are unconditional (clamped windows, a spare slot at the
    // tail), so the per-iteration count kB is fixed and every iteration ends leaving only its
    // own and the previous iteration's DMAs in flight: three windows of latency for each.
    constexpr int kAd = kDiag<kDiagNoAdma> ? 0 : alpha_dma_count<T, ALGO>();
    constexpr int kB = kF + 1 + kAd;
    TD_STAMP(p3);
    vm_wait<0>();   // the F pass's last (unused) staging
    if constexpr (ALGO == 0) {
        // Log-MAP (round 4): no tempmax stream.  Iteration j (wa = tl - j) converts the tiles of
        // wa, copies alpha of wa-1 (folded at j+3) into LDS slot (wa-1) % 4 first and stages the
        // tiles three windows lower, then waits until the previous iteration's alpha copy (window
        // wa) has landed and forms beta's tempmax of wa from it (tm_from_alpha, beta next
        // iteration): the copy has one iteration of latency instead of three, the tiles two.
        // (Issuing the DMAs ahead of the conversion, with a fourth staging slot, measured 0.8 %
        // slower: the conversion's LDS reads then meet the DMAs' LDS writes.)
        auto bstep0 = [&](int j, int slot) {
            TD_STAMP(b0);
            const int wa = tl - j;
            if constexpr (!kDiag<kDiagNoBConvert>) {
                if (wa >= 0 && wa <= tl - 3) tile_convert(sm, slot, src, wa, lane);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's reads are done before it is re-staged
            TD_STAMP(bc);
            TD_ACC(14, b0, bc);   // stamps build: the loader's slot 14 is its B-pass tile conversion
            if constexpr (kAd > 0) alpha_dma<T, ALGO>(sm, astore, gm, wa - 1, lane);
            tile_dma(sm, slot, src, dst, gm, max(min(wa - 3, tl - 3), 0), lane);
            TD_STAMP(bw);
            if (j == 0)
                vm_wait<kAd + kF>();       // the prologue's copies (window tl, row L) have landed
            else
                vm_wait<kAd + 2 * kF>();   // the previous iteration's alpha copy (window wa) has landed
            TD_STAMP(bt);
            TD_ACC(4, bw, bt);   // stamps build: the loader's slot 4 is its B-pass DMA wait
            if (wa >= 0) tm_from_alpha(sm, wa, lane);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            TD_STAMP(b1);
            TD_ACC(15, bt, b1);   // ... slot 15 its tempmax formation (tm_from_alpha, to its writes' completion)
            wg_sync_lds();
            TD_STAMP(b2);
            TD_ACC(2, b0, b1);
            TD_ACC(3, b1, b2);
        };
        if constexpr (kAd > 0) {
            alpha_dma<T, ALGO>(sm, astore, gm, tl, lane);      // folded at j = 2
            alpha_dma_head<T>(sm, astore, gm, tl + 1, lane);   // alpha_raw[.][L] when the last window is full
        }
        TD_STAMP(p4);
        TD_ACC(12, p3, p4);
        for (int j = 0; j < nB; j += 3) {
            bstep0(j, 0);
            if (j + 1 < nB) bstep0(j + 1, 1);
            if (j + 2 < nB) bstep0(j + 2, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no copy outlives the pass
        return;
    }
    auto bstep = [&](int j, int slot) {
        TD_STAMP(b0);
        const int wa = tl - j;
        if constexpr (!kDiag<kDiagNoBConvert>) {
            if (wa >= 0 && wa <= tl - 3) tile_convert(sm, slot, src, wa, lane);
            if (wa >= 0) tm_convert(sm, slot, wa, lane);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's reads are done before it is re-staged
        TD_STAMP(bc);
        TD_ACC(14, b0, bc);   // stamps build: the loader's slot 14 is its B-pass conversion (tiles + tempmax)
        tile_dma(sm, slot, src, dst, gm, max(min(wa - 3, tl - 3), 0), lane);
        tm_dma(sm, slot, tmstore, gm, wa - 3, lane);
        if constexpr (kAd > 0) alpha_dma<T, ALGO>(sm, astore, gm, wa - 1, lane);
        TD_STAMP(bw);
        vm_wait<2 * kB>();   // everything issued before the previous iteration has landed
        TD_STAMP(b1);
        TD_ACC(4, bw, b1);   // stamps build: the loader's slot 4 is its B-pass DMA wait
        wg_sync_lds();
        TD_STAMP(b2);
        TD_ACC(2, b0, b1);
        TD_ACC(3, b1, b2);
    };
    tile_dma(sm, 0, src, dst, gm, max(tl - 3, 0), lane);   // j = 0: never converted
    tm_dma(sm, 0, tmstore, gm, tl, lane);
    tile_dma(sm, 1, src, dst, gm, max(tl - 3, 0), lane);   // j = 1: never converted
    tm_dma(sm, 1, tmstore, gm, tl - 1, lane);
    tile_dma(sm, 2, src, dst, gm, max(tl - 3, 0), lane);   // j = 2: never converted
    tm_dma(sm, 2, tmstore, gm, tl - 2, lane);
    if constexpr (kAd > 0) alpha_dma<T, ALGO>(sm, astore, gm, tl, lane);   // folded at j = 2
    vm_wait<2 * (kF + 1) + kAd>();   // slot 0 landed
    TD_STAMP(p4);
    TD_ACC(12, p3, p4);
    for (int j = 0; j < nB; j += 3) {
        bstep(j, 0);
        if (j + 1 < nB) bstep(j + 1, 1);
        if (j + 2 < nB) bstep(j + 2, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no copy outlives the pass
}

// One SISO over the workgroup's 8 codewords.  Each role runs its own loops (so only that role's
// state is live in its code); every role executes the same sequence of wg_sync_lds barriers:
// 1 (F prologue) + nT (F iterations) + nB (B iterations).
template <typename T, int ALGO>
__device__ void siso_wg(Smem<T>& sm, const SisoSrc<T>& src, const SisoDst<T>& dst, const Geom& gm, T* astore,
                        T* tmstore, const LaneTables* lt, int wave, int lane, unsigned long long* st)
{
    (void)st;
    if constexpr (kRoleRemat<T>) touch(lane);   // nothing derived from the lane index is SISO-invariant (role remat)
    TD_STAMP(p0);
    const int nT = gm.nT;
    const int tl = nT - 1;
    const int nB = nT + 2;   // B-pass iterations: j = 0 .. nT+1 (wa = tl - j, wb = wa + 1, wf = wa + 2)
    T* ga0 = astore + astore_window_off(gm.g, 0, gm.L);   // row 0 of window 0 of this group
    constexpr size_t aws = (size_t)kW * kLanes;            // window t starts at ga0 + t * aws
    T* gtm0 = tmstore + (size_t)gm.g * gm.L * kCw;

    // ===================================== F pass
    if (wave == 0) {
        const int c = lane >> 3;
        LaneConst<T> lc;
        lane_setup(lt, lane, lc);
        T a = lc.a_init0 ? (T)0 : (T)-kInfty;   // alpha[.][0] (:943,948), its tempmax is 0
        __builtin_amdgcn_s_setprio(kAlphaPrio);
        wg_sync_lds();
        TD_STAMP(p1);
        TD_ACC(11, p0, p1);
        int t0 = 0;
        if constexpr (kAlphaSchedS<T, ALGO>) {
            // windows 1 .. tl-1 are full: running bases and slot index, no per-window address math
            if (tl >= 2) {
                TD_STAMP(f0);
                a = alpha_window<T, ALGO>(a, 0, kW, sm, lut_col(sm, lane), c, lc, ga0, gtm0, st ? st + 4 : nullptr);
                TD_STAMP(f1);
                wg_sync_lds();
                TD_STAMP(f2);
                TD_ACC(0, f0, f1);
                TD_ACC(1, f1, f2);
                const unsigned va[3] = {(unsigned)(lc.st_off[0] * sizeof(T)), (unsigned)(lc.st_off[1] * sizeof(T)),
                                        (unsigned)(lc.st_off[2] * sizeof(T))};
                TmBatch<T> tbh{(T)0, lane & 7, (unsigned)(((lane & 7) * kCw + c) * sizeof(T)),
                               (unsigned)((tm2_slot(lane & 7) * kCw + c) * sizeof(T))};
                T* sa = ga0 + aws + (size_t)kArow0 * kLanes;   // window 1, row kArow0 (astore_row)
                T* stm = gtm0 + (size_t)kW * kCw;
                const T* lut = lut_col(sm, lane);
                unsigned long long* chain_st = st ? st + 4 : nullptr;
                (void)chain_st;
                int tb = 1;
                for (int t = 1; t < tl; ++t) {
                    TD_STAMP(f0);
                    StepIn<T> op[3];
                    op[0] = alpha_in<T, 0>(sm, tb, 0, c, lc);
                    op[1] = alpha_in<T, 1>(sm, tb, 1, c, lc);
                    __builtin_amdgcn_sched_barrier(0);   // the window's first reads issue first
                    TD_CHAIN_T0(c0);
                    const T a0 = a;
                    unsigned miss = 0;
                    AlphaSchedS<T, ALGO, 0>::run(a, op, sm, tb, lut, c, lc, sa, stm, va, tbh, miss);
                    if constexpr (kASpec<T, ALGO>) {
#ifdef TD_ASPEC_REDO
                        miss = 1;
#endif
                        if (__builtin_amdgcn_ballot_w64(miss != 0))   // a bucket mismatch: the window again, committed order
                            a = alpha_window<T, ALGO>(a0, t, kW, sm, lut, c, lc, ga0 + (size_t)t * aws,
                                                      gtm0 + (size_t)t * kW * kCw);
                    }
                    TD_CHAIN_ACC(c0);
                    sa += aws;
                    stm += (size_t)kW * kCw;
                    tb = tb == 2 ? 0 : tb + 1;
                    TD_STAMP(f1);
                    wg_sync_lds();
                    TD_STAMP(f2);
                    TD_ACC(0, f0, f1);
                    TD_ACC(1, f1, f2);
                }
                t0 = tl;
            }
        }
        for (int t = t0; t < nT; ++t) {
            TD_STAMP(f0);
            a = alpha_window<T, ALGO>(a, t, window_len(gm, t), sm, lut_col(sm, lane), c, lc, ga0 + (size_t)t * aws,
                                      gtm0 + (size_t)t * kW * kCw, st ? st + 4 : nullptr);
            if (t == tl) {
                if constexpr (ALGO == 0) {   // alpha_raw[.][L] at row L (labels of phase L mod 3): its max is tempmax[L]
                    const int ph = gm.L % 3;   // constant indices only: a runtime index into lc moves it to scratch
                    ga0[(size_t)gm.L * kLanes + (ph == 0 ? lc.st_off[0] : ph == 1 ? lc.st_off[1] : lc.st_off[2])] = a;
                } else {
                    gtm0[(size_t)(gm.L - 1) * kCw + c] = group_max8(a);   // tempmax[L]
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // scratch visible to the loader
            }
            TD_STAMP(f1);
            wg_sync_lds();
            TD_STAMP(f2);
            TD_ACC(0, f0, f1);
            TD_ACC(1, f1, f2);
        }
        __builtin_amdgcn_s_setprio(0);   // in the B pass the beta wave goes first
    } else if (wave == 2) {
        // Loader: every input travels HBM -> LDS by DMA into a staging slot, and this wave converts
        // landed slots into the ring (no VGPR is ever the target of a load in flight).
        // Invariant: every iteration ends with a wait that leaves only its own DMAs in flight.
        // F pass iteration t: convert window t+1 (staged two iterations ago, slot (t+1) % 3) and
        // stage window t+3 into slot t % 3, which window t left one iteration ago.
        constexpr int kF = kTileDma<T>;
        auto fstep = [&](int t) {
            TD_STAMP(f0);
            if (t + 1 <= tl) tile_convert(sm, (t + 1) % 3, src, t + 1, lane);
            if (!kFSkip<ALGO> || t + 3 <= tl) {
                tile_dma(sm, t % 3, src, dst, gm, min(t + 3, tl), lane);
                vm_wait<kF>();   // window t+2 has landed
            } else {
                vm_wait<0>();    // no staging past the last window: nothing is left in flight at the pass end
            }
            TD_STAMP(f1);
            wg_sync_lds();
            TD_STAMP(f2);
            TD_ACC(0, f0, f1);
            TD_ACC(1, f1, f2);
        };
        tile_dma(sm, 0, src, dst, gm, 0, lane);
        vm_wait<0>();
        TD_STAMP(p2);
        TD_ACC(13, p0, p2);
        tile_convert(sm, 0, src, 0, lane);
        tile_dma(sm, 1, src, dst, gm, min(1, tl), lane);
        tile_dma(sm, 2, src, dst, gm, min(2, tl), lane);
        vm_wait<kF>();
        wg_sync_lds();
        TD_STAMP(p1);
        TD_ACC(11, p0, p1);
        for (int t = 0; t < nT; ++t) fstep(t);
        if constexpr (kBLoaderWave<ALGO> == 2) {
            bpass_loader<T, ALGO>(sm, src, dst, gm, astore, tmstore, lane, tl, nB, st);
            return;
        }
    } else if (dst.sys2_out) {
        // waves 1 and 3, first SISO: SISO2's systematic input sys2[g][i][c] = sys1[g][pi(i)][c]
        // (i < K; :1109-1113), one element of window t per lane (kTile - 64 of 128 lanes in the
        // second wave) with pi(i) from the ring slot of window t (Wp[.][k][1], staged by the
        // loader), loaded in iteration t and stored in t+1, so no wave ever waits on HBM before a
        // barrier.  This is demux_perm_kernel's work, done by the waves the F pass leaves idle.
        wg_sync_lds();
        TD_STAMP(p1);
        TD_ACC(11, p0, p1);
        const int e = (wave == 1 ? 0 : kLanes) + lane;
        const int ec = min(e, kTile - 1);
        const int k = ec >> 3, c = ec & 7;
        const T* s1 = src.sys + (size_t)gm.g * gm.L * kCw + c;
        T* s2 = dst.sys2_out + (size_t)gm.g * gm.L * kCw + c;
        T v = (T)0;
        int ip = -1;   // row of the pending store
        for (int t = 0; t < nT; ++t) {
            TD_STAMP(f0);
            const int pi_i = min(max(sm.Wp[t % 3][k][1], 0), gm.K - 1);   // spare rows past K: any valid row
            const T nv = s1[(size_t)pi_i * kCw];
            if (ip >= 0) s2[(size_t)ip * kCw] = v;
            const int i = t * kW + k;
            ip = (e < kTile && i < gm.K) ? i : -1;
            v = nv;
            TD_STAMP(f1);
            wg_sync_lds();
            TD_STAMP(f2);
            TD_ACC(0, f0, f1);
            TD_ACC(1, f1, f2);
        }
        if (ip >= 0) s2[(size_t)ip * kCw] = v;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // sys2 complete before the SISO's end barrier
    } else {
        wg_sync_lds();   // waves 1 and 3 idle in the F pass: keep the barrier count
        TD_STAMP(p1);
        TD_ACC(11, p0, p1);
        for (int t = 0; t < nT; ++t) {
            TD_STAMP(f0);
            TD_STAMP(f1);
            wg_sync_lds();
            TD_STAMP(f2);
            TD_ACC(0, f0, f1);
            TD_ACC(1, f1, f2);
        }
    }

    // ===================================== B pass (waves 0, 1, 3)
    if (kBLoaderWave<ALGO> == 3 && wave == 3) {
        bpass_loader<T, ALGO>(sm, src, dst, gm, astore, tmstore, lane, tl, nB, st);
    } else if (wave == 1) {
        // beta over window wb = tl - j + 1 (its tempmax was staged last iteration)
        LaneConst<T> lc;
        lane_setup(lt, lane, lc);
        const int phL = gm.L % 3;   // beta[.][L] lives in the labeling of phase L mod 3
        T beta = (src.terminated && !((lc.b_init0 >> phL) & 1)) ? (T)-kInfty : (T)0;   // :944,951-959
        int j0 = 0;
        if constexpr (ALGO == 0 && !kDiag<kDiagNoBeta>) {
            if (tl >= 1) {
                // j = 0 (nothing) and j = 1 (window tl, maybe partial: the rolled loop), then the full
                // windows wb = tl-1 .. 0 (j = 2 .. nB-2) with running slot counters
                for (int j = 0; j < 2; ++j) {
                    TD_STAMP(b0);
                    if (j == 1)
                        beta = beta_window<T, ALGO, false>(beta, tl, window_len(gm, tl), sm, lut_col(sm, lane), lane >> 3,
                                                           lc, st ? st + 4 : nullptr);
                    TD_STAMP(b1);
                    wg_sync_lds();
                    TD_STAMP(b2);
                    TD_ACC(2, b0, b1);
                    TD_ACC(3, b1, b2);
                }
                const T* lut = lut_col(sm, lane);
                int tb = (tl - 1) % 3, xb = (tl - 1) & 1;
                for (int wb = tl - 1; wb >= 0; --wb) {
                    TD_STAMP(b0);
                    beta = beta_window_full<T, ALGO>(beta, tb, xb, sm, lut, lane >> 3, lc, st ? st + 4 : nullptr);
                    tb = tb == 0 ? 2 : tb - 1;
                    xb ^= 1;
                    TD_STAMP(b1);
                    wg_sync_lds();
                    TD_STAMP(b2);
                    TD_ACC(2, b0, b1);
                    TD_ACC(3, b1, b2);
                }
                j0 = tl + 2;   // j = nB - 1 (wb = -1): beta idle, the folds finish window 0
            }
        }
        for (int j = j0; j < nB; ++j) {
            TD_STAMP(b0);
            const int wb = tl - j + 1;
            if (!kDiag<kDiagNoBeta> && wb >= 0 && wb <= tl)
                beta = beta_window<T, ALGO>(beta, wb, window_len(gm, wb), sm, lut_col(sm, lane), lane >> 3, lc,
                                            st ? st + 4 : nullptr);
            TD_STAMP(b1);
            wg_sync_lds();
            TD_STAMP(b2);
            TD_ACC(2, b0, b1);
            TD_ACC(3, b1, b2);
        }
    } else {
        // waves 0 and 3: fold window wf = tl - j + 2, one item per lane
        constexpr int kFA = kFoldAOf<T, ALGO>;
        int fe = (wave == 0 ? 0 : kFA) + lane;
        int nfold = wave == 0 ? kFA : kTile - kFA;
        if constexpr (!kFoldRows<ALGO> && kTile - kTile / 3 <= kLanes) {
            // (kW = 12 only: with 15-step windows the other two phases hold 80 items, more than a wave.)
            // Items by recompute depth when alpha rows are not all kept: wave A (beside the loader)
            // takes the 32 items of the phase furthest from a kept row (pd), the fold wave beside
            // the other workgroup's beta (F1) the 64 items of the other two phases.  Max-Log-MAP
            // keeping phase 0: A recomputes two steps, F1 at most one; with items in step order
            // every wave paid two (+0.4 %, config 3).
            constexpr int pd = kCkDeepest<ALGO>, pa = pd == 0 ? 1 : 0, pb = pd == 2 ? 1 : 2;
            const int q = lane >> 3;
            fe = wave == 0 ? (3 * q + pd) * kCw + (lane & 7) : (3 * (q >> 1) + ((q & 1) ? pb : pa)) * kCw + (lane & 7);
            nfold = wave == 0 ? kTile / 3 : kTile - kTile / 3;
        }
        if constexpr (kMlDepthSplit<T, ALGO>) {
            // 15-step windows, Max-Log-MAP (phase 0 kept): 40 items of each recompute depth.  Wave A
            // takes the 40 depth-2 items (steps 2, 5, .., 14) and 24 of depth 1 (steps 1, 4, 7), the
            // other fold wave the remaining 16 of depth 1 (steps 10, 13) and the 40 of depth 0
            // (steps 0, 3, .., 12), so it runs one recompute step instead of two (in step order both
            // waves held lanes of every depth, and the divergent loop ran twice in both)
            const int l = lane;
            int k;
            if (wave == 0)
                k = l < 40 ? 3 * (l >> 3) + 2 : 3 * ((l - 40) >> 3) + 1;
            else
                k = l < 16 ? 3 * (3 + (l >> 3)) + 1 : 3 * (min(l - 16, 39) >> 3);
            fe = k * kCw + (l & 7);
            nfold = wave == 0 ? 64 : 56;
        }
        int j0 = 0;
        if ((ALGO == 0 || kMlFast<T, ALGO>) && !dst.llr && !dst.le_dump && dst.ext_mode >= 2 && tl >= 1) {
            // iterations 0, 1 fold nothing, 2 folds the last window (maybe partial): generic below;
            // here iterations 3 .. nB-1, i.e. the full windows wf = tl-1 .. 0
            for (int j = 0; j < 3; ++j) {
                TD_STAMP(b0);
                const int wf = tl - j + 2;
                if (lane < nfold && wf <= tl && (fe >> 3) < window_len(gm, wf))
                    fold_item<T, ALGO>(sm, lut_col(sm, lane), wf, fe, dst, gm);
                TD_STAMP(b1);
                wg_sync_lds();
                TD_STAMP(b2);
                TD_ACC(2, b0, b1);
                TD_ACC(3, b1, b2);
            }
            FoldLane<T> fl;
            fl.k = fe >> 3;
            fl.c = fe & 7;
            const int ke = min(fl.k, kW - 1);   // spare lanes: any valid row (they fold nothing)
            fl.G = &sm.G[0][ke][fl.c][0];
            fl.Wp = &sm.Wp[0][ke][0];
            fl.Bv = &sm.Bv[0][ke][fl.c * 8];
            if constexpr (kFoldRows<ALGO>) {
                fl.Av = &sm.Av[0][ke][fl.c * 8];
            } else {
                int ks;
                const int r = ck_row_of<ALGO>(ke, ks);
                fl.Av = &sm.Av[0][r][fl.c * 8];
                fl.arot = av_rot<ALGO>(r, fl.c);
                fl.rec = ke - ks;
                fl.Gr = &sm.G[0][ks][fl.c][0];
            }
            fl.ext = dst.ext + (size_t)gm.g * dst.ext_len * kCw + fl.c;
            const int b_ = gm.g * kCw + fl.c;
            fl.bits = (dst.bits && b_ < gm.B) ? dst.bits + (size_t)b_ * dst.bits_stride + (size_t)dst.bits_row * gm.K
                                              : nullptr;
            const T* lut = lut_col(sm, lane);
            int wf = tl - 1, s3 = wf % 3, s4 = wf % kAvSlots, s2 = wf & 1;
            for (int j = 3; j < nB; ++j, --wf) {
                TD_STAMP(b0);
                if (!kDiag<kDiagNoFold> && lane < nfold)
                    fold_item_fast<T, ALGO>(fl, lut, s3, s4, s2, wf * kW, dst.ext_len, gm.K);
                s3 = s3 == 0 ? 2 : s3 - 1;
                s4 = s4 == 0 ? kAvSlots - 1 : s4 - 1;
                s2 ^= 1;
                TD_STAMP(b1);
                wg_sync_lds();
                TD_STAMP(b2);
                TD_ACC(2, b0, b1);
                TD_ACC(3, b1, b2);
            }
            j0 = nB;
        }
        for (int j = j0; j < nB; ++j) {
            TD_STAMP(b0);
            const int wf = tl - j + 2;
            if (!kDiag<kDiagNoFold> && lane < nfold && wf >= 0 && wf <= tl && (fe >> 3) < window_len(gm, wf))
                fold_item<T, ALGO>(sm, lut_col(sm, lane), wf, fe, dst, gm);
            TD_STAMP(b1);
            wg_sync_lds();
            TD_STAMP(b2);
            TD_ACC(2, b0, b1);
            TD_ACC(3, b1, b2);
        }
    }
}

template <typename T>
__device__ __forceinline__ void lut_to_lds(const DecodeParams<T>& p, Smem<T>& sm, int tid)
{
    for (int e = tid; e < kLutElems<T>; e += kWaves * kLanes) sm.lut[e] = lut_elem<T>(p.lut, e);
}

template <typename T>
__device__ __forceinline__ const T* lut_col(const Smem<T>& sm, int lane)
{
    return lut_origin(sm.lut + (lane % kLutCols<T>));
}

template <typename T>
__device__ __forceinline__ Smem<T>* smem()
{
    extern __shared__ __attribute__((aligned(16))) unsigned char td_smem[];
    return reinterpret_cast<Smem<T>*>(td_smem);
}

// VALU issue priority of the beta wave (ties on a SIMD go to the higher priority, then the older
// wave).  Log-MAP: beta bounds the B pass, so it goes first (2; fp32 log-MAP measured best at 0
// before its table went to 32 columns, 2 since: 1414 -> 1436).  Max-Log-MAP: the folds and the
// loader bound the B pass and beta yields (0).
template <typename T, int ALGO>
__device__ __forceinline__ void set_beta_prio()
{
    __builtin_amdgcn_s_setprio(ALGO == 1 ? 0 : 2);
}

struct WgPos {
    int role;       // 0 = A, 1 = B (beta), 2 = F0 (loader), 3 = F1 (fold)
    int lane;
    int g;          // codeword group index
    int slot_key;   // this CU's occupancy word, and the slot taken (4: none)
    int slot;
};

// Roles by placement.  Two workgroups share a CU (three or four in turbo_decode_kernel3 / 4), and a
// recursion wave should share its SIMD with a light role of the other workgroup: A with F0 (the
// loader), B with F1 (the fold wave, idle in the F pass).  The waves read their SIMD from HW_ID and
// the workgroup takes a free slot (0..3) of its CU in a per-CU occupancy word (atomicOr; released at
// the end, wg_release); role = SIMD for slot 0 and SIMD ^ 2 for slot 1, which gives the pairs A/F0,
// B/F1 on every SIMD whatever order the workgroups arrived in (deriving the pairing from the
// dispatch round instead cost 4 % after a kernel with many small blocks had shifted the placement;
// the pairing A/F1 + B/F0 measured 0.7 % slower, and beta beside a loader -- alpha alone on its SIMD
// in the F pass -- 1.3 % slower).  If two waves of the workgroup share a SIMD, the wave index stands
// in for the SIMD.  role_cus = 0 or no slot words: role = wave.
__device__ __forceinline__ WgPos wg_pos(int role_cus, unsigned* slots)
{
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    const int g = (int)blockIdx.x;
    if (role_cus > 0 && slots) {
        __shared__ int s_simd[kWaves];
        __shared__ int s_slot;
        const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
        const int simd = (int)((hw >> 4) & 3);
        const int key = (int)((((xcc & 7) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15));
        if (threadIdx.x == 0) {
            int slot = 0;   // the first free of slots 0..3 (4: none)
            while (slot < 4 && (atomicOr(&slots[key], 1u << slot) & (1u << slot))) ++slot;
            s_slot = slot;
        }
        if (lane == 0) s_simd[wave] = simd;
        __syncthreads();
        bool distinct = true;
#pragma unroll
        for (int a = 0; a < kWaves; ++a)
#pragma unroll
            for (int b = a + 1; b < kWaves; ++b) distinct = distinct && s_simd[a] != s_simd[b];
        const int slot = s_slot;
        const int base = distinct ? simd : wave;
        // slots 2, 3 (turbo_decode_kernel3 / 4): role = SIMD ^ 1, SIMD ^ 3, so that the workgroups'
        // alpha chains (and their beta chains) sit on different SIMDs
        const int rx = slot == 1 ? 2 : (slot == 2 ? 1 : (slot == 3 ? 3 : 0));
        return WgPos{base ^ rx, lane, g, key, slot};
    }
    return WgPos{wave, lane, g, 0, 4};   // slot 4: none (wg_release)
}

// end of the kernel: give the CU slot back (all waves of the workgroup are past their work)
__device__ __forceinline__ void wg_release(const WgPos& w, unsigned* slots)
{
    if (w.slot < 4) {
        __syncthreads();
        if (threadIdx.x == 0) atomicAnd(&slots[w.slot_key], ~(1u << w.slot));
    }
}

// The whole turbo decode of 8 codewords per workgroup (TurboDecoding, log_map.cpp:1146-1280).
template <typename T, int ALGO>
__device__ __forceinline__ void turbo_decode_body(const DecodeParams<T>& p)
{
    const WgPos w = wg_pos(p.role_cus, p.cu_slots);
    Smem<T>& sm = *smem<T>();
    const int wave = w.role, lane = w.lane;
    lut_to_lds(p, sm, wave * kLanes + lane);
    if (wave == 1) set_beta_prio<T, ALGO>();   // beta first; alpha raises itself in the F pass
    __syncthreads();

    Geom gm{p.K, p.L, p.nT, p.B, w.g, p.G, p.pi, p.pinv};
    unsigned long long st[kStampSlots] = {};
#ifdef TD_STAMPS
    const unsigned long long k_cyc0 = __builtin_amdgcn_s_memtime(), k_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // launch clock: workgroup 0 reads the shader clock (s_memtime) and the 100 MHz real-time counter
    // (s_memrealtime) at its start and end -- two scalar reads each, wave-uniform branch -- and its
    // first lane writes them with one vector store (td_clock_read: the sustained clock of the launch)
    const bool clk = p.clk && blockIdx.x == 0;
    unsigned long long clk_c0 = 0, clk_r0 = 0;
    if (clk) {
        clk_c0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
    }
    // SISO pass s = 2*it + dec
    for (int s = 0; s < 2 * p.iters; ++s) {
        const int it = s >> 1, dec = s & 1;
        const bool want_bits = dec == 1 && (p.all_iters || it == p.iters - 1);
        // decoder 1: La = deinterleaved Le of decoder 2 (:1221), zero before the first
        //            iteration (:1212-1215); its Le is written interleaved (ext12[pinv[i]]),
        //            i.e. already as decoder 2's La (:1242).
        // decoder 2: La read in order; its Le is written deinterleaved (ext21[pi[i]], = the
        //            next La of decoder 1); decisions deinterleaved (:1261-1264).
        SisoSrc<T> src{dec ? p.sys2 : p.sys1, dec ? p.par2 : p.par1, dec ? p.ext12 : p.ext21, p.K,
                       (dec == 0 && it == 0) ? 0 : p.K, 1};
        SisoDst<T> dst{dec ? p.ext21 : p.ext12, dec ? 2 : 3, p.K, nullptr, p.le_dump,
                       want_bits ? p.bits : nullptr, p.all_iters ? it : 0, p.all_iters ? p.iters * p.K : p.K,
                       s, p.iters * 2 * p.L, (s == 0 && p.sys2_in_turbo) ? p.sys2 : nullptr};
        TD_STAMP(s0);
        siso_wg<T, ALGO>(sm, src, dst, gm, p.astore, p.tmstore, p.lane, wave, lane, st);
        TD_STAMP(s1);
        __syncthreads();   // extrinsic stores of this SISO visible to the next one's loads
        TD_STAMP(s2);
        TD_ACC(9, s0, s1);
        TD_ACC(10, s1, s2);
    }
    if (clk) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            const ulonglong4 v = make_ulonglong4(clk_c0, clk_r0, c1, r1);
            *reinterpret_cast<ulonglong4*>(p.clk) = v;
        }
    }
#ifdef TD_STAMPS
    st[6] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    st[5] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    st[7] = __builtin_amdgcn_s_memtime() - k_cyc0;
    st[8] = __builtin_amdgcn_s_memrealtime() - k_rt0;
    if (p.stamps && lane == 0)
        for (int q = 0; q < kStampSlots; ++q)
            p.stamps[((size_t)w.g * kWaves + wave) * kStampSlots + q] = st[q];
#endif
    wg_release(w, p.cu_slots);
}

template <typename T, int ALGO>
__global__ __launch_bounds__(kWaves * 64, 2) void turbo_decode_kernel(DecodeParams<T> p)
{
    turbo_decode_body<T, ALGO>(p);
}

// Large batches (more groups than two per CU): three workgroups per CU -- 24 codewords, 12 waves,
// three per SIMD -- where the build fits them: at most 168 VGPRs without scratch (the build fails
// on scratch) and a third of the CU's LDS.  fp32 fits (role remat: fp32 log-MAP 191 -> 78 VGPRs).
// fp64 does not: its Smem (the 4-window alpha ring alone is 30 KB) is more than a third of the CU's
// LDS.  Measured (B = 12288, one box): fp32 Max-Log-MAP 2370 -> 3357 Mbit/s, fp32
// log-MAP 1641 -> 2265.
template <typename T, int ALGO>
constexpr bool kOcc3 = 3 * (sizeof(Smem<T>) + 64) <= 160 * 1024 && (kRoleRemat<T> || (sizeof(T) == 4 && ALGO == 1));
template <typename T, int ALGO>
__global__ __launch_bounds__(kWaves * 64, 3) void turbo_decode_kernel3(DecodeParams<T> p)
{
    if constexpr (kOcc3<T, ALGO>) turbo_decode_body<T, ALGO>(p);
}

// More than three groups per CU: four workgroups per CU (16 waves, at most 128 VGPRs, a quarter of
// the LDS) where they fit: fp32 with 12-step windows (36.7 KB of LDS, 67-79 VGPRs with role remat).
template <typename T, int ALGO>
constexpr bool kOcc4 = 4 * (sizeof(Smem<T>) + 64) <= 160 * 1024 && kRoleRemat<T>;
// fp32 four per CU from the 12-step-window build when this one's Smem does not fit four (launch_turbo4_w12)
#ifdef TD_W12_TU
template <typename T, int ALGO>
constexpr bool kOcc4W12 = false;
#else
template <typename T, int ALGO>
constexpr bool kOcc4W12 = !kOcc4<T, ALGO> && sizeof(T) == 4 && kW != 12;
#endif
template <typename T, int ALGO>
__global__ __launch_bounds__(kWaves * 64, 4) void turbo_decode_kernel4(DecodeParams<T> p)
{
    if constexpr (kOcc4<T, ALGO>) turbo_decode_body<T, ALGO>(p);
}

// td_reserve's workspace-placement probe (td_api.cpp place_ws): the same code as
// turbo_decode_kernel under its own symbol, so that kernel traces and PMC passes of a decode list
// the one-iteration probe launches apart from the decode's own launches.  (Decodes at three or four
// workgroups per CU are probed with their own kernel, launch_turbo_algo.)
template <typename T, int ALGO>
__global__ __launch_bounds__(kWaves * 64, 2) void turbo_placement_probe_kernel(
    DecodeParams<T> p)
{
    turbo_decode_body<T, ALGO>(p);
}

// Standalone SISO (Log_MAP_decoder) over interleaved [G][L][8] inputs.
template <typename T, int ALGO>
__global__ __launch_bounds__(kWaves * 64, 2) void siso_kernel(DecodeParams<T> p, const T* la,
                                                                                          int terminated)
{
    const WgPos w = wg_pos(p.role_cus, p.cu_slots);
    Smem<T>& sm = *smem<T>();
    const int wave = w.role, lane = w.lane;
    lut_to_lds(p, sm, wave * kLanes + lane);
    if (wave == 1) set_beta_prio<T, ALGO>();
    __syncthreads();
    Geom gm{p.K, p.L, p.nT, p.B, w.g, p.G, p.pi, p.pinv};
    SisoSrc<T> s{p.sys1, p.par1, la, p.L, p.L, terminated};
    SisoDst<T> d{nullptr, 0, 0, p.llr_out, nullptr, nullptr, 0, 0, 0, 0, nullptr};
    siso_wg<T, ALGO>(sm, s, d, gm, p.astore, p.tmstore, p.lane, wave, lane, nullptr);
    wg_release(w, p.cu_slots);
}

#ifdef TD_WIN_TU
// The sub-block schedule is compiled in its own translation unit (td_kernels_win.hip, built with the
// max-ILP machine scheduler: build.py WIN_FLAGS); td_kernels.hip and td_kernels_w12.hip skip it.
// ================================================================== sub-block schedule
// BASELINE config 5 / SURVEY.md 8f row 3: the trellis of each codeword is cut into nS sub-blocks
// of W steps (the last one also takes the remainder, e.g. the 3 tail steps) decoded in parallel.
// A sub-block's alpha starts g steps early and its beta g steps late (overlap warm-up), from
//   * equal metrics, or
//   * NII (next-iteration initialisation): the metrics the neighbouring sub-block's chain had at
//     that position in the previous iteration (ITTC/CUDA/turboDecoderBianJieZhi.cu:248,302-304,
//     312,397-400 -- g = 0 there);
// only the codeword's first alpha and last beta start from the true initial / terminated states.
// The SISOs run in the reference's serial order (one launch pair per SISO) or concurrently (both
// in one launch pair, each using the other's extrinsic of the previous iteration:
// turboDecoderBianJieZhi.cu:642-690), and the extrinsic may be scaled (0.77 there, :423-434).
// The arithmetic is oracle/turbo_oracle_window.inc's, which the tests compare with bit for bit:
// log_map.cpp's steps and left-fold LLR (:975-1039), each chain normalised (:986-1000) only after
// producing the metric of a position p with (p - sW) a multiple of S (max* is shift-invariant).
//
// Layout (round 5).  A lane owns one codeword and a RUN of M consecutive sub-blocks [s0, s1) of one
// decoder; a wave holds 64 consecutive codewords of one run, so every wave walks the same
// positions and everything but the codeword is wave-uniform.  Two kernels per SISO:
//   sw_alpha_kernel  alpha forward over the run, a checkpoint every S positions of each sub-block
//                    to HBM (lane-contiguous).  Over the last g positions of sub-block s the lane
//                    also runs sub-block s+1's warm-up chain on the same inputs, so the inputs of a
//                    warm-up are read once for two chains (the round-4 kernel, one sub-block per
//                    lane, read them twice);
//   sw_beta_kernel   beta backward over the run in segments of S positions: the segment's alpha
//                    recomputed from its checkpoint into registers, then beta and the LLR fold;
//                    over the first g positions of sub-block s, s-1's beta warm-up chain runs beside.
// Both prefetch the next segment's inputs (and checkpoint) one segment ahead: alpha into registers,
// beta by LDS DMA with its extrinsic / decision stores deferred to the next segment's start.  SISO2's
// decisions go to a [K][Bp] byte array (a wave's 64 codewords adjacent) that bits_transpose_kernel
// turns into [B][K]: written directly, each byte of a wave store landed on its own cache line.
// launch_window_algo runs the batch in two parts on two streams, so one part's alpha (HBM-heavy)
// co-runs with the other's beta (VALU-heavy), and sizes the lane runs so that one beta round covers
// both parts.  Round 4's single kernel (one sub-block per lane, loads waited at each segment start,
// the interleaver index loaded and waited before every extrinsic store) ran config 5 at 2306-2328
// Mbit/s; these kernels run it at about 2620.
template <typename T>
struct WinArgs {
    int W, g;              // sub-block length, overlap
    int nS;                // sub-blocks per codeword (the last is L - (nS-1)W long, W..2W-1)
    int M, nR;             // sub-blocks per lane run, runs per decoder (nR = ceil(nS / M))
    int Bp;                // the batch's codewords rounded up to whole waves (row stride of bitsT / ckpt)
    int cw0, ncw;          // this launch's slice of the batch: waves of 64 codewords [cw0, cw0 + ncw)
    int ncp;               // checkpoint slots per sub-block (ceil(longest sub-block / S))
    T ext_scale;
    int dec;               // serial: this launch's SISO; -1: both (concurrent schedule)
    int it;                // iteration
    int la_len;            // La valid for steps < la_len (0 before any extrinsic exists)
    int nii;               // boundary metrics from nii_rd (after the first iteration)
    const T* la[2];        // per decoder: La, wide [B/64][K][64] (dec 0 natural order, dec 1 interleaved)
    T* le[2];              // per decoder: Le out, scattered to the other decoder's order
    const T* nii_rd;       // [2 dec][B][nS][2][8]: alpha (0) / beta (1) at the chain's start
    T* nii_wr;
    T* ckpt[2];            // per decoder: [nS][Bp/64][ncp][8][64] alpha checkpoints
    uint8_t* bitsT;        // [K][Bp] SISO2's decisions (natural-order rows); null: none this launch
    uint8_t* bits1;        // B = 1: SISO2's decisions straight into the caller's row (no transpose)
    int hand;              // B = 1, one sub-block a lane: the alpha kernel runs beta's warm-up (sw_alpha_lps_kernel)
    int clk;               // workgroup 0 of this beta launch samples the clock into p.clk (td_clock_read)
};

template <typename T>
struct SwIn {
    T P, Q, ys, la;
};
template <typename T>
struct SwRaw {
    T ys, yp, la;
};

// The windowed kernels' max* table (round 5): three tables (thr, vlo, vhi = vlo of the next bucket) of
// [bucket][32 columns]; lane l reads column l % 32 of each with one ds_read_b64 at a common row
// address, so the 32 lanes an LDS cycle serves hit 64 distinct banks whatever their buckets: 3 x 2 LDS
// cycles a max*, conflict-free.  (The exact kernel's layout, a ds_read2_b64 and a ds_read_b64 on 16
// columns, takes 8 + 2-4: SQ_LDS_BANK_CONFLICT was 15-16 % of the windowed kernels' LDS cycles with it.)
// The tables sit an odd number of 8-byte words apart, more than 2040 B, so the compiler cannot merge
// two reads into a ds_read2 / ds_read2st64 (4x16-lane groups on 32 banks).  The row address is the
// same one lshl_add of the clamped bucket field as before.
template <typename T>
struct SwLut {
    static constexpr int kCols = 32;
    static constexpr int kRow = kCols * (int)sizeof(T);           // bytes per bucket row
    static constexpr int kRows = kLutSize + 1;                     // + a pad row (clamped field)
    static constexpr int kTab = kRows * kRow;
    static constexpr int kOffV = kTab + (int)sizeof(T);
    static constexpr int kOffH = 2 * kOffV + (int)sizeof(T);
    static constexpr int kBytes = kOffH + kTab;
};
static_assert(SwLut<double>::kOffV % 512 && (SwLut<double>::kOffH - SwLut<double>::kOffV) % 512 &&
                  SwLut<double>::kOffH % 512 && SwLut<double>::kOffV > 2040, "no ds_read2 merging");

// The one-read table (ALGO 2, round 6; td_tables.h build_qlut): one value per bucket of the finer grid
// (exponent + kQBits mantissa bits), the same 32 replicated columns, so one conflict-free ds_read_b64
// per max* and no threshold compare / select.
template <typename T>
struct SwQLut {
    static constexpr int kCols = 32;
    static constexpr int kRow = kCols * (int)sizeof(T);
    static constexpr int kBytes = kQRows * kRow;
};
// LDS bytes of the windowed kernels' max* table for ALGO (0: three-read exact, 1: none, 2: one-read)
template <typename T, int ALGO>
constexpr int sw_lut_bytes()
{
    return ALGO == 0 ? SwLut<T>::kBytes : (ALGO == 2 ? SwQLut<T>::kBytes : 16);
}

template <typename T, int ALGO>
__device__ __forceinline__ void sw_lut_fill(char* lut_s, const DecodeParams<T>& p)
{
    if constexpr (ALGO == 2) {
        using Lq = SwQLut<T>;
        for (int e = threadIdx.x; e < kQRows * Lq::kCols; e += blockDim.x)
            *reinterpret_cast<T*>(lut_s + (e / Lq::kCols) * Lq::kRow + (e % Lq::kCols) * (int)sizeof(T)) =
                p.qlut[e / Lq::kCols];
    } else if constexpr (ALGO == 0) {
        using Lt = SwLut<T>;
        for (int e = threadIdx.x; e < Lt::kRows * Lt::kCols; e += blockDim.x) {
            const int q = e / Lt::kCols, o = q * Lt::kRow + (e % Lt::kCols) * (int)sizeof(T);
            const LutEntry<T>& last = p.lut[kLutSize - 1];
            *reinterpret_cast<T*>(lut_s + o) = q < kLutSize ? (T)p.lut[q].thr : (T)INFINITY;
            *reinterpret_cast<T*>(lut_s + Lt::kOffV + o) = q < kLutSize ? (T)p.lut[q].vlo : (T)last.vhi;
            *reinterpret_cast<T*>(lut_s + Lt::kOffH + o) = q < kLutSize ? (T)p.lut[q].vhi : (T)last.vhi;
        }
    }
    __syncthreads();
}
// this lane's table origin: its column, shifted down by the first bucket's field value
template <typename T, int ALGO>
__device__ __forceinline__ const char* sw_lut_lane(const char* lut_s, int lane)
{
    if constexpr (ALGO == 2)
        return lut_s + (lane % SwQLut<T>::kCols) * (int)sizeof(T) - QBucketBits<T>::base * SwQLut<T>::kRow;
    return lut_s + (lane % SwLut<T>::kCols) * (int)sizeof(T) - BucketBits<T>::base * SwLut<T>::kRow;
}
// the one-read table's clamped row field of d (sign outside the field, as bucket_dev)
template <typename T>
__device__ __forceinline__ int qbucket_dev(T d)
{
    using QB = QBucketBits<T>;
    unsigned hi;
    if constexpr (sizeof(T) == 8)
        hi = (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
    else
        hi = (unsigned)__float_as_int(d);
    const int q = (int)__builtin_amdgcn_ubfe(hi, QB::shift, QB::width);
    return min(max(q, QB::base), QB::base + kQRows - 1);
}
// max* of the windowed schedule: ALGO 0 E_algorithm (log_map.cpp:779-801) in the exact bucket form of
// mstar; ALGO 1 max (Max-Log-MAP); ALGO 2 the one-read table (td_tables.h build_qlut)
template <typename T, int ALGO>
__device__ __forceinline__ T sw_mstar(T x, T y, const char* lut)
{
    if constexpr (ALGO == 1) {
        return vmax(x, y);
    } else if constexpr (ALGO == 2) {
        const T d = y - x;
        return vmax(x, y) + *reinterpret_cast<const T*>(lut + qbucket_dev<T>(d) * SwQLut<T>::kRow);
    } else {
        using Lt = SwLut<T>;
        const T d = y - x;
        const char* r = lut + bucket_dev<T>(d) * Lt::kRow;
        const T thr = *reinterpret_cast<const T*>(r);
        const T lo = *reinterpret_cast<const T*>(r + Lt::kOffV);
        const T hi = *reinterpret_cast<const T*>(r + Lt::kOffH);
        return vmax(x, y) + (fabs(d) >= thr ? hi : lo);
    }
}

// The windowed schedule's arrays are WIDE (round 5): [B/64][L][64] and [B/64][K][64], the 64 codewords
// of a wave adjacent per step, so a wave's load of one step is one 512-byte row (4 whole cache lines)
// and its extrinsic store one 512-byte row at the interleaved position.  (The exact schedule keeps its
// 8-codeword groups; sw_demux_kernel writes this layout.)  Round 4 read the 8-codeword layout: eight
// 64-byte pieces per wave load, half a cache line each.
constexpr int kSwCw = 64;
// cache policy of the windowed kernels' streams (TD_SW_NT bits): 1 checkpoint stores nt, 2 the beta
// kernel's checkpoint DMA sc0 sc1 nt, 4 its input DMA sc0 sc1 nt, 8 the alpha kernel's input loads nt,
// 16 the beta kernel's extrinsic stores nt.
// The checkpoints are written once and read once, a launch later: kept out of L2 / MALL (3) config 5
// runs 3410-3415 against 3335-3343 Mbit/s (+2.2 %, one box, 2 interleaved rounds); the inputs, which
// both kernels read, lose with nt (7: level, 15: -0.5 %; profiles/r06/ab_window_cache_policy.txt); the
// extrinsic stores with nt (19) another +1.6 % (3208-3210 against 3157-3160, profiles/r06/ab_extrinsic_nt.txt)
#ifndef TD_SW_NT
#define TD_SW_NT 19
#endif
template <typename T>
__device__ __forceinline__ void sw_ck_store(T* p, T v)
{
    if constexpr ((TD_SW_NT & 1) != 0)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <int BIT>
__device__ __forceinline__ void sw_dma(unsigned lds, const void* src)
{
    if constexpr ((TD_SW_NT & BIT) != 0)
        dma16_stream(lds, src);
    else
        dma16(lds, src);
}
// channel + a-priori of (codeword b, step i) of decoder `dec` (steps outside [0, L) clamped)
// A wave's 64 codewords are the wide group cwv (wave-uniform) and its lanes, so every address is a
// wave-uniform base plus the lane: no per-lane 64-bit pointer stays live across the loops (with the
// codeword index per lane the compiler hoisted one per array and the beta kernel spilled into AGPRs).
template <typename T>
__device__ __forceinline__ SwRaw<T> sw_raw(const DecodeParams<T>& p, const WinArgs<T>& a, int dec, int cwv, int lane,
                                          int i)
{
    const int ic = min(max(i, 0), p.L - 1);
    const size_t row = (size_t)cwv * p.L + ic, rowk = (size_t)cwv * p.K + min(ic, p.K - 1);
    SwRaw<T> r;
    if constexpr ((TD_SW_NT & 8) != 0) {
        r.ys = __builtin_nontemporal_load(&(dec ? p.sys2 : p.sys1)[row * kSwCw + lane]);
        r.yp = __builtin_nontemporal_load(&(dec ? p.par2 : p.par1)[row * kSwCw + lane]);
        r.la = __builtin_nontemporal_load(&a.la[dec][rowk * kSwCw + lane]);
    } else {
        r.ys = (dec ? p.sys2 : p.sys1)[row * kSwCw + lane];
        r.yp = (dec ? p.par2 : p.par1)[row * kSwCw + lane];
        r.la = a.la[dec][rowk * kSwCw + lane];
    }
    return r;
}
// the step's P, Q (see "gamma") with La zero where no extrinsic exists (la_ok: i < la_len)
template <typename T>
__device__ __forceinline__ SwIn<T> sw_cvt(const SwRaw<T>& r, bool la_ok)
{
    const T la = la_ok ? r.la : (T)0;
    const T hla = la / (T)2;
    return SwIn<T>{(r.ys + r.yp) + hla, (r.ys - r.yp) + hla, r.ys, la};
}

// gamma of the transition leaving state s with input u: +-(P or Q), see "gamma"
template <typename T>
__device__ __forceinline__ T sw_g(const SwIn<T>& x, int s)
{
    return kTrellisQ[s] ? x.Q : x.P;
}

// metrics -= their max (log_map.cpp:995-1000), every S positions of the chain's sub-block
template <typename T>
__device__ __forceinline__ void sw_normalise(T (&v)[8])
{
    const T m = vmax(vmax(vmax(v[0], v[1]), vmax(v[2], v[3])), vmax(vmax(v[4], v[5]), vmax(v[6], v[7])));
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] - m;
}

// alpha[.][i] -> alpha[.][i+1] (log_map.cpp:975-985)
template <typename T, int ALGO>
__device__ __forceinline__ void sw_alpha_step(T (&a)[8], const SwIn<T>& x, const char* lut)
{
    T n[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        n[j] = sw_mstar<T, ALGO>(a[p0] - sw_g(x, p0), a[p1] + sw_g(x, p1), lut);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = n[j];
}
// two independent chains on the same step: one code block, so their 16 max* interleave
template <typename T, int ALGO>
__device__ __forceinline__ void sw_alpha_step2(T (&a)[8], T (&c)[8], const SwIn<T>& x, const char* lut)
{
    T n[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        n[j] = sw_mstar<T, ALGO>(a[p0] - sw_g(x, p0), a[p1] + sw_g(x, p1), lut);
        m[j] = sw_mstar<T, ALGO>(c[p0] - sw_g(x, p0), c[p1] + sw_g(x, p1), lut);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = n[j];
        c[j] = m[j];
    }
}

// beta[.][i+1] -> beta[.][i] (log_map.cpp:1004-1016)
template <typename T, int ALGO>
__device__ __forceinline__ void sw_beta_step(T (&b)[8], const SwIn<T>& x, const char* lut)
{
    T n[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const T G = sw_g(x, j);
        n[j] = sw_mstar<T, ALGO>(b[kTrellisNext[j][0]] - G, b[kTrellisNext[j][1]] + G, lut);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = n[j];
}
template <typename T, int ALGO>
__device__ __forceinline__ void sw_beta_step2(T (&b)[8], T (&c)[8], const SwIn<T>& x, const char* lut)
{
    T n[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const T G = sw_g(x, j);
        n[j] = sw_mstar<T, ALGO>(b[kTrellisNext[j][0]] - G, b[kTrellisNext[j][1]] + G, lut);
        m[j] = sw_mstar<T, ALGO>(c[kTrellisNext[j][0]] - G, c[kTrellisNext[j][1]] + G, lut);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        b[j] = n[j];
        c[j] = m[j];
    }
}

// A scheduling fence between the positions of a fast segment: without it the scheduler hoists the
// next position's table reads into the current one and the beta kernel needs 298 VGPRs (one wave per
// SIMD); with it a position's live set is the per-position path's.
#ifndef TD_SW_FENCE
#define TD_SW_FENCE 1
#endif
__device__ __forceinline__ void sw_fence()
{
    if constexpr (TD_SW_FENCE) __builtin_amdgcn_sched_barrier(0);
}

// LLR of step i (log_map.cpp:1024-1039): the two left folds of E over the 8 next states
template <typename T, int ALGO>
__device__ __forceinline__ T sw_llr(const T (&a)[8], const T (&b)[8], const SwIn<T>& x, const char* lut)
{
    T t0[8], t1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
        t0[j] = (a[p0] - sw_g(x, p0)) + b[j];
        t1[j] = (a[p1] + sw_g(x, p1)) + b[j];
    }
    T r0 = sw_mstar<T, ALGO>(t0[0], t0[1], lut), r1 = sw_mstar<T, ALGO>(t1[0], t1[1], lut);
#pragma unroll
    for (int j = 2; j < 8; ++j) {
        r0 = sw_mstar<T, ALGO>(r0, t0[j], lut);
        r1 = sw_mstar<T, ALGO>(r1, t1[j], lut);
    }
    return r1 - r0;
}

template <typename T>
__device__ __forceinline__ void sw_set(T (&v)[8], int slot0_only, T x0)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (j == 0 || !slot0_only) ? x0 : (T)-kInfty;
}
// a chain's NII start metrics, waited for here: a load left pending past the (rare) branch that issues
// it made the compiler wait vmcnt(0) at every later use of the chain -- the next segment's prefetch
// included
template <typename T>
__device__ __forceinline__ void sw_load_nii(T (&v)[8], const T* src)
{
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(v[j]));
}

// the lane's task: decoder, run [s0, s1), codeword b (dead lanes of a partial wave compute on the
// last codeword and store nothing)
struct SwTask {
    int dec, s0, s1, cwv, b;
    bool live;
};
template <typename T>
__device__ __forceinline__ bool sw_task(const DecodeParams<T>& p, const WinArgs<T>& a, SwTask& t)
{
    const int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const int cw_waves = a.ncw, per_dec = a.nR * cw_waves;
    if (wv >= (a.dec < 0 ? 2 : 1) * per_dec) return false;
    t.dec = a.dec < 0 ? wv / per_dec : a.dec;
    const int r = wv % per_dec;
    t.cwv = a.cw0 + r % cw_waves;   // absolute wave of 64 codewords
    t.s0 = (r / cw_waves) * a.M;
    t.s1 = min(t.s0 + a.M, a.nS);
    // padding lanes (b >= B) decode the zeros the demux wrote for them: every array they store to is
    // sized for whole waves (Bp), and only the Le dump, sized B, skips them
    t.b = t.cwv * 64 + (threadIdx.x & 63);
    t.live = t.b < p.B;
    return true;
}


// a use of v that the compiler must wait for (s_waitcnt on its load) before anything after this
// statement, memory operations included
template <typename T>
__device__ __forceinline__ void sw_wait_on(const T& v)
{
    asm volatile("" ::"v"(v) : "memory");
}

__device__ __forceinline__ int sw_end(int s, int nS, int W, int L) { return s == nS - 1 ? L : (s + 1) * W; }
__device__ __forceinline__ int floor_div(int x, int m) { return x >= 0 ? x / m : -((-x + m - 1) / m); }

template <typename T>
__device__ __forceinline__ T* sw_ck(const WinArgs<T>& a, const SwTask& t, int s, int c)
{
    return a.ckpt[t.dec] + (((size_t)s * (a.Bp >> 6) + t.cwv) * a.ncp + c) * 512 + (threadIdx.x & 63);
}

// ---- alpha: forward over the run, checkpoints every S positions of each sub-block
// (s_setprio 2 on the alpha waves, to issue ahead of a co-resident beta wave, measured level: not kept)
#ifndef TD_SW_ALPHA_WAVES
#define TD_SW_ALPHA_WAVES 0
#endif
#if TD_SW_ALPHA_WAVES
#define TD_SW_ALPHA_ATTR __attribute__((amdgpu_waves_per_eu(TD_SW_ALPHA_WAVES)))
#else
#define TD_SW_ALPHA_ATTR
#endif
template <typename T, int ALGO, int S>
__global__ __launch_bounds__(256) TD_SW_ALPHA_ATTR void sw_alpha_kernel(DecodeParams<T> p, WinArgs<T> a)
{
    __shared__ alignas(16) char lut_s[sw_lut_bytes<T, ALGO>()];
    if constexpr (ALGO != 1) sw_lut_fill<T, ALGO>(lut_s, p);
    SwTask t;
    if (!sw_task(p, a, t)) return;
    const int lane = threadIdx.x & 63;
    const char* lut = sw_lut_lane<T, ALGO>(lut_s, lane);
    const int W = a.W, g = a.g, nS = a.nS, L = p.L, dec = t.dec, cwv = t.cwv;
    T* const niw = a.nii_wr + ((size_t)dec * a.Bp + t.b) * nS * 16;
    const T* const nir = a.nii_rd + ((size_t)dec * a.Bp + t.b) * nS * 16;
    const bool use_nii = a.nii && a.it > 0;
    const int base0 = t.s0 * W;

    // the chain of sub-block s0 starts at i0 (clamped to 0)
    T al[8], bl[8];
    const int i0 = base0 - g;
    if (i0 <= 0)
        sw_set(al, 1, (T)0);
    else if (use_nii)
        sw_load_nii(al, nir + (size_t)t.s0 * 16);
    else
        sw_set(al, 0, (T)0);
    sw_set(bl, 0, (T)0);
    const int ps = max(i0, 0);

    // per sub-block bookkeeping (wave-uniform)
    int s = t.s0, st = 0, en = 0, qb = 0, need = 0;
    bool hasB = false;
    auto enter = [&](int ns) {
        s = ns;
        st = s * W;
        en = sw_end(s, nS, W, L);
        hasB = s + 1 < t.s1;                     // the next sub-block's chain runs in this lane
        qb = st + W - g;                         // its start = the NII alpha position of s+1
        const int lc = st + ((en - st - 1) / S) * S;   // last checkpoint
        need = s < nS - 1 ? max(lc, qb) : lc;    // alpha wanted up to here
    };
    enter(t.s0);
    if (s < nS - 1 && qb < 0 && t.live)          // (g > W) the NII position lies before step 0
#pragma unroll
        for (int j = 0; j < 8; ++j) niw[(size_t)(s + 1) * 16 + j] = j == 0 ? (T)0 : (T)-kInfty;
    const int stop = [&] {                        // the run's last position with work
        const int sl = t.s1 - 1, stl = sl * W, enl = sw_end(sl, nS, W, L);
        const int lc = stl + ((enl - stl - 1) / S) * S;
        return sl < nS - 1 ? max(lc, stl + W - g) : lc;
    }();

    int bp = base0 + floor_div(ps - base0, S) * S;
    SwRaw<T> nx[S];
#pragma unroll
    for (int m = 0; m < S; ++m) nx[m] = sw_raw(p, a, dec, cwv, lane, bp + m);
    for (; bp <= stop; bp += S) {
        // the segment's inputs from the prefetch registers, then the next segment's loads into them
        // (converting first keeps one copy of them live: no register moves at the loop edge)
        SwIn<T> x[S];
#pragma unroll
        for (int m = 0; m < S; ++m) x[m] = sw_cvt(nx[m], bp + m < a.la_len);
#pragma unroll
        for (int m = 0; m < S; ++m) nx[m] = sw_raw(p, a, dec, cwv, lane, bp + S + m);
        // Fast segments (all but about one in eight): whole, no chain start or NII position inside, each
        // chain stepping at every position or at none -- one straight block, the two chains' max*
        // interleaved.  The others take the per-position path below.
        const bool qin = (hasB || s < nS - 1) && qb >= bp && qb < bp + S;
        const bool aAll = bp + S <= need, aNone = bp >= need;
        const bool bAll = hasB && bp > qb, bNone = !hasB || bp + S <= qb;
        if (bp >= ps && bp + S - 1 <= stop && !qin && (aAll || aNone) && (bAll || bNone) && !(aNone && bNone)) {
            if (bp >= st) {                               // checkpoint alpha[bp] (normalised)
                T* ck = sw_ck(a, t, s, (bp - st) / S);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if constexpr (!kDiag<kDiagSwNoCk>) sw_ck_store(ck + j * 64, al[j]);
            }
            if (aAll && bAll) {
#pragma unroll
                for (int m = 0; m < S; ++m) {
                    sw_alpha_step2<T, ALGO>(al, bl, x[m], lut);
                    sw_fence();
                }
                sw_normalise(al);
                sw_normalise(bl);
            } else if (aAll) {
#pragma unroll
                for (int m = 0; m < S; ++m) {
                    sw_alpha_step<T, ALGO>(al, x[m], lut);
                    sw_fence();
                }
                sw_normalise(al);
            } else {
#pragma unroll
                for (int m = 0; m < S; ++m) {
                    sw_alpha_step<T, ALGO>(bl, x[m], lut);
                    sw_fence();
                }
                sw_normalise(bl);
            }
        } else {
            // sub-block s+1's chain starts at qb: set once at the segment's start (the positions below qb
            // leave it alone), as a branch, not per-position selects (see the beta kernel)
            if (hasB && qb >= bp && qb < bp + S && qb >= ps && qb <= stop) {
                asm volatile("" ::: "memory");
                if (qb <= 0)
                    sw_set(bl, 1, (T)0);
                else if (use_nii)
                    sw_load_nii(bl, nir + (size_t)(s + 1) * 16);
                else
                    sw_set(bl, 0, (T)0);
            }
#pragma unroll
            for (int m = 0; m < S; ++m) {
                const int pos = bp + m;
                if (pos < ps || pos > stop) continue;
                if (m == 0 && pos >= st && pos < en) {       // checkpoint alpha[pos] (normalised)
                    T* ck = sw_ck(a, t, s, (pos - st) / S);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if constexpr (!kDiag<kDiagSwNoCk>) sw_ck_store(ck + j * 64, al[j]);
                }
                if (s < nS - 1 && pos == qb && t.live)
#pragma unroll
                    for (int j = 0; j < 8; ++j) niw[(size_t)(s + 1) * 16 + j] = al[j];
                const bool doA = pos < need, doB = hasB && pos >= qb;
                if (doA && doB)
                    sw_alpha_step2<T, ALGO>(al, bl, x[m], lut);
                else if (doA)
                    sw_alpha_step<T, ALGO>(al, x[m], lut);
                else if (doB)
                    sw_alpha_step<T, ALGO>(bl, x[m], lut);
                if (m == S - 1) {                            // alpha[bp + S]: an aligned position
                    if (doA) sw_normalise(al);
                    if (doB) sw_normalise(bl);
                }
            }
        }
        if (hasB && bp + S == en) {                      // hand over to sub-block s+1
            if (qb >= en) {                              // g = 0: its chain starts at its first position
                if (t.live)                              // (alpha[en] of this chain is its NII metric)
#pragma unroll
                    for (int j = 0; j < 8; ++j) niw[(size_t)(s + 1) * 16 + j] = al[j];
                if (use_nii)
                    sw_load_nii(bl, nir + (size_t)(s + 1) * 16);
                else
                    sw_set(bl, 0, (T)0);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) al[j] = bl[j];
            enter(s + 1);
        }
    }
}

// ---- alpha for a batch of one codeword (the drop-in's frame): the chain's 8 states across 8 lanes
// (state j in lane j of each group of 8 lanes; the groups mirror each other, lanes 0-7 store), the two
// predecessors fetched by ds_bpermute.  A lone sw_alpha_kernel wave issues a step's 8 max* from one lane
// (about 650 cycles a step); here each lane does one.  Per state the operations and their order are
// sw_alpha_step's; the normalising max (sw_normalise) is exact in any order.
template <typename T>
__device__ __forceinline__ T sw_lane_get(T v, int src)   // v of lane src
{
    if constexpr (sizeof(T) == 8) {
        const long long w = __double_as_longlong((double)v);
        const int lo = __builtin_amdgcn_ds_bpermute(src * 4, (int)w);
        const int hi = __builtin_amdgcn_ds_bpermute(src * 4, (int)(w >> 32));
        return (T)__longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
    } else {
        return (T)__int_as_float(__builtin_amdgcn_ds_bpermute(src * 4, __float_as_int((float)v)));
    }
}
constexpr unsigned sw_pack_last(int u)   // kTrellisLast[.][u] as 8 nibbles (runtime-indexable)
{
    unsigned r = 0;
    for (int j = 0; j < 8; ++j) r |= (unsigned)kTrellisLast[j][u] << (4 * j);
    return r;
}
constexpr unsigned sw_pack_q()           // kTrellisQ as 8 bits
{
    unsigned r = 0;
    for (int j = 0; j < 8; ++j) r |= (kTrellisQ[j] ? 1u : 0u) << j;
    return r;
}
constexpr unsigned sw_pack_next(int u)   // kTrellisNext[.][u] as 8 nibbles
{
    unsigned r = 0;
    for (int j = 0; j < 8; ++j) r |= (unsigned)kTrellisNext[j][u] << (4 * j);
    return r;
}
constexpr unsigned kSwLast0 = sw_pack_last(0), kSwLast1 = sw_pack_last(1), kSwQ = sw_pack_q();
constexpr unsigned kSwNext0 = sw_pack_next(0), kSwNext1 = sw_pack_next(1);
constexpr int kSwLpsChunk = 160;   // sw_alpha_lps_kernel's input chunk (positions): W + 2g + S of config 5 in fp32
struct SwLps {
    int j, p0, p1;   // this lane's state; its two predecessors' lanes
    bool q0, q1;     // their gammas take Q (kTrellisQ)
};
template <typename T, int ALGO>
__device__ __forceinline__ T sw_lps_step(T v, const SwIn<T>& x, const SwLps& l, const char* lut)
{
    const T u0 = sw_lane_get(v, l.p0), u1 = sw_lane_get(v, l.p1);
    return sw_mstar<T, ALGO>(u0 - (l.q0 ? x.Q : x.P), u1 + (l.q1 ? x.Q : x.P), lut);
}
template <typename T>
__device__ __forceinline__ T sw_lps_norm(T v, int lane)
{
    T m = vmax(v, sw_lane_get(v, lane ^ 1));
    m = vmax(m, sw_lane_get(m, lane ^ 2));
    m = vmax(m, sw_lane_get(m, lane ^ 4));
    return v - m;
}

template <typename T, int ALGO, int S>
__global__ __launch_bounds__(256) void sw_alpha_lps_kernel(DecodeParams<T> p, WinArgs<T> a)
{
    __shared__ alignas(16) char lut_s[sw_lut_bytes<T, ALGO>()];
    __shared__ T lin_s[4][3][kSwLpsChunk];   // per wave: codeword 0's ys, yp, La of a chunk of positions
    if constexpr (ALGO != 1) sw_lut_fill<T, ALGO>(lut_s, p);
    SwTask t;
    if (!sw_task(p, a, t)) return;
    const int lane = threadIdx.x & 63;
    const char* lut = sw_lut_lane<T, ALGO>(lut_s, lane);
    T (&lin)[3][kSwLpsChunk] = lin_s[threadIdx.x >> 6];
    SwLps l;
    l.j = lane & 7;
    l.p0 = (lane & ~7) + (int)((kSwLast0 >> (4 * l.j)) & 7);
    l.p1 = (lane & ~7) + (int)((kSwLast1 >> (4 * l.j)) & 7);
    l.q0 = (kSwQ >> (l.p0 & 7)) & 1;
    l.q1 = (kSwQ >> (l.p1 & 7)) & 1;
    const int W = a.W, g = a.g, nS = a.nS, L = p.L, dec = t.dec, cwv = t.cwv, b0 = cwv * 64;
    const bool wr = lane < 8 && b0 < p.B;          // lanes 0-7 store codeword 0's states
    T* const niw = a.nii_wr + ((size_t)dec * a.Bp + b0) * nS * 16;
    const T* const nir = a.nii_rd + ((size_t)dec * a.Bp + b0) * nS * 16;
    const bool use_nii = a.nii && a.it > 0;
    const int base0 = t.s0 * W;
    auto set = [&](bool slot0_only, T x0) -> T { return (l.j == 0 || !slot0_only) ? x0 : (T)-kInfty; };
    auto load_nii = [&](const T* src) -> T {
        T v = src[l.j];
        asm volatile("" ::"v"(v));
        return v;
    };

    T al, bl;
    const int i0 = base0 - g;
    if (i0 <= 0)
        al = set(true, (T)0);
    else if (use_nii)
        al = load_nii(nir + (size_t)t.s0 * 16);
    else
        al = set(false, (T)0);
    bl = set(false, (T)0);
    const int ps = max(i0, 0);

    int s = t.s0, st = 0, en = 0, qb = 0, need = 0;
    bool hasB = false;
    auto enter = [&](int ns) {
        s = ns;
        st = s * W;
        en = sw_end(s, nS, W, L);
        hasB = s + 1 < t.s1;
        qb = st + W - g;
        const int lc = st + ((en - st - 1) / S) * S;
        need = s < nS - 1 ? max(lc, qb) : lc;
    };
    enter(t.s0);
    if (s < nS - 1 && qb < 0 && wr) niw[(size_t)(s + 1) * 16 + lane] = lane == 0 ? (T)0 : (T)-kInfty;
    const int stop = [&] {
        const int sl = t.s1 - 1, stl = sl * W, enl = sw_end(sl, nS, W, L);
        const int lc = stl + ((enl - stl - 1) / S) * S;
        return sl < nS - 1 ? max(lc, stl + W - g) : lc;
    }();
    auto ck_store = [&](int c) {                     // checkpoint alpha (normalised), column of codeword 0
        if (wr) (sw_ck(a, t, s, c) - lane)[lane * 64] = al;
    };
    // a.hand (one sub-block a lane): lanes 8-15 run this sub-block's beta warm-up chain, positions
    // en + g - 1 down to en, beside alpha -- the same exchange-and-max* step with the beta trellis
    // (sw_beta_step: b[next0] - G, b[next1] + G, G = gamma of the state), normalised where the beta
    // kernel normalises it -- and leave beta[en] in column 1 of the sub-block's first checkpoint slot
    // (unused with one codeword), where sw_beta_kernel<LF> starts from it.
    const bool hand = a.hand && s < nS - 1;
    const bool wl = hand && (lane >> 3) == 1;
    const int nw = hand ? g : 0;
    int kw = 0;
    if (wl) {
        l.p0 = 8 + (int)((kSwNext0 >> (4 * l.j)) & 7);
        l.p1 = 8 + (int)((kSwNext1 >> (4 * l.j)) & 7);
        l.q0 = l.q1 = (kSwQ >> l.j) & 1;
    }
    if (hand) {
        const T w0 = use_nii ? nir[(size_t)s * 16 + 8 + l.j] : (T)0;   // the chain of s starts at en + g
        if (wl) al = w0;
    }

    int bp = base0 + floor_div(ps - base0, S) * S;
    // The inputs come a chunk of kSwLpsChunk positions at a time into LDS, every lane loading its share
    // at once: one memory latency a chunk.  (A lone wave's steps are short enough here that loads issued
    // one segment ahead were waited for at every segment.)
    int c0 = bp, c1 = bp;                            // the chunk [c0, c1) in lin
    auto load_chunk = [&](int from) {
        c0 = from;
        c1 = from + kSwLpsChunk;
        for (int k = lane; k < kSwLpsChunk; k += 64) {
            const SwRaw<T> r = sw_raw(p, a, dec, cwv, 0, c0 + k);
            lin[0][k] = r.ys;
            lin[1][k] = r.yp;
            lin[2][k] = r.la;
        }
        __builtin_amdgcn_wave_barrier();
    };
    static_assert(kSwLpsChunk % S == 0, "whole segments a chunk");
    for (; bp <= stop; bp += S) {
        if (bp >= c1) load_chunk(bp);
        SwIn<T> x[S];
#pragma unroll
        for (int m = 0; m < S; ++m) {
            const SwRaw<T> r{lin[0][bp - c0 + m], lin[1][bp - c0 + m], lin[2][bp - c0 + m]};
            x[m] = sw_cvt(r, bp + m < a.la_len);
        }
        if (hasB && qb >= bp && qb < bp + S && qb >= ps && qb <= stop) {
            asm volatile("" ::: "memory");
            if (qb <= 0)
                bl = set(true, (T)0);
            else if (use_nii)
                bl = load_nii(nir + (size_t)(s + 1) * 16);
            else
                bl = set(false, (T)0);
        }
#pragma unroll
        for (int m = 0; m < S; ++m) {
            const int pos = bp + m;
            if (pos < ps || pos > stop) continue;
            if (m == 0 && pos >= st && pos < en) ck_store((pos - st) / S);
            if (s < nS - 1 && pos == qb && wr) niw[(size_t)(s + 1) * 16 + lane] = al;
            const bool doA = pos < need, doB = hasB && pos >= qb;
            const bool wact = kw < nw;
            const int pw = en + g - 1 - kw;                  // the warm-up chain's position
            T na = al, nbv = bl;
            if (doA || wact) {
                SwIn<T> xs = x[m];
                if (wact) {
                    const int iw = min(max(pw - c0, 0), kSwLpsChunk - 1);
                    const SwRaw<T> r{lin[0][iw], lin[1][iw], lin[2][iw]};
                    const SwIn<T> xw = sw_cvt(r, pw < a.la_len);
                    if (wl) xs = xw;
                }
                const T n = sw_lps_step<T, ALGO>(al, xs, l, lut);
                if (wl ? wact : doA) na = n;
            }
            if (doB) nbv = sw_lps_step<T, ALGO>(bl, x[m], l, lut);
            al = na;
            bl = nbv;
            const bool nA = m == S - 1 && doA, nW = wact && (pw - base0) % S == 0;
            if (nA || nW) {
                const T nv = sw_lps_norm(al, lane);
                if (wl ? nW : nA) al = nv;
            }
            if (m == S - 1 && doB) bl = sw_lps_norm(bl, lane);
            if (wact) ++kw;
        }
        if (hasB && bp + S == en) {
            if (qb >= en) {
                if (wr) niw[(size_t)(s + 1) * 16 + lane] = al;
                if (use_nii)
                    bl = load_nii(nir + (size_t)(s + 1) * 16);
                else
                    bl = set(false, (T)0);
            }
            al = bl;
            enter(s + 1);
        }
    }
    if (wl && b0 < p.B) (sw_ck(a, t, s, 0) - lane)[l.j * 64 + 1] = al;   // beta[en] for sw_beta_kernel<LF>
}

// ---- beta + LLR: backward over the run in segments of S positions
#ifndef TD_SW_BETA_WAVES
#define TD_SW_BETA_WAVES 0
#endif
#if TD_SW_BETA_WAVES
#define TD_SW_BETA_ATTR __attribute__((amdgpu_waves_per_eu(TD_SW_BETA_WAVES)))
#else
#define TD_SW_BETA_ATTR
#endif
// LF (lane folds; a batch of one codeword, the drop-in's frame): every lane of the wave runs codeword
// 0's chains, and the S LLRs of a segment are folded side by side, position m in lane m, once the
// segment's beta steps are done -- one fold latency a segment instead of S (the folds are the beta
// kernel's longest dependent chains: 2 x 7 table max* a position).  Same operations, same order.
template <typename T, int ALGO, int S, bool LF>
__global__ __launch_bounds__(256) TD_SW_BETA_ATTR void sw_beta_kernel(DecodeParams<T> p, WinArgs<T> a, const int* __restrict__ pi,
                                                      const int* __restrict__ pinv)
{
    __shared__ alignas(16) char lut_s[sw_lut_bytes<T, ALGO>()];
    __shared__ alignas(16) T ck_lds[4 * 8 * 64];   // per wave: the next segment's checkpoint (DMA slot)
    __shared__ alignas(16) T in_lds[4 * 3 * S * 64];   // per wave: the next segment's ys, yp, La rows (DMA slot)
    __shared__ alignas(16) int ix_lds[4 * 64];         // per wave: the next segment's interleaver entries (DMA slot)
    if constexpr (ALGO != 1) sw_lut_fill<T, ALGO>(lut_s, p);
    SwTask t;
    if (!sw_task(p, a, t)) return;
    const int lane = threadIdx.x & 63;
    const char* lut = sw_lut_lane<T, ALGO>(lut_s, lane);
    const int W = a.W, g = a.g, nS = a.nS, L = p.L, K = p.K, dec = t.dec, cwv = t.cwv;
    const int col = LF ? 0 : lane;                // this lane's codeword within the wave
    const int b = LF ? t.cwv * 64 : t.b;
    T* const niw = a.nii_wr + ((size_t)dec * a.Bp + b) * nS * 16;
    const T* const nir = a.nii_rd + ((size_t)dec * a.Bp + b) * nS * 16;
    const bool use_nii = a.nii && a.it > 0;
    const int base0 = t.s0 * W;
    const int* const perm = dec ? pi : pinv;
    T* const le = a.le[dec] + (size_t)cwv * K * kSwCw;
    uint8_t* const bitsT = dec ? a.bitsT : nullptr;
    uint8_t* const bits1 = LF && dec ? a.bits1 : nullptr;
    const int bcol = LF ? t.cwv * 64 : t.cwv * 64 + lane;
    // clock sample (as turbo_decode_kernel's): workgroup 0's shader clock and 100 MHz counter at its
    // start and end, two scalar reads each, written by its first lane with one vector store
    const bool clk = a.clk && p.clk && blockIdx.x == 0;
    unsigned long long clk_c0 = 0, clk_r0 = 0;
    if (clk) {
        clk_c0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
    }

    int s = t.s1 - 1, st = 0, en = 0, qb = 0;
    bool hasB = false;
    auto enter = [&](int ns) {
        s = ns;
        st = s * W;
        en = sw_end(s, nS, W, L);
        hasB = s > t.s0;                          // the previous sub-block's chain runs in this lane
        qb = min(st + g, L);                      // its start (= the NII beta position of s-1)
    };
    enter(t.s1 - 1);
    // the chain of sub-block s1-1 starts at e = end + g (clamped to L)
    T be[8], bb[8];
    const int e = en + g;
    if (e >= L)
        sw_set(be, 1, (T)0);
    else if (use_nii)
        sw_load_nii(be, nir + (size_t)s * 16 + 8);
    else
        sw_set(be, 0, (T)0);
    sw_set(bb, 0, (T)0);
    if (s > 0 && st + g >= L && t.live)           // NII position at or past L: the terminated state
#pragma unroll
        for (int j = 0; j < 8; ++j) niw[(size_t)(s - 1) * 16 + 8 + j] = j == 0 ? (T)0 : (T)-kInfty;
    const int pe = min(e, L) - 1;                 // first position stepped

    // Segment prefetch, one segment ahead, all of it by DMA into this wave's LDS slots
    // (global_load_lds_dwordx4, 1 KB a wave instruction): the segment's three input rows (ys, yp, La:
    // S consecutive 64-codeword rows each, contiguous in the wide layout) and, for a segment of a
    // sub-block's own range, its checkpoint (8 x 64 lane-contiguous values).  Nothing in flight sits in
    // a VGPR: with the inputs loaded into registers the allocator copied a pending load into the
    // loop-carried register right after issuing it, so the wave waited for the prefetch it had just
    // issued (vmcnt) in every segment.  Rows past the array ends stay inside the workspace (td_api.cpp:
    // kWideSlack); their values are never used (positions >= L are not stepped, La >= K is masked).
    // Ordering: the extrinsic / decision stores of a segment are issued at the start of the next one,
    // before its DMA, so one `s_waitcnt vmcnt(0)` at each segment start covers exactly this segment's
    // DMA and the stores before it, all issued a segment earlier.
    auto seg_sub = [&](int sbp) {                 // sub-block whose chain covers segment sbp
        return sbp >= en ? s : min(t.s0 + (sbp - base0) / W, t.s1 - 1);
    };
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    T* const ckslot = ck_lds + wave * 8 * 64;
    T* const inslot = in_lds + wave * 3 * S * 64;
    const unsigned ckslot_lds = __builtin_amdgcn_readfirstlane(lds_addr(ckslot));   // DMA bases (M0): wave-uniform
    const unsigned inslot_lds = __builtin_amdgcn_readfirstlane(lds_addr(inslot));
    constexpr int kRowBytes = kSwCw * (int)sizeof(T);
    constexpr int kInDma = S * kRowBytes / 1024;                    // DMA instructions per input array
    static_assert(S * kRowBytes % 1024 == 0, "whole 1 KB DMA chunks");
    int bp = base0 + floor_div(pe - base0, S) * S;
    if constexpr (LF) {
        // a.hand: sw_alpha_lps_kernel ran this chain's warm-up and left beta[en] in column 1 of the
        // sub-block's first checkpoint slot; start at the sub-block's last segment from it
        if (a.hand && s < nS - 1) {
            const T* hb = sw_ck(a, t, s, 0) - lane + 1;
#pragma unroll
            for (int j = 0; j < 8; ++j) be[j] = hb[j * 64];
            bp = en - S;
        }
    }
    // the segment's interleaver entries (wave-uniform: scalar loads), one segment ahead
    int* const ixslot = ix_lds + wave * 64;                           // the next segment's perm / pi entries
    const unsigned ixslot_lds = __builtin_amdgcn_readfirstlane(lds_addr(ixslot));
    auto prefetch = [&](int nbp) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // the slots' previous reads are done
        // The interleaver entries by DMA too (lane l < S: perm, S <= l < 2S: pi, of position nbp + l % S),
        // waited for with the rest at the next segment's start.  As scalar loads they were waited out at
        // the lgkmcnt(0) above or at the first table read after it (scalar loads complete out of order,
        // so while one is in flight every LDS wait of the wave is an lgkmcnt(0)).
        dma4(ixslot_lds, (lane & S ? pi : perm) + min(nbp + (lane & (S - 1)), K - 1));
        const int ns = seg_sub(nbp), nst = ns * W;
        if (nbp >= base0 && nbp < sw_end(ns, nS, W, L)) {
            const char* src = reinterpret_cast<const char*>(sw_ck(a, t, ns, (nbp - nst) / S) - lane) + lane * 16;
            constexpr int kDma = 8 * 64 * (int)sizeof(T) / 1024;
#pragma unroll
            for (int q = 0; q < kDma; ++q)
                if constexpr (!kDiag<kDiagSwNoCk>) sw_dma<2>(ckslot_lds + q * 1024, src + q * 1024);
        }
        const size_t row = (size_t)cwv * L + nbp, rowk = (size_t)cwv * K + nbp;
        const char* src0 = reinterpret_cast<const char*>((dec ? p.sys2 : p.sys1) + row * kSwCw) + lane * 16;
        const char* src1 = reinterpret_cast<const char*>((dec ? p.par2 : p.par1) + row * kSwCw) + lane * 16;
        const char* src2 = reinterpret_cast<const char*>(a.la[dec] + rowk * kSwCw) + lane * 16;
#pragma unroll
        for (int q = 0; q < kInDma; ++q) {
            sw_dma<4>(inslot_lds + q * 1024, src0 + q * 1024);
            sw_dma<4>(inslot_lds + S * kRowBytes + q * 1024, src1 + q * 1024);
            sw_dma<4>(inslot_lds + 2 * S * kRowBytes + q * 1024, src2 + q * 1024);
        }
    };
    prefetch(bp);
    // the previous segment's extrinsics and decisions, stored at the start of the next one
    T dlev[S];
    int dbit[S], dpm[S], dpk[S];
    bool dst[S];
#pragma unroll
    for (int m = 0; m < S; ++m) dst[m] = false;
    // LF: lane m < S keeps position m's extrinsic, decision and write positions
    T lf_lev = 0;
    int lf_bit = 0, lf_pm = 0, lf_pk = 0, cur_pm = 0, cur_pk = 0;
    bool lf_st = false;
    auto flush = [&] {
        if constexpr (LF) {
            if (lf_st) {
                le[(size_t)lf_pm * kSwCw] = lf_lev;
                if (bitsT) bitsT[(size_t)lf_pk * a.Bp + bcol] = (uint8_t)lf_bit;
                if (bits1) bits1[lf_pk] = (uint8_t)lf_bit;
            }
        } else {
#pragma unroll
            for (int m = 0; m < S; ++m)
                if (dst[m] && t.live) {
                    if constexpr ((TD_SW_NT & 16) != 0)
                        __builtin_nontemporal_store(dlev[m], &le[(size_t)dpm[m] * kSwCw + lane]);
                    else
                        le[(size_t)dpm[m] * kSwCw + lane] = dlev[m];
                    if (bitsT) bitsT[(size_t)dpk[m] * a.Bp + bcol] = (uint8_t)dbit[m];
                }
        }
    };
    int pm[S], pk[S];
    // one position's LLR, extrinsic and decision (beta = beta[pos + 1]), kept for the flush
    auto llr_out = [&](int pos, const T (&al)[8], const SwIn<T>& xm, int m) {
        const T llr = sw_llr<T, ALGO>(al, be, xm, lut);
        const T lev = (llr - xm.la - (T)2 * xm.ys) * a.ext_scale;
        dlev[m] = lev;
        dbit[m] = llr < (T)0 ? 0 : 1;
        dst[m] = pos < K;
        if (p.le_dump && t.live) p.le_dump[(size_t)b * p.iters * 2 * L + (size_t)(2 * a.it + dec) * L + pos] = lev;
    };
    for (; bp >= base0; bp -= S) {
        SwIn<T> x[S];
        T as[S][8];
        const bool main = bp < en;                        // the segment lies in sub-block s's own range
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this segment's DMA (and the stores before it)
        flush();
        if constexpr (LF) {
            lf_st = false;
            cur_pm = ixslot[lane & (S - 1)];          // lane m: position m's write positions
            cur_pk = ixslot[S + (lane & (S - 1))];
        }
#pragma unroll
        for (int m = 0; m < S; ++m) {
            SwRaw<T> r;
            r.ys = inslot[m * 64 + col];
            r.yp = inslot[(S + m) * 64 + col];
            r.la = inslot[(2 * S + m) * 64 + col];
            x[m] = sw_cvt(r, bp + m < a.la_len);
            pm[m] = __builtin_amdgcn_readfirstlane(ixslot[m]);
            pk[m] = __builtin_amdgcn_readfirstlane(ixslot[S + m]);
            dst[m] = false;
            dpm[m] = pm[m];
            dpk[m] = pk[m];
        }
        if (main)
#pragma unroll
            for (int j = 0; j < 8; ++j) as[0][j] = ckslot[j * 64 + col];
        if (bp - S >= base0) prefetch(bp - S);
        if (main) {                                       // alpha of the segment from its checkpoint
#pragma unroll
            for (int m = 1; m < S; ++m) {                 // (past en in the last segment: computed, unused)
#pragma unroll
                for (int j = 0; j < 8; ++j) as[m][j] = as[m - 1][j];
                sw_alpha_step<T, ALGO>(as[m], x[m - 1], lut);
                sw_fence();
            }
        }
        const int nb = st + g;                            // NII beta position of s-1
        // Sub-block s-1's chain starts at qb (its first step at qb - 1).  Its metrics are set once at
        // the segment's start: the positions above qb - 1 leave them alone, so this equals setting
        // them at qb - 1.  A branch, not a select (the empty asm keeps the compiler from if-converting
        // it into 16 v_cndmask + 16 v_mov at every position: 8 % of the kernel's VALU).
        if (hasB && qb - 1 >= bp && qb - 1 < bp + S && qb - 1 <= pe) {
            asm volatile("" ::: "memory");
            if (qb >= L)
                sw_set(bb, 1, (T)0);
            else if (use_nii)
                sw_load_nii(bb, nir + (size_t)(s - 1) * 16 + 8);
            else
                sw_set(bb, 0, (T)0);
        }
        T asel[LF ? 8 : 1], bsel[LF ? 8 : 1];           // LF: lane m's position's alpha, beta[pos + 1], inputs
        SwIn<T> xsel{};
        bool sel = false;
#pragma unroll
        for (int m = S - 1; m >= 0; --m) {
            const int pos = bp + m;
            if (pos > pe) continue;
            if constexpr (LF) {
                if (main && pos < en && lane == m) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        asel[j] = as[m][j];
                        bsel[j] = be[j];
                    }
                    xsel = x[m];
                    sel = true;
                }
            } else if (main && pos < en) {
                llr_out(pos, as[m], x[m], m);
            }
            const bool doB = hasB && pos < qb;
            if (doB)
                sw_beta_step2<T, ALGO>(be, bb, x[m], lut);
            else
                sw_beta_step<T, ALGO>(be, x[m], lut);
            if (m == 0) {                                 // beta[bp]: an aligned position
                sw_normalise(be);
                if (doB) sw_normalise(bb);
            }
            if (s > 0 && pos == nb && t.live)
#pragma unroll
                for (int j = 0; j < 8; ++j) niw[(size_t)(s - 1) * 16 + 8 + j] = be[j];
        }
        if constexpr (LF) {                               // the segment's S folds, one per lane
            if (!sel)
#pragma unroll
                for (int j = 0; j < 8; ++j) asel[j] = bsel[j] = (T)0;   // (computed and dropped)
            const T llr = sw_llr<T, ALGO>(asel, bsel, xsel, lut);
            const T lev = (llr - xsel.la - (T)2 * xsel.ys) * a.ext_scale;
            const int pos = bp + lane;
            lf_lev = lev;
            lf_bit = llr < (T)0 ? 0 : 1;
            lf_pm = cur_pm;
            lf_pk = cur_pk;
            lf_st = sel && pos < K && b < p.B;
            if (p.le_dump && sel && b < p.B)
                p.le_dump[(size_t)b * p.iters * 2 * L + (size_t)(2 * a.it + dec) * L + pos] = lev;
        }
        if (hasB && bp == st) {                           // hand over to sub-block s-1
            if (qb <= st) {                               // g = 0: its chain starts at its end
                if (use_nii)
                    sw_load_nii(bb, nir + (size_t)(s - 1) * 16 + 8);
                else
                    sw_set(bb, 0, (T)0);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) be[j] = bb[j];
            enter(s - 1);
            if (s > 0 && st + g == en && t.live)          // g = W: the NII position is this chain's start
#pragma unroll
                for (int j = 0; j < 8; ++j) niw[(size_t)(s - 1) * 16 + 8 + j] = be[j];
        }
    }
    flush();
    if (clk) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) *reinterpret_cast<ulonglong4*>(p.clk) = make_ulonglong4(clk_c0, clk_r0, c1, r1);
    }
}

// Demultiplex + x0.5 (log_map.cpp:1202-1205, 1083-1127) of the stream [B][3K+12] into the windowed
// schedule's wide arrays.  A block transposes 64 codewords x kSwDemuxSteps steps through LDS: each
// codeword's 3 x 16 values are one contiguous 384-byte piece of its row, each output row is 512
// bytes.  SISO2's systematic input (sys1 at pi, :1109-1113) is written in the same pass, row i of
// sys1 going to sys2 row pinv(i), so no gather follows (the 8-codeword layout needs demux_perm_kernel).
// The last x-block writes the three tail steps of both encoders (:1119-1123).
constexpr int kSwDemuxSteps = 16;
template <typename T>
__global__ __launch_bounds__(256) void sw_demux_kernel(DecodeParams<T> p, const T* __restrict__ flow)
{
    __shared__ T tile[kSwCw][3 * kSwDemuxSteps + 1];
    const int K = p.K, L = p.L, n = 3 * K + 4 * kMemory;
    const int gw = blockIdx.y, i0 = blockIdx.x * kSwDemuxSteps;
    const T h = (T)0.5;
    if (i0 >= K) {   // the tail block: steps K .. K+2 of the four streams
        for (int e = threadIdx.x; e < kSwCw * kMemory; e += blockDim.x) {
            const int c = e & 63, j = e >> 6, b = gw * kSwCw + c;
            T v[4] = {0, 0, 0, 0};
            if (b < p.B)
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = flow[(size_t)b * n + 3 * K + (u >> 1) * 2 * kMemory + 2 * j + (u & 1)] * h;
            const size_t off = ((size_t)gw * L + K + j) * kSwCw + c;
            p.sys1[off] = v[0];
            p.par1[off] = v[1];
            p.sys2[off] = v[2];
            p.par2[off] = v[3];
        }
        return;
    }
    const int ns = min(kSwDemuxSteps, K - i0);
    for (int e = threadIdx.x; e < kSwCw * 3 * kSwDemuxSteps; e += blockDim.x) {
        const int c = e / (3 * kSwDemuxSteps), q = e % (3 * kSwDemuxSteps), b = gw * kSwCw + c;
        tile[c][q] = (b < p.B && q < 3 * ns) ? flow[(size_t)b * n + 3 * i0 + q] * h : (T)0;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kSwCw * ns; e += blockDim.x) {
        const int c = e & 63, k = e >> 6, i = i0 + k;
        const size_t row = (size_t)gw * L;
        const T ys = tile[c][3 * k];
        p.sys1[(row + i) * kSwCw + c] = ys;
        p.par1[(row + i) * kSwCw + c] = tile[c][3 * k + 1];
        p.par2[(row + i) * kSwCw + c] = tile[c][3 * k + 2];
        p.sys2[(row + p.pinv[i]) * kSwCw + c] = ys;
    }
}

template <typename T>
hipError_t launch_window_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st)
{
    const int Bp = (p.B + kSwCw - 1) / kSwCw * kSwCw;
    hipLaunchKernelGGL(sw_demux_kernel<T>, dim3((p.K + kSwDemuxSteps - 1) / kSwDemuxSteps + 1, Bp / kSwCw), dim3(256),
                       0, st, p, flow);
    return hipGetLastError();
}

// SISO2's decisions [K][Bp] (rows in natural order) -> bits [B][K] (row stride `stride`): 64 x 64-byte
// tiles through LDS, 16-byte loads and stores
__global__ __launch_bounds__(256) void bits_transpose_kernel(const uint8_t* __restrict__ src, int K, int Bp, int B,
                                                             uint8_t* __restrict__ dst, long long stride)
{
    __shared__ uint8_t tile[64][64 + 16];
    const int k0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int r = threadIdx.x >> 2, q = (threadIdx.x & 3) * 16;
    if (k0 + r < K) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)(k0 + r) * Bp + b0 + q);
        *reinterpret_cast<uint4*>(&tile[r][q]) = v;
    }
    __syncthreads();
    const int b = b0 + r;
    if (b >= B) return;
    uint8_t o[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) o[u] = tile[q + u][r];
    uint8_t* d = dst + (size_t)b * stride + k0 + q;
    if (k0 + q + 16 <= K && ((reinterpret_cast<size_t>(d) & 15) == 0)) {
        *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(o);
    } else {
        for (int u = 0; u < 16 && k0 + q + u < K; ++u) d[u] = o[u];
    }
}

// checkpoint spacing S: the segment's alpha stays in registers.  fp64: 4 (round 4: 2 measured -12 %,
// 3 and 5 -6 %); fp32: 8.
#ifndef TD_SW_SEG64
#define TD_SW_SEG64 4
#endif
template <typename T>
constexpr int sw_seg()
{
    return sizeof(T) == 4 ? 8 : TD_SW_SEG64;
}

// sub-blocks per lane run: one (M = 1) while a launch has fewer than kSwRunWaves one-sub-block waves,
// else as many as keep about that many waves; runs need g <= W (two chains at most) and W a multiple
// of S (every sub-block start is a segment start).  Each run's first chain starts g steps early on
// its own (and its last ends g steps late), so fewer, longer runs do less work: at config 5 (96
// sub-blocks, 512 waves of codewords) M = 24 leaves 4 runs a codeword, 2 % extra steps against M = 6's
// 7.8 %, and 2048 waves a SISO -- one round of the beta kernel's 2048 slots (2 waves a SIMD) over the
// two halves.  Measured (round 5, same box, forced run lengths, now td_debug_window_layout): M = 6 2462, 8 2467, 12 2553, 20 2525
// (1.25 rounds), 24 2628, 32 2236 (3/4 of the slots), 48 1559 Mbit/s.
#ifndef TD_SW_RUN_WAVES
#define TD_SW_RUN_WAVES 2048
#endif
constexpr int kSwRunWaves = TD_SW_RUN_WAVES;

int window_run(int L, int W, int g, int B, int ndec, int S, int force)
{
    const int nS = window_subblocks(L, W);
    if (g > W || W % S != 0) return 1;
    if (force > 0) return force < nS ? force : nS;
    const long long waves = (long long)nS * ((B + 63) / 64) * ndec;
    const long long m = waves / kSwRunWaves;
    return m < 1 ? 1 : (m > nS ? nS : (int)m);
}

// Two halves of the batch on two streams (round 5).  The alpha kernel streams inputs and checkpoints
// (HBM-heavy, light VALU) and the beta kernel is VALU- and LDS-heavy with light traffic; back to back on
// one stream each leaves the other resource idle.  The halves are independent codewords, so half B runs
// on a second stream one alpha launch behind half A, and the GPU co-schedules one half's alpha with the
// other's beta.  Used when each half keeps at least kSwHalfWaves waves of 64 codewords and a second
// stream is given (td_api.cpp); SISO2's decisions of every wanted iteration are transposed after the
// join (all_iters decodes keep one stream: their per-iteration transposes would re-join the halves).
#ifndef TD_SW_HALF_WAVES
#define TD_SW_HALF_WAVES 64
#endif
constexpr int kSwHalfWaves = TD_SW_HALF_WAVES;

template <typename T, int ALGO>
hipError_t launch_window_algo(const DecodeParams<T>& p, const WindowParams& w, const WindowBufs<T>& wb, hipStream_t st,
                              const WindowStreams& ws)
{
    constexpr int S = sw_seg<T>();
    const int W = w.window;
    const int nS = window_subblocks(p.L, W);
    const int ndec = w.concurrent ? 2 : 1;
    WinArgs<T> a{};
    a.W = W;
    a.g = w.overlap;
    a.nS = nS;
    a.Bp = (p.B + 63) / 64 * 64;
    a.ncp = (p.L - (nS - 1) * W + S - 1) / S;
    a.ext_scale = (T)w.ext_scale;
    a.nii = w.nii;
    a.ckpt[0] = wb.ckpt[0];
    a.ckpt[1] = wb.ckpt[1];
    const size_t nii_half = (size_t)2 * a.Bp * nS * 16;
    const int cw_total = a.Bp / 64;
    // batch parts: 2 by default (td_debug_window_layout: measured 3 and 4 slower, profiles/r05/sweep_window_layout.txt)
    const int want = w.parts > 0 ? min(w.parts, kSwMaxParts) : 2;
    const int nparts = (ws.st[1] && !p.all_iters) ? max(1, min(want, cw_total / kSwHalfWaves)) : 1;
    const bool split = nparts > 1;
    struct Part {
        int cw0, ncw, M, nR, blocks, Ma, nRa, blocksa;
        hipStream_t s;
    } part[kSwMaxParts];
    for (int h = 0; h < nparts; ++h) {
        Part& q = part[h];
        q.cw0 = (int)((long long)cw_total * h / nparts);
        q.ncw = (int)((long long)cw_total * (h + 1) / nparts) - q.cw0;
        q.M = window_run(p.L, W, w.overlap, cw_total * 64, ndec, S, w.run);   // sized on the whole batch (both halves co-run)
        q.nR = (nS + q.M - 1) / q.M;
        q.blocks = (int)(((long long)q.nR * q.ncw * ndec + 3) / 4);
        q.Ma = w.run_a > 0 ? window_run(p.L, W, w.overlap, cw_total * 64, ndec, S, w.run_a) : q.M;
        q.nRa = (nS + q.Ma - 1) / q.Ma;
        q.blocksa = (int)(((long long)q.nRa * q.ncw * ndec + 3) / 4);
        q.s = h == 0 ? st : ws.st[h];
    }
    auto check = [] { return hipGetLastError(); };
    bool forked[kSwMaxParts] = {}, recorded[kSwMaxParts] = {};
    // one codeword, one sub-block a lane: beta's warm-up runs in the alpha kernel (sw_alpha_lps_kernel)
    a.hand = p.B == 1 && !split && part[0].M == 1 && part[0].Ma == 1 && w.overlap > 0 && w.overlap + S <= W &&
             W % S == 0 && W + 2 * w.overlap + S <= kSwLpsChunk;
    for (int it = 0; it < p.iters; ++it) {
        a.it = it;
        a.nii_rd = wb.nii + (size_t)((it + 1) & 1) * nii_half;
        a.nii_wr = wb.nii + (size_t)(it & 1) * nii_half;
        const bool want_bits = p.all_iters || it == p.iters - 1;
        // a single codeword's decisions go straight to its row (sw_beta_kernel<LF>), without the
        // [K][Bp] staging and bits_transpose_kernel launch (15 a drop-in frame at 15 us each)
        const bool direct = p.B == 1 && !split;
        a.bitsT = want_bits && !direct ? wb.bitsT : nullptr;
        a.bits1 = want_bits && direct ? p.bits + (p.all_iters ? (size_t)it * p.K : 0) : nullptr;
        for (int dec = 0; dec < (w.concurrent ? 1 : 2); ++dec) {
            if (w.concurrent) {   // Jacobi: both SISOs read the other's Le of iteration it-1
                a.dec = -1;
                a.la_len = it == 0 ? 0 : p.K;
                a.la[0] = wb.ext21[(it + 1) & 1];
                a.la[1] = wb.ext12[(it + 1) & 1];
                a.le[0] = wb.ext12[it & 1];
                a.le[1] = wb.ext21[it & 1];
            } else {
                a.dec = dec;
                a.la_len = (it == 0 && dec == 0) ? 0 : p.K;
                a.la[0] = a.le[1] = wb.ext21[0];
                a.la[1] = a.le[0] = wb.ext12[0];
            }
            for (int h = 0; h < nparts; ++h) {
                const Part& q = part[h];
                a.cw0 = q.cw0;
                a.ncw = q.ncw;
                a.clk = h == 0 && it == p.iters - 1 && dec == (w.concurrent ? 0 : 1);   // one writer per decode
                if (h > 0 && !forked[h]) {   // part h starts one alpha launch behind part h-1
                    hipError_t e = hipStreamWaitEvent(q.s, ws.fork[h], 0);
                    if (e != hipSuccess) return e;
                    forked[h] = true;
                }
                a.M = q.Ma;
                a.nR = q.nRa;
                if (p.B == 1)   // the drop-in's single frame: states across lanes
                    hipLaunchKernelGGL((sw_alpha_lps_kernel<T, ALGO, S>), dim3(q.blocksa), dim3(256), 0, q.s, p, a);
                else
                    hipLaunchKernelGGL((sw_alpha_kernel<T, ALGO, S>), dim3(q.blocksa), dim3(256), 0, q.s, p, a);
                a.M = q.M;
                a.nR = q.nR;
                if (h + 1 < nparts && !recorded[h + 1]) {
                    hipError_t e = hipEventRecord(ws.fork[h + 1], q.s);
                    if (e != hipSuccess) return e;
                    recorded[h + 1] = true;
                }
                if (p.B == 1)   // the drop-in's single frame: lane folds
                    hipLaunchKernelGGL((sw_beta_kernel<T, ALGO, S, true>), dim3(q.blocks), dim3(256), 0, q.s, p, a, p.pi,
                                       p.pinv);
                else
                    hipLaunchKernelGGL((sw_beta_kernel<T, ALGO, S, false>), dim3(q.blocks), dim3(256), 0, q.s, p, a, p.pi,
                                       p.pinv);
                hipError_t e = check();
                if (e != hipSuccess) return e;
            }
        }
        if (want_bits && (p.all_iters || !split) && !direct) {
            const long long stride = p.all_iters ? (long long)p.iters * p.K : p.K;
            hipLaunchKernelGGL(bits_transpose_kernel, dim3((p.K + 63) / 64, a.Bp / 64), dim3(256), 0, st, wb.bitsT,
                               p.K, a.Bp, p.B, p.bits + (p.all_iters ? (size_t)it * p.K : 0), stride);
            hipError_t e = check();
            if (e != hipSuccess) return e;
        }
    }
    if (split) {   // join the other parts back into the caller's stream, then the decisions
        for (int h = 1; h < nparts; ++h) {
            hipError_t e = hipEventRecord(ws.join[h], ws.st[h]);
            if (e == hipSuccess) e = hipStreamWaitEvent(st, ws.join[h], 0);
            if (e != hipSuccess) return e;
        }
        hipError_t e;
        hipLaunchKernelGGL(bits_transpose_kernel, dim3((p.K + 63) / 64, a.Bp / 64), dim3(256), 0, st, wb.bitsT, p.K,
                           a.Bp, p.B, p.bits, (long long)p.K);
        e = check();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

size_t window_ckpt_elems(int B, int L, int W, bool f32)
{
    const int S = f32 ? sw_seg<float>() : sw_seg<double>();
    const int nS = window_subblocks(L, W);
    const size_t ncp = (size_t)(L - (nS - 1) * W + S - 1) / S;
    return (size_t)nS * ((B + 63) / 64) * ncp * 8 * 64;
}

size_t window_bits_bytes(int B, int K) { return (size_t)K * ((B + 63) / 64) * 64; }

template <typename T>
hipError_t launch_window(const DecodeParams<T>& p, const WindowParams& w, const WindowBufs<T>& wb, hipStream_t st,
                         const WindowStreams& ws)
{
    if (p.algo == 1) return launch_window_algo<T, 1>(p, w, wb, st, ws);
    return w.exact_table ? launch_window_algo<T, 0>(p, w, wb, st, ws) : launch_window_algo<T, 2>(p, w, wb, st, ws);
}

#endif  // TD_WIN_TU

constexpr int kDemuxBlocks = 32768;   // grid cap of demux_kernel (grid-stride loop beyond); 8192: 0.230 ms, 32768: 0.212 (config 2)

// Demultiplex + x0.5 (log_map.cpp:1202-1205, 1083-1127) of the reference stream layout into the
// batch-interleaved arrays, in two passes:
//   demux_kernel       one thread per (group, step, codeword): sys1, par1, par2 and the tail rows
//                      of sys2, straight from the stream (each wave reads 8 codewords x 8 steps);
//   demux_perm_kernel  sys2[g][i][.] = sys1[g][pi(i)][.] for i < K: SISO2's systematic input is
//                      SISO1's interleaved (:1109-1113), the same 0.5-scaled value.  Each 8-lane
//                      group reads one 64-B row, and all blocks of a codeword group run on one XCD
//                      (blocks go to XCDs round-robin), so the group's 393 KB of sys1 is gathered
//                      from that XCD's L2 instead of from HBM 8 bytes at a time.
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
        T ys1 = 0, yp1 = 0, yp2 = 0;
        if (b < p.B) {
            const T* r = flow + (size_t)b * n;
            const T h = (T)0.5;
            if (i < K) {
                ys1 = r[3 * i] * h;
                yp1 = r[3 * i + 1] * h;
                yp2 = r[3 * i + 2] * h;
            } else {
                const int j = i - K;
                ys1 = r[3 * K + 2 * j] * h;
                yp1 = r[3 * K + 2 * j + 1] * h;
                p.sys2[e] = r[3 * K + 2 * kMemory + 2 * j] * h;
                yp2 = r[3 * K + 2 * kMemory + 2 * j + 1] * h;
            }
        } else if (i >= K) {
            p.sys2[e] = 0;
        }
        p.sys1[e] = ys1;
        p.par1[e] = yp1;
        p.par2[e] = yp2;
    }
}

constexpr int kPermBlock = 256;
template <typename T>
__global__ __launch_bounds__(kPermBlock) void demux_perm_kernel(DecodeParams<T> p, int blocks_per_group)
{
    const int b = blockIdx.x;
    const int xcd = b % 8, r = b / 8;                              // XCD-major: group g on XCD g % 8
    const int g = (r / blocks_per_group) * 8 + xcd;
    const int e = (r % blocks_per_group) * kPermBlock + (int)threadIdx.x;   // (step, codeword) in the group
    if (g >= p.G || e >= p.K * kCw) return;
    const int i = e >> 3, c = e & 7;
    const size_t row = (size_t)g * p.L;
    p.sys2[(row + i) * kCw + c] = p.sys1[(row + p.pi[i]) * kCw + c];
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

// LDS per workgroup: the Smem of its groups, but never less than a third of the CU's 160 KiB, so
// that at most two workgroups share a CU whatever the kernel's register count (the role pairing
// per SIMD, wg_pos, and the load balance of B/8 workgroups over 256 CUs assume two).
constexpr size_t kMinWgLds = 160 * 1024 / 3 + 1024;
template <typename T>
constexpr size_t wg_lds()
{
    return sizeof(Smem<T>) > kMinWgLds ? sizeof(Smem<T>) : kMinWgLds;
}
static_assert(2 * (sizeof(Smem<double>) + 64) <= 160 * 1024, "two workgroups per CU");


// turbo_decode_kernel3's LDS: never less than a quarter of the CU's plus 1 KB, so that at most three
// of its workgroups share a CU (the fp32 Smem alone would let four in)
template <typename T>
constexpr size_t wg_lds3()
{
    return sizeof(Smem<T>) > 160 * 1024 / 4 + 1024 ? sizeof(Smem<T>) : 160 * 1024 / 4 + 1024;
}

// Workgroups per CU for a decode of p.G groups: the fewest expected kernel time over the occupancies
// the build has (2; 3 and 4 where kOcc3 / kOcc4), counting whole dispatch rounds of N groups per CU
// at the measured time of a round with N per CU (fp32, relative to N = 2; one box, K = 6144: log-MAP
// 1.17 for 3, 1.39 for 4; Max-Log-MAP 1.07, 1.29) and the last partial round at the time of its own
// groups per CU.
template <typename T, int ALGO>
int occupancy_pick(const DecodeParams<T>& p)
{
    if (!p.occ3 || p.role_cus <= 0 || p.G <= 2 * p.role_cus) return 2;
    // (four per CU run the 12-step-window build: relative to two per CU with 15-step windows, 1.42)
    const double t_rel[5] = {1.0, 1.0, 1.0, ALGO == 1 ? 1.07 : 1.17, kW == 12 ? (ALGO == 1 ? 1.29 : 1.39) : 1.42};
    auto est = [&](int n) {
        const long per_round = (long)n * p.role_cus;
        const long full = p.G / per_round, rem = p.G % per_round;
        const int last = (int)((rem + p.role_cus - 1) / p.role_cus);
        return full * t_rel[n] + (rem ? t_rel[last] : 0.0);
    };
    int best = 2;
    if (kOcc3<T, ALGO> && est(3) < est(best)) best = 3;
    if ((kOcc4<T, ALGO> || kOcc4W12<T, ALGO>) && est(4) < est(best)) best = 4;
    return best;
}

template <typename T, int ALGO>
hipError_t launch_kernel4(const DecodeParams<T>& p, hipStream_t st)
{
    hipError_t e = allow_smem(reinterpret_cast<const void*>(&turbo_decode_kernel4<T, ALGO>), sizeof(Smem<T>));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((turbo_decode_kernel4<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), sizeof(Smem<T>), st, p);
    return hipGetLastError();
}

template <typename T, int ALGO>
hipError_t launch_turbo_algo(const DecodeParams<T>& p, hipStream_t st, bool probe)
{
    // the placement probe times the kernel the decode will run: at two per CU under its own symbol (the
    // traces list it apart); at three or four per CU (fp32 batches beyond one dispatch round) the
    // decode's own kernel3 / kernel4
    const int occ = occupancy_pick<T, ALGO>(p);
    if (occ == 4) {
        if constexpr (kOcc4<T, ALGO>) return launch_kernel4<T, ALGO>(p, st);
#ifndef TD_W12_TU
        else if constexpr (kOcc4W12<T, ALGO>) return launch_turbo4_w12<T, ALGO>(p, st);
#endif
        else return hipErrorInvalidConfiguration;
    }
    if (occ == 3) {
        hipError_t e = allow_smem(reinterpret_cast<const void*>(&turbo_decode_kernel3<T, ALGO>), wg_lds3<T>());
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((turbo_decode_kernel3<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), wg_lds3<T>(), st, p);
        return hipGetLastError();
    }
    const void* k = probe ? reinterpret_cast<const void*>(&turbo_placement_probe_kernel<T, ALGO>)
                          : reinterpret_cast<const void*>(&turbo_decode_kernel<T, ALGO>);
    hipError_t e = allow_smem(k, wg_lds<T>());
    if (e != hipSuccess) return e;
    if (probe)
        hipLaunchKernelGGL((turbo_placement_probe_kernel<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), wg_lds<T>(), st, p);
    else
        hipLaunchKernelGGL((turbo_decode_kernel<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), wg_lds<T>(), st, p);
    return hipGetLastError();
}

template <typename T, int ALGO>
hipError_t launch_siso_algo(const DecodeParams<T>& p, const T* la, int terminated, hipStream_t st)
{
    hipError_t e = allow_smem(reinterpret_cast<const void*>(&siso_kernel<T, ALGO>), wg_lds<T>());
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((siso_kernel<T, ALGO>), dim3(p.G), dim3(kWaves * kLanes), wg_lds<T>(), st, p, la, terminated);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_demux(const DecodeParams<T>& p, const T* flow, hipStream_t st)
{
    const size_t total = (size_t)p.G * p.L * kCw;
    int gblocks = (int)((total + 255) / 256);
    if (gblocks > kDemuxBlocks) gblocks = kDemuxBlocks;
    hipLaunchKernelGGL(demux_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, flow);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (p.sys2_in_turbo) return hipSuccess;
    const int bpg = (p.K * kCw + kPermBlock - 1) / kPermBlock;
    const long long pblocks = (long long)((p.G + 7) / 8) * 8 * bpg;
    hipLaunchKernelGGL(demux_perm_kernel<T>, dim3((unsigned)pblocks), dim3(kPermBlock), 0, st, p, bpg);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_turbo(const DecodeParams<T>& p, hipStream_t st, bool probe)
{
    return p.algo == 1 ? launch_turbo_algo<T, 1>(p, st, probe) : launch_turbo_algo<T, 0>(p, st, probe);
}

template <typename T>
hipError_t launch_siso(const DecodeParams<T>& p, const T* recs, const T* la, T* la_ws, int terminated, T* llr,
                       hipStream_t st)
{
    const size_t total = (size_t)p.G * p.L * kCw;
    int gblocks = (int)((total + 255) / 256);
    if (gblocks > kDemuxBlocks) gblocks = kDemuxBlocks;
    hipLaunchKernelGGL(siso_in_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, recs, la, la_ws);
    hipError_t e = p.algo == 1 ? launch_siso_algo<T, 1>(p, la_ws, terminated, st)
                               : launch_siso_algo<T, 0>(p, la_ws, terminated, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(siso_out_kernel<T>, dim3(gblocks), dim3(256), 0, st, p, llr);
    return hipGetLastError();
}

#if !defined(TD_W12_TU) && !defined(TD_WIN_TU)
template hipError_t launch_demux<double>(const DecodeParams<double>&, const double*, hipStream_t);
template hipError_t launch_demux<float>(const DecodeParams<float>&, const float*, hipStream_t);
template hipError_t launch_turbo<double>(const DecodeParams<double>&, hipStream_t, bool);
template hipError_t launch_turbo<float>(const DecodeParams<float>&, hipStream_t, bool);
template hipError_t launch_siso<double>(const DecodeParams<double>&, const double*, const double*, double*, int,
                                        double*, hipStream_t);
template hipError_t launch_siso<float>(const DecodeParams<float>&, const float*, const float*, float*, int, float*,
                                       hipStream_t);

int window_steps() { return kW; }
#endif
#ifdef TD_WIN_TU
template hipError_t launch_window_demux<double>(const DecodeParams<double>&, const double*, hipStream_t);
template hipError_t launch_window_demux<float>(const DecodeParams<float>&, const float*, hipStream_t);
template hipError_t launch_window<double>(const DecodeParams<double>&, const WindowParams&, const WindowBufs<double>&,
                                         hipStream_t, const WindowStreams&);
template hipError_t launch_window<float>(const DecodeParams<float>&, const WindowParams&, const WindowBufs<float>&,
                                        hipStream_t, const WindowStreams&);
#endif

}  // namespace td / td_w12

#ifdef TD_W12_TU
namespace td {
template <typename T, int ALGO>
hipError_t launch_turbo4_w12(const DecodeParams<T>& p, hipStream_t st)
{
    static_assert(td_w12::kOcc4<T, ALGO>, "the 12-step-window build has the four-per-CU kernel");
    DecodeParams<T> q = p;
    q.nT = (q.L + td_w12::kW - 1) / td_w12::kW;   // windows of this build
    return td_w12::launch_kernel4<T, ALGO>(q, st);
}
template hipError_t launch_turbo4_w12<float, 0>(const DecodeParams<float>&, hipStream_t);
template hipError_t launch_turbo4_w12<float, 1>(const DecodeParams<float>&, hipStream_t);
}  // namespace td
#endif
