// td_tables.h -- code tables shared by the host API and the gfx950 kernels.
//
//  * trellis of the LTE 8-state RSC, built from the octal generators exactly as
//    gen_g_matrix/gen_trellis do (ITTC/log_map.cpp:114-169, 247-269, 281-337);
//  * the QPP permutation (gen_qpp_index, log_map.cpp:616-624);
//  * the max* bucket table: an exact, branch-free form of E_algorithm's 16-step linear
//    scan (log_map.cpp:14-18, 779-801), see build_lut.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

namespace td {

constexpr int kStates = 8;
constexpr int kMemory = 3;        // M_num_reg (log_map.cpp:28)
constexpr double kInfty = 1e20;   // INFTY (log_map.h:74-76)

// log_map.cpp:14-18
constexpr double kIdx[16] = {0.0,    0.08824, 0.19587, 0.31026, 0.43275, 0.56508, 0.70963, 0.86972,
                             1.0502, 1.2587,  1.5078,  1.8212,  2.2522,  2.9706,  3.6764,  4.3758};
constexpr double kTab[16] = {0.69315, 0.65, 0.6, 0.55, 0.5, 0.45, 0.4, 0.35,
                             0.3,     0.25, 0.2, 0.15, 0.1, 0.05, 0.025, 0.0125};

template <typename T>
struct alignas(4 * sizeof(T)) LutEntry {
    T thr, vlo, vhi, pad;
};

// Trellis (TURBO_TRELLIS, log_map.h:58-66) plus the per-state constants the kernels use.
struct Trellis {
    int nextout[kStates][4];
    int nextstat[kStates][2];
    int lastout[kStates][4];
    int laststat[kStates][2];
};

// The LTE trellis (13/15 octal, G_ROW_1/2 of log_map.h:35-36) as compile-time tables for the
// LLR fold: laststat[next][u] and "the parity output of a transition out of p makes its branch
// metric +-Q" (p in {2,3,4,5}; +-P otherwise).  td_create checks build_trellis(13, 15) against them.
constexpr int kTrellisLast[kStates][2] = {{0, 1}, {3, 2}, {4, 5}, {7, 6}, {1, 0}, {2, 3}, {5, 4}, {6, 7}};
constexpr int kTrellisQ[kStates] = {0, 0, 1, 1, 1, 1, 0, 0};
// nextstat[s][u] (log_map.h:58-66) of the same trellis
constexpr int kTrellisNext[kStates][2] = {{0, 4}, {4, 0}, {5, 1}, {1, 5}, {2, 6}, {6, 2}, {7, 3}, {3, 7}};

// gen_g_matrix (log_map.cpp:114-169): octal -> 4 binary taps, MSB first. false on a non-octal digit.
inline bool octal_taps(int g, int* taps)
{
    for (int j = 0; j < 4; ++j) taps[j] = 0;
    int pos = 1, i = 0;
    while (g > 0) {
        int low = g % 10;
        if (low > 7) return false;
        g /= 10;
        for (i = 4 - (pos - 1) * 3 - 1; i >= 0 && i >= 4 - pos * 3; --i) {
            taps[i] = low % 2;
            low /= 2;
        }
        ++pos;
        if (i < 0) break;
    }
    return true;
}

// gen_trellis (log_map.cpp:281-337) for generators (feedback, forward) in octal.
inline bool build_trellis(int g_fb_oct, int g_ff_oct, Trellis& t)
{
    int fb[4], ff[4];
    if (!octal_taps(g_fb_oct, fb) || !octal_taps(g_ff_oct, ff)) return false;
    for (int s = 0; s < kStates; ++s) {
        for (int u = 0; u < 2; ++u) {
            int st[3] = {(s >> 2) & 1, (s >> 1) & 1, s & 1};   // int2bin, MSB first
            int ak = fb[0] * u;
            for (int k = 1; k < 4; ++k) ak += fb[k] * st[k - 1];
            ak %= 2;
            int out = ff[0] * ak;   // encode_bit, log_map.cpp:247-269
            for (int j = 1; j < 4; ++j) out = (out + ff[j] * st[j - 1]) % 2;
            st[2] = st[1];
            st[1] = st[0];
            st[0] = ak;
            t.nextout[s][2 * u] = 2 * u - 1;
            t.nextout[s][2 * u + 1] = 2 * out - 1;
            t.nextstat[s][u] = st[0] * 4 + st[1] * 2 + st[2];
        }
    }
    for (int s = 0; s < kStates; ++s)
        for (int u = 0; u < 2; ++u) {
            int ns = t.nextstat[s][u];
            t.laststat[ns][u] = s;
            t.lastout[ns][2 * u] = t.nextout[s][2 * u];
            t.lastout[ns][2 * u + 1] = t.nextout[s][2 * u + 1];
        }
    return true;
}

// true when t is the trellis the kernels' compile-time tables describe
inline bool trellis_is_lte(const Trellis& t)
{
    for (int j = 0; j < kStates; ++j)
        for (int u = 0; u < 2; ++u) {
            const int p = kTrellisLast[j][u];
            if (t.laststat[j][u] != p) return false;
            // u == 1 with parity +1, or u == 0 with parity -1: +-P; otherwise +-Q (see td_kernels.hip "gamma")
            const int o = t.nextout[p][2 * u + 1];
            if ((((u == 1) == (o == 1)) ? 0 : 1) != kTrellisQ[p]) return false;
            if (t.nextstat[j][u] != kTrellisNext[j][u]) return false;
        }
    return true;
}

// gen_qpp_index (log_map.cpp:616-624), int32 arithmetic as the reference (valid for K <= 10000).
inline void build_qpp(int K, int f1, int f2, int* pi)
{
    for (int i = 0; i < K; ++i) pi[i] = (f1 * i + (((f2 * i) % K) * i) % K) % K;
}

// Bucket geometry of the max* table.  The bucket index comes straight from the bits of
// d = |y - x|: exponent + top 2 mantissa bits (4 buckets per octave), clamped to [0, 28]:
//   bucket 0      d < 2^-4 * 1.25 (below the first threshold 0.08824)
//   buckets 1..27 [2^e (1 + m/4), 2^e (1 + (m+1)/4)),  e = -4..2
//   bucket 28     d >= 8                                 (f = 0)
// Every bucket holds at most one threshold (checked by lut_one_threshold_per_bucket at td_create;
// the closest pairs are 1.0502 | 1.2587 | 1.5078 | 1.8212 in [1, 2), one per quarter octave), so
//   f(d) = (d >= thr[q]) ? vhi[q] : vlo[q]
// reproduces the reference's linear scan (log_map.cpp:779-801) for every d >= 0.  (Three mantissa
// bits, 57 buckets, give the same results with a table twice the size in LDS.)
constexpr int kLutSize = 29;

template <typename T>
struct BucketBits;
template <>
struct BucketBits<double> {   // bits 18..30 of the high dword: 11 exponent + 2 mantissa bits
    static constexpr int shift = 18, width = 13, base = (1023 - 4) << 2;
};
template <>
struct BucketBits<float> {    // bits 21..30: 8 exponent + 2 mantissa bits
    static constexpr int shift = 21, width = 10, base = (127 - 4) << 2;
};

inline int bucket_of_bits(unsigned hi, int shift, int width, int base)
{
    int q = (int)((hi >> shift) & ((1u << width) - 1)) - base;
    return q < 0 ? 0 : (q > kLutSize - 1 ? kLutSize - 1 : q);
}

inline unsigned high_word(double d)
{
    unsigned long long b;
    std::memcpy(&b, &d, sizeof b);
    return (unsigned)(b >> 32);
}
inline unsigned high_word(float d)
{
    unsigned b;
    std::memcpy(&b, &d, sizeof b);
    return b;
}

// The bucket table for precision T.  Thresholds and values are the reference's doubles
// rounded once to T (exact for T = double).
template <typename T>
inline void build_lut(LutEntry<T>* lut)
{
    using BB = BucketBits<T>;
    T thr[16], val[16];
    for (int k = 0; k < 16; ++k) {
        thr[k] = (T)kIdx[k];
        val[k] = (T)kTab[k];
    }
    val[15] = (T)0;   // d >= idx[15] -> 0 (log_map.cpp:784-787); table[15] is unreachable
    for (int q = 0; q < kLutSize; ++q) {
        int base = 0, in_bucket = -1;
        for (int k = 1; k < 16; ++k) {
            const int qk = bucket_of_bits(high_word(thr[k]), BB::shift, BB::width, BB::base);
            if (qk < q) ++base;
            if (qk == q) in_bucket = k;
        }
        lut[q].thr = in_bucket >= 0 ? thr[in_bucket] : (T)INFINITY;
        lut[q].vlo = val[base];
        lut[q].vhi = val[base + 1 <= 15 ? base + 1 : 15];
        lut[q].pad = (T)0;
    }
}

// No bucket holds two thresholds (build_lut would keep only the last one).
template <typename T>
inline bool lut_one_threshold_per_bucket()
{
    using BB = BucketBits<T>;
    int n[kLutSize] = {};
    for (int k = 1; k < 16; ++k) ++n[bucket_of_bits(high_word((T)kIdx[k]), BB::shift, BB::width, BB::base)];
    for (int q = 0; q < kLutSize; ++q)
        if (n[q] > 1) return false;
    return true;
}

// The device keeps only thr and vlo per bucket and reads vhi[q] as vlo[q+1] (the value just past
// bucket q's threshold is the value at the start of bucket q+1; buckets without a threshold never
// read vhi); true for every table build_lut makes -- checked by td_create.
template <typename T>
inline bool lut_vhi_is_next_vlo(const LutEntry<T>* lut)
{
    for (int q = 0; q + 1 < kLutSize; ++q)   // vhi matters only below a finite threshold
        if (lut[q].thr < (T)INFINITY && lut[q].vhi != lut[q + 1].vlo) return false;
    return true;
}

// Host evaluation of the bucket max* exactly as the device evaluates it (td_kernels.hip mstar).
template <typename T>
inline T maxstar_lut_host(T x, T y, const LutEntry<T>* lut)
{
    using BB = BucketBits<T>;
    T d = y - x;
    d = d < (T)0 ? -d : d;
    const T m = x > y ? x : y;
    const int q = bucket_of_bits(high_word(d), BB::shift, BB::width, BB::base);
    const T hi = q + 1 < kLutSize ? lut[q + 1].vlo : lut[q].vhi;
    return m + (d >= lut[q].thr ? hi : lut[q].vlo);
}

// ---- The windowed schedule's one-read max* table (round 6; td_set_window_maxstar).
// The sub-block schedule is BER-gated, not bit-exact (its boundaries already change the arithmetic),
// so its max* may take the reference's 16-step correction (log_map.cpp:14-18, 779-801) with each
// threshold moved to the nearest edge of a finer bucket grid: exponent + kQBits mantissa bits of d
// (8 buckets an octave), one correction value per bucket -- the reference's value at the bucket's
// midpoint.  Then f(d) is ONE table read at the bucket's row: no threshold read, compare and select
// (3 of a table max*'s 11 VALU and 2 of its 3 LDS reads).  The correction differs from E_algorithm's
// only for d within half a bucket (6.25 % of d) of one of its 15 thresholds, by one table step.
//   row 0             d < 2^-4 (1 + 2^-kQBits) (and every smaller d)
//   rows 1 .. 7*2^k-1 [2^e (1 + m/2^k), 2^e (1 + (m+1)/2^k)),  e = -4..2
//   row 7*2^k         d >= 8  (f = 0)
constexpr int kQBits = 3;
constexpr int kQRows = (7 << kQBits) + 1;

template <typename T>
struct QBucketBits;
template <>
struct QBucketBits<double> {   // bits 17..30 of the high dword: 11 exponent + 3 mantissa bits
    static constexpr int shift = 20 - kQBits, width = 11 + kQBits, base = (1023 - 4) << kQBits;
};
template <>
struct QBucketBits<float> {    // bits 20..30: 8 exponent + 3 mantissa bits
    static constexpr int shift = 23 - kQBits, width = 8 + kQBits, base = (127 - 4) << kQBits;
};

inline int qbucket_of_bits(unsigned hi, int shift, int width, int base)
{
    int q = (int)((hi >> shift) & ((1u << width) - 1)) - base;
    return q < 0 ? 0 : (q > kQRows - 1 ? kQRows - 1 : q);
}

// E_algorithm's correction f(d) for d >= 0 (log_map.cpp:784-797: the linear scan; 0 past the last index)
inline double reference_correction(double d)
{
    if (d >= kIdx[15]) return 0.0;
    int i = 1;
    while (i < 16 && !(d < kIdx[i])) ++i;
    return kTab[i - 1];
}

// the table: row q's value = the reference's correction at the row's midpoint (rounded once to T)
template <typename T>
inline void build_qlut(T* v)
{
    for (int q = 0; q < kQRows; ++q) {
        if (q == kQRows - 1) {
            v[q] = (T)0;
            continue;
        }
        const int e = q >> kQBits, m = q & ((1 << kQBits) - 1);
        const double lo = std::ldexp(1.0 + (double)m / (1 << kQBits), e - 4);
        const double hi = std::ldexp(1.0 + (double)(m + 1) / (1 << kQBits), e - 4);
        v[q] = (T)reference_correction(0.5 * (lo + hi));
    }
}

// Host evaluation of the one-read max* as the windowed kernels evaluate it (td_kernels.hip sw_mstar)
template <typename T>
inline T maxstar_qlut_host(T x, T y, const T* v)
{
    using QB = QBucketBits<T>;
    const T d = y - x;
    const T m = x > y ? x : y;
    return m + v[qbucket_of_bits(high_word(d), QB::shift, QB::width, QB::base)];
}

}  // namespace td
