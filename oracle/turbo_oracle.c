/*
 * turbo_oracle.c -- CPU restatement of the reference turbo codec.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
 * product path.  See turbo_oracle.h for the contract and the reference citations.
 */
#include "turbo_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- max* tables
 * log_map.cpp:14-18 (lookup_index_Log_MAP / lookup_table_Log_MAP) */
static const double k_idx[16] = {0.0,    0.08824, 0.19587, 0.31026, 0.43275, 0.56508,
                                 0.70963, 0.86972, 1.0502,  1.2587,  1.5078,  1.8212,
                                 2.2522, 2.9706,  3.6764,  4.3758};
static const double k_tab[16] = {0.69315, 0.65, 0.6,  0.55, 0.5,   0.45,  0.4,  0.35,
                                 0.3,     0.25, 0.2,  0.15, 0.1,   0.05,  0.025, 0.0125};

/* E_algorithm, log_map.cpp:779-801 */
double tdo_maxstar(double x, double y)
{
    double temp = (y - x) > 0 ? (y - x) : (x - y);
    int i;
    if (temp >= 4.3758) {
        temp = 0;
    } else {
        for (i = 0; i < 16 && temp >= k_idx[i]; i++) {
        }
        temp = k_tab[i - 1];   /* i >= 1 for every non-NaN temp (k_idx[0] = 0) */
    }
    return (x > y ? x : y) + temp;
}

double tdo_maxstar_seq(const double* v, int n)
{
    double t = tdo_maxstar(v[0], v[1]);
    for (int i = 2; i < n; i++) t = tdo_maxstar(t, v[i]);
    return t;
}

/* fp32 restatement of the same table: thresholds and values rounded to float once. */
float tdo_maxstar_f32(float x, float y)
{
    float temp = (y - x) > 0 ? (y - x) : (x - y);
    int i;
    if (temp >= (float)4.3758) {
        temp = 0;
    } else {
        for (i = 0; i < 16 && temp >= (float)k_idx[i]; i++) {
        }
        temp = (float)k_tab[i - 1];
    }
    return (x > y ? x : y) + temp;
}

/* The windowed schedule's one-read max* (TDO_ALGO_LOGMAP_Q; not the reference's -- the sub-block
 * schedule is BER-gated).  The buckets of d = |y - x|: exponent + 3 mantissa bits (8 an octave); row 0
 * holds every d below 2^-4 * 9/8, row 56 every d >= 8; rows 1..55 are [2^e (1 + m/8), 2^e (1 + (m+1)/8))
 * with e = q/8 - 4, m = q % 8.  A row's correction is E_algorithm's (above) at the row's midpoint, 0 in
 * row 56.  The row comes from the bits of d exactly as the kernels take it (sign outside the field). */
#define TDO_QBITS 3
#define TDO_QROWS ((7 << TDO_QBITS) + 1)
static double q_correction(int q)
{
    if (q >= TDO_QROWS - 1) return 0.0;
    const int e = q >> TDO_QBITS, m = q & ((1 << TDO_QBITS) - 1);
    const double lo = ldexp(1.0 + (double)m / (1 << TDO_QBITS), e - 4);
    const double hi = ldexp(1.0 + (double)(m + 1) / (1 << TDO_QBITS), e - 4);
    const double mid = 0.5 * (lo + hi);
    if (mid >= 4.3758) return 0.0;
    int i;
    for (i = 0; i < 16 && mid >= k_idx[i]; i++) {
    }
    return k_tab[i - 1];
}
static int q_row(uint32_t hi, int shift, int width, int base)
{
    int q = (int)((hi >> shift) & ((1u << width) - 1)) - base;
    return q < 0 ? 0 : (q > TDO_QROWS - 1 ? TDO_QROWS - 1 : q);
}
double tdo_maxstar_q(double x, double y)
{
    const double d = y - x;
    uint64_t b;
    memcpy(&b, &d, sizeof b);
    const int q = q_row((uint32_t)(b >> 32), 20 - TDO_QBITS, 11 + TDO_QBITS, (1023 - 4) << TDO_QBITS);
    return (x > y ? x : y) + q_correction(q);
}
float tdo_maxstar_q_f32(float x, float y)
{
    const float d = y - x;
    uint32_t b;
    memcpy(&b, &d, sizeof b);
    const int q = q_row(b, 23 - TDO_QBITS, 8 + TDO_QBITS, (127 - 4) << TDO_QBITS);
    return (x > y ? x : y) + (float)q_correction(q);
}

/* ---------------------------------------------------------------- code tables */

/* gen_g_matrix, log_map.cpp:114-169: octal generator -> 4 binary taps, MSB first */
static int octal_taps(int g, int k_col, int* taps)
{
    int pos = 1, i = 0;
    for (int j = 0; j < k_col; j++) taps[j] = 0;
    while (g > 0) {
        int low = g % 10;
        if (low > 7) return 0;
        g /= 10;
        for (i = k_col - (pos - 1) * 3 - 1; i >= 0 && i >= k_col - pos * 3; i--) {
            taps[i] = low % 2;
            low /= 2;
        }
        pos++;
        if (i < 0) break;
    }
    return 1;
}

/* encode_bit, log_map.cpp:247-269: feed-forward output, then shift the register */
static int encode_bit(const int* gf, int inbit, int* stat)
{
    int out = gf[0] * inbit;
    for (int j = 1; j < 4; j++) out = (out + gf[j] * stat[j - 1]) % 2;
    for (int j = 2; j > 0; j--) stat[j] = stat[j - 1];
    stat[0] = inbit;
    return out;
}

/* gen_trellis, log_map.cpp:281-337 */
int tdo_build_trellis(int g_feedback_octal, int g_forward_octal, tdo_trellis* t)
{
    int fb[4], ff[4];
    if (!octal_taps(g_feedback_octal, 4, fb) || !octal_taps(g_forward_octal, 4, ff)) return 0;
    memcpy(t->g_fb, fb, sizeof fb);
    memcpy(t->g_ff, ff, sizeof ff);
    for (int s = 0; s < TDO_NSTATES; s++) {
        for (int u = 0; u < 2; u++) {
            int st[3] = {(s >> 2) & 1, (s >> 1) & 1, s & 1};   /* int2bin, MSB first (:185-197) */
            int ak = fb[0] * u;
            for (int k = 1; k < 4; k++) ak += fb[k] * st[k - 1];
            ak %= 2;
            int outbit = encode_bit(ff, ak, st);
            t->nextout[s][2 * u] = 2 * u - 1;
            t->nextout[s][2 * u + 1] = 2 * outbit - 1;
            t->nextstat[s][u] = st[0] * 4 + st[1] * 2 + st[2];   /* bin2int (:213-231) */
        }
    }
    for (int s = 0; s < TDO_NSTATES; s++) {
        for (int u = 0; u < 2; u++) {
            int ns = t->nextstat[s][u];
            t->laststat[ns][u] = s;
            t->lastout[ns][2 * u] = t->nextout[s][2 * u];
            t->lastout[ns][2 * u + 1] = t->nextout[s][2 * u + 1];
        }
    }
    return 1;
}

/* gen_qpp_index, log_map.cpp:616-624 (int32 arithmetic exactly as the reference) */
void tdo_qpp(int K, int f1, int f2, int* pi)
{
    for (int i = 0; i < K; i++) pi[i] = (f1 * i + (((f2 * i) % K) * i) % K) % K;
}

/* rsc_encode (terminated), log_map.cpp:451-512; rsc[2*(K+3)] */
static void rsc_encode(const tdo_trellis* t, const int* src, int* rsc, int K)
{
    int st[3] = {0, 0, 0};
    for (int i = 0; i < K + TDO_MREG; i++) {
        int dk;
        if (i < K) {
            dk = src[i];
        } else {   /* trellis termination: drive the register to zero (:483-491) */
            dk = 0;
            for (int j = 1; j < 4; j++) dk += t->g_fb[j] * st[j - 1];
            dk %= 2;
        }
        int ak = t->g_fb[0] * dk;
        for (int j = 1; j < 4; j++) ak += t->g_fb[j] * st[j - 1];
        ak %= 2;
        int out = encode_bit(t->g_ff, ak, st);
        rsc[2 * i] = dk;
        rsc[2 * i + 1] = out;
    }
}

/* encoderm_turbo, log_map.cpp:530-583 (stream layout x,p1,p2 ; tail1 (x,p)x3 ; tail2 (x,p)x3) */
void tdo_turbo_encode(const tdo_trellis* t, const int* pi, const int* src, int K, int* coded)
{
    const int Lt = K + TDO_MREG;
    int* r1 = (int*)malloc(sizeof(int) * 2 * Lt);
    int* r2 = (int*)malloc(sizeof(int) * 2 * Lt);
    int* in2 = (int*)malloc(sizeof(int) * K);
    rsc_encode(t, src, r1, K);
    for (int i = 0; i < K; i++) in2[i] = src[pi[i]];   /* randominterleaver_int, :54-63 */
    rsc_encode(t, in2, r2, K);
    for (int i = 0; i < K; i++) {
        coded[3 * i] = r1[2 * i];
        coded[3 * i + 1] = r1[2 * i + 1];
        coded[3 * i + 2] = r2[2 * i + 1];
    }
    for (int i = 0; i < 2 * TDO_MREG; i++) {
        coded[3 * K + i] = r1[2 * K + i];
        coded[3 * K + 2 * TDO_MREG + i] = r2[2 * K + i];
    }
    free(r1);
    free(r2);
    free(in2);
}

/* ---------------------------------------------------------------- channel */

void tdo_bpsk_map(const int* bits, int n, double* oi, double* oq)
{
    for (int i = 0; i < n; i++) {
        oq[i] = 0.0;
        oi[i] = (bits[i] == 1) ? 1.0 : -1.0;
    }
}

void tdo_mgrns(double mean, double sigma, double seed, int n, double* a)
{
    const double s = 65536.0, w = 2053.0, v = 13849.0;
    for (int k = 0; k < n; k++) {
        double t = 0.0;
        for (int i = 1; i <= 12; i++) {
            seed = seed * w + v;
            int m = (int)(seed / s);
            seed = seed - m * s;
            t = t + seed / s;
        }
        a[k] = mean + (double)(sigma * (t - 6.0));
    }
}

void tdo_awgn(const double* send, double* r, double sigma, int n, double seed)
{
    double* noise = (double*)malloc(sizeof(double) * n);
    tdo_mgrns(0, sigma, seed, n, noise);
    for (int i = 0; i < n; i++) r[i] = send[i] + noise[i];
    free(noise);
}

static double sqr_dis(double ar, double ai, double br, double bi)
{
    double dr = ar - br, di = ai - bi;   /* calculate_sqr_dis, modanddem.cpp:73-84 */
    return dr * dr + di * di;
}

void tdo_bpsk_demod(const double* yi, const double* yq, int n, double Kf, double* out)
{
    static const double map_i[2] = {-1, 1}, map_q[2] = {0, 0};
    for (int i = 0; i < n; i++) {
        double m1 = 0x7fffffffffff, m2 = 0x7fffffffffff;
        for (int j = 0; j < 2; j++) {
            double d = sqr_dis(yi[i], yq[i], map_i[j], map_q[j]);
            if (j & 1) {
                if (d < m1) m1 = d;
            } else {
                if (d < m2) m2 = d;
            }
        }
        out[i] = -Kf * (m1 - m2);
    }
}

/* Constellations of modanddem.cpp:7-71, indexed by the symbol's label (module's bit order). */
static const double k_qpsk_i[4] = {0.7071, 0.7071, -0.7071, -0.7071};
static const double k_qpsk_q[4] = {0.7071, -0.7071, 0.7071, -0.7071};
static const double k_8psk_i[8] = {-0.7071, -1, 0, 0.7071, 0, -0.7071, 0.7071, 1};
static const double k_8psk_q[8] = {0.7071, 0, 1, 0.7071, -1, -0.7071, -0.7071, 0};
static const double k_16qam_a = 0.948683, k_16qam_b = 0.316228;
static const double k_64qam[4] = {0.4629, 0.1543, 0.7615, 1.0801};

/* constellation point of label j for M bits per symbol */
static void constellation(int M, int j, double* ci, double* cq)
{
    switch (M) {
    case 1: *ci = j ? 1.0 : -1.0; *cq = 0.0; break;
    case 2: *ci = k_qpsk_i[j]; *cq = k_qpsk_q[j]; break;
    case 3: *ci = k_8psk_i[j]; *cq = k_8psk_q[j]; break;
    case 4: {   /* i from the two high label bits {-a,-b,a,b}, q from the two low bits {-a,-b,a,b} */
        const double lv[4] = {-k_16qam_a, -k_16qam_b, k_16qam_a, k_16qam_b};
        *ci = lv[j >> 2];
        *cq = lv[j & 3];
        break;
    }
    default: {  /* 64QAM: sign from bit 5 (i) / bit 2 (q), level from bits 4-3 (i) / 1-0 (q) */
        *ci = ((j >> 5) & 1 ? -1.0 : 1.0) * k_64qam[(j >> 3) & 3];
        *cq = ((j >> 2) & 1 ? -1.0 : 1.0) * k_64qam[j & 3];
        break;
    }
    }
}

int tdo_modulate(const int* bits, int N, int M, double* oi, double* oq)
{
    if (M != 1 && M != 2 && M != 3 && M != 4 && M != 6) return -1;
    for (int s = 0; s < N / M; s++) {
        int j = 0;
        if (M == 3)   /* _8psk_module: the symbol's first bit is the label's LSB (:135) */
            for (int b = 0; b < 3; b++) j |= bits[3 * s + b] << b;
        else          /* the others: first bit is the MSB (:113,:150,:165) */
            for (int b = 0; b < M; b++) j = j * 2 + bits[M * s + b];
        constellation(M, j, &oi[s], &oq[s]);
    }
    return 0;
}

int tdo_demodulate(const double* yi, const double* yq, int nsym, int M, double Kf, double* out)
{
    if (M != 1 && M != 2 && M != 3 && M != 4 && M != 6) return -1;
    const double big = 0x7fffffffffff, small = 0x7fffffff;   /* the functions' initial minima */
    for (int i = 0; i < nsym; i++)
        for (int b = 0; b < M; b++) {
            /* output bit b of the symbol is label bit (M-1-b), except 8PSK's (label bit b) */
            const int mask = M == 3 ? 1 << b : 1 << (M - 1 - b);
            double m1 = (M <= 2) ? big : small;
            double m2 = (M == 1 || (M == 2 && b == 0)) ? big : small;
            for (int j = 0; j < (1 << M); j++) {
                double ci, cq;
                constellation(M, j, &ci, &cq);
                const double d = sqr_dis(yi[i], yq[i], ci, cq);
                if (j & mask) {
                    if (d < m1) m1 = d;
                } else {
                    if (d < m2) m2 = d;
                }
            }
            out[(size_t)M * i + b] = -Kf * (m1 - m2);
        }
    return 0;
}

/* glibc srandom_r/random_r, TYPE_3 (degree 31, separation 3) */
void tdo_glibc_srand(tdo_glibc_rand* g, unsigned seed)
{
    if (seed == 0) seed = 1;
    g->tbl[0] = (int32_t)seed;
    long word = (long)seed;
    for (int i = 1; i < 31; i++) {
        long hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        g->tbl[i] = (int32_t)word;
    }
    g->f = 3;
    g->b = 0;
    for (int k = 0; k < 310; k++) (void)tdo_glibc_rand_next(g);
}

int tdo_glibc_rand_next(tdo_glibc_rand* g)
{
    uint32_t val = (uint32_t)g->tbl[g->f] + (uint32_t)g->tbl[g->b];
    g->tbl[g->f] = (int32_t)val;
    g->f = (g->f + 1) % 31;
    g->b = (g->b + 1) % 31;
    return (int)(val >> 1);
}

/* AWGN's seed expression, log_map.cpp:1392 */
static double awgn_seed(tdo_glibc_rand* g)
{
    const double RM = 2147483647.0;
    return (double)(3.0 - (double)((tdo_glibc_rand_next(g) & 2147483647) / RM) / 10e6);
}

/* main.cpp:174 (sigma) and :183-202 (one frame) */
void tdo_make_frame(const tdo_trellis* t, const int* pi, int K, double ebn0_db, tdo_glibc_rand* g,
                    int* src, double* flow)
{
    const int n = 3 * K + 4 * TDO_MREG;
    const double rate = (double)K / (double)n;
    const double sigma = pow(10, -ebn0_db / 20) * sqrt(0.5 / (rate * 1));
    int* coded = (int*)malloc(sizeof(int) * n);
    double *si = (double*)malloc(sizeof(double) * n), *sq = (double*)malloc(sizeof(double) * n);
    double *ri = (double*)malloc(sizeof(double) * n), *rq = (double*)malloc(sizeof(double) * n);
    for (int i = 0; i < K; i++) src[i] = tdo_glibc_rand_next(g) % 2;
    tdo_turbo_encode(t, pi, src, K, coded);
    tdo_bpsk_map(coded, n, si, sq);
    tdo_awgn(si, ri, sigma, n, awgn_seed(g));
    tdo_awgn(sq, rq, sigma, n, awgn_seed(g));
    tdo_bpsk_demod(ri, rq, n, 1 / (2 * pow(sigma, 2)), flow);
    free(coded);
    free(si);
    free(sq);
    free(ri);
    free(rq);
}

void tdo_make_frame_mod(const tdo_trellis* t, const int* pi, int K, double ebn0_db, int M, tdo_glibc_rand* g,
                        int* src, double* flow)
{
    const int n = 3 * K + 4 * TDO_MREG, nsym = n / M;
    const double rate = (double)K / (double)nsym;
    const double sigma = pow(10, -ebn0_db / 20) * sqrt(0.5 / (rate * M));
    int* coded = (int*)malloc(sizeof(int) * n);
    double *si = (double*)malloc(sizeof(double) * nsym), *sq = (double*)malloc(sizeof(double) * nsym);
    double *ri = (double*)malloc(sizeof(double) * nsym), *rq = (double*)malloc(sizeof(double) * nsym);
    for (int i = 0; i < K; i++) src[i] = tdo_glibc_rand_next(g) % 2;
    tdo_turbo_encode(t, pi, src, K, coded);
    tdo_modulate(coded, nsym * M, M, si, sq);
    tdo_awgn(si, ri, sigma, nsym, awgn_seed(g));
    tdo_awgn(sq, rq, sigma, nsym, awgn_seed(g));
    tdo_demodulate(ri, rq, nsym, M, 1 / (2 * pow(sigma, 2)), flow);
    free(coded);
    free(si);
    free(sq);
    free(ri);
    free(rq);
}

/* demultiplex on doubles (exported for the tests) */
static void demux_f64(const double* rec, int K, const int* pi, double* yk);
void tdo_demultiplex(const double* flow, int K, const int* pi, double* yk) { demux_f64(flow, K, pi, yk); }

/* ---------------------------------------------------------------- SISO + turbo (generic) */
#define REAL double
#define SFX f64
#define MAXSTAR(x, y) tdo_maxstar((x), (y))
#define MAXSTAR_Q(x, y) tdo_maxstar_q((x), (y))
#include "turbo_oracle_siso.inc"
#include "turbo_oracle_window.inc"
#undef REAL
#undef SFX
#undef MAXSTAR
#undef MAXSTAR_Q

#define REAL float
#define SFX f32
#define MAXSTAR(x, y) tdo_maxstar_f32((x), (y))
#define MAXSTAR_Q(x, y) tdo_maxstar_q_f32((x), (y))
#include "turbo_oracle_siso.inc"
#include "turbo_oracle_window.inc"
#undef REAL
#undef SFX
#undef MAXSTAR
#undef MAXSTAR_Q

/* ---------------------------------------------------------------- batch + threads */
typedef struct {
    const tdo_trellis* t;
    const int* pi;
    int K, iters, algo, f32, B, tid, nthreads;
    const void* flow;
    uint8_t* bits;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* j = (batch_job*)arg;
    const int n = 3 * j->K + 4 * TDO_MREG;
    int* out = (int*)malloc(sizeof(int) * (size_t)j->K * j->iters);
    for (int b = j->tid; b < j->B; b += j->nthreads) {
        if (j->f32)
            tdo_turbo_decode_f32(j->t, j->pi, (const float*)j->flow + (size_t)b * n, j->K, j->iters, j->algo,
                                 out, NULL);
        else
            tdo_turbo_decode_f64(j->t, j->pi, (const double*)j->flow + (size_t)b * n, j->K, j->iters, j->algo,
                                 out, NULL);
        const int* last = out + (size_t)(j->iters - 1) * j->K;
        for (int i = 0; i < j->K; i++) j->bits[(size_t)b * j->K + i] = (uint8_t)last[i];
    }
    free(out);
    return NULL;
}

int tdo_decode_batch(int K, int f1, int f2, int iters, int algo, int f32, const void* flow, int B,
                     uint8_t* bits, int nthreads)
{
    tdo_trellis t;
    if (!tdo_build_trellis(13, 15, &t)) return -1;
    int* pi = (int*)malloc(sizeof(int) * K);
    tdo_qpp(K, f1, f2, pi);
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    batch_job* jobs = (batch_job*)malloc(sizeof(batch_job) * nthreads);
    for (int k = 0; k < nthreads; k++) {
        batch_job j = {&t, pi, K, iters, algo, f32, B, k, nthreads, flow, bits};
        jobs[k] = j;
        pthread_create(&th[k], NULL, batch_worker, &jobs[k]);
    }
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    free(th);
    free(jobs);
    free(pi);
    return 0;
}

/* ---------------------------------------------------------------- synthetic workload
 * DESIGN.md "Synthetic input": per-codeword glibc-rand stream seeded by
 * (seed ^ block index), then exactly main.cpp's frame (source, encode, BPSK, 2x AWGN, demod). */
void tdo_synth_batch(int K, int f1, int f2, double ebn0_db, uint64_t seed, int B, int* src, double* flow)
{
    tdo_trellis t;
    tdo_build_trellis(13, 15, &t);
    int* pi = (int*)malloc(sizeof(int) * K);
    tdo_qpp(K, f1, f2, pi);
    const int n = 3 * K + 4 * TDO_MREG;
    tdo_glibc_rand g;
    for (int b = 0; b < B; b++) {
        uint64_t s = seed ^ (uint64_t)b;
        tdo_glibc_srand(&g, (unsigned)(s ^ (s >> 32)));
        tdo_make_frame(&t, pi, K, ebn0_db, &g, src + (size_t)b * K, flow + (size_t)b * n);
    }
    free(pi);
}
