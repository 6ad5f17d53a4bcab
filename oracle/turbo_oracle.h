/*
 * turbo_oracle.h -- CPU restatement of the reference turbo codec (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle for the MI355X turbo decoder.  It restates, in plain C,
 * the algorithm of /root/reference/ITTC/log_map.cpp (+ the BPSK parts of
 * ITTC/modanddem.cpp).  Every function cites the reference file:line it follows.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the reported CPU baseline.  The product path
 * (turbo_decoder_cuda_amd, libturbo_mi355x.so) never links or calls it.
 *
 * Pinning: the restatement is checked against the compiled reference
 * (oracle/_ref, built by oracle/Makefile from the reference's own sources) through the
 * golden vectors in tests/golden/ (generator: oracle/gen_golden.py).
 *
 * Deliberate deviation (documented in DESIGN.md): the reference reads `tempmax`
 * uninitialised (log_map.cpp:925,989); the restatement uses tempmax[i] = max_j alpha[j][i]
 * (what the reference computes whenever the garbage is below the true maximum).
 */
#ifndef TURBO_ORACLE_H
#define TURBO_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TDO_NSTATES 8
#define TDO_MREG 3           /* M_num_reg, log_map.cpp:28 */
#define TDO_INFTY 1e20       /* INFTY, log_map.h:74-76 */

/* algorithm selector */
#define TDO_ALGO_LOGMAP 0    /* table Jacobian max*  (TYPE_DECODER 1, log_map.h:26) */
#define TDO_ALGO_MAXLOG 1    /* max* == max          (TYPE_DECODER 2, log_map.h:27; not implemented in the ref) */
#define TDO_ALGO_LOGMAP_Q 2  /* the windowed schedule's one-read table (td_set_window_maxstar TD_WMAXSTAR_FAST):
                                E_algorithm's correction at the midpoint of d's bucket, 8 buckets an octave */

/* Trellis tables, same meaning as TURBO_TRELLIS (log_map.h:58-66). */
typedef struct {
    int nextout[TDO_NSTATES][4];   /* [s][2u] = 2u-1 (systematic), [s][2u+1] = parity (+-1) */
    int nextstat[TDO_NSTATES][2];
    int lastout[TDO_NSTATES][4];
    int laststat[TDO_NSTATES][2];
    int g_fb[4], g_ff[4];          /* generator taps (TURBO_G.g_matrix rows, log_map.h:44-48) */
} tdo_trellis;

/* log_map.cpp:114-169 (gen_g_matrix) + :281-337 (gen_trellis). Returns 0 on a non-octal generator. */
int tdo_build_trellis(int g_feedback_octal, int g_forward_octal, tdo_trellis* t);
/* log_map.cpp:616-624 */
void tdo_qpp(int K, int f1, int f2, int* pi);

/* log_map.cpp:451-512 rsc_encode (terminated) ; :530-583 encoderm_turbo ; coded has 3K+12 ints */
void tdo_turbo_encode(const tdo_trellis* t, const int* pi, const int* src, int K, int* coded);

/* modanddem.cpp:88-102 (_bpsk_module) */
void tdo_bpsk_map(const int* bits, int n, double* out_i, double* out_q);
/* log_map.cpp:1359-1374 (mgrns): CLT-12 Gaussian from a linear congruential generator */
void tdo_mgrns(double mean, double sigma, double seed, int n, double* a);
/* log_map.cpp:1388-1400 (AWGN) with the seed supplied by the caller instead of rand() */
void tdo_awgn(const double* send, double* r, double sigma, int n, double seed);
/* modanddem.cpp:189-224 (_bpsk_demodule): out = -Kf*(d(y,+1)^2 - d(y,-1)^2) */
void tdo_bpsk_demod(const double* yi, const double* yq, int n, double Kf, double* out);
/* glibc random_r TYPE_3 (the rand() the reference's main.cpp:170,185 and AWGN :1392 call) */
typedef struct { int32_t tbl[31]; int f, b; } tdo_glibc_rand;
void tdo_glibc_srand(tdo_glibc_rand* g, unsigned seed);
int tdo_glibc_rand_next(tdo_glibc_rand* g);
/* One frame of main.cpp:183-202 (source, encode, BPSK, AWGN I/Q, demod) driven by a glibc rand() stream. */
void tdo_make_frame(const tdo_trellis* t, const int* pi, int K, double ebn0_db, tdo_glibc_rand* g,
                    int* src, double* flow);

/* modanddem.cpp:175-187 (module) for M = 1, 2, 3, 4, 6 bits per symbol: N bits -> N/M symbols
 * (_bpsk/_qpsk/_8psk/_16qam/_64qam_module, :88-173; constellations :7-71).  Returns 0, -1 on a bad M. */
int tdo_modulate(const int* bits, int N, int M, double* out_i, double* out_q);
/* modanddem.cpp:674-685 (demodule): max-log bit LLRs of nsym symbols, out[M*nsym]
 * (_bpsk/_qpsk/_8psk/_16qam/_64qam_demodule, :189-671).  Returns 0, -1 on a bad M. */
int tdo_demodulate(const double* yi, const double* yq, int nsym, int M, double Kf, double* out);
/* One frame of main.cpp:183-202 with MODULATION = M and SYMBOL_NUM = (3K+12)/M (the argv
 * configuration, main.cpp:13-15): rate = K/SYMBOL_NUM, sigma = 10^(-EbN0/20) sqrt(0.5/(rate M)). */
void tdo_make_frame_mod(const tdo_trellis* t, const int* pi, int K, double ebn0_db, int M, tdo_glibc_rand* g,
                        int* src, double* flow);

/* Jacobian max* with the 16-step table, log_map.cpp:14-18,779-801 */
double tdo_maxstar(double x, double y);
/* left fold, log_map.cpp:817-829 */
double tdo_maxstar_seq(const double* v, int n);
float tdo_maxstar_f32(float x, float y);
/* TDO_ALGO_LOGMAP_Q's max* (restated from its definition: DESIGN.md 8.3, td_tables.h build_qlut) */
double tdo_maxstar_q(double x, double y);
float tdo_maxstar_q_f32(float x, float y);

/* log_map.cpp:1083-1127: flow (already scaled by 0.5) -> yk[4L] */
void tdo_demultiplex(const double* flow, int K, const int* pi, double* yk);

/* log_map.cpp:898-1047 (Log_MAP_decoder); algo = TDO_ALGO_* */
void tdo_siso_f64(const tdo_trellis* t, const double* recs, const double* La, int terminated,
                  double* LLR, int L, int algo);
void tdo_siso_f32(const tdo_trellis* t, const float* recs, const float* La, int terminated,
                  float* LLR, int L, int algo);

/*
 * log_map.cpp:1146-1280 (TurboDecoding) for one codeword, `iters` iterations.
 * flow[3K+12] channel LLRs (NOT modified; the x0.5 of :1202-1205 is applied to a copy).
 * out[iters*K]      hard bits per iteration (natural order), as the reference's flow_decoded.
 * le_dump (nullable)[iters][2][L]: extrinsic Le after SISO1 / SISO2 of each iteration
 *                   (SISO2's in its own, interleaved, order), as log_map.cpp:1234-1238,1255-1259.
 */
void tdo_turbo_decode_f64(const tdo_trellis* t, const int* pi, const double* flow, int K, int iters,
                          int algo, int* out, double* le_dump);
void tdo_turbo_decode_f32(const tdo_trellis* t, const int* pi, const float* flow, int K, int iters,
                          int algo, int* out, float* le_dump);

/*
 * The sub-block (sliding-window) schedule of td_set_window (BASELINE config 5), restated on
 * log_map.cpp's arithmetic (turbo_oracle_window.inc has the definition and the citations):
 * sub-blocks of W steps, overlap g, chains normalised every nrm positions of their sub-block
 * (the HIP kernel's checkpoint spacing: 4 fp64, 8 fp32), NII boundaries, serial or concurrent
 * SISOs, extrinsic scale.  Same outputs as tdo_turbo_decode_*.
 */
void tdo_turbo_decode_window_f64(const tdo_trellis* t, const int* pi, const double* flow, int K, int iters,
                                 int algo, int W, int g, int nrm, int nii, int concurrent, double scale,
                                 int* out, double* le_dump);
void tdo_turbo_decode_window_f32(const tdo_trellis* t, const int* pi, const float* flow, int K, int iters,
                                 int algo, int W, int g, int nrm, int nii, int concurrent, double scale,
                                 int* out, float* le_dump);
void tdo_window_siso_f64(const tdo_trellis* t, const double* ys, const double* yp, const double* La, int L, int W,
                         int g, int nrm, int algo, int use_nii, const double* nii_a, const double* nii_b,
                         double* new_a, double* new_b, double* LLR);
void tdo_window_siso_f32(const tdo_trellis* t, const float* ys, const float* yp, const float* La, int L, int W,
                         int g, int nrm, int algo, int use_nii, const float* nii_a, const float* nii_b,
                         float* new_a, float* new_b, float* LLR);

/*
 * Batch front-end used for the CPU baseline and the parity tests: B codewords, each flow row
 * of 3K+12 values (f64 or f32 by `f32`), nthreads host threads (codewords dealt round-robin).
 * bits[B][K] = final-iteration hard bits (uint8).  Returns 0.
 */
int tdo_decode_batch(int K, int f1, int f2, int iters, int algo, int f32, const void* flow, int B,
                     uint8_t* bits, int nthreads);

/* Synthetic input (BASELINE workload): B codewords, counter-seeded, BPSK/AWGN(mgrns), f64 LLR. */
void tdo_synth_batch(int K, int f1, int f2, double ebn0_db, uint64_t seed, int B, int* src,
                     double* flow);

#ifdef __cplusplus
}
#endif
#endif
