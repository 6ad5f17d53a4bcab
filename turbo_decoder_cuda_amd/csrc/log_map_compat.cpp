// log_map_compat.cpp -- drop-in replacement for ITTC/log_map.cpp at link level.
//
// Exports the C++ symbols ITTC/main.cpp takes from log_map.o:
//   int  M_num_reg                                      log_map.cpp:28
//   void TurboCodingInit()                              log_map.cpp:349-434
//   void TurboEnCoding(int*, int*, int)                 log_map.cpp:700-730 (encoderm_turbo :530-583)
//   void TurboDecoding(double*, int*, int)              log_map.cpp:1146-1280
//   void TurboCodingRelease()                           log_map.cpp:1330-1345
//   void AWGN(double*, double*, double, int)            log_map.cpp:1388-1400 (mgrns :1359-1374)
//   void Log_MAP_decoder(double*, double*, int, double*, int)   log_map.cpp:898-1047
// and reads the caller's globals source_length / f1 / f2 (ITTC/main.h:6-11) without defining
// them.  The decode runs on the MI355X through the C ABI (include/turbo_mi355x.h); nothing
// here decodes on the CPU.  Reference behaviour kept on purpose:
//   * TurboDecoding scales flow[] by 0.5 in place (log_map.cpp:1202-1205) and fills
//     out[N_ITERATION*K], one row of hard bits per iteration (:1261-1264);
//   * failures print a message and exit(1), as the reference does (:288-292, 357-368);
//   * AWGN draws its seed from the process's rand() exactly like the reference.
// Environment, read when the handle opens (TurboCodingInit, or a new K): TD_DEVICE (HIP ordinal,
// default 0), TD_ITERATIONS (default 15 = N_ITERATION), TD_ALGO ("logmap" | "maxlog").
// Opt-in low-latency schedule (default: the exact schedule, bit-exact with log_map.cpp):
//   TD_WINDOW=W     sub-blocks of W trellis steps decoded in parallel (td_set_window); the frame's
//                   time is then one sub-block's chains instead of the whole trellis's
//   TD_OVERLAP=g    warm-up steps of each sub-block's alpha / beta (default min(30, 3W))
//   TD_NII=1        boundary metrics from the previous iteration
//   TD_CONCURRENT=1 both SISOs at once (Jacobi); TD_EXT_SCALE=s extrinsic scale (default 1)
//   TD_WINDOW_MAXSTAR=exact  log_map.cpp's E_algorithm in the windowed log-MAP schedule (default: the
//                   one-read table, td_set_window_maxstar)
// A windowed schedule changes the arithmetic (sub-block boundaries): its results are gated by
// the BER curve, not bit-exact.  Log_MAP_decoder always runs the exact SISO.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "turbo_mi355x.h"

extern int source_length;   // defined by the caller (ITTC/main.h:6)
extern int f1, f2;          // ITTC/main.h:9

int M_num_reg = 3;          // log_map.cpp:28 (memory of the 13/15 RSC)

namespace {

td_handle* g_h = nullptr;
int g_K = 0, g_iters = 15;

[[noreturn]] void die(const char* what, int rc)
{
    std::printf("turbo_mi355x: %s failed (%d): %s\n", what, rc, td_last_error());
    std::exit(1);
}

int env_int(const char* name, int dflt)
{
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

double env_double(const char* name, double dflt)
{
    const char* v = std::getenv(name);
    return v && *v ? std::atof(v) : dflt;
}

// TD_WINDOW & co. (see the file header): the exact schedule unless TD_WINDOW is set and non-zero
void set_schedule(td_handle* h)
{
    const int W = env_int("TD_WINDOW", 0);
    if (W == 0) return;
    td_window_params w{};
    w.window = W;
    w.overlap = env_int("TD_OVERLAP", W > 0 && 3 * W < 30 ? 3 * W : 30);
    w.nii = env_int("TD_NII", 0);
    w.concurrent = env_int("TD_CONCURRENT", 0);
    w.ext_scale = env_double("TD_EXT_SCALE", 1.0);
    const char* ms = std::getenv("TD_WINDOW_MAXSTAR");
    int rc = td_set_window_maxstar(h, ms && std::strcmp(ms, "exact") == 0 ? TD_WMAXSTAR_EXACT : TD_WMAXSTAR_FAST);
    if (rc) die("td_set_window_maxstar (TD_WINDOW_MAXSTAR)", rc);
    rc = td_set_window(h, &w);
    if (rc) die("td_set_window (TD_WINDOW / TD_OVERLAP / TD_EXT_SCALE)", rc);
}

void open_handle(int K)
{
    if (g_h && g_K == K) return;
    if (g_h) td_destroy(g_h);
    g_h = nullptr;
    const char* a = std::getenv("TD_ALGO");
    td_params p{};
    p.K = K;
    p.f1 = f1;
    p.f2 = f2;
    p.iterations = g_iters;
    p.algo = (a && std::strcmp(a, "maxlog") == 0) ? TD_ALGO_MAXLOG : TD_ALGO_LOGMAP;
    p.precision = TD_F64;
    p.device = env_int("TD_DEVICE", 0);
    const int rc = td_create(&g_h, &p);
    if (rc) die("td_create", rc);
    set_schedule(g_h);
    g_K = K;
}

// 13/15 RSC, trellis-terminated (rsc_encode / encode_bit, log_map.cpp:247-269, 451-528).
// Writes K+3 (systematic, parity) pairs.
void rsc(const int* u, int K, int* sys, int* par)
{
    int s0 = 0, s1 = 0, s2 = 0;   // s0 = newest register bit
    for (int i = 0; i < K + 3; ++i) {
        const int fb = (s1 + s2) & 1;              // feedback taps 1011 (13 octal)
        const int d = i < K ? u[i] : fb;           // tail bits drive the register to zero
        const int ak = (d + fb) & 1;
        par[i] = (ak + s0 + s2) & 1;               // forward taps 1101 (15 octal)
        sys[i] = d;
        s2 = s1;
        s1 = s0;
        s0 = ak;
    }
}

}  // namespace

void TurboCodingInit()
{
    // main.cpp sizes flow_decoded as N_ITERATION (15) rows of K (main.cpp:153) and TurboDecoding
    // writes one row per iteration: more than 15 would write past the caller's buffer.
    g_iters = env_int("TD_ITERATIONS", 15);
    if (g_iters < 1 || g_iters > 15) {
        std::printf("turbo_mi355x: TD_ITERATIONS=%d is outside [1, 15] (N_ITERATION rows of flow_decoded)\n", g_iters);
        std::exit(1);
    }
    open_handle(source_length);
}

void TurboCodingRelease()
{
    if (g_h) td_destroy(g_h);
    g_h = nullptr;
    g_K = 0;
}

// encoderm_turbo stream layout (log_map.cpp:566-578): (x, p1, p2) per info bit, then the
// first encoder's 3 tail (x, p) pairs, then the second encoder's.
void TurboEnCoding(int* source, int* coded_source, int K)
{
    std::vector<int> pi(K), ui(K), s1(K + 3), p1(K + 3), s2(K + 3), p2(K + 3);
    int rc = td_qpp_table(K, f1, f2, pi.data());
    if (rc) die("td_qpp_table", rc);
    for (int i = 0; i < K; ++i) ui[i] = source[pi[i]];
    rsc(source, K, s1.data(), p1.data());
    rsc(ui.data(), K, s2.data(), p2.data());
    for (int i = 0; i < K; ++i) {
        coded_source[3 * i] = s1[i];
        coded_source[3 * i + 1] = p1[i];
        coded_source[3 * i + 2] = p2[i];
    }
    for (int t = 0; t < 3; ++t) {
        coded_source[3 * K + 2 * t] = s1[K + t];
        coded_source[3 * K + 2 * t + 1] = p1[K + t];
        coded_source[3 * K + 6 + 2 * t] = s2[K + t];
        coded_source[3 * K + 6 + 2 * t + 1] = p2[K + t];
    }
}

void TurboDecoding(double* flow_for_decode, int* flow_decoded, int flow_length)
{
    const int K = (flow_length - 12) / 3;   // log_map.cpp:1160
    open_handle(K);
    const int rc = td_decode_host(g_h, flow_for_decode, 1, flow_decoded, nullptr);
    if (rc) die("td_decode_host", rc);
    for (int i = 0; i < flow_length; ++i) flow_for_decode[i] *= 0.5;   // the reference's side effect
}

void Log_MAP_decoder(double* recs, double* La, int terminated, double* LLR, int L)
{
    if (!g_h) open_handle(L > 3 ? L - 3 : 1);
    const int rc = td_siso_host(g_h, recs, La, terminated, LLR, L, 1);
    if (rc) die("td_siso_host", rc);
}

// mgrns (log_map.cpp:1359-1374): sum of 12 LCG uniforms per sample (CLT), support +-6 sigma.
static void mgrns(double mean, double sigma, double seed, int n, double* a)
{
    const double s = 65536.0, w = 2053.0, v = 13849.0;
    for (int k = 0; k < n; ++k) {
        double t = 0.0;
        for (int i = 0; i < 12; ++i) {
            seed = seed * w + v;
            const int m = (int)(seed / s);
            seed = seed - m * s;
            t = t + seed / s;
        }
        a[k] = mean + sigma * (t - 6.0);
    }
}

void AWGN(double* send, double* r, double sigma, int totallength)
{
    std::vector<double> noise(totallength > 0 ? totallength : 0);
    const double seed = 3.0 - (double)((rand() & RAND_MAX) / (double)RAND_MAX) / 10e6;
    mgrns(0, sigma, seed, totallength, noise.data());
    for (int i = 0; i < totallength; ++i) r[i] = send[i] + noise[i];
}
