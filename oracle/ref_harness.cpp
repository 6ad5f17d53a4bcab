// ref_harness.cpp -- TEST INFRASTRUCTURE.  Drives the *compiled reference* (the unmodified
// /root/reference/ITTC/log_map.cpp + modanddem.cpp, linked by oracle/Makefile into
// oracle/_ref/ref_harness) to produce golden vectors.  No reference source is copied here:
// this file only declares the reference's exported C++ symbols and calls them in the order
// ITTC/main.cpp and TurboDecoding (log_map.cpp:1146-1280) do.
//
// Modes (all binary output is little-endian, written to the file named last):
//   frames K f1 f2 ebn0 seed nframes iters out    -- main.cpp:170-221 frames + per-iteration Le dumps
//   siso L terminated seed out                    -- one Log_MAP_decoder call (log_map.cpp:898)
//   maxstar n seed out                            -- E_algorithm on random + edge pairs (:779)
//   ber K f1 f2 iters ebn0 maxframes minerr seed  -- BER/BLER via TurboDecoding (prints one line)
//   time K f1 f2 nframes                          -- ms per TurboDecoding call (15 iterations)
//   demod M nsym seed out                         -- demodule() on random + constellation-point symbols
//   framesmod K f1 f2 M ebn0 seed nframes out     -- main.cpp frames with MODULATION = M (src, flow)
//   decode K f1 f2 iters nthreads in out          -- the CPU baseline of bench.py: frames read from `in`
//                                                    (nframes x (3K+12) doubles) decoded through the
//                                                    reference's functions in TurboDecoding's order,
//                                                    frames spread over threads; writes the last
//                                                    iteration's bits (uint8) and prints the wall time
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// ---- globals the reference expects from ITTC/main.h:6-11 (defined by the caller, as main.cpp does)
int source_length;
int MODULATION;
int length_after_code;
int f1, f2;
int SYMBOL_NUM;

// ---- reference symbols (C++ linkage), log_map.cpp / modanddem.cpp
void TurboCodingInit();
void TurboEnCoding(int* source, int* coded_source, int source_length);
void TurboDecoding(double* flow_for_decode, int* flow_decoded, int flow_length);
void TurboCodingRelease();
void AWGN(double* send, double* r, double sigma, int totallength);
void module(int* a, double* outi, double* outq, int N, int modu_index);
void demodule(double* symbol_i, double* symbol_q, int symbol_len, double* out, double Kf, int modu_index);
void Log_MAP_decoder(double* recs_turbo, double* La_turbo, int terminated, double* LLR_all_turbo, int len_total);
void demultiplex(double* rec_turbo, int len_info, double* yk_turbo);
void randominterleaver_double(double* data_unintlvr, double* interleaverddata, int* index_randomintlvr, int length);
void random_deinterlvr_double(double* data_unintlvr, double* interleaverddata, int* index_randomintlvr, int length);
void random_deinterlvr_int(int* data_unintlvr, int* interleaverddata, int* index_randomintlvr, int length);
void decision(double* LLR_seq, int length, int* output);
double E_algorithm(double x, double y);
extern int* index_randomintlvr;
extern int M_num_reg;

static const int kRefIters = 15;   // N_ITERATION, log_map.h:30

static void setup(int K, int a, int b, int M = 1)
{
    MODULATION = M;   // the argv configuration of main.cpp:13-15
    source_length = K;
    length_after_code = 3 * K + 12;
    SYMBOL_NUM = length_after_code / M;
    f1 = a;
    f2 = b;
    TurboCodingInit();
}

// main.cpp:174,183-202 -- one frame into src/flow (rand() stream already seeded)
static void make_frame(int K, double ebn0, int* src, double* flow)
{
    const int n = 3 * K + 4 * M_num_reg;
    double rate = (double)source_length / (double)SYMBOL_NUM;
    double sigma = pow(10, -ebn0 / 20) * sqrt(0.5 / (rate * MODULATION));
    std::vector<int> coded(n);
    std::vector<double> mi(n), mq(n), ri(n), rq(n);
    for (int i = 0; i < K; i++) src[i] = rand() % 2;
    TurboEnCoding(src, coded.data(), K);
    module(coded.data(), mi.data(), mq.data(), SYMBOL_NUM * MODULATION, MODULATION);
    AWGN(mi.data(), ri.data(), sigma, SYMBOL_NUM);
    AWGN(mq.data(), rq.data(), sigma, SYMBOL_NUM);
    demodule(ri.data(), rq.data(), SYMBOL_NUM, flow, 1 / (2 * pow(sigma, 2)), MODULATION);
}

// TurboDecoding's iteration loop (log_map.cpp:1200-1265) replayed through the exported
// functions so that the extrinsic Le after every SISO can be captured.
static void replay(int K, const double* flow_in, int iters, double* le, int* bits)
{
    const int L = K + M_num_reg, n = 3 * K + 4 * M_num_reg;
    std::vector<double> flow(flow_in, flow_in + n), yk(4 * L), La(L, 0.0), Le(L, 0.0), LLR(L, 0.0);
    std::vector<int> tempout(L);
    for (int i = 0; i < n; i++) flow[i] *= 0.5;
    demultiplex(flow.data(), K, yk.data());
    for (int it = 0; it < iters; it++) {
        random_deinterlvr_double(La.data(), Le.data(), index_randomintlvr, K);
        for (int i = K; i < L; i++) La[i] = 0;
        Log_MAP_decoder(yk.data(), La.data(), 1, LLR.data(), L);
        for (int i = 0; i < L; i++) Le[i] = LLR[i] - La[i] - 2 * (yk[2 * i]);
        memcpy(le + ((size_t)it * 2 + 0) * L, Le.data(), sizeof(double) * L);
        randominterleaver_double(Le.data(), La.data(), index_randomintlvr, K);
        for (int i = K; i < L; i++) La[i] = 0;
        Log_MAP_decoder(yk.data() + 2 * L, La.data(), 1, LLR.data(), L);
        for (int i = 0; i < L; i++) Le[i] = LLR[i] - La[i] - 2 * (yk[2 * L + 2 * i]);
        memcpy(le + ((size_t)it * 2 + 1) * L, Le.data(), sizeof(double) * L);
        decision(LLR.data(), L, tempout.data());
        random_deinterlvr_int(bits + (size_t)K * it, tempout.data(), index_randomintlvr, K);
    }
}

static FILE* must_open(const char* p)
{
    FILE* f = fopen(p, "wb");
    if (!f) {
        perror(p);
        exit(2);
    }
    return f;
}

static int mode_frames(int argc, char** argv)
{
    if (argc != 10) return 2;
    int K = atoi(argv[2]), a = atoi(argv[3]), b = atoi(argv[4]);
    double ebn0 = atof(argv[5]);
    unsigned seed = (unsigned)strtoul(argv[6], 0, 10);
    int nf = atoi(argv[7]), iters = atoi(argv[8]);
    setup(K, a, b);
    const int L = K + 3, n = 3 * K + 12;
    FILE* f = must_open(argv[9]);
    srand(seed);
    std::vector<int> src(K), bits((size_t)iters * K), direct((size_t)kRefIters * K);
    std::vector<double> flow(n), work(n), le((size_t)iters * 2 * L);
    int mismatch = 0;
    for (int fr = 0; fr < nf; fr++) {
        make_frame(K, ebn0, src.data(), flow.data());
        replay(K, flow.data(), iters, le.data(), bits.data());
        work = flow;
        TurboDecoding(work.data(), direct.data(), n);   // cross-check the replay
        for (int it = 0; it < iters && it < kRefIters; it++)
            mismatch += memcmp(&bits[(size_t)it * K], &direct[(size_t)it * K], sizeof(int) * K) != 0;
        fwrite(src.data(), sizeof(int), K, f);
        fwrite(flow.data(), sizeof(double), n, f);
        fwrite(le.data(), sizeof(double), le.size(), f);
        fwrite(bits.data(), sizeof(int), bits.size(), f);
    }
    fclose(f);
    TurboCodingRelease();
    printf("replay_vs_TurboDecoding_mismatching_rows %d\n", mismatch);
    return 0;
}

static double urand() { return rand() / (double)RAND_MAX; }

static int mode_siso(int argc, char** argv)
{
    if (argc != 6) return 2;
    int L = atoi(argv[2]), term = atoi(argv[3]);
    srand((unsigned)strtoul(argv[4], 0, 10));
    setup(L - 3, 1, 0);   // tables only; K/pi unused by Log_MAP_decoder
    std::vector<double> recs(2 * L), La(L), LLR(L);
    for (int i = 0; i < 2 * L; i++) recs[i] = (urand() * 2 - 1) * 3.0;
    for (int i = 0; i < L; i++) La[i] = (urand() * 2 - 1) * 6.0;
    Log_MAP_decoder(recs.data(), La.data(), term, LLR.data(), L);
    FILE* f = must_open(argv[5]);
    fwrite(recs.data(), sizeof(double), recs.size(), f);
    fwrite(La.data(), sizeof(double), La.size(), f);
    fwrite(LLR.data(), sizeof(double), LLR.size(), f);
    fclose(f);
    TurboCodingRelease();
    return 0;
}

static int mode_maxstar(int argc, char** argv)
{
    if (argc != 5) return 2;
    int nr = atoi(argv[2]);
    srand((unsigned)strtoul(argv[3], 0, 10));
    static const double th[16] = {0.0,    0.08824, 0.19587, 0.31026, 0.43275, 0.56508, 0.70963, 0.86972,
                                  1.0502, 1.2587,  1.5078,  1.8212,  2.2522,  2.9706,  3.6764,  4.3758};
    std::vector<double> xs, ys;
    for (int k = 0; k < 16; k++)   // pairs whose |y-x| lands exactly on / next to each threshold
        for (int d = -1; d <= 1; d++) {
            double t = th[k];
            double v = d < 0 ? nextafter(t, -1.0) : d > 0 ? nextafter(t, 10.0) : t;
            xs.push_back(0.0); ys.push_back(v);
            xs.push_back(v); ys.push_back(0.0);
            xs.push_back(-5.25); ys.push_back(-5.25 + v);
        }
    for (int i = 0; i < nr; i++) {
        xs.push_back((urand() * 2 - 1) * 20);
        ys.push_back(xs.back() + (urand() * 2 - 1) * 5);
    }
    FILE* f = must_open(argv[4]);
    int m = (int)xs.size();
    std::vector<double> r(m);
    for (int i = 0; i < m; i++) r[i] = E_algorithm(xs[i], ys[i]);
    fwrite(&m, sizeof(int), 1, f);
    fwrite(xs.data(), sizeof(double), m, f);
    fwrite(ys.data(), sizeof(double), m, f);
    fwrite(r.data(), sizeof(double), m, f);
    fclose(f);
    return 0;
}

// BER/BLER at one Eb/N0, main.cpp:172-257 protocol (stop after minerr block errors at the
// measured iteration), rows of TurboDecoding's 15-iteration output.
static int mode_ber(int argc, char** argv)
{
    if (argc != 10) return 2;
    int K = atoi(argv[2]), a = atoi(argv[3]), b = atoi(argv[4]), iters = atoi(argv[5]);
    double ebn0 = atof(argv[6]);
    int maxf = atoi(argv[7]), minerr = atoi(argv[8]);
    setup(K, a, b);
    srand((unsigned)strtoul(argv[9], 0, 10));
    const int n = 3 * K + 12;
    std::vector<int> src(K), out((size_t)kRefIters * K);
    std::vector<double> flow(n);
    long long bit_err[kRefIters] = {0}, blk_err[kRefIters] = {0};
    int nf = 0;
    for (; nf < maxf; nf++) {
        make_frame(K, ebn0, src.data(), flow.data());
        TurboDecoding(flow.data(), out.data(), n);
        for (int it = 0; it < kRefIters; it++) {
            int e = 0;
            for (int i = 0; i < K; i++) e += src[i] != out[(size_t)it * K + i];
            bit_err[it] += e;
            blk_err[it] += e != 0;
        }
        if (blk_err[iters - 1] >= minerr) {
            nf++;
            break;
        }
    }
    printf("ebn0 %.3f frames %d", ebn0, nf);
    for (int it = 0; it < kRefIters; it++) printf(" %lld:%lld", bit_err[it], blk_err[it]);
    printf("\n");
    TurboCodingRelease();
    return 0;
}

static int mode_time(int argc, char** argv)
{
    if (argc != 6) return 2;
    int K = atoi(argv[2]), a = atoi(argv[3]), b = atoi(argv[4]), nf = atoi(argv[5]);
    setup(K, a, b);
    srand(1);
    const int n = 3 * K + 12;
    std::vector<int> src(K), out((size_t)kRefIters * K);
    std::vector<double> flow(n);
    make_frame(K, 1.0, src.data(), flow.data());
    double total = 0;
    for (int fr = 0; fr < nf; fr++) {
        std::vector<double> w = flow;
        auto t0 = std::chrono::steady_clock::now();
        TurboDecoding(w.data(), out.data(), n);
        total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    printf("ms_per_frame_15iter %.3f\n", total / nf);
    TurboCodingRelease();
    return 0;
}

// demodule() (modanddem.cpp:674) on nsym symbols: uniform in [-2, 2]^2, plus every
// constellation point of every modulation exactly, plus points midway between levels
static int mode_demod(int argc, char** argv)
{
    if (argc != 6) return 2;
    int M = atoi(argv[2]), nsym = atoi(argv[3]);
    srand((unsigned)strtoul(argv[4], 0, 10));
    std::vector<int> bits(64 * 6);
    std::vector<double> yi(nsym), yq(nsym), ci(64), cq(64), out((size_t)nsym * M);
    int k = 0;
    const int Ms[5] = {1, 2, 3, 4, 6};
    for (int mi = 0; mi < 5; mi++) {   // the constellation points, through module()
        const int m = Ms[mi];
        for (int j = 0; j < (1 << m); j++)
            for (int b = 0; b < m; b++) bits[(size_t)j * m + b] = (j >> (m - 1 - b)) & 1;
        module(bits.data(), ci.data(), cq.data(), (1 << m) * m, m);
        for (int j = 0; j < (1 << m) && k < nsym; j++, k++) {
            yi[k] = ci[j];
            yq[k] = cq[j];
        }
    }
    for (int j = 0; j < 8 && k < nsym; j++, k++) {   // on the 16QAM / 64QAM decision boundaries
        yi[k] = (j & 1 ? 0.632456 : 0.0) * (j & 2 ? -1 : 1);
        yq[k] = (j & 4 ? 0.3086 : 0.0);
    }
    for (; k < nsym; k++) {
        yi[k] = 4.0 * rand() / RAND_MAX - 2.0;
        yq[k] = 4.0 * rand() / RAND_MAX - 2.0;
    }
    demodule(yi.data(), yq.data(), nsym, out.data(), 1.7, M);
    FILE* f = must_open(argv[5]);
    fwrite(yi.data(), sizeof(double), nsym, f);
    fwrite(yq.data(), sizeof(double), nsym, f);
    fwrite(out.data(), sizeof(double), out.size(), f);
    fclose(f);
    return 0;
}

// TurboDecoding (log_map.cpp:1146-1280) with `iters` iterations instead of the N_ITERATION
// macro, on many frames: the same loop as replay() minus the Le dumps.  The reference is
// re-entrant after TurboCodingInit (read-only globals, per-call mallocs), so threads decode
// frames round-robin.  Output: the hard bits after the last iteration (uint8, natural order).
static void decode_one(int K, const double* flow_in, int iters, unsigned char* out)
{
    const int L = K + M_num_reg, n = 3 * K + 4 * M_num_reg;
    std::vector<double> flow(flow_in, flow_in + n), yk(4 * L), La(L, 0.0), Le(L, 0.0), LLR(L, 0.0);
    std::vector<int> tempout(L), bits(K);
    for (int i = 0; i < n; i++) flow[i] *= 0.5;
    demultiplex(flow.data(), K, yk.data());
    for (int it = 0; it < iters; it++) {
        random_deinterlvr_double(La.data(), Le.data(), index_randomintlvr, K);
        for (int i = K; i < L; i++) La[i] = 0;
        Log_MAP_decoder(yk.data(), La.data(), 1, LLR.data(), L);
        for (int i = 0; i < L; i++) Le[i] = LLR[i] - La[i] - 2 * (yk[2 * i]);
        randominterleaver_double(Le.data(), La.data(), index_randomintlvr, K);
        for (int i = K; i < L; i++) La[i] = 0;
        Log_MAP_decoder(yk.data() + 2 * L, La.data(), 1, LLR.data(), L);
        for (int i = 0; i < L; i++) Le[i] = LLR[i] - La[i] - 2 * (yk[2 * L + 2 * i]);
        decision(LLR.data(), L, tempout.data());
        random_deinterlvr_int(bits.data(), tempout.data(), index_randomintlvr, K);
    }
    for (int i = 0; i < K; i++) out[i] = (unsigned char)bits[i];
}

static int mode_decode(int argc, char** argv)
{
    if (argc != 9) return 2;
    int K = atoi(argv[2]), a = atoi(argv[3]), b = atoi(argv[4]), iters = atoi(argv[5]), nt = atoi(argv[6]);
    setup(K, a, b);
    const size_t n = 3 * (size_t)K + 12;
    FILE* fi = fopen(argv[7], "rb");
    if (!fi) {
        perror(argv[7]);
        return 2;
    }
    std::vector<double> flows;
    {
        std::vector<double> buf(n);
        while (fread(buf.data(), sizeof(double), n, fi) == n) flows.insert(flows.end(), buf.begin(), buf.end());
    }
    fclose(fi);
    const int nf = (int)(flows.size() / n);
    if (nt < 1) nt = 1;
    std::vector<unsigned char> out((size_t)nf * K);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            for (int fr = t; fr < nf; fr += nt) decode_one(K, flows.data() + (size_t)fr * n, iters, out.data() + (size_t)fr * K);
        });
    for (auto& x : th) x.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    FILE* f = must_open(argv[8]);
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    printf("seconds %.6f frames %d threads %d\n", sec, nf, nt);
    TurboCodingRelease();
    return 0;
}

// main.cpp:170-202 frames with MODULATION = M: src [K] int32 + flow [3K+12] double per frame
static int mode_framesmod(int argc, char** argv)
{
    if (argc != 10) return 2;
    int K = atoi(argv[2]), a = atoi(argv[3]), b = atoi(argv[4]), M = atoi(argv[5]);
    double ebn0 = atof(argv[6]);
    unsigned seed = (unsigned)strtoul(argv[7], 0, 10);
    int nf = atoi(argv[8]);
    setup(K, a, b, M);
    const int n = 3 * K + 12;
    FILE* f = must_open(argv[9]);
    srand(seed);
    std::vector<int> src(K);
    std::vector<double> flow(n);
    for (int fr = 0; fr < nf; fr++) {
        make_frame(K, ebn0, src.data(), flow.data());
        fwrite(src.data(), sizeof(int), K, f);
        fwrite(flow.data(), sizeof(double), n, f);
    }
    fclose(f);
    TurboCodingRelease();
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    if (!strcmp(argv[1], "frames")) return mode_frames(argc, argv);
    if (!strcmp(argv[1], "siso")) return mode_siso(argc, argv);
    if (!strcmp(argv[1], "maxstar")) return mode_maxstar(argc, argv);
    if (!strcmp(argv[1], "ber")) return mode_ber(argc, argv);
    if (!strcmp(argv[1], "time")) return mode_time(argc, argv);
    if (!strcmp(argv[1], "demod")) return mode_demod(argc, argv);
    if (!strcmp(argv[1], "framesmod")) return mode_framesmod(argc, argv);
    if (!strcmp(argv[1], "decode")) return mode_decode(argc, argv);
    fprintf(stderr, "unknown mode\n");
    return 2;
}
