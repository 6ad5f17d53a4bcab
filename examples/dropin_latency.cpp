// dropin_latency.cpp -- what the UNCHANGED reference caller gets per frame through the drop-in.
// Plays ITTC/main.cpp's part exactly as main.cpp:221 does: defines the main.h globals, calls
// TurboCodingInit() once, then TurboDecoding(flow, out, 3K+12) one frame per call (out[15][K], the
// N_ITERATION rows; TD_ITERATIONS in the environment sets the compat layer's iteration count), and
// TurboCodingRelease().  Linked against libturbo_logmap_compat.so (csrc/log_map_compat.cpp) in place
// of log_map.o.  The first call (handle creation, staging allocation, code object load) is timed
// apart; the rest are the warm per-frame latency.
//
//   td_dropin_latency K f1 f2 nframes flows.bin bits.bin
//     flows.bin  nframes x (3K+12) doubles (TurboDecoding's input, channel LLRs 2y/sigma^2)
//     bits.bin   nframes x K uint8: the last iteration's row of each frame's out[]
// Prints one JSON object: frames, ms_first, ms_per_frame (mean of frames 1..n-1), ms_min.
//
// Built by turbo_decoder_cuda_amd/build.py (g++, host code only).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int source_length, MODULATION, length_after_code, f1, f2, SYMBOL_NUM;   // ITTC/main.h:6-11
extern int M_num_reg;

void TurboCodingInit();
void TurboDecoding(double* flow_for_decode, int* flow_decoded, int flow_length);
void TurboCodingRelease();

int main(int argc, char** argv)
{
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s K f1 f2 nframes flows.bin bits.bin\n", argv[0]);
        return 2;
    }
    source_length = std::atoi(argv[1]);
    f1 = std::atoi(argv[2]);
    f2 = std::atoi(argv[3]);
    const int nf = std::atoi(argv[4]);
    const int K = source_length, n = 3 * K + 4 * M_num_reg;
    const char* it_env = std::getenv("TD_ITERATIONS");
    const int iters = it_env ? std::atoi(it_env) : 15;
    std::vector<double> flow((size_t)nf * n);
    FILE* f = std::fopen(argv[5], "rb");
    if (!f || std::fread(flow.data(), sizeof(double), flow.size(), f) != flow.size()) {
        std::fprintf(stderr, "read %s failed\n", argv[5]);
        return 2;
    }
    std::fclose(f);
    std::vector<int> out(15 * (size_t)K);   // main.cpp:153: flow_decoded[N_ITERATION][K]
    std::vector<unsigned char> bits((size_t)nf * K);
    TurboCodingInit();
    double first = 0, sum = 0, mn = 1e30;
    for (int fr = 0; fr < nf; ++fr) {
        const auto t0 = std::chrono::steady_clock::now();
        TurboDecoding(flow.data() + (size_t)fr * n, out.data(), n);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (fr == 0) {
            first = ms;
        } else {
            sum += ms;
            mn = ms < mn ? ms : mn;
        }
        for (int i = 0; i < K; ++i) bits[(size_t)fr * K + i] = (unsigned char)out[(size_t)(iters - 1) * K + i];
    }
    TurboCodingRelease();
    f = std::fopen(argv[6], "wb");
    if (!f || std::fwrite(bits.data(), 1, bits.size(), f) != bits.size()) {
        std::fprintf(stderr, "write %s failed\n", argv[6]);
        return 2;
    }
    std::fclose(f);
    std::printf("{\"frames\": %d, \"iterations\": %d, \"ms_first\": %.4f, \"ms_per_frame\": %.4f, \"ms_min\": %.4f}\n", nf,
                iters, first, nf > 1 ? sum / (nf - 1) : first, nf > 1 ? mn : first);
    return 0;
}
