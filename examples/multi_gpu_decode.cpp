// multi_gpu_decode.cpp -- a C++ caller of the C ABI that spreads one batch over several GPUs:
// one td_handle, one host thread and one HIP stream per device ordinal, each
// decoding a contiguous slice of the batch.  The path shards by codeword, so there is no
// exchange between the threads: each slice goes HBM -> decode -> host on its own device.
//
//   multi_gpu_decode K f1 f2 iterations flows.bin bits.bin ORD [ORD ...]
//     flows.bin  B x (3K+12) doubles (ITTC/main.cpp:221's TurboDecoding input, B from the size)
//     bits.bin   B x K uint8 hard decisions of the last iteration, in batch order
//     ORD        HIP device ordinals, one worker thread each (the same ordinal may repeat: two
//                handles on one device then run side by side, each with its own workspace)
//
// Build (host code only; HIP runtime for device buffers and streams):
//   g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include multi_gpu_decode.cpp \
//       -L turbo_decoder_cuda_amd -lturbo_mi355x -L /opt/rocm/lib -lamdhip64 -lpthread \
//       -Wl,-rpath,turbo_decoder_cuda_amd -Wl,-rpath,/opt/rocm/lib
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "turbo_mi355x.h"

namespace {

struct Slice {
    int ordinal;
    long first, count;       // codewords [first, first + count) of the batch
    int rc = 0;
    std::string err;
};

#define CHECK_HIP(x)                                                          \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            s.rc = 3;                                                         \
            s.err = std::string(#x ": ") + hipGetErrorString(e_);             \
            goto done;                                                        \
        }                                                                     \
    } while (0)

// One worker: its own handle on its device, its own stream, its own buffers.
void worker(Slice& s, const td_params& base, const double* flows, uint8_t* bits)
{
    const int K = base.K;
    const size_t n = 3 * (size_t)K + 12;
    td_params p = base;
    p.device = s.ordinal;
    td_handle* h = nullptr;
    hipStream_t st = nullptr;
    void* d_llr = nullptr;
    void* d_bits = nullptr;
    if (s.count == 0) return;
    if (td_create(&h, &p) != TD_OK) {   // binds the handle to p.device
        s.rc = 1;
        s.err = td_last_error();
        return;
    }
    CHECK_HIP(hipSetDevice(s.ordinal));   // this thread's buffers and stream live on the same device
    CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CHECK_HIP(hipMalloc(&d_llr, s.count * n * sizeof(double)));
    CHECK_HIP(hipMalloc(&d_bits, s.count * (size_t)K));
    if (td_reserve(h, (int)s.count) != TD_OK) {
        s.rc = 1;
        s.err = td_last_error();
        goto done;
    }
    CHECK_HIP(hipMemcpyAsync(d_llr, flows + s.first * n, s.count * n * sizeof(double), hipMemcpyHostToDevice, st));
    if (td_decode_device(h, d_llr, (int)s.count, static_cast<uint8_t*>(d_bits), 0, nullptr, st) != TD_OK) {
        s.rc = 1;
        s.err = td_last_error();
        goto done;
    }
    CHECK_HIP(hipMemcpyAsync(bits + s.first * K, d_bits, s.count * (size_t)K, hipMemcpyDeviceToHost, st));
    CHECK_HIP(hipStreamSynchronize(st));
done:
    if (d_llr) (void)hipFree(d_llr);
    if (d_bits) (void)hipFree(d_bits);
    if (st) (void)hipStreamDestroy(st);
    td_destroy(h);
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc < 8) {
        std::fprintf(stderr, "usage: %s K f1 f2 iterations flows.bin bits.bin ORD [ORD ...]\n", argv[0]);
        return 2;
    }
    td_params base{};
    base.K = std::atoi(argv[1]);
    base.f1 = std::atoi(argv[2]);
    base.f2 = std::atoi(argv[3]);
    base.iterations = std::atoi(argv[4]);
    base.algo = TD_ALGO_LOGMAP;
    base.precision = TD_F64;
    const size_t n = 3 * (size_t)base.K + 12;
    FILE* f = std::fopen(argv[5], "rb");
    if (!f) return 2;
    std::fseek(f, 0, SEEK_END);
    const long B = std::ftell(f) / (long)(n * sizeof(double));
    std::fseek(f, 0, SEEK_SET);
    std::vector<double> flows(B * n);
    if (std::fread(flows.data(), sizeof(double), flows.size(), f) != flows.size()) return 2;
    std::fclose(f);
    std::vector<uint8_t> bits((size_t)B * base.K);

    const int nw = argc - 7;
    std::vector<Slice> slices;
    for (int w = 0; w < nw; ++w) {   // contiguous slices, the first B % nw one codeword longer
        const long q = B / nw, r = B % nw;
        slices.push_back(Slice{std::atoi(argv[7 + w]), w * q + (w < r ? w : r), q + (w < r ? 1 : 0)});
    }
    std::vector<std::thread> threads;
    for (auto& s : slices) threads.emplace_back(worker, std::ref(s), std::cref(base), flows.data(), bits.data());
    for (auto& t : threads) t.join();
    int rc = 0;
    for (auto& s : slices)
        if (s.rc) {
            std::fprintf(stderr, "device %d, codewords %ld..%ld: %s\n", s.ordinal, s.first, s.first + s.count - 1,
                         s.err.c_str());
            rc = 1;
        }
    if (rc) return rc;
    FILE* o = std::fopen(argv[6], "wb");
    if (!o || std::fwrite(bits.data(), 1, bits.size(), o) != bits.size()) return 2;
    std::fclose(o);
    std::printf("decoded %ld codewords on %d worker(s)\n", B, nw);
    return 0;
}
