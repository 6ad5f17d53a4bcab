// ubench_window.hip -- achievable VALU issue of the windowed kernels' arithmetic (sw_alpha_kernel /
// sw_beta_kernel, csrc/td_kernels.hip) on gfx950: one codeword chain per lane, fp64 log-MAP steps on the
// three-table max* layout (SwLut: 32 columns, thr / vlo / vhi), inputs read from LDS per step, no HBM.
//   MIX 0: the alpha kernel's core -- one alpha step a position (8 max*), normalised every 4;
//   MIX 1: the beta kernel's core -- per position one alpha-recompute step, one beta step and the LLR's
//          two 7-deep left folds (log_map.cpp:1024-1039), both chains normalised every 4;
//   MIX 2, 3: mixes 0, 1 on a two-read table layout (threshold + a 16-byte (lo, hi) pair);
//   MIX 4, 5: the same two reads from one 1 KiB row a bucket (one row address; thr 2-way conflicted).
// Each mix runs at WPS = 1, 2, 3 waves per SIMD (one workgroup of 4 x WPS waves on each of the 256 CUs,
// held to one a CU by LDS padding), so the issue rate at the beta kernel's two waves per SIMD can be read
// against one and three.  Prints per-wave cycles per position; a PMC pass (SQ_INSTS_VALU) gives the
// instructions, scripts/gpu_r5_ubench_window.sh the issue fraction.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-honor-nans -mllvm -amdgpu-sched-strategy=max-ilp
//       -Iturbo_decoder_cuda_amd/csrc -o scripts/ubench_window scripts/ubench_window.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "td_tables.h"

using td::BucketBits;
using td::kLutSize;
using td::kTrellisLast;
using td::kTrellisNext;
using td::kTrellisQ;

constexpr int kCols = 32, kRow = kCols * 8, kRows = kLutSize + 1, kTab = kRows * kRow;
constexpr int kOffV = kTab + 8, kOffH = 2 * kOffV + 8, kLutBytes = kOffH + kTab;
constexpr int kInSteps = 16;   // input rows cycled through (P, Q per lane)
constexpr int kPos = 4096;     // positions a wave steps

// LAY 0: three tables (the kernels' SwLut), three ds_read_b64 a max*.  LAY 1: the threshold table and
// a (lo, hi) pair table of 16-byte entries [bucket][32 columns], two reads a max* (ds_read_b64 +
// ds_read_b128; the b128 read groups {0-3,12-15,20-27}, ... hit distinct banks for any buckets).
constexpr int kPairOff = (kLutBytes + 15) & ~15;   // pair table: 512-byte rows after the three tables, 16-B aligned
template <int LAY>
__device__ __forceinline__ double mstar(double x, double y, const char* lut, const char* lutp)
{
    const double d = y - x;
    const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
    int q = (int)__builtin_amdgcn_ubfe(hi, BucketBits<double>::shift, BucketBits<double>::width);
    q = min(max(q, BucketBits<double>::base), BucketBits<double>::base + kLutSize - 1);
    if constexpr (LAY == 0) {
        const char* r = lut + q * kRow;
        const double thr = *(const double*)r, lo = *(const double*)(r + kOffV), hv = *(const double*)(r + kOffH);
        return fmax(x, y) + (fabs(d) >= thr ? hv : lo);
    } else if constexpr (LAY == 1) {
        const double thr = *(const double*)(lut + q * kRow);
        const double2 v = *(const double2*)(lutp + q * (2 * kRow));
        return fmax(x, y) + (fabs(d) >= thr ? v.y : v.x);
    } else {   // LAY 2: one 1 KiB row per bucket, [32 columns][thr, pad] then [32 columns][lo, hi]
        const char* r = lutp + q * (4 * kRow);
        const double thr = *(const double*)r;
        const double2 v = *(const double2*)(r + 2 * kRow);
        return fmax(x, y) + (fabs(d) >= thr ? v.y : v.x);
    }
}

__device__ __forceinline__ double g(double P, double Q, int s) { return kTrellisQ[s] ? Q : P; }

__device__ __forceinline__ void norm(double (&v)[8])
{
    const double m = fmax(fmax(fmax(v[0], v[1]), fmax(v[2], v[3])), fmax(fmax(v[4], v[5]), fmax(v[6], v[7])));
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] -= m;
}

template <int MIX_, int WPS>
__global__ __launch_bounds__(256 * WPS) void ub(const double* __restrict__ lut_g, const double* __restrict__ in_g,
                                               double* out, unsigned long long* clk)
{
    constexpr int MIX = MIX_ & 1, LAY = MIX_ >> 1;   // LAY 0, 1, 2
    __shared__ alignas(16) char lut_s[LAY == 2 ? kRows * 4 * kRow : kPairOff + kRows * 2 * kRow];
    __shared__ alignas(16) double in_s[kInSteps * 2 * 64];
    if constexpr (LAY == 2) {
        for (int e = threadIdx.x; e < kRows * kCols; e += blockDim.x) {   // row q, column c: e = q * 32 + c
            char* r = lut_s + (e / kCols) * 4 * kRow + (e % kCols) * 16;
            *(double*)r = lut_g[e];
            *(double*)(r + 2 * kRow) = lut_g[kRows * kCols + e];
            *(double*)(r + 2 * kRow + 8) = lut_g[2 * kRows * kCols + e];
        }
    } else {
        for (int e = threadIdx.x; e < 3 * kRows * kCols; e += blockDim.x) {
            const int t = e / (kRows * kCols), o = e % (kRows * kCols);
            *(double*)(lut_s + (t == 0 ? 0 : t == 1 ? kOffV : kOffH) + o * 8) = lut_g[e];
        }
        for (int e = threadIdx.x; e < kRows * kCols; e += blockDim.x) {   // pair table (lo, hi) from tables 1, 2
            *(double*)(lut_s + kPairOff + e * 16) = lut_g[kRows * kCols + e];
            *(double*)(lut_s + kPairOff + e * 16 + 8) = lut_g[2 * kRows * kCols + e];
        }
    }
    for (int e = threadIdx.x; e < kInSteps * 2 * 64; e += blockDim.x) in_s[e] = in_g[e];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const char* lut = lut_s + (lane % kCols) * 8 - BucketBits<double>::base * kRow;
    const char* lutp = LAY == 2 ? lut_s + (lane % kCols) * 16 - BucketBits<double>::base * 4 * kRow
                                : lut_s + kPairOff + (lane % kCols) * 16 - BucketBits<double>::base * 2 * kRow;
    double a[8], b[8], acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = 0.01 * ((j * 7 + lane) & 15);
        b[j] = 0.02 * ((j * 5 + lane) & 15);
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int p = 0; p < kPos; p += 4) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int row = (p + m) % kInSteps;
            const double P = in_s[(row * 2) * 64 + lane], Q = in_s[(row * 2 + 1) * 64 + lane];
            double n[8];
            if constexpr (MIX == 1) {   // LLR of this position from a and b (before either steps)
                double t0[8], t1[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
                    t0[j] = (a[p0] - g(P, Q, p0)) + b[j];
                    t1[j] = (a[p1] + g(P, Q, p1)) + b[j];
                }
                double r0 = mstar<LAY>(t0[0], t0[1], lut, lutp), r1 = mstar<LAY>(t1[0], t1[1], lut, lutp);
#pragma unroll
                for (int j = 2; j < 8; ++j) {
                    r0 = mstar<LAY>(r0, t0[j], lut, lutp);
                    r1 = mstar<LAY>(r1, t1[j], lut, lutp);
                }
                acc += r1 - r0;
                double nb[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const double G = g(P, Q, j);
                    nb[j] = mstar<LAY>(b[kTrellisNext[j][0]] - G, b[kTrellisNext[j][1]] + G, lut, lutp);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) b[j] = nb[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int p0 = kTrellisLast[j][0], p1 = kTrellisLast[j][1];
                n[j] = mstar<LAY>(a[p0] - g(P, Q, p0), a[p1] + g(P, Q, p1), lut, lutp);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = n[j];
            __builtin_amdgcn_sched_barrier(0);
        }
        norm(a);
        if constexpr (MIX == 1) norm(b);
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = acc;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + b[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

template <int MIX, int WPS>
void run(const double* lut, const double* in, double* out, unsigned long long* clk)
{
    // one workgroup of WPS waves per SIMD on each CU: 256 workgroups, dynamic LDS padding past half the
    // CU's 160 KiB so that no CU takes two
    const int blocks = 256;
    const size_t dyn = 96 * 1024;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&ub<MIX, WPS>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)dyn);
    hipLaunchKernelGGL((ub<MIX, WPS>), dim3(blocks), dim3(256 * WPS), dyn, 0, lut, in, out, clk);   // warm-up
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((ub<MIX, WPS>), dim3(blocks), dim3(256 * WPS), dyn, 0, lut, in, out, clk);
    (void)hipEventRecord(e1, 0);
    if (hipGetLastError() != hipSuccess) std::printf("launch failed\n");
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, sizeof c, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;   // memrealtime: 100 MHz
    const double cyc = (double)c[0] / kPos;                            // one wave's cycles per position
    std::printf("{\"mix\": %d, \"waves_per_simd\": %d, \"waves\": %d, \"positions\": %d, \"kernel_ms\": %.4f, "
                "\"sclk_ghz\": %.4f, \"wave_cycles_per_position\": %.1f}\n",
                MIX, WPS, blocks * 4 * WPS, kPos, ms, ghz, cyc);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main()
{
    // a table of the decoder's shape (thresholds rising through the buckets, two values a row) and
    // inputs of the decoder's magnitudes (|P|, |Q| up to ~4)
    std::vector<double> lut(3 * kRows * kCols), in(kInSteps * 2 * 64);
    for (int q = 0; q < kRows; ++q)
        for (int c = 0; c < kCols; ++c) {
            const double lo = std::ldexp(1.0 + 0.25 * (q & 3), (q >> 2) - 4);   // the bucket's lower edge
            lut[(0 * kRows + q) * kCols + c] = lo * 1.1;
            lut[(1 * kRows + q) * kCols + c] = 0.69 / (1 + q);
            lut[(2 * kRows + q) * kCols + c] = 0.69 / (2 + q);
        }
    unsigned s = 12345;
    for (double& v : in) {
        s = s * 1103515245u + 12345u;
        v = ((s >> 8) & 0xFFFF) / 8192.0 - 4.0;
    }
    double *dl, *di, *dout;
    unsigned long long* dclk;
    (void)hipMalloc(&dl, lut.size() * 8);
    (void)hipMalloc(&di, in.size() * 8);
    (void)hipMalloc(&dout, 256 * 3 * 256 * 8);   // 256 workgroups x up to 768 threads
    (void)hipMalloc(&dclk, 16);
    (void)hipMemcpy(dl, lut.data(), lut.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(di, in.data(), in.size() * 8, hipMemcpyHostToDevice);
    run<0, 1>(dl, di, dout, dclk);
    run<0, 2>(dl, di, dout, dclk);
    run<0, 3>(dl, di, dout, dclk);
    run<1, 1>(dl, di, dout, dclk);
    run<1, 2>(dl, di, dout, dclk);
    run<1, 3>(dl, di, dout, dclk);
    run<2, 2>(dl, di, dout, dclk);   // the two mixes on the (thr, pair) layout
    run<3, 2>(dl, di, dout, dclk);
    run<4, 2>(dl, di, dout, dclk);   // and on one 1 KiB row a bucket (thr at a 16-byte column stride)
    run<5, 2>(dl, di, dout, dclk);
    (void)hipFree(dl);
    (void)hipFree(di);
    (void)hipFree(dout);
    (void)hipFree(dclk);
    return 0;
}
