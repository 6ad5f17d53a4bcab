// ubench_fold.hip -- cycles per LLR fold item of the turbo decoder's B pass on gfx950, one wave per
// workgroup (64 workgroups), everything in LDS: the item's alpha and beta blocks (8 states), its
// (P, Q, ys, La) and the max* table, as the kernel's fold_item_fast reads them.  Each lane folds one
// item per "window" (two E_seq chains of 7 table max* each, then LLR / Le written to LDS).
// V0 the kernel's order (sums, then both chains interleaved); V1 one chain per lane (half the work:
// what a lane does if an item's two chains go to two lanes).
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-honor-nans -o scripts/ubench_fold scripts/ubench_fold.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define NWIN 2000

__device__ __forceinline__ double mstar(double x, double y, const double* lut)
{
    const double d = y - x;
    const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(d) >> 32);
    int q = (int)__builtin_amdgcn_ubfe(hi, 18, 13);
    q = min(max(q, 4076), 4076 + 28) - 4076;
    const int o = q * 32;
    const double thr = lut[o], lo = lut[o + 16], hv = lut[o + 48];
    return fmax(x, y) + (fabs(d) >= thr ? hv : lo);
}

constexpr int kLast[8][2] = {{0, 1}, {3, 2}, {4, 5}, {7, 6}, {1, 0}, {2, 3}, {5, 4}, {6, 7}};
constexpr int kQ[8] = {0, 0, 1, 1, 1, 1, 0, 0};

template <int V>
__global__ void k(double* out, unsigned long long* cyc)
{
    __shared__ double lut_s[30 * 32];
    __shared__ double blk[2][64][8];   // alpha, beta block per lane
    __shared__ double g[64][4];
    __shared__ double res[64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 30 * 32; i += 64) lut_s[i] = ((i / 16) & 1) ? 0.69315 - 0.025 * (i / 32) : 0.08824 * (1 + i / 32);
    for (int j = 0; j < 8; ++j) {
        blk[0][lane][j] = -0.37 * ((lane + 3 * j) % 11);
        blk[1][lane][j] = -0.21 * ((lane * 7 + j) % 13);
    }
    g[lane][0] = 0.3 + 0.01 * lane;
    g[lane][1] = -0.2 + 0.02 * lane;
    g[lane][2] = 0.5;
    g[lane][3] = 0.1;
    __syncthreads();
    const double* lut = lut_s + (lane & 15);
    double acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int w = 0; w < NWIN; ++w) {
        const int e = (lane + w) & 63;   // a different item each window (defeats hoisting)
        const double P = g[e][0], Q = g[e][1], ys = g[e][2], la = g[e][3];
        double a[8], b[8], t0v[8], t1v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] = blk[0][e][j];
            b[j] = blk[1][e][j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int p0 = kLast[j][0], p1 = kLast[j][1];
            t0v[j] = (a[p0] - (kQ[p0] ? Q : P)) + b[j];
            if (V == 0) t1v[j] = (a[p1] + (kQ[p1] ? Q : P)) + b[j];
        }
        double r0 = mstar(t0v[0], t0v[1], lut), r1 = 0;
        if (V == 0) r1 = mstar(t1v[0], t1v[1], lut);
#pragma unroll
        for (int j = 2; j < 8; ++j) {
            r0 = mstar(r0, t0v[j], lut);
            if (V == 0) r1 = mstar(r1, t1v[j], lut);
        }
        const double llr = r1 - r0;
        res[lane] = llr - la - 2.0 * ys;
        acc += llr;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, double* out, unsigned long long* cyc)
{
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<V>, dim3(64), dim3(64), 0, 0, out, cyc);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h[64];
    (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 64; ++i) s += h[i];
    printf("%-40s %8.1f cycles per item (%.1f per trellis step at 12 steps a window)\n", name, s / 64 / NWIN,
           s / 64 / NWIN / 12);
}

int main()
{
    double* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, 64 * 64 * sizeof(double)) != hipSuccess) return 1;
    if (hipMalloc(&cyc, 64 * sizeof(unsigned long long)) != hipSuccess) return 1;
    run<0>("fold item, two chains per lane", out, cyc);
    run<1>("one chain per lane", out, cyc);
    return 0;
}
