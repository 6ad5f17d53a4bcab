// ubench_beta.hip -- cycles per beta step of the turbo decoder's backward recursion on gfx950,
// one chain per wave (64 workgroups of one or two waves), max* table in LDS.
// V0 chain only (operands in registers); V1 + the per-step LDS store of beta (the fold input);
// V2 + operands read from LDS; V3 = V2 with a second wave streaming global_load_lds into LDS.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-honor-nans -o scripts/ubench_beta scripts/ubench_beta.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 6000

template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__device__ __forceinline__ int rowoff(double d)
{
    const int q = (int)__builtin_amdgcn_ubfe((unsigned)(__double_as_longlong(d) >> 32), 17, 14);
    return min(max(q, 8152), 8152 + 56) * 32;
}

template <int V, int C>
__device__ __forceinline__ double step(double b, double sg, double gs, double pg, double gp, double tm, const double* lut,
                                       double* bv)
{
    if (V >= 1 && V < 4) *bv = b;
    const double bp = dpp<C>(b);
    const double xs = fma(sg, gs, b), xp = fma(pg, gp, bp);
    const double d = xp - xs;
    const int o = rowoff(d);
    const double t = lut[o], l = lut[o + 16], h = lut[o + 48];
    if (V >= 4) {   // the store issued behind the table read
        const unsigned a = (unsigned)(size_t)(__attribute__((address_space(3))) double*)bv;
        asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(b) : "memory");
    }
    return (fmax(xs, xp) + (fabs(d) >= t ? h : l)) - tm;
}

template <int V>
__global__ void k(double* out, unsigned long long* cyc, const double* src)
{
    __shared__ double lds[130 * 32];
    __shared__ double ops[2][64 * 4 * 12];
    __shared__ double dma[8][64 * 2];
    for (int i = threadIdx.x; i < 130 * 32; i += blockDim.x) lds[i] = ((i / 16) & 1) ? 0.01 * (i / 32) : 0.05 * (i / 32);
    for (int i = threadIdx.x; i < 2 * 64 * 4 * 12; i += blockDim.x) (&ops[0][0])[i] = 0.01 * (i % 97);
    __syncthreads();
    if (threadIdx.x >= 64) {   // V3: the loader wave streams 1 KiB pieces into LDS continuously
        const unsigned base = (unsigned)(size_t)(__attribute__((address_space(3))) char*)(reinterpret_cast<char*>(&dma[0][0]));
        const int lane = threadIdx.x & 63;
        for (int r = 0; r < N / 2; ++r) {
            unsigned save;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(save) : "s"(base + (r & 7) * 1024), "v"(src + (size_t)(r % 4096) * 128 + lane * 2) : "memory");
            if ((r & 3) == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        return;
    }
    const double* lut = lds - 8152 * 32 + (threadIdx.x & 15);
    const int sl = threadIdx.x & 7;
    const double sg = (sl & 1) ? 1.0 : -1.0, pg = -sg;
    double gs = 0.37 * (sl + 1), gp = 0.21 * (sl + 2), tm = 0.5;
    double b = (sl == 0) ? 0.0 : -3.0 * sl;
    double* bv = &ops[1][threadIdx.x];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i += 3) {
        if (V >= 2 && V != 4) {
            const double* o = &ops[0][(i % 12) * 256 + threadIdx.x];
            gs = o[0]; gp = o[64]; tm = o[128];
        }
        b = step<V, 0x141>(b, sg, gs, pg, gp, tm, lut, bv + ((i + 0) % 12) * 64);
        b = step<V, 0x4E>(b, -sg, gp, pg, gs, tm, lut, bv + ((i + 1) % 12) * 64);
        b = step<V, 0xB1>(b, sg, gp, -pg, gs, tm, lut, bv + ((i + 2) % 12) * 64);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = b;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, double* out, unsigned long long* cyc, const double* src, int threads)
{
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((k<V>), dim3(64), dim3(threads), 0, 0, out, cyc, src);
        hipDeviceSynchronize();
    }
    unsigned long long h[64];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 64; ++i) s += h[i];
    printf("%-44s %8.2f cycles per step\n", name, s / 64 / N);
}

int main()
{
    double *out, *src;
    unsigned long long* cyc;
    if (hipMalloc(&out, 64 * 128 * sizeof(double)) != hipSuccess) return 1;
    if (hipMalloc(&src, (size_t)4097 * 128 * sizeof(double)) != hipSuccess) return 1;
    if (hipMalloc(&cyc, 64 * sizeof(unsigned long long)) != hipSuccess) return 1;
    hipMemset(src, 0, (size_t)4097 * 128 * sizeof(double));
    run<0>("beta chain, operands in registers", out, cyc, src, 64);
    run<1>("+ beta stored to LDS every step", out, cyc, src, 64);
    run<2>("+ operands read from LDS every 3 steps", out, cyc, src, 64);
    run<2>("as above, a loader wave DMA-ing into LDS", out, cyc, src, 128);
    run<4>("store behind the table read (asm), regs", out, cyc, src, 64);
    run<5>("store behind the table read + LDS operands", out, cyc, src, 64);
    return 0;
}
