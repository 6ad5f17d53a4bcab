// ubench_latency.hip -- dependent-chain latencies on gfx950 for the operations on the turbo
// decoder's recursion (one wave per workgroup, 64 workgroups).  Prints cycles per chained op.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-honor-nans -o ubench scripts/ubench_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 4096

template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__global__ void k(double* out, double a, unsigned long long* cyc, int mode)
{
    __shared__ double lds[64 * 4];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 1e-9 * i;
    __syncthreads();
    double x = a * (threadIdx.x + 1);
    float xf = (float)x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (mode) {
        case 0:   // v_add_f64
            for (int i = 0; i < N; ++i) x = x + a;
            break;
        case 1:   // v_fma_f64
            for (int i = 0; i < N; ++i) x = fma(x, 0.999, a);
            break;
        case 2:   // v_max_f64
            for (int i = 0; i < N; ++i) x = fmax(x, a) + 0.0;
            break;
        case 3:   // dpp pair + add
            for (int i = 0; i < N; ++i) x = dpp<0xB1>(x) + a;
            break;
        case 4:   // ds_read_b64 indexed by data + add
            for (int i = 0; i < N; ++i) {
                const int q = (int)(__double_as_longlong(x) >> 40) & 63;
                x = x + lds[q];
            }
            break;
        case 5:   // v_add_f32
            for (int i = 0; i < N; ++i) xf = xf + (float)a;
            break;
        case 6:   // group max: 3 x (dpp pair + max)
            for (int i = 0; i < N; ++i) {
                x = fmax(x, dpp<0xB1>(x));
                x = fmax(x, dpp<0x4E>(x));
                x = fmax(x, dpp<0x141>(x));
                x = x + a;
            }
            break;
        case 7:   // int chain: bfe + med3 + lshl_add
            {
                unsigned u = (unsigned)threadIdx.x;
                for (int i = 0; i < N; ++i) {
                    u = __builtin_amdgcn_ubfe(u * 3u + 7u, 3, 14);
                    u = min(max((int)u, 5), 9000) * 32 + 11;
                }
                x = (double)u;
            }
            break;
        case 9:   // alpha step (maxlog), operands in registers
        case 10:  // alpha step (maxlog), gammas from LDS per step
            {
                const double sg = (threadIdx.x & 1) ? 1.0 : -1.0, pg = -sg;
                double gs = 0.3 * (threadIdx.x & 7), gp = 0.2 * (threadIdx.x & 3);
                for (int i = 0; i < N; ++i) {
                    if (mode == 10) {
                        gs = lds[(i * 8 + (threadIdx.x >> 3)) & 255];
                        gp = lds[(i * 8 + 1 + (threadIdx.x >> 3)) & 255];
                    }
                    const double ap = dpp<0xB1>(x);
                    const double xs = fma(sg, gs, x), xp = fma(pg, gp, ap);
                    double a = fmax(xs, xp);
                    double m = fmax(a, dpp<0xB1>(a));
                    m = fmax(m, dpp<0x4E>(m));
                    m = fmax(m, dpp<0x141>(m));
                    x = a - m;
                }
            }
            break;
        case 11:  // ds_bpermute lookup of a 64-bit value held across lanes (addr from data) + add
            {
                const double tv = 1e-9 * threadIdx.x;
                const int lo = (int)(unsigned)__double_as_longlong(tv), hi = (int)(__double_as_longlong(tv) >> 32);
                for (int i = 0; i < N; ++i) {
                    const int q = ((int)(__double_as_longlong(x) >> 40) & 63) << 2;
                    const int rl = __builtin_amdgcn_ds_bpermute(q, lo), rh = __builtin_amdgcn_ds_bpermute(q, hi);
                    x = x + __longlong_as_double(((long long)(unsigned)rh << 32) | (unsigned)rl);
                }
            }
            break;
        case 12:  // three ds_read_b64 (thr, lo, hi) + cmp/select + add (the max* table path)
            for (int i = 0; i < N; ++i) {
                const int q = (int)(__double_as_longlong(x) >> 40) & 63;
                const double t = lds[q], l = lds[64 + q], h = lds[128 + q];
                x = x + (fabs(x) >= t ? h : l);
            }
            break;
        case 13:  // bucket int ops only: bfe + med3 + lshl (dependent) feeding an add
            for (int i = 0; i < N; ++i) {
                const unsigned hi = (unsigned)((unsigned long long)__double_as_longlong(x) >> 32);
                int q = (int)__builtin_amdgcn_ubfe(hi, 17, 14);
                q = min(max(q, 8152), 8152 + 56);
                x = x + (double)(q * 8);
            }
            break;
        case 14:  // alpha step log-MAP: table max* after the group max (the committed kernel's order)
        case 15:  // alpha step log-MAP: speculative table read from the unnormalised metrics
        case 16:  // as 15 plus the two per-step global stores of alpha and tempmax
            {
                const double sg = (threadIdx.x & 1) ? 1.0 : -1.0, pg = -sg;
                const double gs = 0.3 * (threadIdx.x & 7), gp = 0.2 * (threadIdx.x & 3);
                double* st = out + 4096 + blockIdx.x * 64 + threadIdx.x;
                for (int i = 0; i < N; ++i) {
                    const double an = dpp<0xB1>(x);
                    double m = fmax(x, an);
                    int qu = 0;
                    double t = 0, l = 0, h = 0;
                    if (mode != 14) {
                        const double du = fma(pg, gp, an) - fma(sg, gs, x);
                        qu = min(max((int)__builtin_amdgcn_ubfe((unsigned)(__double_as_longlong(du) >> 32), 17, 14), 8152), 8152 + 56) - 8152;
                        t = lds[qu]; l = lds[64 + qu]; h = lds[128 + qu];
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    m = fmax(m, dpp<0x4E>(m));
                    m = fmax(m, dpp<0x141>(m));
                    const double al = x - m, ap = an - m;
                    if (mode == 16) {
                        asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(st), "v"(al) : "memory");
                        asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(st + 64 * 64), "v"(m) : "memory");
                        st += 64 * 64 * 2;
                    }
                    const double xs = fma(sg, gs, al), xp = fma(pg, gp, ap);
                    const double d = xp - xs;
                    const int q = min(max((int)__builtin_amdgcn_ubfe((unsigned)(__double_as_longlong(d) >> 32), 17, 14), 8152), 8152 + 56) - 8152;
                    if (mode == 14 || q != qu) { t = lds[q]; l = lds[64 + q]; h = lds[128 + q]; }
                    x = fmax(xs, xp) + (fabs(d) >= t ? h : l);
                }
            }
            break;
        case 17:  // issue cost: 8 independent v_add_f64 chains (cycles per 8 adds)
        case 18:  // issue cost: 8 independent v_add_u32 chains (cycles per 8 adds)
            {
                double v[8];
                unsigned w[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) { v[j] = x * (j + 1); w[j] = threadIdx.x * (j + 3); }
                for (int i = 0; i < N; ++i) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (mode == 17) v[j] = v[j] + a; else w[j] = w[j] + (unsigned)i;
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) x += v[j] + (double)w[j];
            }
            break;
        case 8:   // v_add_f64 pairs interleaved (2 independent chains)
            {
                double y = x * 0.5;
                for (int i = 0; i < N; ++i) {
                    x = x + a;
                    y = y + a;
                }
                x += y;
            }
            break;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = x + xf;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, (4096 + 64 * 64 * 2 * (N + 1)) * sizeof(double));
    hipMalloc(&cyc, 64 * sizeof(unsigned long long));
    const char* names[] = {"v_add_f64", "v_fma_f64", "v_max_f64+add0", "dpp64+add_f64", "ds_read_b64(idx)+add",
                           "v_add_f32", "gmax3(dpp+max)+add", "int bfe+med3+lshl", "2x add_f64 interleaved",
                           "alpha step maxlog (regs)", "alpha step maxlog (lds g)", "ds_bpermute x2 lookup+add",
                           "3x ds_read_b64 + sel + add", "bfe+med3+cvt+add",
                           "alpha logmap (table after max)", "alpha logmap (speculative table)", "alpha logmap spec + 2 stores",
                           "8 indep v_add_f64 (per 8)", "8 indep v_add_u32 (per 8)"};
    for (int mode = 0; mode < 19; ++mode) {
        hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, out, 1.0000001, cyc, mode);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, out, 1.0000001, cyc, mode);
        unsigned long long h[64];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 64; ++i) s += h[i];
        printf("%-26s %8.2f cycles per iteration\n", names[mode], s / 64 / N);
    }
    return 0;
}
