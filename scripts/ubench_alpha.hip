// ubench_alpha.hip -- cycles per alpha step of the turbo decoder's forward recursion on gfx950,
// one chain per wave (64 workgroups of one wave), operands in registers, max* table in LDS.
// Variants: 0 table read after the group max (committed order), 1 speculative table read with the
// bucket check, 2 speculative read without the check (timing only), 3 Max-Log-MAP, 4/5 folded
// offsets (5 speculative row), 6 whole correction speculated (row and threshold side) + flag.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-honor-nans -fno-slp-vectorize -o scripts/ubench_alpha scripts/ubench_alpha.hip
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

__device__ __forceinline__ int bucket(double d)
{
    const int q = (int)__builtin_amdgcn_ubfe((unsigned)(__double_as_longlong(d) >> 32), 17, 14);
    return min(max(q, 8152), 8152 + 56) - 8152;
}

// V 4/5: the table address folded into the ds_read offsets (row base = lane column - base bucket,
// one lshl_add), the two candidate sums formed before the select; 5 = speculative read with the
// bucket mismatch OR-ed into a flag checked outside the step (per window in the kernel).
__device__ __forceinline__ int bucket_raw(double d)
{
    const int q = (int)__builtin_amdgcn_ubfe((unsigned)(__double_as_longlong(d) >> 32), 17, 14);
    return min(max(q, 8152), 8152 + 56);
}

template <int V, int C0, int C1, int C2>
__device__ __forceinline__ double step2(double x, double sg, double gs, double pg, double gp, const char* rowb, double* st,
                                        unsigned& flag)
{
    const double an = dpp<C0>(x);
    double m = fmax(x, an);
    double t = 0, l = 0, h = 0;
    int qu = 0;
    if (V == 5) {
        const double du = fma(pg, gp, an) - fma(sg, gs, x);
        qu = bucket_raw(du);
        const char* r = rowb + qu * 128;
        t = *(const double*)r; l = *(const double*)(r + 64 * 128); h = *(const double*)(r + 65 * 128);
        __builtin_amdgcn_sched_barrier(0);
    }
    m = fmax(m, dpp<C1>(m));
    m = fmax(m, dpp<C2>(m));
    const double al = x - m, ap = an - m;
    if (st) {
        asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(st), "v"(al) : "memory");
        asm volatile("global_store_dwordx2 %0, %1, off offset:8" :: "v"(st), "v"(m) : "memory");
    }
    const double xs = fma(sg, gs, al), xp = fma(pg, gp, ap);
    const double d = xp - xs;
    const int q = bucket_raw(d);
    if (V == 4) {
        const char* r = rowb + q * 128;
        t = *(const double*)r; l = *(const double*)(r + 64 * 128); h = *(const double*)(r + 65 * 128);
    } else {
        flag |= (unsigned)(q ^ qu);
    }
    const double mx = fmax(xs, xp);
    const double rl = mx + l, rh = mx + h;
    return fabs(d) >= t ? rh : rl;
}

// V 6: the whole max* correction speculated from the unnormalised difference (row AND threshold
// compare), so the chain after the group max is sub, fma, max, add; the exact difference is only
// checked (same bucket, same side of the row's threshold), OR-ed into a flag read per window.
template <int V, int C0, int C1, int C2>
__device__ __forceinline__ double step3(double x, double sg, double gs, double pg, double gp, const char* rowb, double* st,
                                        unsigned& flag)
{
    const double an = dpp<C0>(x);
    const double du = fma(pg, gp, an) - fma(sg, gs, x);
    const int qu = bucket_raw(du);
    const char* r = rowb + qu * 128;
    const double t = *(const double*)r, l = *(const double*)(r + 64 * 128), h = *(const double*)(r + 65 * 128);
    __builtin_amdgcn_sched_barrier(0);
    double m = fmax(x, an);
    m = fmax(m, dpp<C1>(m));
    m = fmax(m, dpp<C2>(m));
    const double al = x - m, ap = an - m;
    if (st) {
        asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(st), "v"(al) : "memory");
        asm volatile("global_store_dwordx2 %0, %1, off offset:8" :: "v"(st), "v"(m) : "memory");
    }
    const double xs = fma(sg, gs, al), xp = fma(pg, gp, ap);
    if (V == 7) __builtin_amdgcn_sched_barrier(0);
    const double mx = fmax(xs, xp);
    const bool su = fabs(du) >= t;
    const double f = su ? h : l;
    const double d = xp - xs;
    flag |= (unsigned)(bucket_raw(d) ^ qu) | (unsigned)((fabs(d) >= t) != su);
    return mx + f;
}

template <int V, int C0, int C1, int C2>
__device__ __forceinline__ double step(double x, double sg, double gs, double pg, double gp, const double* lut, double* st)
{
    const double an = dpp<C0>(x);
    double m = fmax(x, an);
    double t = 0, l = 0, h = 0;
    int qu = 0;
    if (V == 1 || V == 2) {
        const double du = fma(pg, gp, an) - fma(sg, gs, x);
        qu = bucket(du);
        t = lut[qu * 16]; l = lut[(64 + qu) * 16]; h = lut[(65 + qu) * 16];
        __builtin_amdgcn_sched_barrier(0);
    }
    m = fmax(m, dpp<C1>(m));
    m = fmax(m, dpp<C2>(m));
    const double al = x - m, ap = an - m;
    if (st) {
        asm volatile("global_store_dwordx2 %0, %1, off" :: "v"(st), "v"(al) : "memory");
        asm volatile("global_store_dwordx2 %0, %1, off offset:8" :: "v"(st), "v"(m) : "memory");
    }
    const double xs = fma(sg, gs, al), xp = fma(pg, gp, ap);
    if (V == 3) return fmax(xs, xp);
    const double d = xp - xs;
    if (V == 0) {
        const int q = bucket(d);
        t = lut[q * 16]; l = lut[(64 + q) * 16]; h = lut[(65 + q) * 16];
    } else if (V == 1) {
        const int q = bucket(d);
        if (__builtin_expect(q != qu, 0)) { t = lut[q * 16]; l = lut[(64 + q) * 16]; h = lut[(65 + q) * 16]; }
    }
    return fmax(xs, xp) + (fabs(d) >= t ? h : l);
}

template <int V, int STORE>
__global__ void k(double* out, unsigned long long* cyc)
{
    __shared__ double lds[130 * 16];
    for (int i = threadIdx.x; i < 130 * 16; i += 64) lds[i] = (i / 16 < 64) ? 0.05 * (i / 16) : 0.01 * (i / 16 - 64);
    __syncthreads();
    const double* lut = lds + (threadIdx.x & 15);
    const int sl = threadIdx.x & 7;
    const double sg = (sl & 1) ? 1.0 : -1.0, pg = (sl & 2) ? 1.0 : -1.0;
    const double gs = 0.37 * (sl + 1), gp = 0.21 * (sl + 2);
    double x = (sl == 0) ? 0.0 : -3.0 * sl;
    double* st = STORE ? out + 4096 + (blockIdx.x * 64 + threadIdx.x) * 2 : nullptr;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned flag = 0;
    const char* rowb = (const char*)lut - 8152 * 128;
    if (V >= 6) {
        for (int i = 0; i < N; i += 3) {
            x = step3<V, 0xB1, 0x4E, 0x141>(x, sg, gs, pg, gp, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
            x = step3<V, 0x4E, 0x141, 0xB1>(x, -sg, gp, pg, gs, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
            x = step3<V, 0x141, 0xB1, 0x4E>(x, sg, gp, -pg, gs, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
        }
    } else if (V >= 4) {
        for (int i = 0; i < N; i += 3) {
            x = step2<V, 0xB1, 0x4E, 0x141>(x, sg, gs, pg, gp, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
            x = step2<V, 0x4E, 0x141, 0xB1>(x, -sg, gp, pg, gs, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
            x = step2<V, 0x141, 0xB1, 0x4E>(x, sg, gp, -pg, gs, rowb, st, flag);
            if (STORE) st += 64 * 64 * 2;
        }
    } else
    for (int i = 0; i < N; i += 3) {
        x = step<V, 0xB1, 0x4E, 0x141>(x, sg, gs, pg, gp, lut, st);
        if (STORE) st += 64 * 64 * 2;
        x = step<V, 0x4E, 0x141, 0xB1>(x, -sg, gp, pg, gs, lut, st);
        if (STORE) st += 64 * 64 * 2;
        x = step<V, 0x141, 0xB1, 0x4E>(x, sg, gp, -pg, gs, lut, st);
        if (STORE) st += 64 * 64 * 2;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = x + flag;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, int S>
static void run(const char* name, double* out, unsigned long long* cyc)
{
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((k<V, S>), dim3(64), dim3(64), 0, 0, out, cyc);
        hipDeviceSynchronize();
    }
    unsigned long long h[64];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 64; ++i) s += h[i];
    printf("%-40s %8.2f cycles per step\n", name, s / 64 / N);
}

int main()
{
    double* out;
    unsigned long long* cyc;
    if (hipMalloc(&out, (4096 + (size_t)64 * 64 * 2 * (N + 3)) * sizeof(double)) != hipSuccess) return 1;
    if (hipMalloc(&cyc, 64 * sizeof(unsigned long long)) != hipSuccess) return 1;
    run<0, 0>("table after max", out, cyc);
    run<1, 0>("speculative table, checked", out, cyc);
    run<2, 0>("speculative table, unchecked", out, cyc);
    run<3, 0>("max-log", out, cyc);
    run<0, 1>("table after max + stores", out, cyc);
    run<1, 1>("speculative checked + stores", out, cyc);
    run<3, 1>("max-log + stores", out, cyc);
    run<4, 0>("after max, folded offsets, add-select", out, cyc);
    run<5, 0>("speculative, flag check, folded", out, cyc);
    run<4, 1>("after max folded + stores", out, cyc);
    run<5, 1>("speculative flag folded + stores", out, cyc);
    run<6, 0>("full max* speculation, flag check", out, cyc);
    run<6, 1>("full max* speculation + stores", out, cyc);
    run<7, 0>("full speculation, select after the fmas", out, cyc);
    run<7, 1>("full speculation, select after + stores", out, cyc);
    return 0;
}
