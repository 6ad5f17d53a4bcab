// calib_fetch.hip -- FETCH_SIZE / WRITE_SIZE calibration for the decoder's access width:
// one double (8 B) per lane, 512 contiguous bytes per wave instruction, as the turbo kernel's
// tile loads and extrinsic stores.  Reads 1 GiB, writes 1 GiB; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- ./scripts/calib_fetch   (and WRITE_SIZE)
// hipcc --offload-arch=gfx950 -O3 -o scripts/calib_fetch scripts/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void read8(const double* __restrict__ a, size_t n, double* out)
{
    double s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;   // keeps the loads alive, never stores in practice
}

__global__ void write8(double* __restrict__ a, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}

int main()
{
    const size_t n = (size_t)1 << 27;   // 2^27 doubles = 1 GiB
    double *a, *o;
    if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n, o);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::printf("calib: read8 and write8 over %zu bytes\n", n * 8);
    (void)hipFree(a);
    (void)hipFree(o);
    return 0;
}
