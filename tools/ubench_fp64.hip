// Micro-benchmark (diagnostics): fp64 VALU latency / issue rate on gfx950, measured with
// s_memtime inside the kernel.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 2048

__global__ void dep_chain(double* out, unsigned long long* cyc, double a, double b)
{
    double x = threadIdx.x * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < ITERS; ++i) x = x * a + b;   // mul + add, dependent
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void indep8(double* out, unsigned long long* cyc, double a, double b)
{
    double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,
           x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
    for (int i = 0; i < ITERS; ++i) {
        x0 = x0 * a + b; x1 = x1 * a + b; x2 = x2 * a + b; x3 = x3 * a + b;
        x4 = x4 * a + b; x5 = x5 * a + b; x6 = x6 * a + b; x7 = x7 * a + b;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void div_chain(double* out, unsigned long long* cyc, double a)
{
    double x = 1.0 + threadIdx.x * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) x = a / x;
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(double) * 1024 * 1024);
    hipMalloc(&cyc, sizeof(unsigned long long) * 1024);
    unsigned long long h[1024];
    // grids: 1 block (1 CU) with 64, 128, 256, 512 threads -> 1, 2, 4, 8 waves on the CU
    for (int threads : {64, 128, 256, 512, 1024}) {
        hipLaunchKernelGGL(dep_chain, dim3(1), dim3(threads), 0, 0, out, cyc, 0.999, 1e-3);
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
        printf("dep_chain  waves/CU %2d : %.2f cycles per dependent fp64 op (mul+add pairs: %d)\n",
               threads / 64, (double)h[0] / (2.0 * ITERS), ITERS);
        hipLaunchKernelGGL(indep8, dim3(1), dim3(threads), 0, 0, out, cyc, 0.999, 1e-3);
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
        printf("indep8     waves/CU %2d : %.2f cycles per fp64 instruction per wave\n",
               threads / 64, (double)h[0] / (16.0 * ITERS));
    }
    hipLaunchKernelGGL(div_chain, dim3(1), dim3(64), 0, 0, out, cyc, 1.000001);
    hipDeviceSynchronize();
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("div_chain  1 wave : %.1f cycles per dependent fp64 division\n", (double)h[0] / 256.0);
    // clock: s_memtime ticks vs wall
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(dep_chain, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("memtime ticks %llu in %.3f ms wall (kernel incl. launch)\n", h[0], ms);
    return 0;
}
