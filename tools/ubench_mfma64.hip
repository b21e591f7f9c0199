// Micro-benchmark (diagnostics): fp64 matrix-core rate against fp64 VALU on gfx950, one wave
// per SIMD (one 256-thread workgroup per CU, every CU busy), to decide whether the config-5
// dynamics' 30x30 mass-matrix assembly / Cholesky updates can gain from MFMA.
//   v_mfma_f64_16x16x4_f64: 16 x 16 x 4 x 2 = 2048 flops per wave-instruction
//   v_fma_f64:              64 x 2        =  128 flops per wave-instruction
// Independent accumulators (8 chains) so that the issue rate, not the dependency latency, binds;
// a dependent chain is timed separately (the latency the Cholesky's pivot chain would see).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma64.hip -o tools/ubench_mfma64
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 512
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void mfma_indep(double* out, unsigned long long* cyc, double a0)
{
    d4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
    double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0.0;
    for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

__global__ void mfma_dep(double* out, unsigned long long* cyc, double a0)
{
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

__global__ void vfma_indep(double* out, unsigned long long* cyc, double a0)
{
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
    const double a = a0, b = 1e-3;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, b);
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0.0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

int main()
{
    const int cus = 256;
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(double) * 256 * cus);
    hipMalloc(&cyc, sizeof(unsigned long long) * 4 * cus);
    unsigned long long h[4 * 256];
    struct K { const char* name; void (*f)(double*, unsigned long long*, double); double flops; int chains; };
    const K ks[] = {{"v_mfma_f64_16x16x4f64 x8 independent", mfma_indep, 2048.0, 8},
                    {"v_mfma_f64_16x16x4f64 dependent chain", mfma_dep, 2048.0, 1},
                    {"v_fma_f64 x8 independent", vfma_indep, 128.0, 8}};
    for (const K& k : ks) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipLaunchKernelGGL(k.f, dim3(cus), dim3(256), 0, 0, out, cyc, 0.999);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k.f, dim3(cus), dim3(256), 0, 0, out, cyc, 0.999);
        hipEventRecord(e1, 0);
        hipDeviceSynchronize();
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double mean = 0.0;
        for (int i = 0; i < 4 * cus; ++i) mean += (double)h[i];
        mean /= 4 * cus;
        const double insts = (double)ITERS * k.chains;
        const double tf = k.flops * insts * 4 * cus / (ms * 1e-3) / 1e12;
        printf("%-40s %.2f cycles per wave-instruction, %.1f flops/cycle/SIMD, chip %.1f TF/s (%.3f ms)\n",
               k.name, mean / insts, k.flops * insts / mean, tf, ms);
    }
    return 0;
}
