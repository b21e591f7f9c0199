// Micro-benchmark (diagnostics): VALU issue cost per wave and per SIMD on gfx950, by waves per
// SIMD, for the instruction kinds the QP kernel issues: independent v_fma_f32,
// v_pk_fma_f32 (two floats per lane), v_fma_f64, v_mov_b32_dpp, ds_bpermute_b32.  One workgroup
// of 256 w threads on one CU = w waves per SIMD; s_memtime around ITERS x 8 independent ops.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_issue.hip -o tools/ubench_issue
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 1024

typedef float f2 __attribute__((ext_vector_type(2)));

template <int K>
__global__ void bench(float* out, unsigned long long* cyc, float a, float b)
{
    const int t = threadIdx.x;
    float x[8];
    f2 y[8];
    double z[8];
    int w[8];
    for (int i = 0; i < 8; ++i) {
        x[i] = t * 1e-3f + i;
        y[i] = f2{x[i], x[i] + 0.5f};
        z[i] = x[i];
        w[i] = t + i;
    }
    const f2 a2{a, a}, b2{b, b};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (K == 0) x[i] = __builtin_fmaf(x[i], a, b);
            if (K == 1) y[i] = __builtin_elementwise_fma(y[i], a2, b2);
            if (K == 2) z[i] = __builtin_fma(z[i], (double)a, (double)b);
            if (K == 3) w[i] = __builtin_amdgcn_update_dpp(w[i], w[i], 0x134, 0xF, 0xF, false);
            if (K == 4) w[i] = __builtin_amdgcn_ds_bpermute(((t + 1) & 63) << 2, w[i]);
        }
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += x[i] + y[i].x + y[i].y + (float)z[i] + (float)w[i];
    out[blockIdx.x * blockDim.x + t] = s;
    if ((t & 63) == 0) cyc[t >> 6] = t1 - t0;
}

int main()
{
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * 4096);
    hipMalloc(&cyc, sizeof(unsigned long long) * 64);
    unsigned long long h[64];
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32 (2 floats)", "v_fma_f64", "v_mov_b32_dpp",
                           "ds_bpermute_b32"};
    for (int k = 0; k < 5; ++k) {
        for (int w : {1, 2, 3, 4}) {
            auto kern = k == 0 ? bench<0> : k == 1 ? bench<1> : k == 2 ? bench<2> : k == 3 ? bench<3> : bench<4>;
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(kern, dim3(1), dim3(256 * w), 0, 0, out, cyc, 0.999f, 1e-3f);
            hipDeviceSynchronize();
            hipMemcpy(h, cyc, sizeof(unsigned long long) * 4 * w, hipMemcpyDeviceToHost);
            double mx = 0, mean = 0;
            for (int i = 0; i < 4 * w; ++i) {
                mx = h[i] > mx ? h[i] : mx;
                mean += h[i];
            }
            mean /= 4 * w;
            const double ops = 8.0 * ITERS;
            printf("%-26s waves/SIMD %d: %.2f cycles per op per wave (mean), SIMD: %.2f cycles per wave-op\n",
                   names[k], w, mean / ops, mx / (ops * w));
        }
    }
    return 0;
}
