#include <hip/hip_runtime.h>
__device__ double dpp_f64(double v, int ctrl_dummy);
template <int CTRL> __device__ __forceinline__ double dppd(double v) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// raw results [0] of the swaps (diagnostic of the instruction semantics)
__device__ __forceinline__ double swap16(double v) {
    long long b = __double_as_longlong(v);
    auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (unsigned)lo[0]);
}
__device__ __forceinline__ double swap32(double v) {
    long long b = __double_as_longlong(v);
    auto lo = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (unsigned)lo[0]);
}
__global__ void k(double* x, double* out) {
    int l = threadIdx.x;
    double v = x[l];
    out[l] = dppd<0xB1>(v);
    out[64 + l] = dppd<0x4E>(v);
    out[128 + l] = dppd<0x141>(v);
    out[192 + l] = dppd<0x140>(v);
    out[256 + l] = swap16(v);
    out[320 + l] = swap32(v);
}
int main() {
    double h[64], *x, *o; double r[384];
    for (int i = 0; i < 64; ++i) h[i] = i;
    hipMalloc(&x, 512); hipMalloc(&o, 384 * 8);
    hipMemcpy(x, h, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, x, o);
    hipMemcpy(r, o, 384 * 8, hipMemcpyDeviceToHost);
    const char* names[6] = {"quad[1032]", "quad[2301]", "half_mirror", "row_mirror", "swap16", "swap32"};
    for (int t = 0; t < 6; ++t) {
        int ok_xor = 1;
        printf("%-12s:", names[t]);
        for (int i = 0; i < 20; ++i) printf(" %d", (int)r[64 * t + i]);
        printf(" ... lane32->%d lane63->%d\n", (int)r[64*t+32], (int)r[64*t+63]);
    }
    return 0;
}
