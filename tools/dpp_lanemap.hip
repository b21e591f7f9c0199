// Lane mapping of the cross-lane moves the DPP scan tree uses (gfx950): prints, per primitive, the
// source lane each destination lane received (x = lane id; -1 = kept its "old" value).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o)
{
    const int l = threadIdx.x;
    const int x = l;
    o[0 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false);   // row_bcast:15, rows 1,3
    o[1 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false);   // row_bcast:31, rows 2,3
    o[2 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x150, 0x5, 0xF, false);   // row_newbcast:0, rows 0,2
    o[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false);   // row_shr:2
    o[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, x, 0x108, 0xF, 0xF, false);   // row_shl:8
    auto s = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    o[5 * 64 + l] = s[0];
    o[6 * 64 + l] = s[1];
    auto t = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    o[7 * 64 + l] = t[0];
    o[8 * 64 + l] = t[1];
    o[9 * 64 + l] = __builtin_amdgcn_readlane(x, 32);
}
int main()
{
    int* d;
    int h[10 * 64];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[10] = {"row_bcast15 rm0xA", "row_bcast31 rm0xC", "row_newbcast0 rm0x5", "row_shr2", "row_shl8",
                          "permlane16_swap[0]", "permlane16_swap[1]", "permlane32_swap[0]", "permlane32_swap[1]",
                          "readlane32"};
    for (int p = 0; p < 10; ++p) {
        printf("%-20s", nm[p]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[p * 64 + l]);
        printf("\n");
    }
    hipFree(d);
    return 0;
}
