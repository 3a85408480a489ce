// dpp_lab.hip -- which lane does each gfx950 DPP wave shift read? (experiment only)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    int l = threadIdx.x;
    out[0 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x130, 0xF, 0xF, false);  // wave_shl:1
    out[1 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x138, 0xF, 0xF, false);  // wave_shr:1
    out[2 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x134, 0xF, 0xF, false);  // wave_rol:1
    out[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x13C, 0xF, 0xF, false);  // wave_ror:1
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x101, 0xF, 0xF, false);  // row_shl:1
    out[5 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x111, 0xF, 0xF, false);  // row_shr:1
}
int main() {
    int* d; int h[6 * 64];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    const char* nm[6] = {"wave_shl1", "wave_shr1", "wave_rol1", "wave_ror1", "row_shl1", "row_shr1"};
    for (int r = 0; r < 6; ++r) {
        printf("%s:", nm[r]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
