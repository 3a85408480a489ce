// atomic_lab.hip -- experiment (NOT product code): cost of one returning device-scope
// atomicAdd per packet on a per-slot counter table (the fixed-capacity slot-bucket idea
// for the device switch), against a plain scattered store of the same shape.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void k_bucket(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* __restrict__ cnt,
                         uint32_t* __restrict__ slots, int K, int mode) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const uint32_t k = keys[p];
        if (mode == 0) {
            const uint32_t pos = atomicAdd(&cnt[k], 1u);
            slots[(size_t)k * K + (pos < (uint32_t)K ? pos : K - 1)] = p;
        } else if (mode == 1) {
            atomicAdd(&cnt[k], 1u);                 // non-returning
        } else {
            slots[(size_t)k * K] = p;                // plain scattered store
        }
    }
}

extern "C" int lab_bucket(const uint32_t* keys, uint32_t n, uint32_t* cnt, uint32_t* slots, int K,
                          int mode, int grid, int block, void* stream) {
    hipLaunchKernelGGL(k_bucket, dim3(grid), dim3(block), 0, (hipStream_t)stream, keys, n, cnt, slots,
                       K, mode);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
