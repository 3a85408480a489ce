// store_policy_lab.hip -- experiment harness (NOT product code): the headline W = 8 reduce
// (4 chunks per worker per thread, 512 workgroups, nt loads -- k_sum_reduce_i32_vec<8,4,true>'s
// geometry) with its 16-byte stores issued under different cache-policy bits, to see whether
// the lines a launch leaves dirty cost the NEXT dependent launch (MI355X_MICROARCH.md: a
// kernel boundary costs + B / 6 TB/s when the predecessor leaves B bytes dirty).
//   variant 0: nt (the product), 1: sc0 sc1 (write-through, system scope), 2: sc1 nt,
//   3: sc0 sc1 nt, 4: default policy, 5: sc1
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lab {
using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

template <int P>
__device__ __forceinline__ void store16(u32x4* p, u32x4 v) {
    if constexpr (P == 0) {
        __builtin_nontemporal_store(v, p);
    } else if constexpr (P == 1) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (P == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (P == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (P == 4) {
        *p = v;
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    }
}

template <int P>
__global__ __launch_bounds__(kBlock) void k_reduce8(const uint32_t* const* __restrict__ inp_unused,
                                                    const u32x4* __restrict__ i0, const u32x4* __restrict__ i1,
                                                    const u32x4* __restrict__ i2, const u32x4* __restrict__ i3,
                                                    const u32x4* __restrict__ i4, const u32x4* __restrict__ i5,
                                                    const u32x4* __restrict__ i6, const u32x4* __restrict__ i7,
                                                    u32x4* __restrict__ out, size_t n4) {
    constexpr int U = 4;
    const u32x4* in[8] = {i0, i1, i2, i3, i4, i5, i6, i7};
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    size_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = __builtin_nontemporal_load(in[0] + i + u * stride);
#pragma unroll
        for (int w = 1; w < 8; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += __builtin_nontemporal_load(in[w] + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) store16<P>(out + i + u * stride, acc[u]);
    }
    for (; i < n4; i += stride) {
        u32x4 acc = __builtin_nontemporal_load(in[0] + i);
#pragma unroll
        for (int w = 1; w < 8; ++w) acc += __builtin_nontemporal_load(in[w] + i);
        store16<P>(out + i, acc);
    }
}
}  // namespace lab

extern "C" int lab_reduce8(int variant, int grid, void* const* bufs, void* out, size_t n4, void* stream) {
    using namespace lab;
    hipStream_t s = (hipStream_t)stream;
    const u32x4* b[8];
    for (int w = 0; w < 8; ++w) b[w] = (const u32x4*)bufs[w];
#define L(P) hipLaunchKernelGGL(k_reduce8<P>, dim3(grid), dim3(kBlock), 0, s, nullptr, b[0], b[1], b[2], b[3], \
                                b[4], b[5], b[6], b[7], (u32x4*)out, n4)
    switch (variant) {
        case 0: L(0); break;
        case 1: L(1); break;
        case 2: L(2); break;
        case 3: L(3); break;
        case 4: L(4); break;
        case 5: L(5); break;
        default: return -1;
    }
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
