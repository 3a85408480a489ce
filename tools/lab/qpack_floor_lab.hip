// qpack_floor_lab.hip -- experiment harness (NOT product code): the one-launch worker pack
// (k_qpack_nga_multi_v256<8>) against COPY kernels moving the same bytes with no arithmetic:
//   1: the product's layout (a wave per 1040-byte row, 9 aligned 1 KiB loads, 8 body stores
//      at row + 16 and a lane-0 header store per worker), the loaded bits stored as they are;
//   2: the ideal stream copy of the same volume (8 x 1 KiB stores at row starts of a
//      1,024-byte stride: aligned, no header chunk).
// tools/lab/qpack_floor_lab.py times them interleaved with the product call.
#include "../../distributed-training-ina_amd/csrc/ina_kernels.hip"

namespace lab {
using namespace ina;

template <bool kRows>
__global__ __launch_bounds__(kBlock) void k_copy_qpm(QPackGroup a, const float* __restrict__ base,
                                                     uint32_t stride, uint32_t np) {
    const int lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * kBlock) >> 6;
    for (uint32_t p = (blockIdx.x * kBlock + threadIdx.x) >> 6; p < np; p += nwaves) {
        const size_t e0 = (size_t)p * 256 + 4 * (size_t)lane;
        const u32x4 b = *reinterpret_cast<const u32x4*>(base + e0);
        u32x4 v[kQpGroup];
#pragma unroll
        for (int g = 0; g < kQpGroup; ++g)
            v[g] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.x[g] + e0));
#pragma unroll
        for (int g = 0; g < kQpGroup; ++g) {
            const u32x4 o = u32x4{v[g].x ^ b.x, v[g].y ^ b.y, v[g].z ^ b.z, v[g].w ^ b.w};
            u32x4* row = reinterpret_cast<u32x4*>(a.pkts[g] + (size_t)p * stride);
            if (kRows) {
                packet_store(o, row + 1 + lane);
                if (lane == 0) packet_store(o, row);
            } else {
                packet_store(o, row + lane);
            }
        }
    }
}
}  // namespace lab

extern "C" int lab_copy(int which, const float* const* xs, const float* base, uint8_t* const* outs,
                        uint32_t stride, uint32_t np, void* stream) {
    ina::QPackGroup a{};
    for (int g = 0; g < ina::kQpGroup; ++g) {
        a.x[g] = xs[g];
        a.pkts[g] = outs[g];
    }
    const dim3 grid((np * 64 + ina::kBlock - 1) / ina::kBlock), blk(ina::kBlock);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (which == 1) hipLaunchKernelGGL(lab::k_copy_qpm<true>, grid, blk, 0, s, a, base, stride, np);
    else hipLaunchKernelGGL(lab::k_copy_qpm<false>, grid, blk, 0, s, a, base, stride, np);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
