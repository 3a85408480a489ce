// ew16_lab.hip -- experiment harness (NOT product code): the int16 elementwise kernels
// (quantise fp32 -> int16 with slot flags, dequantise int16 -> fp32) and the fused C2
// quantise + reduce against COPY kernels that move exactly the same bytes with the same
// per-lane layout and no arithmetic -- the floor those kernels could reach on this box.
// tools/lab/ew16_lab.py times them interleaved, back to back on two rotating input sets.
#include "../../distributed-training-ina_amd/csrc/ina_kernels.hip"

namespace lab {
using namespace ina;

// 4 B in -> 2 B out per value, the split layout of k_quantize_i16_vec (a wave covers 512
// values, lane l the 4 at 4l of each 256-value half): 16 B loads, 8 B stores
__global__ __launch_bounds__(kBlock) void k_copy_4to2_split(const float* __restrict__ x,
                                                            uint16_t* __restrict__ y, size_t n) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    const int lane = (int)(tid & 63);
    const size_t nreg = n / 512;
    for (size_t r = tid >> 6; r < nreg; r += stride >> 6) {
        const size_t eA = r * 512 + 4 * (size_t)lane, eB = eA + 256;
        const u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x + eA));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x + eB));
        u32x2 oa, ob;
        oa.x = (u.x >> 16) | (u.y & 0xFFFF0000u);
        oa.y = (u.z >> 16) | (u.w & 0xFFFF0000u);
        ob.x = (v.x >> 16) | (v.y & 0xFFFF0000u);
        ob.y = (v.z >> 16) | (v.w & 0xFFFF0000u);
        __builtin_nontemporal_store(oa, reinterpret_cast<u32x2*>(y + eA));
        __builtin_nontemporal_store(ob, reinterpret_cast<u32x2*>(y + eB));
    }
}

// the same bytes, consecutive layout: lane owns 8 consecutive values (32 B in, 16 B out)
__global__ __launch_bounds__(kBlock) void k_copy_4to2_row(const float* __restrict__ x,
                                                          uint16_t* __restrict__ y, size_t n) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n / 8; i += stride) {
        const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x) + 2 * i);
        const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x) + 2 * i + 1);
        u32x4 o;
        o.x = (a.x >> 16) | (a.y & 0xFFFF0000u);
        o.y = (a.z >> 16) | (a.w & 0xFFFF0000u);
        o.z = (b.x >> 16) | (b.y & 0xFFFF0000u);
        o.w = (b.z >> 16) | (b.w & 0xFFFF0000u);
        __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(y) + i);
    }
}

// 2 B in -> 4 B out per value (k_dequantize_i16's layout: 8 B loads, 16 B stores)
__global__ __launch_bounds__(kBlock) void k_copy_2to4(const uint16_t* __restrict__ x,
                                                      float* __restrict__ y, size_t n) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n / 4; i += stride) {
        const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(x) + i);
        u32x4 r;
        r.x = v.x << 16; r.y = v.x & 0xFFFF0000u; r.z = v.y << 16; r.w = v.y & 0xFFFF0000u;
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4*>(y) + i);
    }
}

// W = 4 streams of 16 B in, one 16 B out (C2's bytes), integer add of the bits only
__global__ __launch_bounds__(kBlock) void k_copy_w4(PtrPack<float> in, int32_t* __restrict__ out,
                                                    size_t n) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n / 4; i += stride) {
        u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[0]) + i);
#pragma unroll
        for (int w = 1; w < 4; ++w) a += __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w]) + i);
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(out) + i);
    }
}
}  // namespace lab

// which: 0 product quantise_i16 (flags), 1 copy 4->2 split, 2 copy 4->2 row,
//        3 product dequantise_i16, 4 copy 2->4, 5 product C2 quant_reduce<4>, 6 copy W=4,
//        7 product sum_reduce<4,1,true> (int32 bits, no quantise)
extern "C" int lab_run(int which, int grid, const void* const* bufs, void* out, size_t n, void* ovf,
                       void* stream) {
    using namespace ina;
    hipStream_t s = (hipStream_t)stream;
    PtrPack<float> pk;
    PtrPack<int32_t> pki;
    for (int w = 0; w < INA_MAX_WORKERS; ++w) {
        pk.p[w] = w < 4 ? (const float*)bufs[w] : nullptr;
        pki.p[w] = w < 4 ? (const int32_t*)bufs[w] : nullptr;
    }
    const float* x = (const float*)bufs[0];
    switch (which) {
        case 0: hipLaunchKernelGGL(k_quantize_i16_vec, dim3(grid), dim3(kBlock), 0, s, x, (int16_t*)out, n,
                                   8192.0f, 256, 32, (uint8_t*)ovf); break;
        case 1: hipLaunchKernelGGL(lab::k_copy_4to2_split, dim3(grid), dim3(kBlock), 0, s, x, (uint16_t*)out, n); break;
        case 2: hipLaunchKernelGGL(lab::k_copy_4to2_row, dim3(grid), dim3(kBlock), 0, s, x, (uint16_t*)out, n); break;
        case 3: hipLaunchKernelGGL(k_dequantize_i16, dim3(grid), dim3(kBlock), 0, s, (const int16_t*)bufs[0],
                                   (float*)out, n, 1.0f / 8192.0f, 1); break;
        case 4: hipLaunchKernelGGL(lab::k_copy_2to4, dim3(grid), dim3(kBlock), 0, s, (const uint16_t*)bufs[0],
                                   (float*)out, n); break;
        case 5: hipLaunchKernelGGL(k_quant_reduce_i32<4>, dim3(grid), dim3(kBlock), 0, s, pk, 4, (int32_t*)out, n,
                                   65536.0f, 1); break;
        case 6: hipLaunchKernelGGL(lab::k_copy_w4, dim3(grid), dim3(kBlock), 0, s, pk, (int32_t*)out, n); break;
        case 7: hipLaunchKernelGGL((k_sum_reduce_i32_vec<4, 1, true>), dim3(grid), dim3(kBlock), 0, s, pki,
                                   (int32_t*)out, n / 4, n); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
