// reduce_lab.hip -- experiment harness (NOT product code): variants of the W-way
// int32 streaming reduce, timed side by side by tools/lab/reduce_lab.py to pick
// the structure the product kernel (csrc/ina_kernels.hip) uses.
#include <hip/hip_runtime.h>
#include <cstdint>

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
constexpr int MAXW = 16;
struct Ptrs { const u32x4* p[MAXW]; };

#define GLOBAL_AS __attribute__((address_space(1)))
#define LDS_AS __attribute__((address_space(3)))

template <typename T> __device__ __forceinline__ T ldnt(const T* p) { return __builtin_nontemporal_load(p); }

// v1: grid-stride, U chunks spaced by the grid stride (the product form)
template <int W, int U, int B>
__global__ __launch_bounds__(B) void v_gridstride(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    size_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ldnt(in.p[0] + i + u * stride);
#pragma unroll
        for (int w = 1; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += ldnt(in.p[w] + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + i + u * stride);
    }
    for (; i < n4; i += stride) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// v2: block-contiguous tiles: block b handles tiles b, b+G, ...; a tile is U*B chunks
// contiguous, loaded as U consecutive 16-byte-per-lane rows
template <int W, int U, int B>
__global__ __launch_bounds__(B) void v_tile(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tile = (size_t)U * B;
    const size_t ntiles = n4 / tile;
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        size_t base = t * tile + threadIdx.x;
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ldnt(in.p[0] + base + u * B);
#pragma unroll
        for (int w = 1; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += ldnt(in.p[w] + base + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + base + u * B);
    }
    for (size_t i = ntiles * tile + (size_t)blockIdx.x * B + threadIdx.x; i < n4; i += (size_t)gridDim.x * B) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// v3: each block streams one contiguous span (persistent chunking)
template <int W, int U, int B>
__global__ __launch_bounds__(B) void v_span(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    size_t per = (n4 + gridDim.x - 1) / gridDim.x;
    per = (per + (size_t)U * B - 1) / ((size_t)U * B) * ((size_t)U * B);
    size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * B < hi; i += (size_t)U * B) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ldnt(in.p[0] + i + u * B);
#pragma unroll
        for (int w = 1; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += ldnt(in.p[w] + i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + i + u * B);
    }
    for (; i < hi; i += B) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// v4: LDS-DMA staging (global_load_lds_dwordx4, nt), one W x 1 KiB stage per wave
template <int W, int B, int AUX>
__global__ __launch_bounds__(B) void v_ldsdma(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    __shared__ __attribute__((aligned(16))) u32x4 stage[B / 64][W][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t wave_id = ((size_t)blockIdx.x * B + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * B) >> 6;
    const size_t nrows = n4 / 64;
    for (size_t r = wave_id; r < nrows; r += nwaves) {
        size_t i = r * 64 + lane;
#pragma unroll
        for (int w = 0; w < W; ++w)
            __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(in.p[w] + i),
                                             (LDS_AS void*)&stage[wv][w][0], 16, 0, AUX);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 a = stage[wv][0][lane];
#pragma unroll
        for (int w = 1; w < W; ++w) a += stage[wv][w][lane];
        __builtin_nontemporal_store(a, out + i);
    }
    for (size_t i = nrows * 64 + (size_t)blockIdx.x * B + threadIdx.x; i < n4; i += (size_t)gridDim.x * B) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// v5: LDS-DMA, two stages per wave: rows r and r+nwaves in flight together
template <int W, int B, int AUX>
__global__ __launch_bounds__(B) void v_ldsdma2(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    __shared__ __attribute__((aligned(16))) u32x4 stage[B / 64][2][W][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t wave_id = ((size_t)blockIdx.x * B + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * B) >> 6;
    const size_t nrows = n4 / 64;
    size_t r = wave_id;
    for (; r + nwaves < nrows; r += 2 * nwaves) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int w = 0; w < W; ++w)
                __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(in.p[w] + (r + s * nwaves) * 64 + lane),
                                                 (LDS_AS void*)&stage[wv][s][w][0], 16, 0, AUX);
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W) : "memory");
        {
            u32x4 a = stage[wv][0][0][lane];
#pragma unroll
            for (int w = 1; w < W; ++w) a += stage[wv][0][w][lane];
            __builtin_nontemporal_store(a, out + r * 64 + lane);
        }
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");   // the store above is the youngest
        {
            u32x4 a = stage[wv][1][0][lane];
#pragma unroll
            for (int w = 1; w < W; ++w) a += stage[wv][1][w][lane];
            __builtin_nontemporal_store(a, out + (r + nwaves) * 64 + lane);
        }
    }
    for (; r < nrows; r += nwaves) {
        size_t i = r * 64 + lane;
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
    for (size_t i = nrows * 64 + (size_t)blockIdx.x * B + threadIdx.x; i < n4; i += (size_t)gridDim.x * B) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}


// v8: explicit "all loads, then adds" with an optional scheduling fence (SB) so the
// compiler cannot interleave the adds (and full vmcnt(0) waits) between load pairs
template <int W, int U, int B, int SB>
__global__ __launch_bounds__(B) void v_gs_sb(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    size_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 v[W][U];
#pragma unroll
        for (int w = 0; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) v[w][u] = ldnt(in.p[w] + i + u * stride);
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 a = v[0][u];
#pragma unroll
            for (int w = 1; w < W; ++w) a += v[w][u];
            __builtin_nontemporal_store(a, out + i + u * stride);
        }
    }
    for (; i < n4; i += stride) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// ceilings: W-stream read with a negligible write; 1->1 copy
template <int W, int B>
__global__ __launch_bounds__(B) void v_readonly(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    u32x4 a = {0, 0, 0, 0};
    for (size_t i = tid; i < n4; i += stride) {
#pragma unroll
        for (int w = 0; w < W; ++w) a += ldnt(in.p[w] + i);
    }
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u) out[tid] = a;
}

template <int B>
__global__ __launch_bounds__(B) void v_copy(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    for (size_t i = tid; i < n4; i += stride) __builtin_nontemporal_store(ldnt(in.p[0] + i), out + i);
}

// v10: product form with nt loads but a default-policy store (the fp32 PS combine, which
// streams 6.7 TB/s, stores that way); v12: nt loads, store through a buffer resource with
// cache-policy aux bits (AUXS)
template <int W, int U, int B>
__global__ __launch_bounds__(B) void v_gs_plainst(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    size_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ldnt(in.p[0] + i + u * stride);
#pragma unroll
        for (int w = 1; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += ldnt(in.p[w] + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) out[i + u * stride] = a[u];
    }
    for (; i < n4; i += stride) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        out[i] = a;
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// v11: buffer loads/stores, 4 GiB windows per stream, AUXL/AUXS cache-policy bits
template <int W, int U, int B, int AUXL, int AUXS>
__global__ __launch_bounds__(B) void v_gs_buf(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    __amdgpu_buffer_rsrc_t r[W];
#pragma unroll
    for (int w = 0; w < W; ++w) r[w] = mk_rsrc(in.p[w], (uint32_t)(n4 * 16));
    __amdgpu_buffer_rsrc_t ro = mk_rsrc(out, (uint32_t)(n4 * 16));
    const uint32_t tid = blockIdx.x * B + threadIdx.x, stride = gridDim.x * B;
    uint32_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 a[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r[0], (i + u * stride) * 16, 0, AUXL));
#pragma unroll
        for (int w = 1; w < W; ++w)
#pragma unroll
            for (int u = 0; u < U; ++u)
                a[u] += __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r[w], (i + u * stride) * 16, 0, AUXL));
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, a[u]), ro, (i + u * stride) * 16, 0, AUXS);
    }
    for (; i < n4; i += stride) {
        u32x4 a = ldnt(in.p[0] + i);
#pragma unroll
        for (int w = 1; w < W; ++w) a += ldnt(in.p[w] + i);
        __builtin_nontemporal_store(a, out + i);
    }
}

// copy-class policy variants (LD/ST: 1 = nt, 0 = default), 4 chunks in flight per thread
template <int B, int LD, int ST>
__global__ __launch_bounds__(B) void v_copy_pol(Ptrs in, u32x4* __restrict__ out, size_t n4) {
    const size_t tid = (size_t)blockIdx.x * B + threadIdx.x, stride = (size_t)gridDim.x * B;
    size_t i = tid;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        u32x4 a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = LD ? ldnt(in.p[0] + i + u * stride) : in.p[0][i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (ST) __builtin_nontemporal_store(a[u], out + i + u * stride);
            else out[i + u * stride] = a[u];
        }
    }
    for (; i < n4; i += stride) out[i] = in.p[0][i];
}

using Kfn = void (*)(Ptrs, u32x4*, size_t);

template <int B>
static Kfn pick(int variant, int U) {
    switch (variant) {
        case 1: return U == 1 ? v_gridstride<8, 1, B> : U == 2 ? v_gridstride<8, 2, B> : U == 4 ? v_gridstride<8, 4, B> : U == 6 ? v_gridstride<8, 6, B> : v_gridstride<8, 8, B>;
        case 2: return U == 1 ? v_tile<8, 1, B> : U == 2 ? v_tile<8, 2, B> : v_tile<8, 4, B>;
        case 3: return U == 1 ? v_span<8, 1, B> : U == 2 ? v_span<8, 2, B> : v_span<8, 4, B>;
        case 4: return U == 1 ? v_ldsdma<8, B, 0> : v_ldsdma<8, B, 2>;
        case 5: if constexpr (B <= 512 && (B % 64) == 0) return U == 1 ? v_ldsdma2<8, B, 0> : v_ldsdma2<8, B, 2>; else return nullptr;
        case 6: return v_readonly<8, B>;
        case 7: return v_copy<B>;
        case 8: return U == 2 ? v_gs_sb<8, 2, B, 0> : v_gs_sb<8, 4, B, 0>;
        case 9: return U == 2 ? v_gs_sb<8, 2, B, 1> : v_gs_sb<8, 4, B, 1>;
        case 10: return U == 2 ? v_gs_plainst<8, 2, B> : v_gs_plainst<8, 4, B>;
        case 12: return U == 0 ? v_copy_pol<B, 0, 0> : U == 1 ? v_copy_pol<B, 0, 1> : U == 2 ? v_copy_pol<B, 1, 0> : v_copy_pol<B, 1, 1>;
        case 11: return U == 2 ? v_gs_buf<8, 4, B, 2, 2> : U == 4 ? v_gs_buf<8, 4, B, 2, 0> : U == 5 ? v_gs_buf<8, 4, B, 2, 1> : v_gs_buf<8, 4, B, 0, 2>;
    }
    return nullptr;
}

extern "C" int lab_launch(int variant, int W, int U, int B, int grid, const void* const* bufs,
                          void* out, size_t n4, void* stream) {
    if (W != 8) return -1;
    Ptrs p;
    for (int w = 0; w < MAXW; ++w) p.p[w] = w < W ? (const u32x4*)bufs[w] : nullptr;
    Kfn k = B == 256 ? pick<256>(variant, U) : B == 512 ? pick<512>(variant, U) : B == 1024 ? pick<1024>(variant, U) : B == 768 ? pick<768>(variant, U) : B == 128 ? pick<128>(variant, U) : nullptr;
    if (!k) return -2;
    hipLaunchKernelGGL(k, dim3(grid), dim3(B), 0, (hipStream_t)stream, p, (u32x4*)out, n4);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
