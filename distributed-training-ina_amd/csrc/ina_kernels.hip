// ina_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the INA aggregation path
// and the extern "C" entry points declared in include/ina.h.
//
// Reference behaviour each kernel reproduces (Fangjin98/distributed-training-INA):
//   k_sum_reduce_*      processor.p4:14-24 (x32, ngaa.p4:87-168): per-slot bit<32> add
//   k_quantize_*        float_to_int (absent; DataManager.py:9,37) -- build-defined
//   k_dequantize_*      int_to_float (absent; NGAPacket.py:5,118) -- build-defined
//   k_ps_combine_f32    aggregate(), launch.py:42-52 / launch_async.py:42-57
//   k_pack_nga_*        DataManager._send_data, DataManager.py:111-165 + headers.p4:27-80
//   k_unpack_nga_*      NGAHeader/NGAPayload, NGAPacket.py:62-118 (layout of headers.p4)
//   k_pack_c128         send_gradients packet loop, communicator.cc:23-37
//
// All of these are HBM-streaming kernels (no contraction -> no MFMA): 16 B per lane
// per access (global_load_dwordx4), 256-thread workgroups, grid-stride loops over
// a grid capped near 8 workgroups per CU, non-temporal loads and write-through (sc1)
// stores for data that is touched exactly once (ina_device.h).  Integer sums use uint32 arithmetic (defined wraparound).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstring>

#include "ina.h"
#include "ina_internal.h"
#include "ina_device.h"

namespace ina {

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
using u32x2 = uint32_t __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// error reporting
// ---------------------------------------------------------------------------
static thread_local char g_err[256] = "";

int set_error(int code, const char* fmt, const char* detail) {
    snprintf(g_err, sizeof g_err, fmt, detail ? detail : "");
    return code;
}

static int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
        return INA_EHIP;
    }
    return INA_OK;
}

// ---------------------------------------------------------------------------
// tuning (grid cap / unroll), overridable for sweeps through ina_set_tuning()
// ---------------------------------------------------------------------------
static std::atomic<int> g_max_blocks{16384};  // default-cap kernels (C4 int16 fused: 16384 beat 8192 by 3 %)
// sum-reduce: measured best on MI355X (tools/lab/reduce_lab.py, reduce_w_lab.py,
// interleaved A/B): 4 x 16 B per worker per thread in flight and 64*W 256-thread
// workgroups (W = 2, 4: 256; W = 8: 512; W = 16: 1024).  0 = that rule; >0 overrides.
static std::atomic<int> g_reduce_blocks{0};
static std::atomic<int> g_unroll{0};   // 0 = per-W choice (launch_reduce_u)
// 16-byte chunks in flight per thread in the one-in one-out elementwise kernels
// (quantise, dequantise, PS apply): one, with the 8192-workgroup grid striding, beat 2
// and 4 -- quantise 40.9 -> 37.6 us, dequantise 41.2 -> 36.8 (tools/lab/ew_lab.py)
#ifndef INA_EW_U
#define INA_EW_U 1
#endif
constexpr int kEwU = INA_EW_U;
// PS combine kernels, W <= 4 (tools/lab/ew_lab.py, C2 size): one chunk in flight --
// fp32 combine 94.3 -> 91.9 us at 256 workgroups, INA combine 106.4 -> 93.2 us at 8192
#ifndef INA_COMB_U
#define INA_COMB_U 1
#endif
#ifndef INA_COMBI_U
#define INA_COMBI_U 1
#endif
#ifndef INA_QR_U
#define INA_QR_U 1     // fused quantise + reduce, W <= 8: C2 91.8 -> 86.7 us (ew_lab)
#endif
// the flat packet kernels (pack, fused quantise + pack, unpack; one 16-byte chunk per thread,
// grid-striding) and the fused quantise + reduce for W > 8: 16,384 workgroups beat 8,192 by
// 1-3 % on two boxes (pack 34.9 -> 33.9 us, worker pack 51.5 -> 50.8, unpack 36.6 -> 35.6;
// a covering grid of ~26k is slower again; profiles/r03/lab/pack_grid_lab.log)
static std::atomic<int> g_stream_blocks{16384};
// the one-in one-out elementwise kernels (quantise, dequantise, PS apply, the int16 wire
// kernels of ina_shard.hip): one 16-byte chunk per thread, the grid covering the whole
// array -- no grid-stride loop.  At a 1 GiB bucket (config 5) that is 330-340 us (80 %)
// against 416-425 us (64 %) with an 8192-workgroup grid striding; at config-2 size it is
// within +-1 us of it (tools/lab/ew_grid_lab.py, profiles/r02/lab/ew_grid_lab.json)
static std::atomic<int> g_ew_blocks{1 << 24};
int ew_grid_cap() { return g_ew_blocks.load(); }
// PS combine kernels (W+2 streams), measured per kernel (bench_extra grid sweeps and
// ew_lab): the fp32 combine runs best at 256 workgroups (6.6-6.7 TB/s vs 6.0 at 512),
// the INA combine (quantiser in the loop) with one chunk in flight at 8192
static std::atomic<int> g_combine_blocks{256};
static std::atomic<int> g_combine_ina_blocks{8192};
static std::atomic<int> g_nontemporal{1};
// flat packet kernels index 16-byte chunks in 32 bits: a launch covers at most this many
// chunks and longer batches go in packet ranges (tunable so tests reach the split path)
static std::atomic<int64_t> g_launch_chunks{0x7FFFFFFF};

static inline unsigned grid_for(size_t work_items, int per_thread, int cap_override = 0) {
    size_t per_block = (size_t)kBlock * (size_t)per_thread;
    size_t blocks = (work_items + per_block - 1) / per_block;
    size_t cap = (size_t)(cap_override > 0 ? cap_override : g_max_blocks.load());
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    return (unsigned)blocks;
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// grid cap of the reductions that finish with one atomic per workgroup on one word
constexpr int kFaninBlocks = 256;

// ---------------------------------------------------------------------------
// memory helpers
// ---------------------------------------------------------------------------
template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT) stream_store(v, p);
    else *p = v;
}

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// ---------------------------------------------------------------------------
// quantiser (build-defined, see include/ina.h): sat(rne(x * 2^k)), NaN -> 0
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t q32(float x, float s) {
    float y = __builtin_rintf(x * s);
    int32_t r = (int32_t)y;                         // in-range lanes only are selected
    r = (y >= 2147483648.0f) ? INT32_MAX : r;
    r = (y < -2147483648.0f) ? INT32_MIN : r;
    return (y != y) ? 0 : r;
}

// returns the int16 value widened to int32; *sat |= clamped-or-NaN
#ifndef INA_Q16_MED3
#define INA_Q16_MED3 1
#endif
// int16 kernels: a wave covers 512 values as two 256-value halves (16 B per lane per
// load, contiguous per instruction) -- C4 fused quantise+reduce 289 -> 251 us against
// 8 consecutive values per lane (32-B lane stride; tools/lab/ew_lab.py, lab/q16_lab.log)
#ifndef INA_Q16_SPLIT
#define INA_Q16_SPLIT 1
#endif
__device__ __forceinline__ int32_t q16(float x, float s, bool& sat) {
    float y = __builtin_rintf(x * s);
#if INA_Q16_MED3
    // one v_med3_f32 clamps; a clamped value, +-inf or NaN differs from y
    const float c = __builtin_amdgcn_fmed3f(y, -32768.0f, 32767.0f);
    sat |= !(c == y);
    return (y != y) ? 0 : (int32_t)c;
#else
    bool in = (y <= 32767.0f) && (y >= -32768.0f);  // false for NaN
    sat |= !in;
    int32_t r = in ? (int32_t)y : 0;
    r = (y > 32767.0f) ? 32767 : r;
    r = (y < -32768.0f) ? -32768 : r;
    return r;
#endif
}

__device__ __forceinline__ int32_t sat16(int32_t a, bool& sat) {
    bool hi = a > 32767, lo = a < -32768;
    sat |= hi | lo;
    return hi ? 32767 : (lo ? -32768 : a);
}

// ---------------------------------------------------------------------------
// per-slot overflow flags: thread t owns 8 consecutive values; a slot of V values
// (V % 8 == 0, V/8 a power of two <= 64) is V/8 adjacent lanes of one wave.  The
// group's first lane writes the slot flag from a wave ballot -- one writer per slot,
// no atomics, no pre-zeroing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void write_slot_flags8(unsigned long long m, bool active, size_t elem0,
                                                  int V, int lanes_per_slot,
                                                  uint8_t* __restrict__ ovf) {
    int lane = threadIdx.x & 63;
    int g0 = lane & ~(lanes_per_slot - 1);
    unsigned long long gm = (lanes_per_slot == 64) ? ~0ull : (((1ull << lanes_per_slot) - 1ull) << g0);
    if (active && (lane & (lanes_per_slot - 1)) == 0) ovf[elem0 / (size_t)V] = (m & gm) ? 1 : 0;
}

// the same for the split layout (a wave owns 512 values, lane l holds 4 at 4l of each
// 256-value half): a slot is V/4 adjacent lanes of one half, or both halves at V = 512
__device__ __forceinline__ void write_slot_flags_split(unsigned long long ma, unsigned long long mb,
                                                       size_t eA, size_t eB, size_t n, int V,
                                                       uint8_t* __restrict__ ovf) {
    if (V >= 512) {
        write_slot_flags8(ma | mb, eA < n, eA, V, 64, ovf);
    } else {
        write_slot_flags8(ma, eA < n, eA, V, V / 4, ovf);
        write_slot_flags8(mb, eB < n, eB, V, V / 4, ovf);
    }
}

static inline bool slot_ballot_ok(int V) {
    if (V % 8) return false;
    int l = V / 8;
    return l >= 1 && l <= 64 && (l & (l - 1)) == 0;
}


// Cross-lane moves by one lane are DPP row moves (measured on gfx950, tools/lab/dpp_lab.hip):
// update_dpp(old, x, 0x130 wave_shl:1) -> lane i reads lane i+1 (lane 63 gets `old`);
// 0x138 wave_shr:1 -> lane i reads lane i-1 (lane 0 gets `old`).  One VALU op instead of
// an LDS ds_bpermute, and `old` supplies the value from outside the wave.

template <int W>
constexpr int kUnrW = W > 0 ? W : 1;

// Grid-stride loop over 16-byte chunks with UU independent chunks per thread per
// iteration (chunks i, i+stride, ..., all loads issued before use), then a 1-chunk
// remainder loop: the geometry the reduce lab measured fastest (tools/lab).
template <int U, typename Body>
__device__ __forceinline__ void chunk_loop(size_t n4, Body&& body) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    size_t i = tid;
    for (; i + (U - 1) * stride < n4; i += U * stride) body.template operator()<U>(i, stride);
    for (; i < n4; i += stride) body.template operator()<1>(i, stride);
}

// ===========================================================================
// 1. W-way int32 sum-reduce (the headline kernel)
// ===========================================================================
template <int W, int U, bool NT>
__device__ __forceinline__ void sum_reduce_body(const PtrPack<int32_t>& in, int32_t* __restrict__ out,
                                                size_t n4, size_t n) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    size_t i = tid;
    // full iterations: U independent 16-byte chunks per thread, all W*U loads in flight
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc[u] = ld<NT>(reinterpret_cast<const u32x4*>(in.p[0]) + i + u * stride);
#pragma unroll
        for (int w = 1; w < W; ++w) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                acc[u] += ld<NT>(reinterpret_cast<const u32x4*>(in.p[w]) + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            st<NT>(reinterpret_cast<u32x4*>(out) + i + u * stride, acc[u]);
    }
    for (; i < n4; i += stride) {
        u32x4 acc = ld<NT>(reinterpret_cast<const u32x4*>(in.p[0]) + i);
#pragma unroll
        for (int w = 1; w < W; ++w) acc += ld<NT>(reinterpret_cast<const u32x4*>(in.p[w]) + i);
        st<NT>(reinterpret_cast<u32x4*>(out) + i, acc);
    }
    // scalar tail (n % 4 values)
    size_t t = 4 * n4 + tid;
    if (t < n) {
        uint32_t a = (uint32_t)in.p[0][t];
#pragma unroll
        for (int w = 1; w < W; ++w) a += (uint32_t)in.p[w][t];
        out[t] = (int32_t)a;
    }
}

template <int W, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_sum_reduce_i32_vec(PtrPack<int32_t> in,
                                                               int32_t* __restrict__ out,
                                                               size_t n4, size_t n) {
    sum_reduce_body<W, U, NT>(in, out, n4, n);
}

// the same reduce launched by the PCIe pipeline (ina_sum_reduce_host_i32) on its chunks:
// its own symbol only so that rocprof attributes the pipeline's launches apart from the
// device-resident bulk reduce (same body, same geometry)
template <int W, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_host_chunk_reduce_i32(PtrPack<int32_t> in,
                                                                  int32_t* __restrict__ out,
                                                                  size_t n4, size_t n) {
    sum_reduce_body<W, U, NT>(in, out, n4, n);
}

// runtime-W vector kernel (W not in the specialised set)
__global__ __launch_bounds__(kBlock) void k_sum_reduce_i32_vec_dyn(PtrPack<int32_t> in, int W,
                                                                   int32_t* __restrict__ out,
                                                                   size_t n4, size_t n) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = tid; i < n4; i += stride) {
        u32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[0]) + i);
        int w = 1;
        for (; w + 3 < W; w += 4) {
            u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w]) + i);
            u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w + 1]) + i);
            u32x4 c = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w + 2]) + i);
            u32x4 d = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w + 3]) + i);
            acc += (a + b) + (c + d);
        }
        for (; w < W; ++w) acc += __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w]) + i);
        stream_store(acc, reinterpret_cast<u32x4*>(out) + i);
    }
    size_t t = 4 * n4 + tid;
    if (t < n) {
        uint32_t a = 0;
        for (int w = 0; w < W; ++w) a += (uint32_t)in.p[w][t];
        out[t] = (int32_t)a;
    }
}

// unaligned fallback: one element per thread
__global__ __launch_bounds__(kBlock) void k_sum_reduce_i32_scalar(PtrPack<int32_t> in, int W,
                                                                  int32_t* __restrict__ out,
                                                                  size_t n) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint32_t a = 0;
        for (int w = 0; w < W; ++w) a += (uint32_t)in.p[w][i];
        out[i] = (int32_t)a;
    }
}

template <int W, int U>
static void launch_reduce_w(const PtrPack<int32_t>& pk, int32_t* out, size_t n4, size_t n,
                            hipStream_t s, bool host) {
    int cap = g_reduce_blocks.load();
    // 64 workgroups per worker stream, clamped to [256, 1024] -- except W = 16 (768: 3 per
    // CU beat 4, 278.8 vs 300.2 us) and W = 2 with one chunk (512); tools/lab/reduce_w_sweep.py
    if (cap <= 0)
        cap = W == 16 ? 768 : (W == 2 && U == 1) ? 512 : (W * 64 < 256 ? 256 : (W * 64 > 1024 ? 1024 : W * 64));
    unsigned g = grid_for(n4, U, cap);
    const bool nt = g_nontemporal.load();
    if (host && nt)
        hipLaunchKernelGGL((k_host_chunk_reduce_i32<W, U, true>), dim3(g), dim3(kBlock), 0, s, pk, out, n4, n);
    else if (host)
        hipLaunchKernelGGL((k_host_chunk_reduce_i32<W, U, false>), dim3(g), dim3(kBlock), 0, s, pk, out, n4, n);
    else if (nt)
        hipLaunchKernelGGL((k_sum_reduce_i32_vec<W, U, true>), dim3(g), dim3(kBlock), 0, s, pk, out, n4, n);
    else
        hipLaunchKernelGGL((k_sum_reduce_i32_vec<W, U, false>), dim3(g), dim3(kBlock), 0, s, pk, out, n4, n);
}

template <int W>
static void launch_reduce_u(const PtrPack<int32_t>& pk, int32_t* out, size_t n4, size_t n,
                            hipStream_t s, bool host) {
    int u = g_unroll.load();
    if (u == 0) u = W <= 4 ? 1 : 4;   // auto: 1 chunk per stream for W <= 4 (86.5 vs 90.4 us at W = 4)
    switch (u) {
        case 1: launch_reduce_w<W, 1>(pk, out, n4, n, s, host); break;
        case 2: launch_reduce_w<W, 2>(pk, out, n4, n, s, host); break;
        default: launch_reduce_w<W, 4>(pk, out, n4, n, s, host); break;
    }
}

// ===========================================================================
// 2. quantise / dequantise
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_quantize_i32(const float* __restrict__ x,
                                                         int32_t* __restrict__ q, size_t n,
                                                         float s, int vec) {
    size_t n4 = vec ? n / 4 : 0;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    u32x4* q4 = reinterpret_cast<u32x4*>(q);
    chunk_loop<kEwU>(n4, [&]<int UU>(size_t i, size_t st) {
        f32x4 v[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) v[u] = __builtin_nontemporal_load(x4 + i + u * st);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            u32x4 r;
            r.x = (uint32_t)q32(v[u].x, s); r.y = (uint32_t)q32(v[u].y, s);
            r.z = (uint32_t)q32(v[u].z, s); r.w = (uint32_t)q32(v[u].w, s);
            stream_store(r, q4 + i + u * st);
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        q[i] = q32(x[i], s);
}

// int16: thread owns 8 values (two float4 loads, one 16-byte store)
__global__ __launch_bounds__(kBlock) void k_quantize_i16_vec(const float* __restrict__ x,
                                                             int16_t* __restrict__ q, size_t n,
                                                             float s, int V, int lanes_per_slot,
                                                             uint8_t* __restrict__ ovf) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
#if INA_Q16_SPLIT
    // a wave owns 512 consecutive values, lane l the 4 at 4l of each 256-value half (one
    // contiguous KiB per load instruction); see k_quant_reduce_i16
    const int lane = (int)(tid & 63);
    const size_t nreg = (n + 511) / 512;
    for (size_t r = tid >> 6; r < nreg; r += stride >> 6) {
        const size_t eA = r * 512 + 4 * (size_t)lane, eB = eA + 256;
        bool sa = false, sb = false;
        if (r * 512 + 512 <= n) {                 // wave-uniform
            f32x4 u = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + eA));
            f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + eB));
            u32x2 oa, ob;
            oa.x = (uint32_t)(uint16_t)q16(u.x, s, sa) | ((uint32_t)q16(u.y, s, sa) << 16);
            oa.y = (uint32_t)(uint16_t)q16(u.z, s, sa) | ((uint32_t)q16(u.w, s, sa) << 16);
            ob.x = (uint32_t)(uint16_t)q16(v.x, s, sb) | ((uint32_t)q16(v.y, s, sb) << 16);
            ob.y = (uint32_t)(uint16_t)q16(v.z, s, sb) | ((uint32_t)q16(v.w, s, sb) << 16);
            stream_store(oa, reinterpret_cast<u32x2*>(q + eA));
            stream_store(ob, reinterpret_cast<u32x2*>(q + eB));
        } else {
            for (size_t j = eA; j < eA + 4 && j < n; ++j) q[j] = (int16_t)q16(x[j], s, sa);
            for (size_t j = eB; j < eB + 4 && j < n; ++j) q[j] = (int16_t)q16(x[j], s, sb);
        }
        const unsigned long long ma = __ballot(sa), mb = __ballot(sb);   // wave-convergent
        if (ovf) write_slot_flags_split(ma, mb, eA, eB, n, V, ovf);
    }
#else
    const size_t n8 = (n + 7) / 8;
    // uniform trip count per wave so every lane reaches the ballot together
    const size_t wave0 = tid & ~(size_t)63;
    for (size_t base = wave0; base < n8; base += stride) {
        size_t i = base + (tid & 63);
        bool sat = false;
        if (i < n8) {
            size_t e = 8 * i;
            int32_t r[8];
            if (e + 8 <= n) {
                f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + e));
                f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + e) + 1);
                r[0] = q16(a.x, s, sat); r[1] = q16(a.y, s, sat); r[2] = q16(a.z, s, sat); r[3] = q16(a.w, s, sat);
                r[4] = q16(b.x, s, sat); r[5] = q16(b.y, s, sat); r[6] = q16(b.z, s, sat); r[7] = q16(b.w, s, sat);
                u32x4 o;
                o.x = (uint32_t)(uint16_t)r[0] | ((uint32_t)r[1] << 16);
                o.y = (uint32_t)(uint16_t)r[2] | ((uint32_t)r[3] << 16);
                o.z = (uint32_t)(uint16_t)r[4] | ((uint32_t)r[5] << 16);
                o.w = (uint32_t)(uint16_t)r[6] | ((uint32_t)r[7] << 16);
                stream_store(o, reinterpret_cast<u32x4*>(q + e));
            } else {
                for (size_t j = e; j < n; ++j) q[j] = (int16_t)q16(x[j], s, sat);
            }
        }
        unsigned long long m = __ballot(sat);   // wave-convergent: uniform trip count
        if (ovf) write_slot_flags8(m, i < n8, 8 * i, V, lanes_per_slot, ovf);
    }
#endif
}

// generic int16 path (unaligned or V without a ballot layout): byte flags via a
// pre-zeroed array and benign same-value stores
__global__ __launch_bounds__(kBlock) void k_quantize_i16_scalar(const float* __restrict__ x,
                                                                int16_t* __restrict__ q, size_t n,
                                                                float s, int V,
                                                                uint8_t* __restrict__ ovf) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        bool sat = false;
        q[i] = (int16_t)q16(x[i], s, sat);
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
}

__global__ __launch_bounds__(kBlock) void k_dequantize_i32(const int32_t* __restrict__ sv,
                                                           float* __restrict__ y, size_t n,
                                                           float inv, int vec) {
    size_t n4 = vec ? n / 4 : 0;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(sv);
    f32x4* y4 = reinterpret_cast<f32x4*>(y);
    chunk_loop<kEwU>(n4, [&]<int UU>(size_t i, size_t st) {
        u32x4 v[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) v[u] = __builtin_nontemporal_load(s4 + i + u * st);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            f32x4 r;
            r.x = (float)(int32_t)v[u].x * inv; r.y = (float)(int32_t)v[u].y * inv;
            r.z = (float)(int32_t)v[u].z * inv; r.w = (float)(int32_t)v[u].w * inv;
            stream_store(r, y4 + i + u * st);
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = (float)sv[i] * inv;
}

// int16 -> fp32: lane holds 4 values (8-byte load, 16-byte store), so each instruction of
// a wave reads 512 B and writes 1 KiB contiguous; vec = 0 for unaligned buffers
__global__ __launch_bounds__(kBlock) void k_dequantize_i16(const int16_t* __restrict__ sv,
                                                           float* __restrict__ y, size_t n,
                                                           float inv, int vec) {
    size_t n4 = vec ? n / 4 : 0;
    const u32x2* s4 = reinterpret_cast<const u32x2*>(sv);
    f32x4* y4 = reinterpret_cast<f32x4*>(y);
    chunk_loop<kEwU>(n4, [&]<int UU>(size_t i, size_t st) {
        u32x2 v[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) v[u] = __builtin_nontemporal_load(s4 + i + u * st);
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            f32x4 r;
            r.x = (float)(int16_t)(v[u].x & 0xFFFFu) * inv; r.y = (float)((int32_t)v[u].x >> 16) * inv;
            r.z = (float)(int16_t)(v[u].y & 0xFFFFu) * inv; r.w = (float)((int32_t)v[u].y >> 16) * inv;
            stream_store(r, y4 + i + u * st);
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = (float)sv[i] * inv;
}

// ===========================================================================
// 3. fused quantise + reduce (configs 2 and 4) and the int16 narrow reduce
// ===========================================================================
template <int W>
__global__ __launch_bounds__(kBlock) void k_quant_reduce_i32(PtrPack<float> in, int Wd,
                                                             int32_t* __restrict__ out,
                                                             size_t n, float s, int vec) {
    const int nw = W > 0 ? W : Wd;
    size_t n4 = vec ? n / 4 : 0;
    u32x4* o4 = reinterpret_cast<u32x4*>(out);
    if constexpr (W > 0) {
        chunk_loop<(W <= 8 ? INA_QR_U : 2)>(n4, [&]<int UU>(size_t i, size_t st) {
            f32x4 v[W][UU];
#pragma unroll
            for (int w = 0; w < W; ++w)
#pragma unroll
                for (int u = 0; u < UU; ++u)
                    v[w][u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w]) + i + u * st);
#pragma unroll
            for (int u = 0; u < UU; ++u) {
                u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    acc.x += (uint32_t)q32(v[w][u].x, s); acc.y += (uint32_t)q32(v[w][u].y, s);
                    acc.z += (uint32_t)q32(v[w][u].z, s); acc.w += (uint32_t)q32(v[w][u].w, s);
                }
                stream_store(acc, o4 + i + u * st);
            }
        });
    } else {
        const size_t stride = (size_t)gridDim.x * kBlock;
        for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
            u32x4 acc = {0u, 0u, 0u, 0u};
            for (int w = 0; w < nw; ++w) {
                f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w]) + i);
                acc.x += (uint32_t)q32(v.x, s); acc.y += (uint32_t)q32(v.y, s);
                acc.z += (uint32_t)q32(v.z, s); acc.w += (uint32_t)q32(v.w, s);
            }
            stream_store(acc, o4 + i);
        }
    }
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint32_t a = 0;
        for (int w = 0; w < nw; ++w) a += (uint32_t)q32(in.p[w][i], s);
        out[i] = (int32_t)a;
    }
}

// int16: thread owns 8 values; each worker value saturates at quantisation (wire
// width), exact int32 sum, one final saturation; per-slot flag = any saturation.
template <int W>
__global__ __launch_bounds__(kBlock) void k_quant_reduce_i16(PtrPack<float> in, int Wd,
                                                             int16_t* __restrict__ out, size_t n,
                                                             float s, int V, int lanes_per_slot,
                                                             uint8_t* __restrict__ ovf) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    const int nw = W > 0 ? W : Wd;
    constexpr int UNR = W > 0 ? W : 1;
#if INA_Q16_SPLIT
    // a wave owns 512 consecutive values: lane l holds 4l..4l+3 of each 256-value half, so
    // every load instruction of the wave reads 1 KiB contiguous (16 B per lane, no 32-B
    // lane stride); the two halves' saturation ballots give the slot flags
    const int lane = (int)(tid & 63);
    const size_t nreg = (n + 511) / 512;
    for (size_t r = tid >> 6; r < nreg; r += stride >> 6) {
        const size_t eA = r * 512 + 4 * (size_t)lane, eB = eA + 256;
        bool sa = false, sb = false;
        if (r * 512 + 512 <= n) {                 // wave-uniform
            int32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll UNR
            for (int w = 0; w < nw; ++w) {
                f32x4 u = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w] + eA));
                f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w] + eB));
                a[0] += q16(u.x, s, sa); a[1] += q16(u.y, s, sa);
                a[2] += q16(u.z, s, sa); a[3] += q16(u.w, s, sa);
                a[4] += q16(v.x, s, sb); a[5] += q16(v.y, s, sb);
                a[6] += q16(v.z, s, sb); a[7] += q16(v.w, s, sb);
            }
            u32x2 oa, ob;
            oa.x = (uint32_t)(uint16_t)sat16(a[0], sa) | ((uint32_t)sat16(a[1], sa) << 16);
            oa.y = (uint32_t)(uint16_t)sat16(a[2], sa) | ((uint32_t)sat16(a[3], sa) << 16);
            ob.x = (uint32_t)(uint16_t)sat16(a[4], sb) | ((uint32_t)sat16(a[5], sb) << 16);
            ob.y = (uint32_t)(uint16_t)sat16(a[6], sb) | ((uint32_t)sat16(a[7], sb) << 16);
            stream_store(oa, reinterpret_cast<u32x2*>(out + eA));
            stream_store(ob, reinterpret_cast<u32x2*>(out + eB));
        } else {
            for (size_t j = eA; j < eA + 4 && j < n; ++j) {
                int32_t a = 0;
                for (int w = 0; w < nw; ++w) a += q16(in.p[w][j], s, sa);
                out[j] = (int16_t)sat16(a, sa);
            }
            for (size_t j = eB; j < eB + 4 && j < n; ++j) {
                int32_t a = 0;
                for (int w = 0; w < nw; ++w) a += q16(in.p[w][j], s, sb);
                out[j] = (int16_t)sat16(a, sb);
            }
        }
        const unsigned long long ma = __ballot(sa), mb = __ballot(sb);   // wave-convergent
        if (ovf) write_slot_flags_split(ma, mb, eA, eB, n, V, ovf);
    }
#else
    const size_t n8 = (n + 7) / 8;
    const size_t wave0 = tid & ~(size_t)63;
    for (size_t base = wave0; base < n8; base += stride) {
        size_t i = base + (tid & 63);
        bool sat = false;
        if (i < n8) {
            size_t e = 8 * i;
            if (e + 8 <= n) {
                int32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll UNR
                for (int w = 0; w < nw; ++w) {
                    f32x4 u = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w] + e));
                    f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in.p[w] + e) + 1);
                    a[0] += q16(u.x, s, sat); a[1] += q16(u.y, s, sat);
                    a[2] += q16(u.z, s, sat); a[3] += q16(u.w, s, sat);
                    a[4] += q16(v.x, s, sat); a[5] += q16(v.y, s, sat);
                    a[6] += q16(v.z, s, sat); a[7] += q16(v.w, s, sat);
                }
                u32x4 o;
                o.x = (uint32_t)(uint16_t)sat16(a[0], sat) | ((uint32_t)sat16(a[1], sat) << 16);
                o.y = (uint32_t)(uint16_t)sat16(a[2], sat) | ((uint32_t)sat16(a[3], sat) << 16);
                o.z = (uint32_t)(uint16_t)sat16(a[4], sat) | ((uint32_t)sat16(a[5], sat) << 16);
                o.w = (uint32_t)(uint16_t)sat16(a[6], sat) | ((uint32_t)sat16(a[7], sat) << 16);
                stream_store(o, reinterpret_cast<u32x4*>(out + e));
            } else {
                for (size_t j = e; j < n; ++j) {
                    int32_t a = 0;
                    for (int w = 0; w < nw; ++w) a += q16(in.p[w][j], s, sat);
                    out[j] = (int16_t)sat16(a, sat);
                }
            }
        }
        unsigned long long m = __ballot(sat);   // wave-convergent: uniform trip count
        if (ovf) write_slot_flags8(m, i < n8, 8 * i, V, lanes_per_slot, ovf);
    }
#endif
}

__global__ __launch_bounds__(kBlock) void k_quant_reduce_i16_scalar(PtrPack<float> in, int W,
                                                                    int16_t* __restrict__ out,
                                                                    size_t n, float s, int V,
                                                                    uint8_t* __restrict__ ovf) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        bool sat = false;
        int32_t a = 0;
        for (int w = 0; w < W; ++w) a += q16(in.p[w][i], s, sat);
        out[i] = (int16_t)sat16(a, sat);
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
}

// int16 narrow reduce of already-quantised int16 buffers
__global__ __launch_bounds__(kBlock) void k_sum_reduce_i16(PtrPack<int16_t> in, int W,
                                                           int16_t* __restrict__ out, size_t n,
                                                           int V, int lanes_per_slot,
                                                           uint8_t* __restrict__ ovf) {
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    const size_t n8 = (n + 7) / 8;
    const size_t wave0 = tid & ~(size_t)63;
    for (size_t base = wave0; base < n8; base += stride) {
        size_t i = base + (tid & 63);
        bool sat = false;
        if (i < n8) {
            size_t e = 8 * i;
            if (e + 8 <= n) {
                int32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int w = 0; w < W; ++w) {
                    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in.p[w] + e));
                    a[0] += (int16_t)(v.x & 0xFFFF); a[1] += (int16_t)(v.x >> 16);
                    a[2] += (int16_t)(v.y & 0xFFFF); a[3] += (int16_t)(v.y >> 16);
                    a[4] += (int16_t)(v.z & 0xFFFF); a[5] += (int16_t)(v.z >> 16);
                    a[6] += (int16_t)(v.w & 0xFFFF); a[7] += (int16_t)(v.w >> 16);
                }
                u32x4 o;
                o.x = (uint32_t)(uint16_t)sat16(a[0], sat) | ((uint32_t)sat16(a[1], sat) << 16);
                o.y = (uint32_t)(uint16_t)sat16(a[2], sat) | ((uint32_t)sat16(a[3], sat) << 16);
                o.z = (uint32_t)(uint16_t)sat16(a[4], sat) | ((uint32_t)sat16(a[5], sat) << 16);
                o.w = (uint32_t)(uint16_t)sat16(a[6], sat) | ((uint32_t)sat16(a[7], sat) << 16);
                stream_store(o, reinterpret_cast<u32x4*>(out + e));
            } else {
                for (size_t j = e; j < n; ++j) {
                    int32_t a = 0;
                    for (int w = 0; w < W; ++w) a += in.p[w][j];
                    out[j] = (int16_t)sat16(a, sat);
                }
            }
        }
        unsigned long long m = __ballot(sat);   // wave-convergent: uniform trip count
        if (ovf) write_slot_flags8(m, i < n8, 8 * i, V, lanes_per_slot, ovf);
    }
}

__global__ __launch_bounds__(kBlock) void k_sum_reduce_i16_scalar(PtrPack<int16_t> in, int W,
                                                                  int16_t* __restrict__ out,
                                                                  size_t n, int V,
                                                                  uint8_t* __restrict__ ovf) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        bool sat = false;
        int32_t a = 0;
        for (int w = 0; w < W; ++w) a += in.p[w][i];
        out[i] = (int16_t)sat16(a, sat);
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
}

// ===========================================================================
// 4. PS combine (launch.py:42-52), bit-exact fp32 op sequence; built with
//    -ffp-contract=off so no FMA fuses the sub/add/mul.
// ===========================================================================
// W-templated (0 = runtime W) fp32 combine over float4 chunks
template <int W>
__global__ __launch_bounds__(kBlock) void k_ps_combine_f32(const float* __restrict__ local,
                                                           PtrPack<float> paras, int Wd, float ws,
                                                           float* __restrict__ out, size_t n,
                                                           int vec) {
    const int nw = W > 0 ? W : Wd;
    size_t n4 = vec ? n / 4 : 0;
    const f32x4* l4 = reinterpret_cast<const f32x4*>(local);
    f32x4* o4 = reinterpret_cast<f32x4*>(out);
    chunk_loop<(W > 0 && W <= 4) ? INA_COMB_U : 2>(n4, [&]<int UU>(size_t i, size_t st) {
        f32x4 l[UU], acc[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) { l[u] = l4[i + u * st]; acc[u] = f32x4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll kUnrW<W>
        for (int w = 0; w < nw; ++w) {
            f32x4 p[UU];
#pragma unroll
            for (int u = 0; u < UU; ++u)
                p[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(paras.p[w]) + i + u * st);
#pragma unroll
            for (int u = 0; u < UU; ++u) {       // python sum(): 0 + d_0 + d_1 + ...
                acc[u].x = __fadd_rn(acc[u].x, __fsub_rn(p[u].x, l[u].x));
                acc[u].y = __fadd_rn(acc[u].y, __fsub_rn(p[u].y, l[u].y));
                acc[u].z = __fadd_rn(acc[u].z, __fsub_rn(p[u].z, l[u].z));
                acc[u].w = __fadd_rn(acc[u].w, __fsub_rn(p[u].w, l[u].w));
            }
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            f32x4 r;
            r.x = __fadd_rn(l[u].x, __fmul_rn(acc[u].x, ws)); r.y = __fadd_rn(l[u].y, __fmul_rn(acc[u].y, ws));
            r.z = __fadd_rn(l[u].z, __fmul_rn(acc[u].z, ws)); r.w = __fadd_rn(l[u].w, __fmul_rn(acc[u].w, ws));
            o4[i + u * st] = r;
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        float l = local[i];
        float acc = 0.0f;
        for (int w = 0; w < nw; ++w) acc = __fadd_rn(acc, __fsub_rn(paras.p[w][i], l));
        out[i] = __fadd_rn(l, __fmul_rn(acc, ws));
    }
}

__global__ __launch_bounds__(kBlock) void k_ps_apply_i32(const float* __restrict__ local,
                                                         const int32_t* __restrict__ sum,
                                                         float inv, float ws,
                                                         float* __restrict__ out, size_t n, int vec) {
    size_t n4 = vec ? n / 4 : 0;
    chunk_loop<kEwU>(n4, [&]<int UU>(size_t i, size_t st) {
        f32x4 l[UU];
        u32x4 q[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            l[u] = reinterpret_cast<const f32x4*>(local)[i + u * st];
            q[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sum) + i + u * st);
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            f32x4 r;
            r.x = __fadd_rn(l[u].x, __fmul_rn(__fmul_rn((float)(int32_t)q[u].x, inv), ws));
            r.y = __fadd_rn(l[u].y, __fmul_rn(__fmul_rn((float)(int32_t)q[u].y, inv), ws));
            r.z = __fadd_rn(l[u].z, __fmul_rn(__fmul_rn((float)(int32_t)q[u].z, inv), ws));
            r.w = __fadd_rn(l[u].w, __fmul_rn(__fmul_rn((float)(int32_t)q[u].w, inv), ws));
            reinterpret_cast<f32x4*>(out)[i + u * st] = r;
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        float d = __fmul_rn((float)sum[i], inv);
        out[i] = __fadd_rn(local[i], __fmul_rn(d, ws));
    }
}

// INA form: out = local + ws * ((float)sum_w q(paras[w] - local) * 2^-k), one pass
template <int W>
__global__ __launch_bounds__(kBlock) void k_ps_combine_ina(const float* __restrict__ local,
                                                           PtrPack<float> paras, int Wd, float s,
                                                           float inv, float ws,
                                                           float* __restrict__ out, size_t n,
                                                           int vec) {
    const int nw = W > 0 ? W : Wd;
    size_t n4 = vec ? n / 4 : 0;
    chunk_loop<(W > 0 && W <= 4) ? INA_COMBI_U : 2>(n4, [&]<int UU>(size_t i, size_t st) {
        f32x4 l[UU];
        u32x4 acc[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            l[u] = reinterpret_cast<const f32x4*>(local)[i + u * st];
            acc[u] = u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll kUnrW<W>
        for (int w = 0; w < nw; ++w) {
            f32x4 p[UU];
#pragma unroll
            for (int u = 0; u < UU; ++u)
                p[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(paras.p[w]) + i + u * st);
#pragma unroll
            for (int u = 0; u < UU; ++u) {
                acc[u].x += (uint32_t)q32(__fsub_rn(p[u].x, l[u].x), s);
                acc[u].y += (uint32_t)q32(__fsub_rn(p[u].y, l[u].y), s);
                acc[u].z += (uint32_t)q32(__fsub_rn(p[u].z, l[u].z), s);
                acc[u].w += (uint32_t)q32(__fsub_rn(p[u].w, l[u].w), s);
            }
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            f32x4 r;
            r.x = __fadd_rn(l[u].x, __fmul_rn(__fmul_rn((float)(int32_t)acc[u].x, inv), ws));
            r.y = __fadd_rn(l[u].y, __fmul_rn(__fmul_rn((float)(int32_t)acc[u].y, inv), ws));
            r.z = __fadd_rn(l[u].z, __fmul_rn(__fmul_rn((float)(int32_t)acc[u].z, inv), ws));
            r.w = __fadd_rn(l[u].w, __fmul_rn(__fmul_rn((float)(int32_t)acc[u].w, inv), ws));
            reinterpret_cast<f32x4*>(out)[i + u * st] = r;
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        float l = local[i];
        uint32_t acc = 0;
        for (int w = 0; w < nw; ++w) acc += (uint32_t)q32(__fsub_rn(paras.p[w][i], l), s);
        float y = __fmul_rn((float)(int32_t)acc, inv);
        out[i] = __fadd_rn(l, __fmul_rn(y, ws));
    }
}

// ===========================================================================
// 5. NGA-V packets (15-byte BE header, V BE words, zero tail)
// ===========================================================================
struct NgaHdr {
    uint32_t bitmap, seq0, num_slots;
    uint32_t flags_count_sw;   // count | flags << 8 | switch_id << 16
    int V;
};

// Value sources of the pack kernels: stored int32 words, or fp32 gradients (optionally
// minus a base vector: the worker's delta p - p_global) quantised on the fly -- the
// fused worker-side quantise + packetise (DataManager.py:37 then 111-165, one pass).
struct SrcI32 {
    const int32_t* __restrict__ v;
    SrcI32 shifted(size_t off) const { return SrcI32{v + off}; }
    __device__ __forceinline__ uint32_t one(size_t e) const { return (uint32_t)v[e]; }
    __device__ __forceinline__ u32x4 four(size_t e) const {
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(v + e));
    }
};
struct SrcQ32 {
    const float* __restrict__ x;
    const float* __restrict__ base;   // may be null
    float s;
    SrcQ32 shifted(size_t off) const { return SrcQ32{x + off, base ? base + off : nullptr, s}; }
    __device__ __forceinline__ uint32_t one(size_t e) const {
        return (uint32_t)q32(base ? __fsub_rn(x[e], base[e]) : x[e], s);
    }
    __device__ __forceinline__ u32x4 four(size_t e) const {
        f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + e));
        if (base) {
            // the base (p_global) is shared: every worker's pack and the PS update read the
            // same vector, so it is loaded with the default policy and stays in the
            // Infinity Cache between them (nt: the steady-state 8-worker step 0.690 ->
            // 0.661 ms; one cold pack unchanged; profiles/r03/lab/qpack_base_lab.log)
            f32x4 b = *reinterpret_cast<const f32x4*>(base + e);
            a.x = __fsub_rn(a.x, b.x); a.y = __fsub_rn(a.y, b.y);
            a.z = __fsub_rn(a.z, b.z); a.w = __fsub_rn(a.w, b.w);
        }
        return u32x4{(uint32_t)q32(a.x, s), (uint32_t)q32(a.y, s), (uint32_t)q32(a.z, s),
                     (uint32_t)q32(a.w, s)};
    }
};

template <typename Src>
__device__ __forceinline__ uint32_t nga_val(const Src& src, size_t n, size_t p, int V, long j) {
    // payload word j of packet p (0 outside [0, V) and past n: zero tail pad)
    if (j < 0 || j >= V) return 0u;
    size_t e = p * (size_t)V + (size_t)j;
    return e < n ? src.one(e) : 0u;
}

// flat pack (stride % 16 == 0, V % 4 == 0, 16-byte aligned source and packets): the
// packet array is written as one contiguous stream of 16-byte chunks, thread per chunk,
// U chunks in flight per thread.  Chunk c (1 <= c <= V/4) of a packet holds wire dwords
// 4c..4c+3 = bytes 2,1,0 of value 4c-4+t and byte 3 of value 4c-3+t (one v_perm each);
// the chunk loads its own 4 values (one 16-byte load, quantised once when the source is
// fp32) and takes value 4c -- the next chunk's first -- from the next lane (DPP
// wave_shl:1; lane 63 loads it).  Chunk 0 is the header plus value 0's top byte.
constexpr uint32_t kSelWire = 0x07000102u;   // perm(next, v): {v.b2, v.b1, v.b0, next.b3}
// 16-byte chunks in flight per thread in the flat packet kernels: one (with an 8192-
// workgroup grid striding over the rest, now 16,384: g_stream_blocks) beat 2, 4 and 8 -- fused worker pack 57.7 -> 54.2
// us, pack 37.5 -> 36.5, unpack 40.4 -> 39.1 (tools/lab/apply_lab.py, lab/pack_u_lab.log)
#ifndef INA_PACK_U
#define INA_PACK_U 1
#endif
#ifndef INA_UNPACK_U
#define INA_UNPACK_U 1
#endif
#ifndef INA_PACK_DESC_SPLIT
#define INA_PACK_DESC_SPLIT 1
#endif
#ifndef INA_UNPACK_HDR_SPLIT
#define INA_UNPACK_HDR_SPLIT 1
#endif

template <typename Src, int U>
__global__ __launch_bounds__(kBlock) void k_pack_nga_flat(Src src, size_t n, NgaHdr h,
                                                          const uint8_t* __restrict__ ovf,
                                                          uint8_t* __restrict__ pkts, uint32_t C,
                                                          uint32_t L, uint32_t nch,
                                                          u32x2* __restrict__ desc) {
    const uint32_t gs = gridDim.x * kBlock;
    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = (blockIdx.x * kBlock + threadIdx.x) & ~63u;
    const size_t V = (size_t)h.V;
    u32x4* ch = reinterpret_cast<u32x4*>(pkts);
#if INA_PACK_DESC_SPLIT
    // descriptors (header bytes 4..11) depend on the packet number alone: a thread per
    // packet writes them, consecutive lanes consecutive entries (coalesced), instead of one
    // 8-byte store from each packet's chunk-0 lane (the unpack header fields' pattern)
    if (desc) {
        const uint32_t np = nch / C;
        const uint32_t count = h.flags_count_sw & 0xFFu, sw = (h.flags_count_sw >> 16) & 0xFFu;
        for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
            const uint32_t seq = h.seq0 + p;
            const uint32_t bi = bswap(seq % h.num_slots), bf = bswap(seq);
            uint32_t flags = (h.flags_count_sw >> 8) & 0xFFu;
            if (ovf && ovf[p]) flags |= INA_FLAG_OVERFLOW;
            desc[p] = u32x2{count | (flags << 8) | (bi << 16), (bi >> 16) | (sw << 16) | (bf << 24)};
        }
    }
#endif
    for (uint32_t base = wave0; base < nch; base += U * gs) {
        u32x4 v[U];
        uint32_t nx0[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = base + u * gs + (uint32_t)lane;
            const uint32_t p = t / C, c = t - p * C;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (t < nch && c >= 1 && c <= L) {
                const size_t e0 = (size_t)p * V + 4 * (size_t)(c - 1);
                if (e0 + 4 <= n) {
                    v[u] = src.four(e0);
                } else {                                   // last packet of the bucket: zero tail
                    v[u].x = e0 < n ? src.one(e0) : 0u;
                    v[u].y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
                    v[u].z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
                }
            }
            nx0[u] = 0u;
            if (lane == 63 && t < nch && c < L) {
                const size_t e = (size_t)p * V + 4 * (size_t)c;
                nx0[u] = e < n ? src.one(e) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = base + u * gs + (uint32_t)lane;
            const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)nx0[u], (int)v[u].x, 0x130,
                                                                      0xF, 0xF, false);
            if (t >= nch) continue;
            const uint32_t p = t / C, c = t - p * C;
            u32x4 o;
            if (c == 0) {
                const uint32_t seq = h.seq0 + p;
                const uint32_t idx = seq % h.num_slots;
                uint32_t flags = (h.flags_count_sw >> 8) & 0xFFu;
                if (ovf && ovf[p]) flags |= INA_FLAG_OVERFLOW;
                const uint32_t count = h.flags_count_sw & 0xFFu, sw = (h.flags_count_sw >> 16) & 0xFFu;
                const uint32_t bi = bswap(idx), bf = bswap(seq);
                o.x = bswap(h.bitmap);
                o.y = count | (flags << 8) | (bi << 16);
                o.z = (bi >> 16) | (sw << 16) | (bf << 24);
                o.w = (bf >> 8) | (nx & 0xFF000000u);        // value 0's top byte at byte 15
                if (desc && !INA_PACK_DESC_SPLIT) desc[p] = u32x2{o.y, o.z};   // header bytes 4..11 (ina.h)
            } else if (c <= L) {
                o.x = __builtin_amdgcn_perm(v[u].y, v[u].x, kSelWire);
                o.y = __builtin_amdgcn_perm(v[u].z, v[u].y, kSelWire);
                o.z = __builtin_amdgcn_perm(v[u].w, v[u].z, kSelWire);
                o.w = __builtin_amdgcn_perm(nx, v[u].w, kSelWire);
            } else {
                o = u32x4{0u, 0u, 0u, 0u};                   // padding chunks
            }
            packet_store(o, ch + t);
        }
    }
}

// Several workers' fused quantise + pack in ONE launch (a GPU hosting a group of the
// job's workers; the packet path's W simulated workers): the flat chunk stream of
// k_pack_nga_flat<SrcQ32>, with every thread producing the same chunk of up to kQpGroup
// workers' packets.  The shared base chunk (p_global) is loaded once for all of them and
// the workers' loads are all in flight together; each worker's output stream stays
// coalesced.  Bytes = the per-worker kernel's, worker by worker.
constexpr int kQpGroup = 8;
// stores: nt like the other packet kernels (write-through and default-policy stores were
// slower in both layouts, profiles/r03/lab/qpack_multi_lab.log)
__device__ __forceinline__ void qpm_store(u32x4 v, u32x4* p) { packet_store(v, p); }
struct QPackGroup {
    const float* x[kQpGroup];
    uint8_t* pkts[kQpGroup];
    u32x2* desc[kQpGroup];          // all null or all set
    uint32_t bitmap[kQpGroup], seq0[kQpGroup], fcs[kQpGroup];   // fcs: count | flags<<8 | sw<<16
};

template <int G>
__global__ __launch_bounds__(kBlock) void k_qpack_nga_multi(QPackGroup a, const float* __restrict__ base,
                                                            size_t n, float s, uint32_t num_slots,
                                                            uint32_t V, uint32_t C, uint32_t L,
                                                            uint32_t nch) {
    const uint32_t gs = gridDim.x * kBlock;
    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = (blockIdx.x * kBlock + threadIdx.x) & ~63u;
    if (a.desc[0]) {                                   // descriptors: thread per packet, coalesced
        const uint32_t np = nch / C;
        for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t seq = a.seq0[g] + p;
                const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
                const uint32_t f = a.fcs[g];
                a.desc[g][p] = u32x2{(f & 0xFFFFu) | (bi << 16),
                                     (bi >> 16) | (((f >> 16) & 0xFFu) << 16) | (bf << 24)};
            }
        }
    }
    for (uint32_t t0 = wave0; t0 < nch; t0 += gs) {
        const uint32_t t = t0 + (uint32_t)lane;
        const uint32_t p = t / C, c = t - p * C;
        const bool body = t < nch && c >= 1 && c <= L;
        const size_t e0 = (size_t)p * V + 4 * (size_t)(c - 1);
        const bool full = body && e0 + 4 <= n;
        u32x4 v[G];
        uint32_t nx0[G];
        f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
        if (full && base) b = *reinterpret_cast<const f32x4*>(base + e0);   // default policy: shared
#pragma unroll
        for (int g = 0; g < G; ++g) {
            v[g] = u32x4{0u, 0u, 0u, 0u};
            if (full) {
                f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.x[g] + e0));
                if (base) {
                    x.x = __fsub_rn(x.x, b.x); x.y = __fsub_rn(x.y, b.y);
                    x.z = __fsub_rn(x.z, b.z); x.w = __fsub_rn(x.w, b.w);
                }
                v[g] = u32x4{(uint32_t)q32(x.x, s), (uint32_t)q32(x.y, s), (uint32_t)q32(x.z, s),
                             (uint32_t)q32(x.w, s)};
            } else if (body) {                         // last packet of the bucket: zero tail
                const SrcQ32 src{a.x[g], base, s};
                v[g].x = e0 < n ? src.one(e0) : 0u;
                v[g].y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
                v[g].z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
            }
            nx0[g] = 0u;
            if (lane == 63 && t < nch && c < L) {      // the next chunk's first value
                const size_t e = (size_t)p * V + 4 * (size_t)c;
                nx0[g] = e < n ? SrcQ32{a.x[g], base, s}.one(e) : 0u;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)nx0[g], (int)v[g].x, 0x130,
                                                                      0xF, 0xF, false);
            if (t >= nch) continue;
            u32x4 o;
            if (c == 0) {
                const uint32_t seq = a.seq0[g] + p;
                const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
                const uint32_t f = a.fcs[g];
                o.x = bswap(a.bitmap[g]);
                o.y = (f & 0xFFFFu) | (bi << 16);
                o.z = (bi >> 16) | (((f >> 16) & 0xFFu) << 16) | (bf << 24);
                o.w = (bf >> 8) | (nx & 0xFF000000u);
            } else if (c <= L) {
                o.x = __builtin_amdgcn_perm(v[g].y, v[g].x, kSelWire);
                o.y = __builtin_amdgcn_perm(v[g].z, v[g].y, kSelWire);
                o.z = __builtin_amdgcn_perm(v[g].w, v[g].z, kSelWire);
                o.w = __builtin_amdgcn_perm(nx, v[g].w, kSelWire);
            } else {
                o = u32x4{0u, 0u, 0u, 0u};
            }
            qpm_store(o, reinterpret_cast<u32x4*>(a.pkts[g]) + t);
        }
    }
}

// Descriptors from the header parameters alone (no packet read): what the pack kernels
// write beside each packet, for up to kQpGroup workers of npk packets each -- so a switch's
// slot sort can start before the payload exists.
struct DescGroup {
    u32x2* desc[kQpGroup];
    uint32_t seq0[kQpGroup], fcs[kQpGroup];
};
__global__ __launch_bounds__(kBlock) void k_nga_make_desc(DescGroup a, int G, uint32_t num_slots,
                                                          uint32_t np) {
    const uint32_t gs = gridDim.x * kBlock;
    for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
        for (int g = 0; g < G; ++g) {
            const uint32_t seq = a.seq0[g] + p;
            const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
            const uint32_t f = a.fcs[g];
            a.desc[g][p] = u32x2{(f & 0xFFFFu) | (bi << 16),
                                 (bi >> 16) | (((f >> 16) & 0xFFu) << 16) | (bf << 24)};
        }
    }
}

// NGA-256 (64 value chunks per packet): a wave per packet.  Lane l holds values 4l..4l+3
// (one aligned 1 KiB load per worker) and writes value chunk l + 1; the next chunk's first
// value comes from lane l + 1 (DPP wave_shl:1), lane 63's is value 256 = the zero past the
// packet, so no lane loads anything twice or alone; lane 0 also writes the header chunk.
// (one launch, 8 workers, config 3: 343 -> 329 us, the steady packet-path step 587 -> 563 us;
// write-through or default-policy stores are slower in both layouts, qpack_multi_lab.log)
#ifndef INA_QPM_PPW
#define INA_QPM_PPW 1
#endif
#ifndef INA_QPM_PPW_BLOCKS
#define INA_QPM_PPW_BLOCKS (1 << 20)      // a covering grid (a wave per packet)
#endif
// (amdgpu_waves_per_eu 6 / 7 -- 74 / 71 VGPRs against 87 -- gained nothing,
// profiles/r03/lab/qpack_occupancy_lab.log)
template <int G>
__global__ __launch_bounds__(kBlock) void k_qpack_nga_multi_v256(QPackGroup a, const float* __restrict__ base,
                                                                 size_t n, float s, uint32_t num_slots,
                                                                 uint32_t stride, uint32_t np) {
    const uint32_t gs = gridDim.x * kBlock;
    const int lane = threadIdx.x & 63;
    if (a.desc[0]) {
        for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t seq = a.seq0[g] + p;
                const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
                const uint32_t f = a.fcs[g];
                a.desc[g][p] = u32x2{(f & 0xFFFFu) | (bi << 16),
                                     (bi >> 16) | (((f >> 16) & 0xFFu) << 16) | (bf << 24)};
            }
        }
    }
    const uint32_t nwaves = gs >> 6, pad = stride / 16 - 65;
    for (uint32_t p = (blockIdx.x * kBlock + threadIdx.x) >> 6; p < np; p += nwaves) {
        const size_t e0 = (size_t)p * 256 + 4 * (size_t)lane;
        const bool full = e0 + 4 <= n;
        u32x4 v[G];
        f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
        if (full && base) b = *reinterpret_cast<const f32x4*>(base + e0);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            v[g] = u32x4{0u, 0u, 0u, 0u};
            if (full) {
                f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.x[g] + e0));
                if (base) {
                    x.x = __fsub_rn(x.x, b.x); x.y = __fsub_rn(x.y, b.y);
                    x.z = __fsub_rn(x.z, b.z); x.w = __fsub_rn(x.w, b.w);
                }
                v[g] = u32x4{(uint32_t)q32(x.x, s), (uint32_t)q32(x.y, s), (uint32_t)q32(x.z, s),
                             (uint32_t)q32(x.w, s)};
            } else {
                const SrcQ32 src{a.x[g], base, s};
                v[g].x = e0 < n ? src.one(e0) : 0u;
                v[g].y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
                v[g].z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[g].x, 0x130, 0xF, 0xF, false);
            u32x4* row = reinterpret_cast<u32x4*>(a.pkts[g] + (size_t)p * stride);
            u32x4 o;
            o.x = __builtin_amdgcn_perm(v[g].y, v[g].x, kSelWire);
            o.y = __builtin_amdgcn_perm(v[g].z, v[g].y, kSelWire);
            o.z = __builtin_amdgcn_perm(v[g].w, v[g].z, kSelWire);
            o.w = __builtin_amdgcn_perm(nx, v[g].w, kSelWire);
            qpm_store(o, row + 1 + lane);
            if (lane == 0) {
                const uint32_t seq = a.seq0[g] + p;
                const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
                const uint32_t f = a.fcs[g];
                u32x4 h;
                h.x = bswap(a.bitmap[g]);
                h.y = (f & 0xFFFFu) | (bi << 16);
                h.z = (bi >> 16) | (((f >> 16) & 0xFFu) << 16) | (bf << 24);
                h.w = (bf >> 8) | (v[g].x & 0xFF000000u);
                qpm_store(h, row);
            }
            if ((uint32_t)lane < pad) qpm_store(u32x4{0u, 0u, 0u, 0u}, row + 65 + lane);
        }
    }
}

// ---- split NGA rows: header rows + payload rows (include/ina.h "split layout") ------------
// The wire datagram is header (15 B) || payload (4V B).  Stored split -- a 16-byte header row
// (the 15 wire bytes + a zero) and a 4V-byte payload row of V big-endian words -- every
// payload row starts 16-byte aligned and covers exactly 4V/128 cache lines, so the packs
// store whole aligned chunks (the packed NGA-256 row's 1,040 bytes touch 9 lines and its
// body stores straddle 16-byte boundaries), and the payload stream of a bucket IS its
// values in order, byte-swapped, zero-padded to whole packets: packing is an elementwise
// pass.  sendmmsg / recvmmsg carry it as two iovecs per datagram (same bytes on the wire).
__device__ __forceinline__ u32x4 nga_hdr_row(uint32_t bitmap, uint32_t fcs, uint32_t seq, uint32_t num_slots) {
    const uint32_t bi = bswap(seq % num_slots), bf = bswap(seq);
    return u32x4{bswap(bitmap), (fcs & 0xFFFFu) | (bi << 16),
                 (bi >> 16) | (((fcs >> 16) & 0xFFu) << 16) | (bf << 24), bf >> 8};
}
__device__ __forceinline__ u32x4 bswap4(u32x4 v) {
    return u32x4{bswap(v.x), bswap(v.y), bswap(v.z), bswap(v.w)};
}

// one worker: payload chunk t = values 4t..4t+3 byte-swapped (zero past n); header rows and
// descriptors a thread per packet
template <typename Src>
__global__ __launch_bounds__(kBlock) void k_pack_nga_split(Src src, size_t n, NgaHdr h,
                                                           const uint8_t* __restrict__ ovf,
                                                           u32x4* __restrict__ hdr, u32x4* __restrict__ pay,
                                                           u32x2* __restrict__ desc, size_t nch, size_t np,
                                                           int vec) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    for (size_t t = tid; t < nch; t += gs) {
        const size_t e0 = 4 * t;
        u32x4 v;
        if (vec && e0 + 4 <= n) {
            v = src.four(e0);
        } else {
            v.x = e0 < n ? src.one(e0) : 0u;
            v.y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
            v.z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
            v.w = e0 + 3 < n ? src.one(e0 + 3) : 0u;
        }
        packet_store(bswap4(v), pay + t);
    }
    for (size_t p = tid; p < np; p += gs) {
        uint32_t fcs = h.flags_count_sw;
        if (ovf && ovf[p]) fcs |= (uint32_t)INA_FLAG_OVERFLOW << 8;
        const u32x4 r = nga_hdr_row(h.bitmap, fcs, h.seq0 + (uint32_t)p, h.num_slots);
        packet_store(r, hdr + p);
        if (desc) desc[p] = u32x2{r.y, r.z};
    }
}

// up to kQpGroup workers' fused quantise(x_w - base) + split pack in one launch: the base
// chunk loaded once for every worker, each worker's payload stream coalesced
struct QPackSplit {
    const float* x[kQpGroup];
    u32x4* hdr[kQpGroup];
    u32x4* pay[kQpGroup];
    u32x2* desc[kQpGroup];          // all null or all set
    uint32_t bitmap[kQpGroup], seq0[kQpGroup], fcs[kQpGroup];
};
template <int G>
__global__ __launch_bounds__(kBlock) void k_qpack_nga_multi_split(QPackSplit a, const float* __restrict__ base,
                                                                  size_t n, float s, uint32_t num_slots,
                                                                  size_t nch, size_t np) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    for (size_t t = tid; t < nch; t += gs) {
        const size_t e0 = 4 * t;
        if (e0 + 4 <= n) {
            f32x4 b = f32x4{0.f, 0.f, 0.f, 0.f};
            if (base) b = *reinterpret_cast<const f32x4*>(base + e0);   // default policy: shared
            f32x4 x[G];
#pragma unroll
            for (int g = 0; g < G; ++g) x[g] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.x[g] + e0));
#pragma unroll
            for (int g = 0; g < G; ++g) {
                f32x4 y = x[g];
                if (base) {
                    y.x = __fsub_rn(y.x, b.x); y.y = __fsub_rn(y.y, b.y);
                    y.z = __fsub_rn(y.z, b.z); y.w = __fsub_rn(y.w, b.w);
                }
                const u32x4 q{(uint32_t)q32(y.x, s), (uint32_t)q32(y.y, s), (uint32_t)q32(y.z, s),
                              (uint32_t)q32(y.w, s)};
                packet_store(bswap4(q), a.pay[g] + t);
            }
        } else {                                       // the bucket's last chunk: zero tail
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const SrcQ32 src{a.x[g], base, s};
                u32x4 v;
                v.x = e0 < n ? src.one(e0) : 0u;
                v.y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
                v.z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
                v.w = e0 + 3 < n ? src.one(e0 + 3) : 0u;
                packet_store(bswap4(v), a.pay[g] + t);
            }
        }
    }
    for (size_t p = tid; p < np; p += gs) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const u32x4 r = nga_hdr_row(a.bitmap[g], a.fcs[g], a.seq0[g] + (uint32_t)p, num_slots);
            packet_store(r, a.hdr[g] + p);
            if (a.desc[g]) a.desc[g][p] = u32x2{r.y, r.z};
        }
    }
}

// split rows -> int32 values (payload byte-swapped back; every payload word, npk * V)
__global__ __launch_bounds__(kBlock) void k_unpack_nga_split_vals(const u32x4* __restrict__ pay, size_t nch,
                                                                  u32x4* __restrict__ vals) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < nch; t += gs)
        stream_store(bswap4(__builtin_nontemporal_load(pay + t)), vals + t);
}

// One worker's NGA-256 packets, a wave per packet (the layout of k_qpack_nga_multi_v256):
// fp32 quantised on the fly (int32 words and the per-packet overflow flag are supported; the
// int32 pack is faster on the flat stream, see pack_nga_launch).
#ifndef INA_PACK_PPW
#define INA_PACK_PPW 1
#endif
template <typename Src>
__global__ __launch_bounds__(kBlock) void k_pack_nga_v256(Src src, size_t n, NgaHdr h,
                                                          const uint8_t* __restrict__ ovf,
                                                          uint8_t* __restrict__ pkts, uint32_t stride,
                                                          uint32_t np, u32x2* __restrict__ desc) {
    const uint32_t gs = gridDim.x * kBlock;
    const int lane = threadIdx.x & 63;
    const uint32_t count = h.flags_count_sw & 0xFFu, sw = (h.flags_count_sw >> 16) & 0xFFu;
    if (desc) {
        for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
            const uint32_t seq = h.seq0 + p;
            const uint32_t bi = bswap(seq % h.num_slots), bf = bswap(seq);
            uint32_t flags = (h.flags_count_sw >> 8) & 0xFFu;
            if (ovf && ovf[p]) flags |= INA_FLAG_OVERFLOW;
            desc[p] = u32x2{count | (flags << 8) | (bi << 16), (bi >> 16) | (sw << 16) | (bf << 24)};
        }
    }
    const uint32_t nwaves = gs >> 6, pad = stride / 16 - 65;
    for (uint32_t p = (blockIdx.x * kBlock + threadIdx.x) >> 6; p < np; p += nwaves) {
        const size_t e0 = (size_t)p * 256 + 4 * (size_t)lane;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        if (e0 + 4 <= n) {
            v = src.four(e0);
        } else {
            v.x = e0 < n ? src.one(e0) : 0u;
            v.y = e0 + 1 < n ? src.one(e0 + 1) : 0u;
            v.z = e0 + 2 < n ? src.one(e0 + 2) : 0u;
        }
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x130, 0xF, 0xF, false);
        u32x4* row = reinterpret_cast<u32x4*>(pkts + (size_t)p * stride);
        u32x4 o;
        o.x = __builtin_amdgcn_perm(v.y, v.x, kSelWire);
        o.y = __builtin_amdgcn_perm(v.z, v.y, kSelWire);
        o.z = __builtin_amdgcn_perm(v.w, v.z, kSelWire);
        o.w = __builtin_amdgcn_perm(nx, v.w, kSelWire);
        packet_store(o, row + 1 + lane);
        if (lane == 0) {
            const uint32_t seq = h.seq0 + p;
            const uint32_t bi = bswap(seq % h.num_slots), bf = bswap(seq);
            uint32_t flags = (h.flags_count_sw >> 8) & 0xFFu;
            if (ovf && ovf[p]) flags |= INA_FLAG_OVERFLOW;
            u32x4 hd;
            hd.x = bswap(h.bitmap);
            hd.y = count | (flags << 8) | (bi << 16);
            hd.z = (bi >> 16) | (sw << 16) | (bf << 24);
            hd.w = (bf >> 8) | (v.x & 0xFF000000u);
            packet_store(hd, row);
        }
        if ((uint32_t)lane < pad) packet_store(u32x4{0u, 0u, 0u, 0u}, row + 65 + lane);
    }
}

// generic path: any stride / alignment, thread per output byte
template <typename Src>
__global__ __launch_bounds__(kBlock) void k_pack_nga_bytes(Src src, size_t n,
                                                           NgaHdr h, const uint8_t* __restrict__ ovf,
                                                           uint8_t* __restrict__ pkts, size_t pstride,
                                                           size_t nbytes) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const int V = h.V;
    for (size_t g = (size_t)blockIdx.x * kBlock + threadIdx.x; g < nbytes; g += gs) {
        size_t p = g / pstride;
        size_t b = g - p * pstride;
        uint32_t seq = h.seq0 + (uint32_t)p;
        uint8_t out = 0;
        if (b < 4) out = (uint8_t)(h.bitmap >> (24 - 8 * b));
        else if (b == 4) out = (uint8_t)(h.flags_count_sw & 0xFF);
        else if (b == 5) out = (uint8_t)(((h.flags_count_sw >> 8) & 0xFF) | ((ovf && ovf[p]) ? INA_FLAG_OVERFLOW : 0));
        else if (b < 10) out = (uint8_t)((seq % h.num_slots) >> (24 - 8 * (b - 6)));
        else if (b == 10) out = (uint8_t)((h.flags_count_sw >> 16) & 0xFF);
        else if (b < 15) out = (uint8_t)(seq >> (24 - 8 * (b - 11)));
        else if (b < 15 + 4 * (size_t)V) {
            size_t q = b - 15;
            out = (uint8_t)(nga_val(src, n, p, V, (long)(q / 4)) >> (24 - 8 * (q % 4)));
        }
        pkts[g] = out;
    }
}

// packet descriptors (include/ina.h): header bytes 4..11 of each packet, gathered; one
// 8-byte result per lane, two dword loads when rows are 4-byte aligned
__global__ __launch_bounds__(kBlock) void k_nga_desc(const uint8_t* __restrict__ pkts, size_t npk,
                                                     size_t pstride, uint64_t* __restrict__ desc) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const bool al4 = (pstride & 3) == 0 && ((uintptr_t)pkts & 3u) == 0;
    for (size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x; p < npk; p += gs) {
        const uint8_t* pk = pkts + p * pstride;
        uint64_t d;
        if (al4) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(pk);
            d = (uint64_t)w[1] | ((uint64_t)w[2] << 32);
        } else {
            d = 0;
            for (int b = 0; b < 8; ++b) d |= (uint64_t)pk[4 + b] << (8 * b);
        }
        desc[p] = d;
    }
}

struct NgaFieldsDev {
    uint32_t* bitmap; uint8_t* count; uint8_t* flags; uint32_t* index; uint8_t* switch_id; uint32_t* frag_id;
};

__device__ __forceinline__ void nga_store_header(const NgaFieldsDev& f, size_t p, uint32_t w0,
                                                 uint32_t w1, uint32_t w2, uint32_t w3) {
    if (f.bitmap) f.bitmap[p] = bswap(w0);
    if (f.count) f.count[p] = (uint8_t)(w1 & 0xFF);
    if (f.flags) f.flags[p] = (uint8_t)((w1 >> 8) & 0xFF);
    if (f.index) f.index[p] = bswap((w1 >> 16) | (w2 << 16));
    if (f.switch_id) f.switch_id[p] = (uint8_t)((w2 >> 16) & 0xFF);
    if (f.frag_id) f.frag_id[p] = bswap((w2 >> 24) | (w3 << 8));
}

// flat unpack: the packet buffer is read as one contiguous array of 16-byte chunks
// (C = stride/16 per packet), thread per chunk, U chunks in flight per thread.  Chunk c
// >= 1 of a packet holds dwords 4c..4c+3 and yields values 4c-4..4c-1 (value j = byte
// 3 of dword 3+j, then bytes 0..2 of dword 4+j: one v_perm each), so the only
// cross-lane input is the previous chunk's dword 3 (DPP wave_shr:1; lane 0 of a wave
// loads it).  Chunk 0 is the header (SoA fields); chunks past V/4 are padding.  Reads
// and writes are both fully contiguous streams.
constexpr uint32_t kSelBE = 0x03040506u;   // perm(hi, lo): {lo.b3, hi.b0, hi.b1, hi.b2} as a BE word

template <int U>
__global__ __launch_bounds__(kBlock) void k_unpack_nga_flat(const uint8_t* __restrict__ pkts,
                                                            uint32_t C, uint32_t L, uint32_t nch,
                                                            NgaFieldsDev f, int hdr,
                                                            int32_t* __restrict__ vals, uint32_t V) {
    const uint32_t gs = gridDim.x * kBlock;
    const int lane = threadIdx.x & 63;
    const uint32_t wave0 = (blockIdx.x * kBlock + threadIdx.x) & ~63u;
    const u32x4* ch = reinterpret_cast<const u32x4*>(pkts);
#if INA_UNPACK_HDR_SPLIT
    // header fields by a thread per packet: consecutive lanes store consecutive SoA
    // entries.  The chunk-0 lane's six narrow stores (one packet per wave, every field
    // line written from many waves) cost 13 % (profiles/r01/lab/unpack_out_lab.log);
    // this pass: 42.6 -> 39.3 us, a separate header kernel 42.0 (profiles/r02/lab/unpack_hdr_lab.log)
    if (hdr) {
        const uint32_t np = nch / C;
        for (uint32_t p = blockIdx.x * kBlock + threadIdx.x; p < np; p += gs) {
            const u32x4 hv = ch[(size_t)p * C];
            nga_store_header(f, p, hv.x, hv.y, hv.z, hv.w);
        }
    }
#endif
    for (uint32_t base = wave0; base < nch; base += U * gs) {
        u32x4 a[U];
        uint32_t pw0[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = base + u * gs + (uint32_t)lane;
            a[u] = t < nch ? __builtin_nontemporal_load(ch + t) : u32x4{0u, 0u, 0u, 0u};
            pw0[u] = 0u;
            if (lane == 0 && t > 0 && t < nch) pw0[u] = reinterpret_cast<const uint32_t*>(ch + t)[-1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = base + u * gs + (uint32_t)lane;
            const uint32_t pw = (uint32_t)__builtin_amdgcn_update_dpp((int)pw0[u], (int)a[u].w, 0x138,
                                                                      0xF, 0xF, false);
            if (t >= nch) continue;
            const uint32_t p = t / C, c = t - p * C;
            if (c == 0) {
                if (hdr && !INA_UNPACK_HDR_SPLIT) nga_store_header(f, p, a[u].x, a[u].y, a[u].z, a[u].w);
            } else if (c <= L && vals) {
                u32x4 o;
                o.x = __builtin_amdgcn_perm(a[u].x, pw, kSelBE);
                o.y = __builtin_amdgcn_perm(a[u].y, a[u].x, kSelBE);
                o.z = __builtin_amdgcn_perm(a[u].z, a[u].y, kSelBE);
                o.w = __builtin_amdgcn_perm(a[u].w, a[u].z, kSelBE);
                // the values are a bulk output: written through, 35.3 -> 34.1 us (nt) on two
                // boxes (tools/lab/unpack_store_lab.py, profiles/r03/lab/unpack_store_lab.log)
                stream_store(o, reinterpret_cast<u32x4*>(vals + (size_t)p * V) + (c - 1));
            }
        }
    }
}

// PS side, fused: for every packet the switch completed (actions[p] == FWD_AGG) decode
// its V summed words, place them by slot = frag_id - seq0 (the sequence numbering of
// DataManager.py:116-130), dequantise and apply the update
//     out[slot*V + j] = local[..] + ws * ((float)sum * 2^-k)
// (aggregate()'s update with the switch's integer sum, launch.py:46-50), and write the
// slot's PS ack header (is_ack=1, fragcheck.p4:26-31) into ack row `slot`.
// A wave owns windows of kApWin packets: one coalesced read of their action bytes, a
// ballot of the completed ones (1 in W of a worker stream, all of them in a stream from
// a hardware switch), then kApB completed packets at a time with all their loads in
// flight: header and chunk loads, then the slots' local rows.  Lane l holds chunk l+1 of a packet and
// decodes values 4l..4l+3 with one v_perm each (the previous chunk's last dword by DPP
// wave_shr:1; header dword 3 for lane 0), the header comes in with a wave-uniform load.
// batch and window measured with tools/lab/apply_lab.py (8 x NGA-256 switch output,
// 1 in 8 packets completed): batch 4 with the local rows prefetched 56.7 us; batch 8
// without prefetch 66.8, with prefetch 81.9 (VGPRs); 16-packet windows spread the
// completed packets of a dense stream over more waves than 64-packet ones
#ifndef INA_APPLY_BATCH
#define INA_APPLY_BATCH 4
#endif
#ifndef INA_APPLY_WIN
#define INA_APPLY_WIN 16
#endif
#ifndef INA_APPLY_MW
#define INA_APPLY_MW 1
#endif
static_assert(64 % INA_APPLY_WIN == 0, "windows tile the wave's 64 lanes");
constexpr int kApB = INA_APPLY_BATCH;
constexpr int kApWin = INA_APPLY_WIN;   // packets per window (<= 64)

__global__ __launch_bounds__(kBlock) void k_apply_completed_nga(
        const uint8_t* __restrict__ pkts, uint32_t npk, uint32_t pstride,
        const uint8_t* __restrict__ actions, uint32_t seq0, uint32_t nslots,
        const float* __restrict__ local, float inv, float ws, float* __restrict__ out, size_t n,
        uint8_t* __restrict__ acks, size_t ack_stride, int V) {
    const int lane = threadIdx.x & 63;
    const int L = V >> 2;
    const bool vl = lane < L;
    const int chn = 1 + (vl ? lane : 0);
    const uint32_t wave = blockIdx.x * (kBlock / 64) + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t nwaves = (gridDim.x * kBlock) >> 6;
#if INA_APPLY_MW
    // one action load covers this wave's next 64 / kApWin windows (lane l: window l /
    // kApWin of the group, packet l % kApWin), so a stream whose completed packets sit in
    // one region does not pay a round trip per empty window
    constexpr uint32_t kG = 64 / kApWin;
    const size_t S = (size_t)nwaves * kApWin;               // distance between a wave's windows
    for (size_t w0 = (size_t)wave * kApWin; w0 < npk; w0 += kG * S) {
        const size_t p = w0 + (size_t)(lane / kApWin) * S + (size_t)(lane % kApWin);
        unsigned long long m = __ballot(p < npk && actions[p] == INA_ACT_FWD_AGG);
#else
    for (uint32_t w0 = wave * kApWin; w0 < npk; w0 += nwaves * kApWin) {
        const uint32_t p = w0 + (uint32_t)lane;
        unsigned long long m = __ballot(lane < kApWin && p < npk && actions[p] == INA_ACT_FWD_AGG);
#endif
        while (m) {
            uint32_t pid[kApB];
            int nb = 0;
#pragma unroll
            for (int b = 0; b < kApB; ++b) {
                if (m) {
                    const uint32_t bit = (uint32_t)__builtin_ctzll(m);
#if INA_APPLY_MW
                    pid[b] = (uint32_t)(w0 + (size_t)(bit / kApWin) * S + (bit % kApWin));
#else
                    pid[b] = w0 + bit;
#endif
                    m &= m - 1;
                    nb = b + 1;
                } else {
                    pid[b] = pid[0];
                }
            }
            u32x4 hv[kApB], a[kApB];
#pragma unroll
            for (int b = 0; b < kApB; ++b) {
                const u32x4* pk = reinterpret_cast<const u32x4*>(pkts + (size_t)pid[b] * pstride);
                hv[b] = pk[0];
                a[b] = __builtin_nontemporal_load(pk + chn);
            }
            // slots from the headers, then every local row of the batch in flight at once
            uint32_t slot[kApB];
            f32x4 l[kApB];
#pragma unroll
            for (int b = 0; b < kApB; ++b) {
                const uint32_t h2 = __builtin_amdgcn_readfirstlane(hv[b].z);
                const uint32_t h3 = __builtin_amdgcn_readfirstlane(hv[b].w);
                slot[b] = b < nb ? bswap((h2 >> 24) | (h3 << 8)) - seq0 : 0xFFFFFFFFu;
                const size_t e = (size_t)slot[b] * (size_t)V + 4 * (size_t)lane;
                l[b] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (slot[b] < nslots && vl && e + 4 <= n) l[b] = *reinterpret_cast<const f32x4*>(local + e);
            }
#pragma unroll
            for (int b = 0; b < kApB; ++b) {
                if (slot[b] >= nslots) continue;               // past the batch, or not this bucket
                if (lane == 0 && acks) {
                    u32x4 hd = hv[b];
                    hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                    *reinterpret_cast<u32x4*>(acks + (size_t)slot[b] * ack_stride) = hd;
                }
                const uint32_t pw = (uint32_t)__builtin_amdgcn_update_dpp((int)hv[b].w, (int)a[b].w,
                                                                          0x138, 0xF, 0xF, false);
                uint32_t v[4];
                v[0] = __builtin_amdgcn_perm(a[b].x, pw, kSelBE);
                v[1] = __builtin_amdgcn_perm(a[b].y, a[b].x, kSelBE);
                v[2] = __builtin_amdgcn_perm(a[b].z, a[b].y, kSelBE);
                v[3] = __builtin_amdgcn_perm(a[b].w, a[b].z, kSelBE);
                if (!vl) continue;
                const size_t e = (size_t)slot[b] * (size_t)V + 4 * (size_t)lane;
                if (e + 4 <= n) {
                    f32x4 r;
                    r.x = __fadd_rn(l[b].x, __fmul_rn(__fmul_rn((float)(int32_t)v[0], inv), ws));
                    r.y = __fadd_rn(l[b].y, __fmul_rn(__fmul_rn((float)(int32_t)v[1], inv), ws));
                    r.z = __fadd_rn(l[b].z, __fmul_rn(__fmul_rn((float)(int32_t)v[2], inv), ws));
                    r.w = __fadd_rn(l[b].w, __fmul_rn(__fmul_rn((float)(int32_t)v[3], inv), ws));
                    // nt, like the fused switch pass's PS output (cold: default 58.0 us,
                    // write-through 57.0, nt 56.5; profiles/r03/lab/apply_store_lab.log)
                    __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(out + e));
                } else {
                    for (int t = 0; t < 4 && e + t < n; ++t)
                        out[e + t] = __fadd_rn(local[e + t], __fmul_rn(__fmul_rn((float)(int32_t)v[t], inv), ws));
                }
            }
        }
    }
}

// header fields only (no values asked for), one thread per packet (coalesced SoA stores)
__global__ __launch_bounds__(kBlock) void k_unpack_nga_hdr(const uint8_t* __restrict__ pkts,
                                                           size_t npk, size_t pstride,
                                                           NgaFieldsDev f) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    for (size_t p = (size_t)blockIdx.x * kBlock + threadIdx.x; p < npk; p += gs) {
        u32x4 a = *reinterpret_cast<const u32x4*>(pkts + p * pstride);
        nga_store_header(f, p, a.x, a.y, a.z, a.w);
    }
}

__device__ __forceinline__ uint32_t be32_at(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

__global__ __launch_bounds__(kBlock) void k_unpack_nga_scalar(const uint8_t* __restrict__ pkts,
                                                              size_t npk, int V, size_t pstride,
                                                              NgaFieldsDev f, int32_t* __restrict__ vals) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const size_t per = (size_t)V + 1;   // slot 0: header, 1..V: values
    for (size_t g = (size_t)blockIdx.x * kBlock + threadIdx.x; g < npk * per; g += gs) {
        size_t p = g / per, j = g - p * per;
        const uint8_t* pk = pkts + p * pstride;
        if (j == 0) {
            if (f.bitmap) f.bitmap[p] = be32_at(pk);
            if (f.count) f.count[p] = pk[4];
            if (f.flags) f.flags[p] = pk[5];
            if (f.index) f.index[p] = be32_at(pk + 6);
            if (f.switch_id) f.switch_id[p] = pk[10];
            if (f.frag_id) f.frag_id[p] = be32_at(pk + 11);
        } else if (vals) {
            vals[p * (size_t)V + j - 1] = (int32_t)be32_at(pk + 15 + 4 * (j - 1));
        }
    }
}

// ===========================================================================
// 6. C-128 packets: 131 BE words per packet (communicator.cc:23-37)
// ===========================================================================
__global__ __launch_bounds__(kBlock) void k_pack_c128(const uint32_t* __restrict__ g, size_t npk,
                                                      uint32_t bitmap, uint32_t agg, int tensor_index,
                                                      uint32_t* __restrict__ out) {
    const size_t gs = (size_t)gridDim.x * kBlock;
    const size_t total = npk * 131;
    for (size_t t = (size_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += gs) {
        size_t p = t / 131;
        uint32_t w = (uint32_t)(t - p * 131);
        uint32_t v;
        if (w == 0) v = bitmap;
        else if (w == 1) v = agg;
        else if (w == 2) v = (uint32_t)(tensor_index + (int)p);
        else v = g[p * 128 + (w - 3)];
        out[t] = bswap(v);
    }
}

// 4 consecutive words per thread: one 16-byte store (the buffer is 16-byte aligned), the
// words' sources found from one 32-bit divide (4-byte gradient loads).  ResNet-50's 199,665
// packets: 38.7 -> 35.7 us against a word per thread; one word per thread over a covering
// grid 46.7 us, 8 words per thread 48.8 us (tools/lab/c128_lab.py, profiles/r02/lab/c128_lab.log)
template <int X>
__global__ __launch_bounds__(kBlock) void k_pack_c128_x4(const uint32_t* __restrict__ g, uint32_t total,
                                                         uint32_t bitmap, uint32_t agg, int tensor_index,
                                                         uint32_t* __restrict__ out) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t t0 = X * c;
    if (t0 >= total) return;
    uint32_t p = t0 / 131u, w = t0 - p * 131u;
    uint32_t r[X];
#pragma unroll
    for (int i = 0; i < X; ++i) {
        uint32_t v = 0;
        if (t0 + i < total) {
            if (w == 0) v = bitmap;
            else if (w == 1) v = agg;
            else if (w == 2) v = (uint32_t)(tensor_index + (int)p);
            else v = g[(size_t)p * 128 + (w - 3)];
        }
        r[i] = bswap(v);
        if (++w == 131u) { w = 0; ++p; }
    }
    if (t0 + X <= total) {
#pragma unroll
        for (int i = 0; i < X; i += 4)
            *reinterpret_cast<u32x4*>(out + t0 + i) = u32x4{r[i], r[i + 1], r[i + 2], r[i + 3]};
    } else {
        for (uint32_t i = 0; t0 + i < total; ++i) out[t0 + i] = r[i];
    }
}


// ===========================================================================
// 7. checksum: sum_i x[i]*(2i+1) mod 2^32 -- wave shuffle + LDS block reduce
// ===========================================================================
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ __launch_bounds__(kBlock) void k_checksum_i32(const int32_t* __restrict__ x, size_t n,
                                                         int vec, uint32_t* __restrict__ out) {
    __shared__ uint32_t part[kBlock / 64];
    const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlock;
    uint32_t acc = 0;
    size_t n4 = vec ? n / 4 : 0;
    for (size_t i = tid; i < n4; i += stride) {
        u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x) + i);
        uint32_t c = (uint32_t)(8 * i + 1);
        acc += v.x * c + v.y * (c + 2) + v.z * (c + 4) + v.w * (c + 6);
    }
    for (size_t i = 4 * n4 + tid; i < n; i += stride) acc += (uint32_t)x[i] * (uint32_t)(2 * i + 1);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int w = 0; w < kBlock / 64; ++w) s += part[w];
        atomicAdd(out, s);
    }
}

// ===========================================================================
// 8. per-bucket absmax for a dynamic scale: max_i |x[i] - base[i]| over finite and
//    infinite values (NaN ignored: the quantiser maps it to 0).  Non-negative floats
//    order like their bit patterns, so blocks combine with one atomicMax on the bits.
// ===========================================================================
__device__ __forceinline__ float absdiff(float x, const float* base, size_t i) {
    return fabsf(base ? __fsub_rn(x, base[i]) : x);
}

#ifndef INA_ABSMAX_U
#define INA_ABSMAX_U 4
#endif
#ifndef INA_ABSMAX_BLOCKS
#define INA_ABSMAX_BLOCKS kFaninBlocks
#endif
__global__ __launch_bounds__(kBlock) void k_absmax_f32(const float* __restrict__ x,
                                                       const float* __restrict__ base, size_t n,
                                                       int vec, uint32_t* __restrict__ out) {
    __shared__ float part[kBlock / 64];
    const size_t n4 = vec ? n / 4 : 0;
    float m = 0.0f;
    chunk_loop<INA_ABSMAX_U>(n4, [&]<int UU>(size_t i, size_t st) {
        f32x4 a[UU], b[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            a[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x) + i + u * st);
            b[u] = base ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base) + i + u * st)
                        : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
            m = fmaxf(m, fabsf(__fsub_rn(a[u].x, b[u].x)));
            m = fmaxf(m, fabsf(__fsub_rn(a[u].y, b[u].y)));
            m = fmaxf(m, fabsf(__fsub_rn(a[u].z, b[u].z)));
            m = fmaxf(m, fabsf(__fsub_rn(a[u].w, b[u].w)));
        }
    });
    const size_t stride = (size_t)gridDim.x * kBlock;
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        m = fmaxf(m, absdiff(x[i], base, i));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = part[0];
        for (int w = 1; w < kBlock / 64; ++w) r = fmaxf(r, part[w]);
        atomicMax(out, __float_as_uint(r));
    }
}

// W workers in one pass (ina_absmax_multi_f32): a thread's 16-byte chunk of base is loaded
// once and compared against the same chunk of every worker, 4 workers' loads in flight at
// a time -- W + 1 streams instead of W launches of 2 (and no per-worker memset + launch)
__global__ __launch_bounds__(kBlock) void k_absmax_multi_f32(PtrPack<float> xs, int W,
                                                             const float* __restrict__ base, size_t n,
                                                             int vec, uint32_t* __restrict__ out) {
    __shared__ float part[kBlock / 64];
    const size_t n4 = vec ? n / 4 : 0;
    const size_t stride = (size_t)gridDim.x * kBlock;
    float m = 0.0f;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
        const f32x4 b = base ? __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base) + i)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
        int w = 0;
        for (; w + 4 <= W; w += 4) {
            f32x4 a[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                a[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(xs.p[w + u]) + i);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                m = fmaxf(m, fabsf(__fsub_rn(a[u].x, b.x)));
                m = fmaxf(m, fabsf(__fsub_rn(a[u].y, b.y)));
                m = fmaxf(m, fabsf(__fsub_rn(a[u].z, b.z)));
                m = fmaxf(m, fabsf(__fsub_rn(a[u].w, b.w)));
            }
        }
        for (; w < W; ++w) {
            const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(xs.p[w]) + i);
            m = fmaxf(m, fabsf(__fsub_rn(a.x, b.x)));
            m = fmaxf(m, fabsf(__fsub_rn(a.y, b.y)));
            m = fmaxf(m, fabsf(__fsub_rn(a.z, b.z)));
            m = fmaxf(m, fabsf(__fsub_rn(a.w, b.w)));
        }
    }
    for (size_t i = 4 * n4 + (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        for (int w = 0; w < W; ++w) m = fmaxf(m, absdiff(xs.p[w][i], base, i));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = part[0];
        for (int w = 1; w < kBlock / 64; ++w) r = fmaxf(r, part[w]);
        atomicMax(out, __float_as_uint(r));
    }
}
#ifndef INA_ABSMAX_MULTI_BLOCKS
#define INA_ABSMAX_MULTI_BLOCKS 512
#endif

}  // namespace ina

// ===========================================================================
// extern "C" entry points
// ===========================================================================
using namespace ina;

static inline hipStream_t hs(ina_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

static int check_k(int k) {
    if (k < -126 || k > 127) return set_error(INA_EINVAL, "k out of range [-126,127]%s", "");
    return INA_OK;
}

template <typename T>
static int fill_pack(PtrPack<T>& pk, const T* const* bufs, int W, bool& all_aligned) {
    if (!bufs || W < 1 || W > INA_MAX_WORKERS)
        return set_error(INA_EINVAL, "W must be in [1, %s]", "64");
    all_aligned = true;
    for (int w = 0; w < W; ++w) {
        if (!bufs[w]) return set_error(INA_EINVAL, "null worker buffer%s", "");
        pk.p[w] = bufs[w];
        all_aligned &= aligned16(bufs[w]);
    }
    for (int w = W; w < INA_MAX_WORKERS; ++w) pk.p[w] = nullptr;
    return INA_OK;
}

template <typename Src>
static int pack_nga_launch(const Src& src, bool src_aligned, size_t n, const ina_nga_params_t* prm,
                           const uint8_t* ovf, uint8_t* pkts, size_t pstride, hipStream_t s,
                           uint64_t* desc = nullptr) {
    if (!prm || prm->V <= 0 || prm->num_slots == 0)
        return set_error(INA_EINVAL, "bad nga params%s", "");
    const int V = prm->V;
    if (pstride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)V)
        return set_error(INA_EINVAL, "stride < 15 + 4V%s", "");
    size_t npk = (n + (size_t)V - 1) / (size_t)V;
    if (npk == 0) return INA_OK;
    if (!pkts) return set_error(INA_EINVAL, "null pointer%s", "");
    NgaHdr h{prm->bitmap, prm->seq0, prm->num_slots,
             (uint32_t)prm->count | ((uint32_t)prm->flags << 8) | ((uint32_t)prm->switch_id << 16), V};
    if (pstride % 16 == 0 && V % 4 == 0 && src_aligned && aligned16(pkts)) {
        // 32-bit chunk indices: huge buckets go in packet ranges
        const size_t C = pstride / 16;
        const size_t per = std::max<size_t>(1, (size_t)g_launch_chunks.load() / C);
        for (size_t p0 = 0; p0 < npk; p0 += per) {
            const size_t np = npk - p0 < per ? npk - p0 : per;
            const size_t v0 = p0 * (size_t)V;
            NgaHdr hp = h;
            hp.seq0 = h.seq0 + (uint32_t)p0;
            // a wave per packet for the fused worker pack (cold, one launch: 53.2 -> 48.9 us);
            // the int32 pack stays on the flat stream (36.5 -> 39.1 us with a wave per
            // packet: one 16-byte load per lane leaves too little in flight),
            // profiles/r03/lab/pack_ppw_lab.log
            if (INA_PACK_PPW && std::is_same_v<Src, SrcQ32> && V == 256 && C <= 65 + 64) {
                hipLaunchKernelGGL((k_pack_nga_v256<Src>), dim3(grid_for(np * 64, 1, 1 << 20)), dim3(kBlock), 0, s,
                                   src.shifted(v0), n - v0, hp, ovf ? ovf + p0 : nullptr, pkts + p0 * pstride,
                                   (uint32_t)pstride, (uint32_t)np,
                                   desc ? reinterpret_cast<u32x2*>(desc + p0) : nullptr);
                continue;
            }
            hipLaunchKernelGGL((k_pack_nga_flat<Src, INA_PACK_U>), dim3(grid_for(np * C, INA_PACK_U, g_stream_blocks)),
                               dim3(kBlock), 0, s, src.shifted(v0), n - v0, hp, ovf ? ovf + p0 : nullptr,
                               pkts + p0 * pstride, (uint32_t)C, (uint32_t)(V / 4), (uint32_t)(np * C),
                               desc ? reinterpret_cast<u32x2*>(desc + p0) : nullptr);
        }
    } else {
        size_t nbytes = npk * pstride;
        hipLaunchKernelGGL(k_pack_nga_bytes<Src>, dim3(grid_for(nbytes, 1)), dim3(kBlock), 0, s, src, n,
                           h, ovf, pkts, pstride, nbytes);
        if (desc)   // the generic layout gathers its descriptors from the written headers
            hipLaunchKernelGGL(k_nga_desc, dim3(grid_for(npk, 1)), dim3(kBlock), 0, s, pkts, npk, pstride,
                               desc);
    }
    return check_launch("pack_nga");
}

extern "C" {

const char* ina_version(void) { return "ina-mi355x 0.2 (gfx950)"; }
const char* ina_last_error_string(void) { return g_err; }

#ifndef INA_LAB_KEYS
#define INA_LAB_KEYS 0
#endif
int ina_set_tuning(int key, int value) {
    switch (key) {
        case 0: if (value < 1) return INA_EINVAL; g_max_blocks = value; return INA_OK;
        case 1: if (value != 0 && value != 1 && value != 2 && value != 4) return INA_EINVAL; g_unroll = value; return INA_OK;
        case 2: g_nontemporal = value ? 1 : 0; return INA_OK;
        case 3: if (value < 0) return INA_EINVAL; g_reduce_blocks = value; return INA_OK;
#if INA_LAB_KEYS
        // grid-cap sweeps (bench_extra.py, tools/lab): lab builds only (make EXTRA=-DINA_LAB_KEYS=1)
        case 4: if (value < 1) return INA_EINVAL; g_stream_blocks = value; return INA_OK;
        case 14: if (value < 1) return INA_EINVAL; g_ew_blocks = value; return INA_OK;
        case 5: if (value < 1) return INA_EINVAL; g_combine_blocks = value; return INA_OK;
        case 6: if (value < 1) return INA_EINVAL; g_combine_ina_blocks = value; return INA_OK;
        case 10: return set_switch_win(value);
#endif
        case 7: return set_h2d_streams(value);
        case 8: if (value < 1) return INA_EINVAL; g_launch_chunks = value; return INA_OK;
        case 9: return set_small_sort(value);
        case 11: return set_ack_fast(value);
        case 12: return set_sort_mode(value);
        case 13: return set_os_rounds(value);
        case 15: return set_tiny_max(value);
        case 16: return set_zero_copy(value);
        case 17: return set_bucket_tile(value);
        case 18: return set_runs(value);
        case 19: return set_pre_all(value);
        case 20: return set_local(value);
        case 21: return set_decide_delay(value);
        default: return INA_EINVAL;
    }
}

}  // extern "C"

namespace ina {
// host = true: the PCIe pipeline's chunks (k_host_chunk_reduce_i32, see above)
int sum_reduce_i32_impl(const int32_t* const* bufs, int W, int32_t* out, size_t n,
                        ina_stream_t stream, bool host) {
    if (n == 0) return INA_OK;
    PtrPack<int32_t> pk;
    bool al;
    if (int rc = fill_pack(pk, bufs, W, al)) return rc;
    if (!out) return set_error(INA_EINVAL, "null out%s", "");
    hipStream_t s = hs(stream);
    if (!(al && aligned16(out))) {
        hipLaunchKernelGGL(k_sum_reduce_i32_scalar, dim3(grid_for(n, 1)), dim3(kBlock), 0, s, pk, W, out, n);
        return check_launch("sum_reduce_i32 scalar");
    }
    size_t n4 = n / 4;
    switch (W) {
        case 1: launch_reduce_u<1>(pk, out, n4, n, s, host); break;
        case 2: launch_reduce_u<2>(pk, out, n4, n, s, host); break;
        case 3: launch_reduce_u<3>(pk, out, n4, n, s, host); break;
        case 4: launch_reduce_u<4>(pk, out, n4, n, s, host); break;
        case 8: launch_reduce_u<8>(pk, out, n4, n, s, host); break;
        case 16: launch_reduce_u<16>(pk, out, n4, n, s, host); break;
        default:
            hipLaunchKernelGGL(k_sum_reduce_i32_vec_dyn, dim3(grid_for(n4, 1)), dim3(kBlock), 0, s,
                               pk, W, out, n4, n);
    }
    return check_launch("sum_reduce_i32");
}
}  // namespace ina

extern "C" {

int ina_sum_reduce_i32(const int32_t* const* bufs, int W, int32_t* out, size_t n,
                       ina_stream_t stream) {
    return sum_reduce_i32_impl(bufs, W, out, n, stream, false);
}

int ina_quantize_f32_i32(const float* x, int32_t* q, size_t n, int k, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    if (!x || !q) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = aligned16(x) && aligned16(q);
    hipLaunchKernelGGL(k_quantize_i32, dim3(grid_for(vec ? n / 4 + 1 : n, kEwU, g_ew_blocks)), dim3(kBlock), 0,
                       hs(stream), x, q, n, ldexpf(1.0f, k), vec);
    return check_launch("quantize_i32");
}

int ina_quantize_f32_i16_sat(const float* x, int16_t* q, size_t n, int k, int V,
                             uint8_t* ovf, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (V <= 0) return set_error(INA_EINVAL, "V must be > 0%s", "");
    if (n == 0) return INA_OK;
    if (!x || !q) return set_error(INA_EINVAL, "null pointer%s", "");
    hipStream_t s = hs(stream);
    float sc = ldexpf(1.0f, k);
    if (aligned16(x) && aligned16(q) && (!ovf || slot_ballot_ok(V))) {
        int lps = slot_ballot_ok(V) ? V / 8 : 1;
        hipLaunchKernelGGL(k_quantize_i16_vec, dim3(grid_for((n + 7) / 8, 1)), dim3(kBlock), 0, s,
                           x, q, n, sc, V, lps, ovf);
    } else {
        if (ovf && hipMemsetAsync(ovf, 0, (n + V - 1) / V, s) != hipSuccess)
            return set_error(INA_EHIP, "memset overflow flags%s", "");
        hipLaunchKernelGGL(k_quantize_i16_scalar, dim3(grid_for(n, 1)), dim3(kBlock), 0, s, x, q, n,
                           sc, V, ovf);
    }
    return check_launch("quantize_i16");
}

int ina_dequantize_i32_f32(const int32_t* sv, float* y, size_t n, int k, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    if (!sv || !y) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = aligned16(sv) && aligned16(y);
    hipLaunchKernelGGL(k_dequantize_i32, dim3(grid_for(vec ? n / 4 + 1 : n, kEwU, g_ew_blocks)), dim3(kBlock), 0,
                       hs(stream), sv, y, n, ldexpf(1.0f, -k), vec);
    return check_launch("dequantize_i32");
}

int ina_dequantize_i16_f32(const int16_t* sv, float* y, size_t n, int k, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    if (!sv || !y) return set_error(INA_EINVAL, "null pointer%s", "");
    const int vec = ((uintptr_t)sv % 8 == 0) && aligned16(y);
    hipLaunchKernelGGL(k_dequantize_i16, dim3(grid_for(vec ? n / 4 + 1 : n, kEwU, g_ew_blocks)),
                       dim3(kBlock), 0, hs(stream), sv, y, n, ldexpf(1.0f, -k), vec);
    return check_launch("dequantize_i16");
}

int ina_sum_reduce_i16_sat(const int16_t* const* bufs, int W, int16_t* out, size_t n, int V,
                           uint8_t* ovf, ina_stream_t stream) {
    if (V <= 0) return set_error(INA_EINVAL, "V must be > 0%s", "");
    if (n == 0) return INA_OK;
    PtrPack<int16_t> pk;
    bool al;
    if (int rc = fill_pack(pk, bufs, W, al)) return rc;
    if (!out) return set_error(INA_EINVAL, "null out%s", "");
    hipStream_t s = hs(stream);
    if (al && aligned16(out) && (!ovf || slot_ballot_ok(V))) {
        int lps = slot_ballot_ok(V) ? V / 8 : 1;
        hipLaunchKernelGGL(k_sum_reduce_i16, dim3(grid_for((n + 7) / 8, 1)), dim3(kBlock), 0, s, pk, W,
                           out, n, V, lps, ovf);
    } else {
        if (ovf && hipMemsetAsync(ovf, 0, (n + V - 1) / V, s) != hipSuccess)
            return set_error(INA_EHIP, "memset overflow flags%s", "");
        hipLaunchKernelGGL(k_sum_reduce_i16_scalar, dim3(grid_for(n, 1)), dim3(kBlock), 0, s, pk, W,
                           out, n, V, ovf);
    }
    return check_launch("sum_reduce_i16");
}

int ina_quantize_reduce_f32_i32(const float* const* bufs, int W, int32_t* out, size_t n, int k,
                                ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    PtrPack<float> pk;
    bool al;
    if (int rc = fill_pack(pk, bufs, W, al)) return rc;
    if (!out) return set_error(INA_EINVAL, "null out%s", "");
    // one worker: the sum is the quantised buffer itself (the same q32), so the tuned
    // one-in one-out kernel runs it (0.75 -> 0.67 ms per GiB with the decode, bench.py C5 layout B)
    if (W == 1) return ina_quantize_f32_i32(bufs[0], out, n, k, stream);
    int vec = al && aligned16(out);
    float sc = ldexpf(1.0f, k);
    // W <= 8: one 16-byte chunk per stream per thread and a grid covering the bucket (C2,
    // back to back: 86.2 us against 88.7 at 8192 workgroups and 87.9-96.7 at 256-2048,
    // tools/lab/ew16_lab.py, profiles/r03/lab/ew16_lab.log); more streams stride
    unsigned g = grid_for(vec ? n / 4 + 1 : n, W <= 8 ? INA_QR_U : 2, W <= 8 ? g_ew_blocks.load() : g_stream_blocks.load());
    hipStream_t s = hs(stream);
    switch (W) {
        case 2: hipLaunchKernelGGL(k_quant_reduce_i32<2>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, vec); break;
        case 4: hipLaunchKernelGGL(k_quant_reduce_i32<4>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, vec); break;
        case 8: hipLaunchKernelGGL(k_quant_reduce_i32<8>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, vec); break;
        case 16: hipLaunchKernelGGL(k_quant_reduce_i32<16>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, vec); break;
        default: hipLaunchKernelGGL(k_quant_reduce_i32<0>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, vec);
    }
    return check_launch("quantize_reduce_i32");
}

int ina_quantize_reduce_f32_i16_sat(const float* const* bufs, int W, int16_t* out, size_t n, int k,
                                    int V, uint8_t* ovf, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (V <= 0) return set_error(INA_EINVAL, "V must be > 0%s", "");
    if (n == 0) return INA_OK;
    PtrPack<float> pk;
    bool al;
    if (int rc = fill_pack(pk, bufs, W, al)) return rc;
    if (!out) return set_error(INA_EINVAL, "null out%s", "");
    hipStream_t s = hs(stream);
    float sc = ldexpf(1.0f, k);
    if (al && aligned16(out) && (!ovf || slot_ballot_ok(V))) {
        int lps = slot_ballot_ok(V) ? V / 8 : 1;
        unsigned g = grid_for((n + 7) / 8, 1);
        switch (W) {
            case 4: hipLaunchKernelGGL(k_quant_reduce_i16<4>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, V, lps, ovf); break;
            case 8: hipLaunchKernelGGL(k_quant_reduce_i16<8>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, V, lps, ovf); break;
            case 16: hipLaunchKernelGGL(k_quant_reduce_i16<16>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, V, lps, ovf); break;
            default: hipLaunchKernelGGL(k_quant_reduce_i16<0>, dim3(g), dim3(kBlock), 0, s, pk, W, out, n, sc, V, lps, ovf);
        }
    } else {
        if (ovf && hipMemsetAsync(ovf, 0, (n + V - 1) / V, s) != hipSuccess)
            return set_error(INA_EHIP, "memset overflow flags%s", "");
        hipLaunchKernelGGL(k_quant_reduce_i16_scalar, dim3(grid_for(n, 1)), dim3(kBlock), 0, s, pk, W,
                           out, n, sc, V, ovf);
    }
    return check_launch("quantize_reduce_i16");
}

int ina_ps_combine_f32(const float* local, const float* const* paras, int W, double weight_step,
                       float* out, size_t n, ina_stream_t stream) {
    if (n == 0) return INA_OK;
    PtrPack<float> pk;
    bool al;
    if (int rc = fill_pack(pk, paras, W, al)) return rc;
    if (!local || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = al && aligned16(local) && aligned16(out);
    unsigned g = grid_for(vec ? n / 4 + 1 : n, W <= 4 ? INA_COMB_U : 2, g_combine_blocks);
    hipStream_t s = hs(stream);
    float ws = (float)weight_step;
    switch (W) {
#define PSC(WW) case WW: hipLaunchKernelGGL(k_ps_combine_f32<WW>, dim3(g), dim3(kBlock), 0, s, local, pk, W, ws, out, n, vec); break;
        PSC(1) PSC(2) PSC(3) PSC(4) PSC(5) PSC(6) PSC(7) PSC(8)
#undef PSC
        default: hipLaunchKernelGGL(k_ps_combine_f32<0>, dim3(g), dim3(kBlock), 0, s, local, pk, W, ws, out, n, vec);
    }
    return check_launch("ps_combine_f32");
}

int ina_ps_apply_i32(const float* local, const int32_t* sum_int, int k, double weight_step,
                     float* out, size_t n, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    if (!local || !sum_int || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = aligned16(local) && aligned16(sum_int) && aligned16(out);
    hipLaunchKernelGGL(k_ps_apply_i32, dim3(grid_for(vec ? n / 4 + 1 : n, kEwU, g_ew_blocks)), dim3(kBlock), 0,
                       hs(stream), local, sum_int, ldexpf(1.0f, -k), (float)weight_step, out, n, vec);
    return check_launch("ps_apply_i32");
}

int ina_ps_combine_ina_f32(const float* local, const float* const* paras, int W, int k,
                           double weight_step, float* out, size_t n, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n == 0) return INA_OK;
    PtrPack<float> pk;
    bool al;
    if (int rc = fill_pack(pk, paras, W, al)) return rc;
    if (!local || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = al && aligned16(local) && aligned16(out);
    unsigned g = grid_for(vec ? n / 4 + 1 : n, W <= 4 ? INA_COMBI_U : 2, g_combine_ina_blocks);
    hipStream_t s = hs(stream);
    float sc = ldexpf(1.0f, k), inv = ldexpf(1.0f, -k), ws = (float)weight_step;
    switch (W) {
#define PSI(WW) case WW: hipLaunchKernelGGL(k_ps_combine_ina<WW>, dim3(g), dim3(kBlock), 0, s, local, pk, W, sc, inv, ws, out, n, vec); break;
        PSI(1) PSI(2) PSI(3) PSI(4) PSI(5) PSI(6) PSI(7) PSI(8)
#undef PSI
        default: hipLaunchKernelGGL(k_ps_combine_ina<0>, dim3(g), dim3(kBlock), 0, s, local, pk, W, sc, inv, ws, out, n, vec);
    }
    return check_launch("ps_combine_ina_f32");
}

int ina_pack_nga_desc(const int32_t* vals, size_t n, const ina_nga_params_t* prm, const uint8_t* ovf,
                      uint8_t* pkts, size_t pstride, ina_nga_desc_t* desc, ina_stream_t stream) {
    if (n && !vals) return set_error(INA_EINVAL, "null pointer%s", "");
    if (desc && ((uintptr_t)desc & 7u)) return set_error(INA_EINVAL, "descriptors must be 8-byte aligned%s", "");
    return pack_nga_launch(SrcI32{vals}, aligned16(vals), n, prm, ovf, pkts, pstride, hs(stream), desc);
}

int ina_pack_nga(const int32_t* vals, size_t n, const ina_nga_params_t* prm, const uint8_t* ovf,
                 uint8_t* pkts, size_t pstride, ina_stream_t stream) {
    return ina_pack_nga_desc(vals, n, prm, ovf, pkts, pstride, nullptr, stream);
}

int ina_quantize_pack_nga_desc(const float* x, const float* base, size_t n, int k,
                               const ina_nga_params_t* prm, uint8_t* pkts, size_t pstride,
                               ina_nga_desc_t* desc, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (n && !x) return set_error(INA_EINVAL, "null pointer%s", "");
    if (desc && ((uintptr_t)desc & 7u)) return set_error(INA_EINVAL, "descriptors must be 8-byte aligned%s", "");
    bool al = aligned16(x) && (!base || aligned16(base));
    return pack_nga_launch(SrcQ32{x, base, ldexpf(1.0f, k)}, al, n, prm, nullptr, pkts, pstride,
                           hs(stream), desc);
}

int ina_quantize_pack_nga(const float* x, const float* base, size_t n, int k,
                          const ina_nga_params_t* prm, uint8_t* pkts, size_t pstride,
                          ina_stream_t stream) {
    return ina_quantize_pack_nga_desc(x, base, n, k, prm, pkts, pstride, nullptr, stream);
}

int ina_nga_make_descriptors(const ina_nga_params_t* prm, int W, size_t npk, ina_nga_desc_t* const* desc,
                             ina_stream_t stream) {
    if (!prm || !desc || W < 1 || W > INA_MAX_WORKERS)
        return set_error(INA_EINVAL, "prm, desc non-null and W in [1, %s]", "64");
    if (npk > 0xFFFFFFFFu) return set_error(INA_EINVAL, "too many packets%s", "");
    for (int w = 0; w < W; ++w) {
        if (prm[w].num_slots == 0 || prm[w].num_slots != prm[0].num_slots)
            return set_error(INA_EINVAL, "every worker needs the same non-zero num_slots%s", "");
        if (!desc[w] || ((uintptr_t)desc[w] & 7u))
            return set_error(INA_EINVAL, "descriptors must be non-null and 8-byte aligned%s", "");
    }
    if (npk == 0) return INA_OK;
    for (int w0 = 0; w0 < W; w0 += kQpGroup) {
        const int G = std::min(kQpGroup, W - w0);
        DescGroup a{};
        for (int g = 0; g < G; ++g) {
            const ina_nga_params_t& q = prm[w0 + g];
            a.desc[g] = reinterpret_cast<u32x2*>(desc[w0 + g]);
            a.seq0[g] = q.seq0;
            a.fcs[g] = (uint32_t)q.count | ((uint32_t)q.flags << 8) | ((uint32_t)q.switch_id << 16);
        }
        hipLaunchKernelGGL(k_nga_make_desc, dim3(grid_for(npk, 1)), dim3(kBlock), 0, hs(stream), a, G,
                           prm[0].num_slots, (uint32_t)npk);
    }
    return check_launch("nga_make_descriptors");
}

int ina_quantize_pack_nga_multi(const float* const* x, int W, const float* base, size_t n, int k,
                                const ina_nga_params_t* prm, uint8_t* const* pkts, size_t pstride,
                                ina_nga_desc_t* const* desc, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (!x || !prm || !pkts || W < 1 || W > INA_MAX_WORKERS)
        return set_error(INA_EINVAL, "x, prm, pkts non-null and W in [1, %s]", "64");
    const int V = prm[0].V;
    if (V <= 0 || prm[0].num_slots == 0) return set_error(INA_EINVAL, "bad nga params%s", "");
    if (pstride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)V)
        return set_error(INA_EINVAL, "stride < 15 + 4V%s", "");
    const size_t npk = (n + (size_t)V - 1) / (size_t)V;
    if (npk == 0) return INA_OK;                       // empty buckets: nothing to write
    bool flat = pstride % 16 == 0 && V % 4 == 0 && (!base || aligned16(base));
    for (int w = 0; w < W; ++w) {
        if (prm[w].V != V || prm[w].num_slots != prm[0].num_slots)
            return set_error(INA_EINVAL, "every worker needs the same V and num_slots%s", "");
        if ((n && !x[w]) || !pkts[w]) return set_error(INA_EINVAL, "null worker buffer%s", "");
        if (desc && (!desc[w] || ((uintptr_t)desc[w] & 7u)))
            return set_error(INA_EINVAL, "descriptors must be non-null and 8-byte aligned%s", "");
        flat &= aligned16(x[w]) && aligned16(pkts[w]);
    }
    hipStream_t s = hs(stream);
    if (!flat) {     // generic layouts: the per-worker byte path, worker by worker
        for (int w = 0; w < W; ++w)
            if (int rc = ina_quantize_pack_nga_desc(x[w], base, n, k, &prm[w], pkts[w], pstride,
                                                    desc ? desc[w] : nullptr, stream))
                return rc;
        return INA_OK;
    }
    const float sc = ldexpf(1.0f, k);
    const size_t C = pstride / 16;
    const size_t per = std::max<size_t>(1, (size_t)g_launch_chunks.load() / C);
    for (int w0 = 0; w0 < W; w0 += kQpGroup) {
        const int G = std::min(kQpGroup, W - w0);
        for (size_t p0 = 0; p0 < npk; p0 += per) {     // 32-bit chunk indices: packet ranges
            const size_t np = npk - p0 < per ? npk - p0 : per;
            const size_t v0 = p0 * (size_t)V;
            QPackGroup a{};
            for (int g = 0; g < G; ++g) {
                const ina_nga_params_t& q = prm[w0 + g];
                a.x[g] = x[w0 + g] + v0;
                a.pkts[g] = pkts[w0 + g] + p0 * pstride;
                a.desc[g] = desc ? reinterpret_cast<u32x2*>(desc[w0 + g] + p0) : nullptr;
                a.bitmap[g] = q.bitmap;
                a.seq0[g] = q.seq0 + (uint32_t)p0;
                a.fcs[g] = (uint32_t)q.count | ((uint32_t)q.flags << 8) | ((uint32_t)q.switch_id << 16);
            }
            const dim3 blk(kBlock);
            const float* bp = base ? base + v0 : nullptr;
            const size_t nn = n - v0;
            if (INA_QPM_PPW && V == 256 && C <= 65 + 64) {          // a wave per packet
                const dim3 grid(grid_for(np * 64, 1, INA_QPM_PPW_BLOCKS));
                switch (G) {
#define INA_QPM(g_) case g_: hipLaunchKernelGGL(k_qpack_nga_multi_v256<g_>, grid, blk, 0, s, a, bp, nn, sc, \
                                                prm[0].num_slots, (uint32_t)pstride, (uint32_t)np); break;
                    INA_QPM(1) INA_QPM(2) INA_QPM(3) INA_QPM(4) INA_QPM(5) INA_QPM(6) INA_QPM(7) INA_QPM(8)
#undef INA_QPM
                }
                continue;
            }
            const dim3 grid(grid_for(np * C, 1, g_stream_blocks));
            const uint32_t ns = prm[0].num_slots, VV = (uint32_t)V, CC = (uint32_t)C, L = (uint32_t)(V / 4),
                           nch = (uint32_t)(np * C);
            switch (G) {
#define INA_QPM(g_) case g_: hipLaunchKernelGGL(k_qpack_nga_multi<g_>, grid, blk, 0, s, a, bp, nn, sc, ns, \
                                                VV, CC, L, nch); break;
                INA_QPM(1) INA_QPM(2) INA_QPM(3) INA_QPM(4) INA_QPM(5) INA_QPM(6) INA_QPM(7) INA_QPM(8)
#undef INA_QPM
            }
        }
    }
    return check_launch("quantize_pack_nga_multi");
}

int ina_nga_descriptors(const uint8_t* pkts, size_t npk, size_t pstride, ina_nga_desc_t* desc,
                        ina_stream_t stream) {
    if (pstride < (size_t)INA_NGA_HDR_BYTES) return set_error(INA_EINVAL, "stride < 15%s", "");
    if (npk == 0) return INA_OK;
    if (!pkts || !desc) return set_error(INA_EINVAL, "null pointer%s", "");
    if ((uintptr_t)desc & 7u) return set_error(INA_EINVAL, "descriptors must be 8-byte aligned%s", "");
    hipLaunchKernelGGL(k_nga_desc, dim3(grid_for(npk, 1)), dim3(kBlock), 0, hs(stream), pkts, npk, pstride,
                       desc);
    return check_launch("nga_descriptors");
}

// ---- split rows (include/ina.h) ----------------------------------------------------------
static int split_geometry(int V, uint32_t num_slots) {
    if (V <= 0 || V % 4 || V > 256 || num_slots == 0)
        return set_error(INA_EINVAL, "split rows need V a multiple of 4 in [4, 256] and num_slots > 0%s", "");
    return INA_OK;
}

int ina_pack_nga_split(const int32_t* vals, size_t n, const ina_nga_params_t* prm, const uint8_t* ovf,
                       uint8_t* hdr, uint8_t* pay, ina_nga_desc_t* desc, ina_stream_t stream) {
    if (!prm) return set_error(INA_EINVAL, "null params%s", "");
    if (int rc = split_geometry(prm->V, prm->num_slots)) return rc;
    const size_t V = (size_t)prm->V, npk = (n + V - 1) / V;
    if (npk == 0) return INA_OK;
    if (!vals || !hdr || !pay) return set_error(INA_EINVAL, "null pointer%s", "");
    if (!aligned16(hdr) || !aligned16(pay) || (desc && ((uintptr_t)desc & 7u)))
        return set_error(INA_EINVAL, "header / payload rows 16-byte aligned, descriptors 8%s", "");
    NgaHdr h{prm->bitmap, prm->seq0, prm->num_slots,
             (uint32_t)prm->count | ((uint32_t)prm->flags << 8) | ((uint32_t)prm->switch_id << 16), prm->V};
    const size_t nch = npk * V / 4;
    hipLaunchKernelGGL((k_pack_nga_split<SrcI32>), dim3(grid_for(std::max(nch, npk), 1, ew_grid_cap())),
                       dim3(kBlock), 0, hs(stream), SrcI32{vals}, n, h, ovf, reinterpret_cast<u32x4*>(hdr),
                       reinterpret_cast<u32x4*>(pay), reinterpret_cast<u32x2*>(desc), nch, npk,
                       aligned16(vals) ? 1 : 0);
    return check_launch("pack_nga_split");
}

int ina_quantize_pack_nga_multi_split(const float* const* x, int W, const float* base, size_t n, int k,
                                      const ina_nga_params_t* prm, uint8_t* const* hdr, uint8_t* const* pay,
                                      ina_nga_desc_t* const* desc, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (!x || !prm || !hdr || !pay || W < 1 || W > INA_MAX_WORKERS)
        return set_error(INA_EINVAL, "x, prm, hdr, pay non-null and W in [1, %s]", "64");
    const int V = prm[0].V;
    if (int rc = split_geometry(V, prm[0].num_slots)) return rc;
    const size_t npk = (n + (size_t)V - 1) / (size_t)V;
    if (npk == 0) return INA_OK;
    if (base && !aligned16(base)) return set_error(INA_EINVAL, "base must be 16-byte aligned%s", "");
    for (int w = 0; w < W; ++w) {
        if (prm[w].V != V || prm[w].num_slots != prm[0].num_slots)
            return set_error(INA_EINVAL, "every worker needs the same V and num_slots%s", "");
        if (!x[w] || !hdr[w] || !pay[w]) return set_error(INA_EINVAL, "null worker buffer%s", "");
        if (!aligned16(x[w]) || !aligned16(hdr[w]) || !aligned16(pay[w]))
            return set_error(INA_EINVAL, "worker buffers and rows must be 16-byte aligned%s", "");
        if (desc && (!desc[w] || ((uintptr_t)desc[w] & 7u)))
            return set_error(INA_EINVAL, "descriptors must be non-null and 8-byte aligned%s", "");
    }
    const float sc = ldexpf(1.0f, k);
    const size_t nch = npk * (size_t)V / 4;
    const dim3 grid(grid_for(std::max(nch, npk), 1, ew_grid_cap())), blk(kBlock);
    hipStream_t s = hs(stream);
    for (int w0 = 0; w0 < W; w0 += kQpGroup) {
        const int G = std::min(kQpGroup, W - w0);
        QPackSplit a{};
        for (int g = 0; g < G; ++g) {
            const ina_nga_params_t& q = prm[w0 + g];
            a.x[g] = x[w0 + g];
            a.hdr[g] = reinterpret_cast<u32x4*>(hdr[w0 + g]);
            a.pay[g] = reinterpret_cast<u32x4*>(pay[w0 + g]);
            a.desc[g] = desc ? reinterpret_cast<u32x2*>(desc[w0 + g]) : nullptr;
            a.bitmap[g] = q.bitmap;
            a.seq0[g] = q.seq0;
            a.fcs[g] = (uint32_t)q.count | ((uint32_t)q.flags << 8) | ((uint32_t)q.switch_id << 16);
        }
        switch (G) {
#define INA_QPS(g_) case g_: hipLaunchKernelGGL(k_qpack_nga_multi_split<g_>, grid, blk, 0, s, a, base, n, sc, \
                                                prm[0].num_slots, nch, npk); break;
            INA_QPS(1) INA_QPS(2) INA_QPS(3) INA_QPS(4) INA_QPS(5) INA_QPS(6) INA_QPS(7) INA_QPS(8)
#undef INA_QPS
        }
    }
    return check_launch("quantize_pack_nga_multi_split");
}

int ina_unpack_nga_split(const uint8_t* hdr, const uint8_t* pay, size_t npk, int V,
                         const ina_nga_fields_t* fields, int32_t* vals, ina_stream_t stream) {
    if (V <= 0 || V % 4 || V > 256) return set_error(INA_EINVAL, "V must be a multiple of 4 in [4, 256]%s", "");
    if (npk == 0) return INA_OK;
    if (!hdr || (vals && !pay)) return set_error(INA_EINVAL, "null pointer%s", "");
    if (!aligned16(hdr) || (pay && !aligned16(pay)) || (vals && !aligned16(vals)))
        return set_error(INA_EINVAL, "rows and values must be 16-byte aligned%s", "");
    hipStream_t s = hs(stream);
    if (fields) {
        NgaFieldsDev f{fields->bitmap, fields->count, fields->flags, fields->index, fields->switch_id,
                       fields->frag_id};
        hipLaunchKernelGGL(k_unpack_nga_hdr, dim3(grid_for(npk, 1)), dim3(kBlock), 0, s, hdr, npk, (size_t)16, f);
    }
    if (vals) {
        const size_t nch = npk * (size_t)V / 4;
        hipLaunchKernelGGL(k_unpack_nga_split_vals, dim3(grid_for(nch, 1, ew_grid_cap())), dim3(kBlock), 0, s,
                           reinterpret_cast<const u32x4*>(pay), nch, reinterpret_cast<u32x4*>(vals));
    }
    return check_launch("unpack_nga_split");
}

int ina_unpack_nga(const uint8_t* pkts, size_t npk, int V, size_t pstride,
                   const ina_nga_fields_t* fields, int32_t* vals, ina_stream_t stream) {
    if (V <= 0 || pstride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)V)
        return set_error(INA_EINVAL, "bad V/stride%s", "");
    if (npk == 0) return INA_OK;
    if (!pkts) return set_error(INA_EINVAL, "null packets%s", "");
    NgaFieldsDev f{};
    if (fields) f = NgaFieldsDev{fields->bitmap, fields->count, fields->flags, fields->index,
                                 fields->switch_id, fields->frag_id};
    hipStream_t s = hs(stream);
    if (vals && V % 4 == 0 && pstride % 16 == 0 && aligned16(pkts) && aligned16(vals)) {
        // flat chunk stream; 32-bit chunk indices, so huge batches go in packet ranges
        const size_t C = pstride / 16;
        const size_t per = std::max<size_t>(1, (size_t)g_launch_chunks.load() / C);
        for (size_t p0 = 0; p0 < npk; p0 += per) {
            const size_t np = npk - p0 < per ? npk - p0 : per;
            NgaFieldsDev fo = f;
            if (fo.bitmap) fo.bitmap += p0;
            if (fo.count) fo.count += p0;
            if (fo.flags) fo.flags += p0;
            if (fo.index) fo.index += p0;
            if (fo.switch_id) fo.switch_id += p0;
            if (fo.frag_id) fo.frag_id += p0;
            hipLaunchKernelGGL(k_unpack_nga_flat<INA_UNPACK_U>, dim3(grid_for(np * C, INA_UNPACK_U, g_stream_blocks)),
                               dim3(kBlock), 0, s, pkts + p0 * pstride, (uint32_t)C, (uint32_t)(V / 4),
                               (uint32_t)(np * C), fo, fields ? 1 : 0, vals + p0 * (size_t)V,
                               (uint32_t)V);
        }
    } else if (!vals && pstride % 16 == 0 && aligned16(pkts)) {
        if (fields)
            hipLaunchKernelGGL(k_unpack_nga_hdr, dim3(grid_for(npk, 1)), dim3(kBlock), 0, s, pkts, npk,
                               pstride, f);
    } else {
        hipLaunchKernelGGL(k_unpack_nga_scalar, dim3(grid_for(npk * ((size_t)V + 1), 1)), dim3(kBlock),
                           0, s, pkts, npk, V, pstride, f, vals);
    }
    return check_launch("unpack_nga");
}

int ina_apply_completed_nga(const uint8_t* pkts, size_t npk, int V, size_t pstride,
                            const uint8_t* actions, uint32_t seq0, const float* local, int k,
                            double weight_step, float* out, size_t n, uint8_t* acks,
                            size_t ack_stride, ina_stream_t stream) {
    if (int rc = check_k(k)) return rc;
    if (V <= 0 || V % 4 || V > 256) return set_error(INA_EINVAL, "V must be a multiple of 4 <= 256%s", "");
    if (pstride % 16 || pstride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)V || !aligned16(pkts))
        return set_error(INA_EINVAL, "packets must be 16-byte aligned rows of stride %% 16 == 0%s", "");
    if (acks && (ack_stride % 16 || !aligned16(acks)))
        return set_error(INA_EINVAL, "ack rows must be 16-byte aligned%s", "");
    if (npk == 0 || n == 0) return INA_OK;
    if (npk > 0x7FFFFFFFu || pstride > 0xFFFFFFFFu) return set_error(INA_EINVAL, "too many packets%s", "");
    if (!actions || !local || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    if (!aligned16(local) || !aligned16(out)) return set_error(INA_EINVAL, "local/out must be 16-byte aligned%s", "");
    const size_t nslots = (n + (size_t)V - 1) / (size_t)V;
    const uint32_t ns32 = nslots > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)nslots;
    const size_t windows = (npk + kApWin - 1) / kApWin;
    unsigned g = (unsigned)std::min<size_t>((windows + 3) / 4, 2048);
    hipLaunchKernelGGL(k_apply_completed_nga, dim3(g), dim3(kBlock), 0, hs(stream), pkts,
                       (uint32_t)npk, (uint32_t)pstride, actions, seq0, ns32, local,
                       ldexpf(1.0f, -k), (float)weight_step, out, n, acks, ack_stride, V);
    return check_launch("apply_completed_nga");
}

int ina_pack_c128(const uint32_t* gradient, int packet_num, int worker_id, uint32_t aggregator_index,
                  int tensor_index, uint8_t* pkts, ina_stream_t stream) {
    if (packet_num < 0) return set_error(INA_EINVAL, "packet_num < 0%s", "");
    if (packet_num == 0) return INA_OK;
    if (!gradient || !pkts) return set_error(INA_EINVAL, "null pointer%s", "");
    if ((uintptr_t)pkts & 3u) return set_error(INA_EINVAL, "packets must be 4-byte aligned%s", "");
    // 1 << (worker_id-1): x86 masks the shift count (communicator.cc:18, UB for 0)
    uint32_t bitmap = 1u << ((unsigned)(worker_id - 1) & 31u);
    size_t total = (size_t)packet_num * 131;
    if (total < 0xFFFFFF00u && aligned16(pkts)) {
        hipLaunchKernelGGL(k_pack_c128_x4<4>, dim3((unsigned)((total / 4 + kBlock) / kBlock)), dim3(kBlock), 0,
                           hs(stream), gradient, (uint32_t)total, bitmap, aggregator_index, tensor_index,
                           reinterpret_cast<uint32_t*>(pkts));
    } else {
        hipLaunchKernelGGL(k_pack_c128, dim3(grid_for(total, 1)), dim3(kBlock), 0, hs(stream), gradient,
                           (size_t)packet_num, bitmap, aggregator_index, tensor_index,
                           reinterpret_cast<uint32_t*>(pkts));
    }
    return check_launch("pack_c128");
}

int ina_absmax_f32(const float* x, const float* base, size_t n, float* out_dev, ina_stream_t stream) {
    if (!out_dev) return set_error(INA_EINVAL, "null out%s", "");
    hipStream_t s = hs(stream);
    if (hipMemsetAsync(out_dev, 0, sizeof(float), s) != hipSuccess)
        return set_error(INA_EHIP, "memset absmax%s", "");
    if (n == 0) return INA_OK;
    if (!x) return set_error(INA_EINVAL, "null pointer%s", "");
    const int vec = aligned16(x) && (!base || aligned16(base));
    // every block ends in one atomicMax on the same word (~11 ns each, serialised, and all
    // blocks end together), so the grid stays small: 256 workgroups 38 us, 2048 47 us, 8192
    // 86 us (ResNet-50 delta); 8 or 16 chunks in flight per lane instead of 4 were slower
    // (profiles/r02/lab/absmax_geometry_lab.log)
    hipLaunchKernelGGL(k_absmax_f32, dim3(grid_for(vec ? n / 4 + 1 : n, INA_ABSMAX_U, INA_ABSMAX_BLOCKS)), dim3(kBlock), 0,
                       s, x, base, n, vec, reinterpret_cast<uint32_t*>(out_dev));
    return check_launch("absmax_f32");
}

int ina_absmax_multi_f32(const float* const* xs, int W, const float* base, size_t n, float* out_dev,
                         ina_stream_t stream) {
    if (!out_dev) return set_error(INA_EINVAL, "null out%s", "");
    PtrPack<float> pk;
    bool al;
    if (int rc = fill_pack(pk, xs, W, al)) return rc;
    hipStream_t s = hs(stream);
    if (hipMemsetAsync(out_dev, 0, sizeof(float), s) != hipSuccess)
        return set_error(INA_EHIP, "memset absmax%s", "");
    if (n == 0) return INA_OK;
    const int vec = al && (!base || aligned16(base));
    hipLaunchKernelGGL(k_absmax_multi_f32, dim3(grid_for(vec ? n / 4 + 1 : n, 1, INA_ABSMAX_MULTI_BLOCKS)),
                       dim3(kBlock), 0, s, pk, W, base, n, vec, reinterpret_cast<uint32_t*>(out_dev));
    return check_launch("absmax_multi_f32");
}

int ina_scale_for(float absmax, int W, int bits, int* k_out) {
    // largest k with W * (absmax * 2^k + 1/2) <= 2^(bits-1) - 1: no worker value and no
    // W-way sum saturates (each quantised value rounds by at most 1/2)
    if (!k_out) return set_error(INA_EINVAL, "null k_out%s", "");
    if (W < 1 || (bits != 16 && bits != 32)) return set_error(INA_EINVAL, "W >= 1, bits 16 or 32%s", "");
    if (!(absmax >= 0.0f) || std::isinf(absmax))
        return set_error(INA_EINVAL, "absmax must be finite and >= 0%s", "");
    const double lim = (bits == 32 ? 2147483647.0 : 32767.0) / (double)W - 0.5;
    if (lim <= 0.0) return set_error(INA_EINVAL, "too many workers for this width%s", "");
    if (absmax == 0.0f) {
        *k_out = 127;
        return INA_OK;
    }
    int k = (int)std::floor(std::log2(lim / (double)absmax));
    k = k < -126 ? -126 : (k > 127 ? 127 : k);
    while (k > -126 && (double)absmax * std::ldexp(1.0, k) > lim) --k;       // guard log2 rounding
    while (k < 127 && (double)absmax * std::ldexp(1.0, k + 1) <= lim) ++k;
    *k_out = k;
    return INA_OK;
}

int ina_checksum_i32(const int32_t* x, size_t n, uint32_t* out_dev, ina_stream_t stream) {
    if (!out_dev) return set_error(INA_EINVAL, "null out%s", "");
    hipStream_t s = hs(stream);
    if (hipMemsetAsync(out_dev, 0, sizeof(uint32_t), s) != hipSuccess)
        return set_error(INA_EHIP, "memset checksum%s", "");
    if (n == 0) return INA_OK;
    if (!x) return set_error(INA_EINVAL, "null pointer%s", "");
    int vec = aligned16(x);
    hipLaunchKernelGGL(k_checksum_i32, dim3(grid_for(vec ? n / 4 + 1 : n, 1, kFaninBlocks)), dim3(kBlock), 0,
                       s, x, n, vec, out_dev);
    return check_launch("checksum_i32");
}

}  // extern "C"

#if INA_STORE_CHECK
namespace ina {
unsigned long long store_violations_kernels() {
    unsigned long long v = 0, z = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_store_violations), sizeof(v)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_store_violations), &z, sizeof(z)) != hipSuccess)
        return ~0ull;                                  // unreadable: report as a violation
    return v;
}
}  // namespace ina
#endif

#if INA_STORE_CHECK
// checked builds only (not in include/ina.h): the stream_store contract violations of every
// source since the last call, cleared by the call
extern "C" int ina_store_check_violations(unsigned long long* count) {
    if (!count) return INA_EINVAL;
    if (hipDeviceSynchronize() != hipSuccess) return INA_EHIP;
    *count = ina::store_violations_kernels() + ina::store_violations_shard() + ina::store_violations_switch();
    return INA_OK;
}
#endif
