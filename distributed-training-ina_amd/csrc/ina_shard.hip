// ina_shard.hip -- the int16 saturating wire under slot-range sharding (SURVEY.md 8e,
// BASELINE config 4 semantics carried across GPUs).
//
// The switch's narrow path marks a slot whose sum does not fit with the ngaa_h overflow
// bit (headers.p4:30) while the Processor add itself is a plain register add
// (processor.p4:14-24).  On one GPU the int16 path accumulates the W workers exactly in
// int32 and saturates once (ina_quantize_reduce_f32_i16_sat).  Across GPUs the sum goes
// through an RCCL reduce-scatter, and saturation is not associative, so the ranks never
// reduce int16 values: each rank widens its saturated int16 quantisation into one int32
// "wire" word
//
//     wire = q16(x) + (sat(x) << 22)      sat = 1 when x clamped or was NaN
//
// and the wires are summed by an ordinary int32 SUM.  With at most 64 ranks the low 22
// bits carry sum q16 in [-2^21, 2^21) exactly and the bits above count the ranks whose
// value saturated, so one collective carries both the sum and the per-element saturation
// flags.  The owner of a shard decodes it once: out = sat16(sum q16), flag = any
// saturation, and the result equals the single-GPU path bit for bit.
//
// Both kernels stream 16 B per lane (global_load_dwordx4, non-temporal: every byte is
// touched once) over a grid-stride loop; HBM-bound at 8 B/value (quantise: 4 in, 4 out)
// and 4 + 2 + 4 B/value (finish: wire in, int16 + fp32 out).
#include <hip/hip_runtime.h>

#include <cmath>

#include "ina.h"
#include "ina_internal.h"
#include "ina_device.h"

namespace ina {
namespace {

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
using u32x2 = uint32_t __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));

constexpr int kBlk = 256;
constexpr int kWireShift = INA_I16_WIRE_SHIFT;   // 22
constexpr int32_t kWireHalf = 1 << (kWireShift - 1);

// the quantiser of ina_quantize_f32_i16_sat: sat16(rne(x * 2^k)), NaN -> 0 (flagged)
__device__ __forceinline__ int32_t q16w(float x, float s) {
    const float y = __builtin_rintf(x * s);
    const float c = __builtin_amdgcn_fmed3f(y, -32768.0f, 32767.0f);   // one v_med3_f32
    const int32_t v = (y != y) ? 0 : (int32_t)c;
    const int32_t sat = !(c == y);               // clamped, +-inf or NaN
    return v + (sat << kWireShift);
}

// decoded shard value: sum q16 and whether anything saturated (a rank, or the sum)
__device__ __forceinline__ int32_t finish1(uint32_t w, bool& sat) {
    const int32_t s = (int32_t)w;
    const int32_t c = (s + kWireHalf) >> kWireShift;     // ranks that saturated (>= 0)
    const int32_t v = s - (int32_t)((uint32_t)c << kWireShift);
    sat |= c != 0;
    const bool hi = v > 32767, lo = v < -32768;
    sat |= hi | lo;
    return hi ? 32767 : (lo ? -32768 : v);
}

__global__ __launch_bounds__(kBlk) void k_quantize_i16_wire(const float* __restrict__ x,
                                                            int32_t* __restrict__ wire, size_t n,
                                                            float s, int vec) {
    const size_t tid = (size_t)blockIdx.x * kBlk + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlk;
    const size_t n4 = vec ? n / 4 : 0;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    u32x4* w4 = reinterpret_cast<u32x4*>(wire);
    for (size_t i = tid; i < n4; i += stride) {
        const f32x4 v = __builtin_nontemporal_load(x4 + i);
        u32x4 r;
        r.x = (uint32_t)q16w(v.x, s); r.y = (uint32_t)q16w(v.y, s);
        r.z = (uint32_t)q16w(v.z, s); r.w = (uint32_t)q16w(v.w, s);
        stream_store(r, w4 + i);
    }
    for (size_t i = 4 * n4 + tid; i < n; i += stride) wire[i] = q16w(x[i], s);
}

// Summed wire shard -> int16 (out16) and/or dequantised fp32 (y), per-slot flags.
// Lane l of a wave holds the 4 values at 4(base + l); with V/4 a power of two <= 64 a
// slot is V/4 adjacent lanes, and the group's first lane writes the slot's flag from a
// wave ballot (one writer per slot: no atomics, no pre-zeroing).  The trip count is
// uniform per wave so the ballot is convergent.
__global__ __launch_bounds__(kBlk) void k_i16_wire_finish_vec(const int32_t* __restrict__ wsum,
                                                              size_t n, float inv, int lps, int V,
                                                              int16_t* __restrict__ out16,
                                                              float* __restrict__ y,
                                                              uint8_t* __restrict__ ovf) {
    const size_t tid = (size_t)blockIdx.x * kBlk + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * kBlk;
    const int lane = threadIdx.x & 63;
    const size_t nch = (n + 3) / 4;
    for (size_t base = tid & ~(size_t)63; base < nch; base += stride) {
        const size_t i = base + lane;
        const size_t e = 4 * i;
        bool sat = false;
        if (e + 4 <= n) {
            const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wsum) + i);
            const int32_t a = finish1(w.x, sat), b = finish1(w.y, sat);
            const int32_t c = finish1(w.z, sat), d = finish1(w.w, sat);
            if (out16) {
                u32x2 o;
                o.x = (uint32_t)(uint16_t)a | ((uint32_t)b << 16);
                o.y = (uint32_t)(uint16_t)c | ((uint32_t)d << 16);
                stream_store(o, reinterpret_cast<u32x2*>(out16 + e));
            }
            if (y) {
                f32x4 f;
                f.x = (float)a * inv; f.y = (float)b * inv; f.z = (float)c * inv; f.w = (float)d * inv;
                stream_store(f, reinterpret_cast<f32x4*>(y + e));
            }
        } else if (e < n) {
            for (size_t j = e; j < n; ++j) {
                const int32_t r = finish1((uint32_t)wsum[j], sat);
                if (out16) out16[j] = (int16_t)r;
                if (y) y[j] = (float)r * inv;
            }
        }
        const unsigned long long m = __ballot(sat);
        if (ovf && e < n && (lane & (lps - 1)) == 0) {
            const int g0 = lane & ~(lps - 1);
            const unsigned long long gm = (lps == 64) ? ~0ull : (((1ull << lps) - 1ull) << g0);
            ovf[e / (size_t)V] = (m & gm) ? 1 : 0;
        }
    }
}

// any alignment / any V: flags pre-zeroed by the caller, saturating elements store 1
__global__ __launch_bounds__(kBlk) void k_i16_wire_finish_scalar(const int32_t* __restrict__ wsum,
                                                                 size_t n, float inv, int V,
                                                                 int16_t* __restrict__ out16,
                                                                 float* __restrict__ y,
                                                                 uint8_t* __restrict__ ovf) {
    const size_t stride = (size_t)gridDim.x * kBlk;
    for (size_t i = (size_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += stride) {
        bool sat = false;
        const int32_t r = finish1((uint32_t)wsum[i], sat);
        if (out16) out16[i] = (int16_t)r;
        if (y) y[i] = (float)r * inv;
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
}

inline unsigned grid_of(size_t items) {
    size_t g = (items + kBlk - 1) / kBlk;
    const size_t cap = (size_t)ew_grid_cap();       // the elementwise kernels' cap (tuning key 14)
    if (g > cap) g = cap;                           // grid-stride beyond
    return g ? (unsigned)g : 1u;
}
inline bool al(const void* p, unsigned a) { return ((uintptr_t)p % a) == 0; }

}  // namespace
}  // namespace ina

using namespace ina;

extern "C" {

int ina_quantize_f32_i16_wire(const float* x, int32_t* wire, size_t n, int k, ina_stream_t stream) {
    if (k < -126 || k > 127) return set_error(INA_EINVAL, "k out of range [-126,127]%s", "");
    if (n == 0) return INA_OK;
    if (!x || !wire) return set_error(INA_EINVAL, "null pointer%s", "");
    const int vec = al(x, 16) && al(wire, 16);
    hipLaunchKernelGGL(k_quantize_i16_wire, dim3(grid_of(vec ? n / 4 + 1 : n)), dim3(kBlk), 0,
                       reinterpret_cast<hipStream_t>(stream), x, wire, n, ldexpf(1.0f, k), vec);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? INA_OK : set_error(INA_EHIP, "quantize_i16_wire: %s", hipGetErrorString(e));
}

int ina_i16_wire_finish(const int32_t* wire_sum, size_t n, int k, int V, int16_t* out16, float* y,
                        uint8_t* overflow_per_slot, ina_stream_t stream) {
    if (k < -126 || k > 127) return set_error(INA_EINVAL, "k out of range [-126,127]%s", "");
    if (V <= 0) return set_error(INA_EINVAL, "V must be > 0%s", "");
    if (n == 0) return INA_OK;
    if (!wire_sum) return set_error(INA_EINVAL, "null pointer%s", "");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float inv = ldexpf(1.0f, -k);
    const int l = V / 4;
    const bool ballot = V % 4 == 0 && l >= 1 && l <= 64 && (l & (l - 1)) == 0;
    const bool vec = al(wire_sum, 16) && (!out16 || al(out16, 8)) && (!y || al(y, 16));
    if (vec && (ballot || !overflow_per_slot)) {
        hipLaunchKernelGGL(k_i16_wire_finish_vec, dim3(grid_of((n + 3) / 4)), dim3(kBlk), 0, s,
                           wire_sum, n, inv, ballot ? l : 1, V, out16, y, overflow_per_slot);
    } else {
        if (overflow_per_slot &&
            hipMemsetAsync(overflow_per_slot, 0, (n + (size_t)V - 1) / (size_t)V, s) != hipSuccess)
            return set_error(INA_EHIP, "memset overflow flags%s", "");
        hipLaunchKernelGGL(k_i16_wire_finish_scalar, dim3(grid_of(n)), dim3(kBlk), 0, s, wire_sum, n,
                           inv, V, out16, y, overflow_per_slot);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? INA_OK : set_error(INA_EHIP, "i16_wire_finish: %s", hipGetErrorString(e));
}

}  // extern "C"

#if INA_STORE_CHECK
namespace ina {
unsigned long long store_violations_shard() {
    unsigned long long v = 0, z = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_store_violations), sizeof(v)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_store_violations), &z, sizeof(z)) != hipSuccess)
        return ~0ull;                                  // unreadable: report as a violation
    return v;
}
}  // namespace ina
#endif
