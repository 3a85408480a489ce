// ina_device.h -- device-side helpers shared by the HIP sources of libina.so.
#pragma once
#include <hip/hip_runtime.h>

namespace ina {

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

// Streaming stores of the one-pass reduce and elementwise kernels.  INA_STORE_SC1 = 1: stores with
// the sc1 cache-policy bit (write-through at system scope), so a launch leaves no dirty lines for the next
// dependent launch's boundary to drain (MI355X_MICROARCH.md: a boundary costs + B / 6 TB/s
// when the predecessor leaves B bytes dirty).  The headline reduce, interleaved on two
// boxes (tools/lab/store_policy_lab.py, profiles/r03/lab/store_policy_lab*.log): back to
// back 151.7 -> 150.9 and 149.2 -> 147.1 us, single launches 157.2 -> 153.1 and
// 152.7 -> 148.5 us against nt stores; default-policy stores 155.8-156.4.
// INA_STORE_SC1 = 0: the non-temporal (nt) stores of rounds 1-2.
//
// The sc1 store is a compiler builtin (`__builtin_amdgcn_raw_buffer_store_b*`, aux bit 4 =
// SC1 on gfx950), never inline asm: the compiler then owns the store's wait states and
// hazards (round 3's asm store needed a hand-placed s_nop -- a VALU overwrite of the data
// VGPRs of a >8-byte store -- and gave wrong W = 16 sums without it).  A buffer store needs
// a wave-uniform base: the wave's first active lane's address (readfirstlane) is the
// resource base and every lane stores at its byte distance from it.
// CONTRACT: at every call site a lane's address is >= the first active lane's (lanes
// store at wave_base + lane * sizeof(T), or at rising packet / slot positions), so the
// distance is small and positive.  Every caller in csrc/ keeps it (a lane below the first
// one would fall outside the resource and its store would be dropped -- which the parity
// tests of every kernel would see).  A per-store check with an ordinary-store fallback
// measured 4-7 % slower on the streaming kernels and 2.3x on the int16 reduce (the branch
// split the unrolled loop and doubled its registers; profiles/r04/lab/store_builtin_lab.log).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "stream_store's SC1 cache-policy bit (aux bit 4) is the gfx942 / gfx950 encoding"
#endif
#ifndef INA_STORE_SC1
#define INA_STORE_SC1 1
#endif
// buffer resource word 3 for a raw (stride 0, untyped) gfx9 buffer: 32-bit data format
constexpr int kRawBufferWord3 = 0x00020000;
constexpr int kAuxSC1 = 16;
// INA_STORE_CHECK = 1 (checked builds: make BUILD=build_chk OUT=... EXTRA=-DINA_STORE_CHECK=1):
// every stream_store verifies the CONTRACT above -- its lane's distance from the wave's base is
// in [0, 2^31 - sizeof(T)] -- and counts each store that breaks it in a per-source device
// counter (ina_store_check_violations reads and clears them; tests/test_gpu_store_views.py and
// the conftest hook of a checked run assert zero).  Counted, not trapped: a trap is a GPU fault,
// and on this pool a faulting kernel can take the machine's GPUs down with it.
#ifndef INA_STORE_CHECK
#define INA_STORE_CHECK 0
#endif
#if INA_STORE_CHECK
static __device__ unsigned long long g_store_violations;   // one per source file
#endif
template <typename T>
__device__ __forceinline__ void stream_store(T v, T* p) {
#if INA_STORE_SC1
    static_assert(sizeof(T) == 16 || sizeof(T) == 8 || sizeof(T) == 4, "16, 8 or 4-byte stores");
    const uint64_t a = (uint64_t)(uintptr_t)p;
    // (readfirstlane returns int: each half goes through uint32_t, or the low half's bit 31
    // would sign-extend into the high half)
    const uint64_t a0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t d = (uint32_t)(a - a0);
#if INA_STORE_CHECK
    const int64_t dist = (int64_t)(a - a0);
    if (dist < 0 || dist > (int64_t)0x7FFFFFFF - (int64_t)sizeof(T))
        atomicAdd(&g_store_violations, 1ull);
#endif
    __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)a0, 0, 0x7FFFFFFF, kRawBufferWord3);
    if constexpr (sizeof(T) == 16)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, (int)d, 0, kAuxSC1);
    else if constexpr (sizeof(T) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)d, 0, kAuxSC1);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)d, 0, kAuxSC1);
#else
    __builtin_nontemporal_store(v, p);
#endif
}

// Packet kernels (pack / unpack of NGA rows) keep non-temporal stores: their rows are the
// next launch's input (the switch, the sender), and write-through made the fused worker
// pack 9 % slower in the packet path (54.7 -> 59.6 us per launch beside the switch,
// profiles/r03/lab/path_store_lab.log).
#ifndef INA_PACKET_STORE
#define INA_PACKET_STORE 0            // 0 non-temporal, 1 write-through (stream_store), 2 default
#endif
template <typename T>
__device__ __forceinline__ void packet_store(T v, T* p) {
#if INA_PACKET_STORE == 1
    stream_store(v, p);
#elif INA_PACKET_STORE == 2
    *p = v;
#else
    __builtin_nontemporal_store(v, p);
#endif
}

}  // namespace ina
