// ina_device.h -- device-side helpers shared by the HIP sources of libina.so.
#pragma once
#include <hip/hip_runtime.h>

namespace ina {

// Streaming stores of the one-pass reduce and elementwise kernels.  INA_STORE_SC1 = 1: `global_store_dwordx{2,4}
// ... sc1` (write-through at system scope), so a launch leaves no dirty lines for the next
// dependent launch's boundary to drain (MI355X_MICROARCH.md: a boundary costs + B / 6 TB/s
// when the predecessor leaves B bytes dirty).  The headline reduce, interleaved on two
// boxes (tools/lab/store_policy_lab.py, profiles/r03/lab/store_policy_lab*.log): back to
// back 151.7 -> 150.9 and 149.2 -> 147.1 us, single launches 157.2 -> 153.1 and
// 152.7 -> 148.5 us against nt stores; default-policy stores 155.8-156.4.
// INA_STORE_SC1 = 0: the non-temporal (nt) stores of rounds 1-2.
#ifndef INA_STORE_SC1
#define INA_STORE_SC1 1
#endif
template <typename T>
__device__ __forceinline__ void stream_store(T v, T* p) {
#if INA_STORE_SC1
    static_assert(sizeof(T) == 16 || sizeof(T) == 8 || sizeof(T) == 4, "16, 8 or 4-byte stores");
    // a VALU write to the data VGPRs of a store of more than 8 bytes needs a wait state
    // after the store; the compiler's hazard recognizer does not see the store inside the
    // asm statement, so the asm carries it (without it: wrong sums at W = 16, whose
    // allocation rewrites a store's data registers right after it)
    if constexpr (sizeof(T) == 16)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (sizeof(T) == 8)
        asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#else
    __builtin_nontemporal_store(v, p);
#endif
}

// Packet kernels (pack / unpack of NGA rows) keep non-temporal stores: their rows are the
// next launch's input (the switch, the sender), and write-through made the fused worker
// pack 9 % slower in the packet path (54.7 -> 59.6 us per launch beside the switch,
// profiles/r03/lab/path_store_lab.log).
template <typename T>
__device__ __forceinline__ void packet_store(T v, T* p) {
    __builtin_nontemporal_store(v, p);
}

}  // namespace ina
