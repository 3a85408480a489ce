// gather_lab.hip -- experiment only: the memory traffic of the switch run kernel
// (k_switch_run2) without its state machine, to price the gather itself.  Same sorted
// (slot, packet id) arrays, same windows of 16 sorted positions per wave, same 8-packet
// batches (lane l: 16-byte chunk l of each packet, the tail chunk 64 in lane b), then per
// segment: a 1,024-byte register row store and, in mode 2, the 1,040-byte forwarded
// packet store over the segment's last packet.  mode 0: reads only; 1: + register rows;
// 2: + forwarded packets.  The payload words are only XOR-folded (no decode), so what is
// left against k_switch_run2 is its decode / count / frag / re-encode work.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/lab/gather_lab.so tools/lab/gather_lab.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ keys,
                                                const uint32_t* __restrict__ ids, uint8_t* pkts,
                                                size_t npk, size_t stride, uint32_t* __restrict__ regs,
                                                uint32_t win, int mode) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (size_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const size_t nwaves = ((size_t)gridDim.x * 256) >> 6;
    for (size_t w0 = wave * win; w0 < npk; w0 += nwaves * win) {
        const size_t i = w0 + (size_t)lane;
        const uint32_t ki = i < npk ? keys[i] : 0xFFFFFFFFu;
        const uint32_t idw = i < npk ? ids[i] : 0u;
        const uint32_t kp = (i > 0 && i <= npk) ? keys[i - 1] : 0xFFFFFFFFu;
        const bool head = (uint32_t)lane < win && i < npk && (i == 0 || kp != ki);
        unsigned long long hm = __ballot(head);
        while (hm) {
            const int hl = __builtin_ctzll(hm);
            hm &= hm - 1;
            const uint32_t slot = __builtin_amdgcn_readlane(ki, hl);
            size_t end;
            {
                unsigned long long dm = __ballot(ki != slot) & ~((2ull << hl) - 1ull);
                if (dm) {
                    end = w0 + (size_t)__builtin_ctzll(dm);
                } else {
                    size_t j0 = w0 + 64;
                    for (;;) {
                        const size_t j = j0 + (size_t)lane;
                        const unsigned long long m = __ballot(j >= npk || keys[j] != slot);
                        if (m) { end = j0 + (size_t)__builtin_ctzll(m); break; }
                        j0 += 64;
                    }
                }
            }
            u32x4 acc = {0u, 0u, 0u, 0u};
            uint32_t last = 0;
            for (size_t q0 = w0 + (size_t)hl; q0 < end; q0 += 8) {
                const int nb = (int)((end - q0) < 8 ? (end - q0) : 8);
                uint32_t pid[8];
                const uint32_t my = lane < nb ? ids[q0 + (size_t)lane] : 0u;
#pragma unroll
                for (int b = 0; b < 8; ++b) pid[b] = __builtin_amdgcn_readlane(my, b < nb ? b : 0);
                uint32_t mypid = pid[0];
#pragma unroll
                for (int b = 1; b < 8; ++b) mypid = lane == b ? pid[b] : mypid;
                const u32x4 tl = *(reinterpret_cast<const u32x4*>(pkts + (size_t)mypid * stride) + 64);
                u32x4 a[8];
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    a[b] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pkts + (size_t)pid[b] * stride) + lane);
#pragma unroll
                for (int b = 0; b < 8; ++b) acc ^= a[b];
                acc ^= tl;
                last = pid[nb - 1];
            }
            if (mode >= 1) reinterpret_cast<u32x4*>(regs + (size_t)slot * 256)[lane] = acc;
            if (mode >= 2) {
                reinterpret_cast<u32x4*>(pkts + (size_t)last * stride)[lane] = acc;
                if (lane == 63) reinterpret_cast<u32x4*>(pkts + (size_t)last * stride)[64] = acc;
            }
        }
    }
}

extern "C" int lab_gather(const uint32_t* keys, const uint32_t* ids, uint8_t* pkts, size_t npk, size_t stride,
                          uint32_t* regs, int win, int mode, void* stream) {
    const size_t per_block = (size_t)win * 4;
    const unsigned gr = (unsigned)((npk + per_block - 1) / per_block);
    hipLaunchKernelGGL(k_gather, dim3(gr), dim3(256), 0, (hipStream_t)stream, keys, ids, pkts, npk, stride, regs,
                       (uint32_t)win, mode);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
