// ina_switch.hip -- the packet-stream aggregator: ngaa.p4's Ingress.apply
// (ngaa.p4:120-196), its count register (64-82), frag check (fragcheck.p4:14-57)
// and the V Processor registers (processor.p4:14-24), restated on the device.
//
// A batch of NGA-V packets in arrival order is grouped by aggregator slot with a
// stable radix sort (slot, arrival) -- slots are independent in the P4 program, so
// per-slot arrival order is all that matters -- and each slot's packets are run
// through the register state machine by ONE wave: the slot's V registers stay in
// VGPRs for the whole segment, each packet is staged through LDS (16-byte loads of
// the padded packet, byte-offset payload words at 15 + 4j extracted with
// v_alignbyte), rewritten there (running sum, collision bit) and stored back.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "ina.h"
#include "ina_internal.h"

namespace ina {

using u32x4s = uint32_t __attribute__((ext_vector_type(4)));

constexpr int kSwBlock = 256;               // 4 waves, one slot segment each
constexpr int kMaxV = 256;                  // 4 payload words per lane
constexpr int kMaxStride = 16 + 4 * kMaxV;  // 1040 B, LDS staging per wave

// Cross-lane moves by one lane as DPP row moves (measured on gfx950, tools/lab/dpp_lab.hip):
// wave_shl:1 -> lane i reads lane i+1 (lane 63 keeps its own value); wave_shr:1 -> lane i
// reads lane i-1 (lane 0 keeps its own).  One VALU op instead of an LDS ds_bpermute.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t rd_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// 1. keys: aggregator slot of each packet, or num_slots (sorts last) for packets
//    that are not this switch's (switch_check miss, ngaa.p4:27-37,184-186)
__global__ void k_switch_keys(const uint8_t* __restrict__ pkts, size_t npk, size_t stride,
                              uint32_t num_slots, int switch_id, uint32_t* __restrict__ keys,
                              uint32_t* __restrict__ ids, uint8_t* __restrict__ actions) {
    size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npk) return;
    const uint8_t* pk = pkts + p * stride;
    bool mine = switch_id >= 0 && pk[10] == (uint8_t)switch_id;
    keys[p] = mine ? rd_be32(pk + 6) % num_slots : num_slots;
    ids[p] = (uint32_t)p;
    if (!mine) actions[p] = INA_ACT_FWD_OTHER;
}

// 2. one wave per slot segment of the sorted stream
__global__ __launch_bounds__(kSwBlock) void k_switch_run(ina_switch_state_t st,
                                                         uint8_t* __restrict__ pkts, size_t npk,
                                                         size_t stride,
                                                         const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ ids,
                                                         uint8_t* __restrict__ actions) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kSwBlock / 64][kMaxStride];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const size_t pos = (size_t)blockIdx.x * (kSwBlock / 64) + wv;
    if (pos >= npk) return;
    const uint32_t slot = keys[pos];
    if (slot >= st.num_slots) return;                      // not ours: already marked
    if (pos > 0 && keys[pos - 1] == slot) return;          // not the segment head
    const int V = st.V;
    uint8_t* lds = stage[wv];
    const bool vec = (stride % 16 == 0) && (((uintptr_t)pkts & 15u) == 0);

    // slot state into registers: count, frag (scalar) and V registers (<= 4 per lane)
    uint32_t cnt = st.count[slot];
    uint32_t frag = st.frag[slot];
    uint32_t reg[kMaxV / 64];
#pragma unroll
    for (int r = 0; r < kMaxV / 64; ++r) {
        int j = lane + 64 * r;
        reg[r] = j < V ? st.regs[(size_t)slot * V + j] : 0u;
    }

    for (size_t q = pos; q < npk && keys[q] == slot; ++q) {
        const uint32_t pid = ids[q];
        uint8_t* pk = pkts + (size_t)pid * stride;
        // stage the packet in LDS
        if (vec) {
            for (size_t b = 16 * (size_t)lane; b < stride; b += 64 * 16)
                *reinterpret_cast<u32x4s*>(lds + b) = *reinterpret_cast<const u32x4s*>(pk + b);
        } else {
            for (size_t b = lane; b < stride; b += 64) lds[b] = pk[b];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t flags = lds[5];
        const uint32_t hcount = lds[4];
        const uint32_t frag_in = rd_be32(lds + 11);
        const bool is_ack = (flags >> 6) & 1u;
        uint8_t act;
        bool rewrite = false;
        if (is_ack) {                                       // reset_id (fragcheck.p4:26-31)
            frag = 0;
            act = INA_ACT_FWD_ACK;
        } else {
            if (frag == 0) frag = frag_in;                  // write_read_id (fragcheck.p4:14-24)
            if (frag != frag_in) {                          // collision (ngaa.p4:177-181)
                if (lane == 0) lds[5] = (uint8_t)(flags | INA_FLAG_COLLISION);
                act = INA_ACT_FWD_COLLISION;
                rewrite = true;
            } else {
                cnt = (cnt + 1u) & 0xFFu;                   // read_add_count (ngaa.p4:66-78)
                if (cnt == hcount) cnt = 0;
                const bool first = (cnt == 1u);
#pragma unroll
                for (int r = 0; r < kMaxV / 64; ++r) {
                    int j = lane + 64 * r;
                    if (j < V) {
                        uint32_t lo = *reinterpret_cast<const uint32_t*>(lds + 12 + 4 * j);
                        uint32_t hi = *reinterpret_cast<const uint32_t*>(lds + 16 + 4 * j);
                        uint32_t v = __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, 3));
                        reg[r] = first ? v : reg[r] + v;    // processor.p4:16-21
                    }
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int r = 0; r < kMaxV / 64; ++r) {
                    int j = lane + 64 * r;
                    if (j < V) {                            // out_value -> payload (processor.p4:22)
                        uint8_t* d = lds + 15 + 4 * j;
                        d[0] = (uint8_t)(reg[r] >> 24); d[1] = (uint8_t)(reg[r] >> 16);
                        d[2] = (uint8_t)(reg[r] >> 8);  d[3] = (uint8_t)reg[r];
                    }
                }
                act = cnt == 0 ? INA_ACT_FWD_AGG : INA_ACT_DROP;   // ngaa.p4:170-175
                rewrite = act != INA_ACT_DROP || st.write_dropped;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (rewrite) {
            if (vec) {
                for (size_t b = 16 * (size_t)lane; b < stride; b += 64 * 16)
                    *reinterpret_cast<u32x4s*>(pk + b) = *reinterpret_cast<const u32x4s*>(lds + b);
            } else {
                for (size_t b = lane; b < stride; b += 64) pk[b] = lds[b];
            }
        }
        if (lane == 0) actions[pid] = act;
        __builtin_amdgcn_wave_barrier();
    }
    // registers back to the slot
    if (lane == 0) {
        st.count[slot] = (uint8_t)cnt;
        st.frag[slot] = frag;
    }
#pragma unroll
    for (int r = 0; r < kMaxV / 64; ++r) {
        int j = lane + 64 * r;
        if (j < V) st.regs[(size_t)slot * V + j] = reg[r];
    }
}


// 2c. register-resident segment processor (stride % 16 == 0, V % 4 == 0, V <= 256).
// Lane l owns payload values 4l..4l+3.  Value j sits at bytes 15+4j, so lane l's
// values are decoded from chunks l and l+1 (16-byte chunk c = bytes 16c..16c+15) and
// chunk c (c >= 1) is re-encoded from lane c-1's values plus lane c's first value.
// Lanes 0..L (L = V/4) load chunks 0..L; when L = 64 the tail chunk 64 is held by
// lane 63 in a second register.  A wave loads up to kB packets of its segment at
// once, runs the P4 state machine over them in arrival order with the slot's
// registers in VGPRs, re-encodes and stores each packet.  Each wave owns windows of
// 64 sorted positions and runs the segments that start in them.
constexpr int kB = 8;

__device__ __forceinline__ uint32_t enc_lo(uint32_t prev, uint32_t v) {
    // LE dword: BE bytes 1..3 of prev followed by BE byte 0 of v
    return (__builtin_bswap32(prev) >> 8) | (v & 0xFF000000u);
}

__global__ __launch_bounds__(kSwBlock) void k_switch_run2(ina_switch_state_t st,
                                                          uint8_t* __restrict__ pkts, size_t npk,
                                                          size_t stride,
                                                          const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ ids,
                                                          uint8_t* __restrict__ actions) {
    const int lane = threadIdx.x & 63;
    const int V = st.V;
    const int L = V >> 2;                       // lanes holding values
    const bool vl = lane < L;
    const bool wide = L == 64;                  // tail chunk lives in lane 63's t[]
    const size_t wave = ((size_t)blockIdx.x * kSwBlock + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * kSwBlock) >> 6;
    const uint32_t NS = st.num_slots;
    // each wave takes windows of 64 sorted positions and processes the segments that
    // START in its window (a segment may run past the window's end)
    for (size_t w0 = wave * 64; w0 < npk; w0 += nwaves * 64) {
        const size_t i = w0 + (size_t)lane;
        const uint32_t ki = i < npk ? keys[i] : NS;
        const uint32_t idw = i < npk ? ids[i] : 0u;     // packet ids of the window, one load
        const uint32_t kp = (i > 0 && i <= npk) ? keys[i - 1] : 0xFFFFFFFFu;
        unsigned long long hm = __ballot(i < npk && ki < NS && (i == 0 || kp != ki));
        while (hm) {
        const int hl = __builtin_ctzll(hm);
        hm &= hm - 1;
        const size_t pos = w0 + (size_t)hl;
        const uint32_t slot = __builtin_amdgcn_readlane(ki, hl);
        // segment end: first later position whose key differs (vector scan)
        size_t end;
        {
            unsigned long long dm = __ballot(ki != slot) & ~((2ull << hl) - 1ull);
            if (dm) {
                end = w0 + (size_t)__builtin_ctzll(dm);
            } else {
                size_t j0 = w0 + 64;
                for (;;) {
                    const size_t j = j0 + (size_t)lane;
                    const bool diff = j >= npk || keys[j] != slot;
                    const unsigned long long m = __ballot(diff);
                    if (m) { end = j0 + (size_t)__builtin_ctzll(m); break; }
                    j0 += 64;
                }
            }
        }
        uint32_t cnt = st.count[slot];
        uint32_t frag = st.frag[slot];
        u32x4s reg = {0u, 0u, 0u, 0u};
        if (vl) reg = *reinterpret_cast<const u32x4s*>(st.regs + (size_t)slot * V + 4 * lane);
        for (size_t q0 = pos; q0 < end; q0 += kB) {
            const int nb = (int)((end - q0) < (size_t)kB ? (end - q0) : (size_t)kB);
            u32x4s a[kB], t[kB];
            uint32_t pid[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const size_t q = q0 + (size_t)b;
                pid[b] = b >= nb ? 0u
                         : (q < w0 + 64 ? __builtin_amdgcn_readlane(idw, (int)(q - w0)) : ids[q]);
                const u32x4s* pk = reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[b] * stride);
                a[b] = (b < nb && lane <= L) ? pk[lane] : u32x4s{0u, 0u, 0u, 0u};
                t[b] = (b < nb && wide && lane == 63) ? pk[64] : u32x4s{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                if (b >= nb) break;
                const uint32_t h1 = __builtin_amdgcn_readlane(a[b].y, 0),
                               h2 = __builtin_amdgcn_readlane(a[b].z, 0),
                               h3 = __builtin_amdgcn_readlane(a[b].w, 0);
                const uint32_t hcount = h1 & 0xFFu, flags = (h1 >> 8) & 0xFFu;
                const uint32_t frag_in = __builtin_bswap32((h2 >> 24) | (h3 << 8));
                uint8_t act;
                if ((flags >> 6) & 1u) {                     // ack: reset_id (fragcheck.p4:26-31)
                    frag = 0;
                    act = INA_ACT_FWD_ACK;
                } else {
                    if (frag == 0) frag = frag_in;           // write_read_id (fragcheck.p4:14-24)
                    if (frag != frag_in) {                   // collision (ngaa.p4:177-181)
                        if (lane == 0) a[b].y |= (uint32_t)INA_FLAG_COLLISION << 8;
                        act = INA_ACT_FWD_COLLISION;
                    } else {
                        cnt = (cnt + 1u) & 0xFFu;            // read_add_count (ngaa.p4:66-78)
                        if (cnt == hcount) cnt = 0;
                        const bool first = cnt == 1u;
                        u32x4s c;                            // chunk l+1
                        c.x = from_next_lane(a[b].x); c.y = from_next_lane(a[b].y);
                        c.z = from_next_lane(a[b].z); c.w = from_next_lane(a[b].w);
                        if (wide && lane == 63) c = t[b];
                        u32x4s v;                            // values 4l..4l+3
                        v.x = __builtin_bswap32(__builtin_amdgcn_alignbyte(c.x, a[b].w, 3));
                        v.y = __builtin_bswap32(__builtin_amdgcn_alignbyte(c.y, c.x, 3));
                        v.z = __builtin_bswap32(__builtin_amdgcn_alignbyte(c.z, c.y, 3));
                        v.w = __builtin_bswap32(__builtin_amdgcn_alignbyte(c.w, c.z, 3));
                        reg = first ? v : reg + v;           // processor.p4:16-21
                        // out_value -> payload (processor.p4:22)
                        u32x4s p;                            // lane l-1's values
                        p.x = from_prev_lane(reg.x); p.y = from_prev_lane(reg.y);
                        p.z = from_prev_lane(reg.z); p.w = from_prev_lane(reg.w);
                        if (lane == 0) {
                            a[b].w = (a[b].w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                        } else if (lane <= L) {
                            a[b].x = enc_lo(p.x, p.y);
                            a[b].y = enc_lo(p.y, p.z);
                            a[b].z = enc_lo(p.z, p.w);
                            a[b].w = lane < L ? enc_lo(p.w, reg.x)
                                              : ((__builtin_bswap32(p.w) >> 8) | (a[b].w & 0xFF000000u));
                        }
                        if (wide && lane == 63) {            // tail chunk 64 from lane 63's values
                            t[b].x = enc_lo(reg.x, reg.y);
                            t[b].y = enc_lo(reg.y, reg.z);
                            t[b].z = enc_lo(reg.z, reg.w);
                            t[b].w = (__builtin_bswap32(reg.w) >> 8) | (t[b].w & 0xFF000000u);
                        }
                        act = cnt == 0 ? INA_ACT_FWD_AGG : INA_ACT_DROP;   // ngaa.p4:170-175
                    }
                }
                if (act != INA_ACT_DROP || st.write_dropped) {
                    u32x4s* pk = reinterpret_cast<u32x4s*>(pkts + (size_t)pid[b] * stride);
                    if (lane <= L) pk[lane] = a[b];
                    if (wide && lane == 63) pk[64] = t[b];
                }
                if (lane == 0) actions[pid[b]] = act;
            }
        }
        if (lane == 0) {
            st.count[slot] = (uint8_t)cnt;
            st.frag[slot] = frag;
        }
        if (vl) *reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * lane) = reg;
        }
    }
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static int end_bit_for(uint32_t num_slots) {
    int b = 1;
    while (b < 32 && ((uint64_t)1 << b) <= (uint64_t)num_slots) ++b;
    return b;   // sentinel value num_slots fits
}

static size_t sort_temp_bytes(size_t npk, uint32_t num_slots) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)npk, 0,
                                       end_bit_for(num_slots));
    return tb;
}

}  // namespace ina

namespace ina {

// 3. ipRoute (ngaa.p4:39-61): exact match of each forwarded packet's IPv4 destination
//    against a table of <= 256 rows staged in LDS; every lane of a wave scans the same
//    row at once (LDS broadcast), first hit wins, a miss is the default drop.
__global__ __launch_bounds__(256) void k_route_ipv4(const uint8_t* __restrict__ actions,
                                                    const uint32_t* __restrict__ dst_ip,
                                                    uint32_t dst_default, size_t npk,
                                                    const uint32_t* __restrict__ keys,
                                                    const int32_t* __restrict__ ports, int nent,
                                                    int32_t* __restrict__ egress) {
    __shared__ uint32_t k_s[INA_ROUTE_MAX];
    __shared__ int32_t p_s[INA_ROUTE_MAX];
    for (int i = threadIdx.x; i < nent; i += blockDim.x) {
        k_s[i] = keys[i];
        p_s[i] = ports[i];
    }
    __syncthreads();
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < npk;
         p += (size_t)gridDim.x * blockDim.x) {
        int32_t port = INA_PORT_DROP;
        if (actions[p] != INA_ACT_DROP) {
            const uint32_t d = dst_ip ? dst_ip[p] : dst_default;
            for (int i = 0; i < nent; ++i) {
                if (k_s[i] == d) {
                    port = p_s[i];
                    break;
                }
            }
        }
        egress[p] = port;
    }
}

}  // namespace ina

using namespace ina;

extern "C" {

size_t ina_switch_scratch_bytes(size_t npkts, uint32_t num_slots) {
    if (npkts == 0 || npkts > 0x7FFFFFFFu || num_slots == 0) return 256;
    return 4 * align_up(npkts * 4, 256) + align_up(sort_temp_bytes(npkts, num_slots), 256) + 256;
}

int ina_switch_process(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                       uint8_t* actions, void* scratch, ina_stream_t stream) {
    if (!st || st->V <= 0 || st->V > kMaxV || st->num_slots == 0)
        return set_error(INA_EINVAL, "bad switch state (V in [1,256])%s", "");
    if (stride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)st->V || stride > (size_t)kMaxStride)
        return set_error(INA_EINVAL, "stride must be in [15+4V, 1040]%s", "");
    if (npk == 0) return INA_OK;
    if (npk > 0x7FFFFFFFu) return set_error(INA_EINVAL, "too many packets%s", "");
    if (!pkts || !actions || !scratch || !st->count || !st->frag || !st->regs)
        return set_error(INA_EINVAL, "null pointer%s", "");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint8_t* base = reinterpret_cast<uint8_t*>(align_up((uintptr_t)scratch, 256));
    size_t arr = align_up(npk * 4, 256);
    uint32_t* k_in = reinterpret_cast<uint32_t*>(base);
    uint32_t* k_out = reinterpret_cast<uint32_t*>(base + arr);
    uint32_t* v_in = reinterpret_cast<uint32_t*>(base + 2 * arr);
    uint32_t* v_out = reinterpret_cast<uint32_t*>(base + 3 * arr);
    void* temp = base + 4 * arr;
    size_t tb = sort_temp_bytes(npk, st->num_slots);

    unsigned g = (unsigned)((npk + 255) / 256);
    hipLaunchKernelGGL(k_switch_keys, dim3(g), dim3(256), 0, s, pkts, npk, stride, st->num_slots,
                       st->switch_id, k_in, v_in, actions);
    if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch keys launch%s", "");
    if (hipcub::DeviceRadixSort::SortPairs(temp, tb, k_in, k_out, v_in, v_out, (int)npk, 0,
                                           end_bit_for(st->num_slots), s) != hipSuccess)
        return set_error(INA_EHIP, "switch radix sort%s", "");
    const bool fast = stride % 16 == 0 && ((uintptr_t)pkts & 15u) == 0 && st->V % 4 == 0 &&
                      st->V <= kMaxV && ((uintptr_t)st->regs & 15u) == 0;
    if (fast) {
        unsigned gr = (unsigned)std::min<size_t>((npk + kSwBlock - 1) / kSwBlock, 2048);
        hipLaunchKernelGGL(k_switch_run2, dim3(gr), dim3(kSwBlock), 0, s, *st, pkts, npk, stride, k_out,
                           v_out, actions);
    } else {
        unsigned gw = (unsigned)((npk + (kSwBlock / 64) - 1) / (kSwBlock / 64));
        hipLaunchKernelGGL(k_switch_run, dim3(gw), dim3(kSwBlock), 0, s, *st, pkts, npk, stride, k_out,
                           v_out, actions);
    }
    if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch run launch%s", "");
    return INA_OK;
}

int ina_route_ipv4(const uint8_t* actions, const uint32_t* dst_ip, uint32_t dst_default,
                   size_t npk, const uint32_t* keys, const int32_t* ports, int nent,
                   int32_t* egress, ina_stream_t stream) {
    if (nent < 0 || nent > INA_ROUTE_MAX)
        return set_error(INA_EINVAL, "route table must have 0..256 rows%s", "");
    if (npk == 0) return INA_OK;
    if (!actions || !egress || (nent > 0 && (!keys || !ports)))
        return set_error(INA_EINVAL, "null pointer%s", "");
    unsigned g = (unsigned)std::min<size_t>((npk + 255) / 256, 2048);
    hipLaunchKernelGGL(k_route_ipv4, dim3(g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       actions, dst_ip, dst_default, npk, keys, ports, nent, egress);
    if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "route launch%s", "");
    return INA_OK;
}

}  // extern "C"
