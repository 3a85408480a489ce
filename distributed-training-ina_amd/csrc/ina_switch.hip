// ina_switch.hip -- the packet-stream aggregator: ngaa.p4's Ingress.apply
// (ngaa.p4:120-196), its count register (64-82), frag check (fragcheck.p4:14-57)
// and the V Processor registers (processor.p4:14-24), restated on the device.
//
// A batch of NGA-V packets in arrival order is grouped by aggregator slot with a
// stable sort (slot, arrival) -- slots are independent in the P4 program, so per-slot
// arrival order is all that matters: by default one global pass on the key's high digit
// and one workgroup per bucket of slots on the low digit (k_rs_local), else LSD digit
// passes or a one-workgroup bitonic sort for small batches.  Each slot's packets are
// then run through the register state machine by ONE wave (k_switch_run2): the slot's V
// registers stay in VGPRs for the whole segment, lane l holds 16-byte chunk l of up to 8
// packets at once, payload words at byte 15 + 4j are decoded with v_alignbyte from the
// neighbouring lane's chunk (DPP), and a forwarded packet is re-encoded from the
// registers.  Layouts that kernel does not take (V % 4 != 0, unaligned rows) run
// k_switch_run, which stages each packet through LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>

#include "ina.h"
#include "ina_internal.h"

namespace ina {

using u32x4s = uint32_t __attribute__((ext_vector_type(4)));
using f32x4s = float __attribute__((ext_vector_type(4)));

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

// threadIdx.x >> 6 is the same in every lane of a wave, but the compiler cannot see
// that: without readfirstlane everything derived from it (chunk/window loops, the
// slot state machine) is treated as divergent -- VGPR state and exec-mask branches.
__device__ __forceinline__ int wave_in_block() {
    return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

__device__ __forceinline__ uint32_t rd_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// ---- stable LSD radix sort of (slot key, packet id) --------------------------------
// The P4 registers see each slot's packets in arrival order, so the batch is grouped by
// slot with a STABLE sort.  Keys need only ceil(log2(num_slots + 1)) bits (18 at 2^17
// slots), so the sort is 1-3 digit passes of <= 9 bits.  A block owns a chunk of 4096
// consecutive items (1024 / 2048 for smaller batches, see sort_plan), its wave w the w-th
// quarter of them (rounds of 64, in order; all loads issued up front):
//   hist     the chunk's digit counts (LDS) -> cnt[digit][chunk]
//   colscan  one wave per digit: exclusive scan along the chunks (in place) + the
//            digit's total
//   scatter  base(digit, chunk, wave) = exclusive scan of the digit totals + the
//            column prefix + the counts of the chunk's earlier waves; inside a round an
//            item's rank is the number of lower lanes with the same digit (ballots over
//            its bits)
// so order is kept across rounds, lanes, waves and chunks.  (rocprim's radix sort ran
// ~130 us at 819,200 pairs: 10 dependent merge passes, or onesweep + lookback resets.)
constexpr int kRsMaxBits = 9;
constexpr int kRsBins = 1 << kRsMaxBits;     // 512
#ifndef INA_RS_WAVES
#define INA_RS_WAVES 4
#endif
#ifndef INA_RS_ROUNDS
#define INA_RS_ROUNDS 16
#endif
constexpr int kRsRounds = INA_RS_ROUNDS;
#ifndef INA_RS_ROUNDS_SMALL
#define INA_RS_ROUNDS_SMALL 4
#endif
#ifndef INA_RS_SMALL_ITEMS
#define INA_RS_SMALL_ITEMS 262144
#endif
#ifndef INA_RS_ROUNDS_MID
#define INA_RS_ROUNDS_MID 8
#endif
#ifndef INA_RS_MID_ITEMS
#define INA_RS_MID_ITEMS 524288
#endif
constexpr int kRsBlock = 64 * INA_RS_WAVES;
constexpr int kRsWaves = kRsBlock / 64;
static_assert(kRsBins % kRsBlock == 0, "digits split evenly over the block's threads");

__device__ __forceinline__ unsigned long long lanes_with_digit(uint32_t d, int bits, bool valid) {
    unsigned long long m = __ballot(valid);
    for (int b = 0; b < bits; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long mb = __ballot(bit);
        m &= bit ? mb : ~mb;
    }
    return m;
}

// inclusive wave64 scan in DPP (no LDS round trips): Hillis-Steele inside each 16-lane
// row with row_shr:1,2,4,8 (bound_ctrl: lanes shifted in from outside the row read 0),
// then row_bcast:15 adds row r-1's last lane into rows 1 and 3 and row_bcast:31 adds
// lane 31 into rows 2 and 3 (GFX9 DPP; disabled rows keep old = 0)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// LDS digit count from every lane of a wave (call convergent; `valid` masks lanes out).
// Neighbouring packets usually share their higher digits (a worker's consecutive slots),
// and 64 same-address LDS atomics serialise, so a wave whose valid lanes all hold one
// digit adds its popcount once.
__device__ __forceinline__ void lds_count(uint32_t* h, uint32_t d, bool valid) {
    const unsigned long long act = __ballot(valid);
    if (!act) return;
    const int first = __builtin_ctzll(act);
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, first);
    const unsigned long long same = __ballot(valid && d == d0);
    if (same == act) {
        if ((int)(threadIdx.x & 63) == first) atomicAdd(&h[d0], (uint32_t)__builtin_popcountll(act));
    } else if (valid) {
        atomicAdd(&h[d], 1u);
    }
}

// Stable scatter of one sort tile (both sort paths): on entry base[w][d] holds wave w's
// count of digit d and gst[d] the tile's first output position for digit d; an item goes
// to gst[d] + the counts of its digit in earlier waves and rounds + its rank among this
// round's lanes with the same digit (ballots over the digit's bits).  Staging the tile in
// LDS first, so each digit leaves as one contiguous run, measured no faster (pass 0
// 15.1 -> 17.9 us, pass 1 17.9 -> 17.3 us at 819,200 packets: the passes are bound by
// their dependent phases, not by the scattered stores; profiles/r02/lab/switch_sort_lab)
template <int R, int NW = kRsWaves>
__device__ __forceinline__ void rs_tile_scatter(const uint32_t (&k)[R], const uint32_t (&v)[R],
                                                size_t i0, size_t n, int shift, int bits,
                                                uint32_t (*base)[kRsBins], const uint32_t* gst,
                                                uint32_t* __restrict__ kout,
                                                uint32_t* __restrict__ vout, int rw = R) {
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const uint32_t nb = 1u << bits;
    constexpr int kThr = NW * 64;
    constexpr int kDPT = (kRsBins + kThr - 1) / kThr;
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kThr;
        if (d >= nb) continue;
        uint32_t b = gst[d];
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const uint32_t cw = base[w][d];
            base[w][d] = b;
            b += cw;
        }
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r >= rw || i0 - (size_t)lane + (size_t)r * 64 >= n) break;   // wave-uniform
        const bool valid = i0 + (size_t)r * 64 < n;
        const uint32_t d = (k[r] >> shift) & (nb - 1);
        const unsigned long long pm = lanes_with_digit(d, bits, valid);
        const uint32_t rank = (uint32_t)__builtin_popcountll(pm & below);
        const uint32_t b0 = base[wv][d];
        if (valid) {
            kout[b0 + rank] = k[r];
            vout[b0 + rank] = v[r];
            if (rank == 0) base[wv][d] = b0 + (uint32_t)__builtin_popcountll(pm);
        }
    }
}

// 1. keys: aggregator slot of each packet, or num_slots (sorts last) for packets that
//    are not this switch's (switch_check miss, ngaa.p4:27-37,184-186); fused with the
//    first digit pass's chunk histogram.
constexpr uint32_t kAckBit = 0x80000000u;
template <int R, bool kDesc, int NW = kRsWaves>
__global__ __launch_bounds__(NW * 64) void k_switch_keys(const uint8_t* __restrict__ pkts,
                                                          const uint2* __restrict__ desc,
                                                          size_t npk, size_t stride,
                                                          uint32_t num_slots, int switch_id,
                                                          uint32_t* __restrict__ keys,
                                                          uint8_t* __restrict__ actions, int bits,
                                                          int shift, uint32_t* __restrict__ hist,
                                                          size_t nch, int ack_hint) {
    __shared__ uint32_t h[kRsBins];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const size_t c = blockIdx.x;
    const uint32_t nb = 1u << bits;
    for (uint32_t d = threadIdx.x; d < nb; d += NW * 64) h[d] = 0;
    __syncthreads();
    const size_t p0 = c * (NW * 64 * R) + (size_t)wv * (64 * R) + (size_t)lane;
    uint32_t idx[R], sid[R], ack[R];
    if (kDesc) {                                               // descriptors: header bytes 4..11
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t p = p0 + (size_t)r * 64;
            const uint2 d = p < npk ? desc[p] : uint2{0u, 0u};
            idx[r] = __builtin_bswap32((d.x >> 16) | (d.y << 16));
            sid[r] = (d.y >> 16) & 0xFFu;
            ack[r] = (d.x >> 14) & 1u;
        }
    } else if ((stride & 3) == 0 && ((uintptr_t)pkts & 3u) == 0) {   // header bytes 4..11
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t p = p0 + (size_t)r * 64;
            uint32_t w1 = 0, w2 = 0;
            if (p < npk) {
                const uint32_t* pk = reinterpret_cast<const uint32_t*>(pkts + p * stride);
                w1 = pk[1];
                w2 = pk[2];
            }
            idx[r] = __builtin_bswap32((w1 >> 16) | (w2 << 16));
            sid[r] = (w2 >> 16) & 0xFFu;
            ack[r] = (w1 >> 14) & 1u;                          // flags byte 5, bit 6
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t p = p0 + (size_t)r * 64;
            idx[r] = p < npk ? rd_be32(pkts + p * stride + 6) : 0u;
            sid[r] = p < npk ? pkts[p * stride + 10] : 0u;
            ack[r] = p < npk ? (pkts[p * stride + 5] >> 6) & 1u : 0u;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const size_t p = p0 + (size_t)r * 64;
        const bool mine = switch_id >= 0 && sid[r] == (uint32_t)(uint8_t)switch_id;
        const uint32_t key = mine ? idx[r] % num_slots : num_slots;
        if (p < npk) {
            // bit 31 carries "PS ack" through the sort (the digit passes never read it)
            keys[p] = key | ((ack_hint && mine && ack[r]) ? kAckBit : 0u);
            if (!mine) actions[p] = INA_ACT_FWD_OTHER;
        }
        lds_count(h, (key >> shift) & (nb - 1), p < npk);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nb; d += NW * 64) hist[d * nch + c] = h[d];
}

// 1b. batches of at most kSmallBatch packets (recvmmsg-sized, where launch latency and not
//     bandwidth is the cost): keys and the whole sort in ONE workgroup.  The (slot, packet
//     id) pairs are unique 64-bit values, so sorting them -- a bitonic network in LDS --
//     gives the stable slot order with no rank bookkeeping; then the run kernel: two
//     launches instead of seven.
constexpr int kSmallBatch = 4096;                 // LDS capacity of the one-workgroup sort
#ifndef INA_SWITCH_SMALL_MAX
#define INA_SWITCH_SMALL_MAX 2048
#endif
static_assert(INA_SWITCH_SMALL_MAX <= kSmallBatch, "small path limited by its LDS");
constexpr int kSmallBlock = 1024;
// ina_set_tuning key 9: the largest batch the one-workgroup sort takes (0: never; 1: the
// default, INA_SWITCH_SMALL_DEFAULT; 2..INA_SWITCH_SMALL_MAX: that many packets).  Above
// ~700 packets the bucket sort is faster (tiny_lab: 1,024 packets 26.6 vs 25.2 us, 2,048
// 37.5 vs 25.3; 512: 23.1 vs 24.0 -- profiles/r02/lab/tiny_lab.log)
#ifndef INA_SWITCH_SMALL_DEFAULT
#define INA_SWITCH_SMALL_DEFAULT 768
#endif
static std::atomic<int> g_small_sort{INA_SWITCH_SMALL_DEFAULT};
#ifndef INA_SWITCH_TINY_MAX
#define INA_SWITCH_TINY_MAX 128                // one-launch path (k_switch_tiny) up to this many packets (tiny_lab: break-even ~150)
#endif
static std::atomic<int> g_switch_win{0};   // ina_set_tuning key 10: run-kernel window (0: auto)
static std::atomic<int> g_ack_fast{1};     // ina_set_tuning key 11: lone-ack lane path (0: off)
// ina_set_tuning key 12, the slot sort: 0 auto (bucket + local for two-digit keys, else the
// digit passes), 1 one-sweep, 2 bucket + local where it applies, 3 hist/colscan/scatter
// digit passes (r01).  Bucket + local measured 265.3 -> 251.0 us against the digit passes
// at 819,200 NGA-256 packets with descriptors (profiles/r02/lab/switch_sort_lab_hyb.json)
static std::atomic<int> g_sort_mode{0};
static std::atomic<int> g_os_rounds{0};    // ina_set_tuning key 13: sort tile rounds (0 auto, 4/8/16)
int set_sort_mode(int v) {
    if (v < 0 || v > 3) return INA_EINVAL;
    g_sort_mode = v;
    return INA_OK;
}
int set_os_rounds(int v) {
    if (v != 0 && v != 4 && v != 8 && v != 16) return INA_EINVAL;
    g_os_rounds = v;
    return INA_OK;
}
int set_ack_fast(int v) {
    g_ack_fast = v ? 1 : 0;
    return INA_OK;
}
int set_switch_win(int v) {
    if (v < 0 || v > 64) return INA_EINVAL;
    g_switch_win = v;
    return INA_OK;
}
static std::atomic<int> g_tiny_max{INA_SWITCH_TINY_MAX};   // ina_set_tuning key 15 (0: off)
int set_tiny_max(int v) {
    if (v < 0 || v > INA_SWITCH_SMALL_MAX) return INA_EINVAL;
    g_tiny_max = v;
    return INA_OK;
}
int set_small_sort(int v) {
    if (v < 0 || v > INA_SWITCH_SMALL_MAX) return INA_EINVAL;
    g_small_sort = v == 1 ? INA_SWITCH_SMALL_DEFAULT : v;
    return INA_OK;
}

// T = uint32_t packs (slot << 12 | id) when num_slots + 1 <= 2^20, else uint64_t (slot << 32
// | id).  Compare-exchange stages with j < 64 pair elements inside one wave's 64-element
// groups, so they need only a wave barrier; the 21 stages with j >= 64 (M = 4096) need
// the workgroup's.
template <typename T, int kIdBits>
__device__ __forceinline__ void switch_sort_small_body(
        const uint8_t* __restrict__ pkts, uint32_t npk, size_t stride, uint32_t num_slots,
        int switch_id, uint8_t* __restrict__ actions, uint32_t* __restrict__ keys,
        uint32_t* __restrict__ ids) {
    __shared__ T v[kSmallBatch];
    uint32_t M = 1;
    while (M < npk) M <<= 1;
    const bool al4 = (stride & 3) == 0 && ((uintptr_t)pkts & 3u) == 0;
    for (uint32_t p = threadIdx.x; p < M; p += kSmallBlock) {
        T c = ~(T)0;                                        // padding sorts last
        if (p < npk) {
            const uint8_t* pk = pkts + (size_t)p * stride;
            uint32_t idx, sid;
            if (al4) {                                      // header bytes 4..11
                const uint32_t w1 = reinterpret_cast<const uint32_t*>(pk)[1];
                const uint32_t w2 = reinterpret_cast<const uint32_t*>(pk)[2];
                idx = __builtin_bswap32((w1 >> 16) | (w2 << 16));
                sid = (w2 >> 16) & 0xFFu;
            } else {
                idx = rd_be32(pk + 6);
                sid = pk[10];
            }
            const bool mine = switch_id >= 0 && sid == (uint32_t)(uint8_t)switch_id;
            const uint32_t key = mine ? idx % num_slots : num_slots;
            if (!mine) actions[p] = INA_ACT_FWD_OTHER;      // switch_check miss, ngaa.p4:184-186
            c = ((T)key << kIdBits) | (T)p;
        }
        v[p] = c;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= M; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < M; i += kSmallBlock) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const T a = v[i], b = v[l];
                    if ((a > b) == ((i & k) == 0)) {
                        v[i] = b;
                        v[l] = a;
                    }
                }
            }
            if (j > 32) {
                __syncthreads();
            } else {                                        // partners in the same wave
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        __syncthreads();
    }
    for (uint32_t p = threadIdx.x; p < npk; p += kSmallBlock) {
        keys[p] = (uint32_t)(v[p] >> kIdBits);
        ids[p] = (uint32_t)(v[p] & (((T)1 << kIdBits) - 1));
    }
}

template <typename T, int kIdBits>
__global__ __launch_bounds__(kSmallBlock) void k_switch_sort_small(
        const uint8_t* __restrict__ pkts, uint32_t npk, size_t stride, uint32_t num_slots,
        int switch_id, uint8_t* __restrict__ actions, uint32_t* __restrict__ keys,
        uint32_t* __restrict__ ids) {
    switch_sort_small_body<T, kIdBits>(pkts, npk, stride, num_slots, switch_id, actions, keys, ids);
}

// later passes: chunk histogram of digit (key >> shift)
template <int R>
__global__ __launch_bounds__(kRsBlock) void k_rs_hist(const uint32_t* __restrict__ keys, size_t n,
                                                      int shift, int bits,
                                                      uint32_t* __restrict__ hist, size_t nch) {
    __shared__ uint32_t h[kRsBins];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const size_t c = blockIdx.x;
    const uint32_t nb = 1u << bits;
    for (uint32_t d = threadIdx.x; d < nb; d += kRsBlock) h[d] = 0;
    __syncthreads();
    const size_t i0 = c * (kRsWaves * 64 * R) + (size_t)wv * (64 * R) + (size_t)lane;
    uint32_t k[R];
#pragma unroll
    for (int r = 0; r < R; ++r) k[r] = i0 + (size_t)r * 64 < n ? keys[i0 + (size_t)r * 64] : 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) lds_count(h, (k[r] >> shift) & (nb - 1), i0 + (size_t)r * 64 < n);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nb; d += kRsBlock) hist[d * nch + c] = h[d];
}

// one wave per digit: cnt[d][*] -> exclusive prefix along the chunks, totals[d]
__global__ __launch_bounds__(kRsBlock) void k_rs_colscan(uint32_t* __restrict__ hist, size_t nch,
                                                         uint32_t nb, uint32_t* __restrict__ totals) {
    const int lane = threadIdx.x & 63;
    const size_t d = (size_t)blockIdx.x * kRsWaves + wave_in_block();
    if (d >= nb) return;
    uint32_t* row = hist + d * nch;
    uint32_t run = 0;
    // 8 x 64 chunks per step (one step up to 2 M packets): the step's loads are all
    // issued before its scans
    constexpr int kCs = 8;
    for (size_t c0 = 0; c0 < nch; c0 += 64 * kCs) {
        uint32_t x[kCs];
#pragma unroll
        for (int q = 0; q < kCs; ++q) {
            const size_t c = c0 + 64 * q + (size_t)lane;
            x[q] = c < nch ? row[c] : 0u;
        }
#pragma unroll
        for (int q = 0; q < kCs; ++q) {
            const size_t c = c0 + 64 * q + (size_t)lane;
            const uint32_t inc = wave_incl_scan(x[q]);
            if (c < nch) row[c] = run + inc - x[q];
            run += __builtin_amdgcn_readlane(inc, 63);
        }
    }
    if (lane == 0) totals[d] = run;
}

// scatter: out position = base(digit, chunk, wave) + items of that digit the wave already
// placed + rank among this round's lanes with the same digit
template <bool kIds, int R, int NW = kRsWaves>
__global__ __launch_bounds__(NW * 64) void k_rs_scatter(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout,
                                                         uint32_t* __restrict__ vout, size_t n,
                                                         int shift, int bits,
                                                         const uint32_t* __restrict__ colpref,
                                                         const uint32_t* __restrict__ totals,
                                                         size_t nch) {
    __shared__ uint32_t base[NW][kRsBins];   // per-wave counts, then per-wave bases
    __shared__ uint32_t dbase[kRsBins];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const size_t c = blockIdx.x;
    const uint32_t nb = 1u << bits;
    const size_t tile0 = c * (NW * 64 * R);
    const size_t i0 = tile0 + (size_t)wv * (64 * R) + (size_t)lane;
    uint32_t k[R], v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const size_t i = i0 + (size_t)r * 64;
        k[r] = i < n ? kin[i] : 0u;
        v[r] = kIds ? (i < n ? vin[i] : 0u) : (uint32_t)i;
    }
    // digit totals and this chunk's column prefixes: loaded with the keys, one round trip
    constexpr int kDPT = (kRsBins + NW * 64 - 1) / (NW * 64);   // digits per thread
    uint32_t tot[kDPT], cpf[kDPT];
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * (NW * 64);
        tot[j] = d < nb ? totals[d] : 0u;
        cpf[j] = d < nb ? colpref[d * nch + c] : 0u;
    }
    for (uint32_t d = lane; d < nb; d += 64) base[wv][d] = 0;
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * (NW * 64);
        if (d < nb) dbase[d] = tot[j];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r)              // this wave's digit counts
        lds_count(base[wv], (k[r] >> shift) & (nb - 1), i0 + (size_t)r * 64 < n);
    if (wv == 0) {                                   // digit bases: exclusive scan of the totals
        uint32_t carry = 0;
        for (uint32_t d0 = 0; d0 < nb; d0 += 64) {
            const uint32_t d = d0 + (uint32_t)lane;
            const uint32_t t = d < nb ? dbase[d] : 0u;
            const uint32_t inc = wave_incl_scan(t);
            if (d < nb) dbase[d] = carry + inc - t;
            carry += __builtin_amdgcn_readlane(inc, 63);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {                 // the tile's first output position per digit
        const uint32_t d = threadIdx.x + (uint32_t)j * (NW * 64);
        if (d < nb) dbase[d] += cpf[j];
    }
    __syncthreads();
    rs_tile_scatter<R, NW>(k, v, i0, n, shift, bits, base, dbase, kout, vout);
}

// ---- bucket + local slot sort (ina_set_tuning key 12 = 2) -----------------------------
// Two-digit keys sorted MSD-first: ONE global pass (keys + histogram, column scan, scatter)
// on the high digit leaves every bucket of 2^lbits consecutive slots contiguous and in
// arrival order; then one workgroup per bucket sorts it stably on the low digit, the
// bucket's whole tile staying in registers and LDS.  The permutation equals the LSD
// passes' (stable by (high, low) digit, arrival order inside a slot), so the run kernel
// sees the same arrays; the second pass's histogram and column-scan launches and its
// global rank bookkeeping are gone.  A bucket larger than one tile (skewed slot use) is
// sorted tile by tile: a counting sweep over the bucket first, then the tiles in order.
#ifndef INA_LOCAL_WAVES
#define INA_LOCAL_WAVES 16
#endif
constexpr int kLcWaves = INA_LOCAL_WAVES;           // waves per bucket workgroup
constexpr int kLcRounds = 64 / kLcWaves > 4 ? 64 / kLcWaves : 4;   // tile = max(4096, 256 x waves) items
template <int NW, int R>
__global__ __launch_bounds__(NW * 64) void k_rs_local(const uint32_t* __restrict__ kin,
                                                      const uint32_t* __restrict__ vin,
                                                      uint32_t* __restrict__ kout,
                                                      uint32_t* __restrict__ vout, int lbits,
                                                      const uint32_t* __restrict__ totals,
                                                      uint32_t skip) {
    constexpr int kThr = NW * 64;
    // the bucket holding nothing but foreign packets (sentinel key num_slots) is not sorted:
    // they sort after every slot anyway and the run kernel skips them (nforeign)
    if (blockIdx.x == skip) return;
    constexpr int kDPT = (kRsBins + kThr - 1) / kThr;
    __shared__ uint32_t base[NW][kRsBins];
    __shared__ uint32_t gst[kRsBins];               // bucket digit counts, then output positions
    __shared__ uint32_t red[NW];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const uint32_t b = blockIdx.x;
    // bucket start = sum of the earlier buckets' totals (high-digit pass)
    uint32_t part = 0;
    for (uint32_t d = threadIdx.x; d < b; d += kThr) part += totals[d];
    part = __builtin_amdgcn_readlane(wave_incl_scan(part), 63);
    if (lane == 0) red[wv] = part;
    const uint32_t cnt = totals[b];
    const uint32_t nb = 1u << lbits;
    for (uint32_t d = threadIdx.x; d < nb; d += kThr) gst[d] = 0;
    __syncthreads();
    if (cnt == 0) return;                           // block-uniform
    uint32_t s0 = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s0 += red[w];
    constexpr uint32_t kTile = (uint32_t)kThr * (uint32_t)R;
    const uint32_t ntile = (cnt + kTile - 1) / kTile;
    const size_t n_end = (size_t)s0 + cnt;
    if (ntile > 1) {                                // bucket digit totals -> output positions
        for (size_t i = (size_t)s0 + (size_t)wv * 64 + (size_t)lane; i - (size_t)lane < n_end; i += kThr)
            lds_count(gst, (i < n_end ? kin[i] : 0u) & (nb - 1), i < n_end);
        __syncthreads();
        if (wv == 0) {
            uint32_t carry = s0;
            for (uint32_t d0 = 0; d0 < nb; d0 += 64) {
                const uint32_t d = d0 + (uint32_t)lane;
                const uint32_t t = d < nb ? gst[d] : 0u;
                const uint32_t inc = wave_incl_scan(t);
                if (d < nb) gst[d] = carry + inc - t;
                carry += __builtin_amdgcn_readlane(inc, 63);
            }
        }
    }
    for (uint32_t t = 0; t < ntile; ++t) {
        // the tile's items split evenly over the waves in order (wave w: rw rounds of 64
        // consecutive items), so a 2,048-item bucket is 2 rounds per wave, not 8 of 4 waves
        const uint32_t tn = min(kTile, cnt - t * kTile);
        const int rw = (int)((tn + (uint32_t)kThr - 1) / (uint32_t)kThr);
        const size_t i0 = (size_t)s0 + (size_t)t * kTile + (size_t)wv * 64 * (size_t)rw + (size_t)lane;
        const size_t t_end = (size_t)s0 + (size_t)t * kTile + tn;
        uint32_t k[R], v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = i0 + (size_t)r * 64;
            const bool ok = r < rw && i < t_end;
            k[r] = ok ? kin[i] : 0u;
            v[r] = ok ? vin[i] : 0u;
        }
        for (uint32_t d = lane; d < nb; d += 64) base[wv][d] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r < rw) lds_count(base[wv], k[r] & (nb - 1), i0 + (size_t)r * 64 < t_end);
        __syncthreads();
        uint32_t tc[kDPT];                          // this tile's count per digit
#pragma unroll
        for (int j = 0; j < kDPT; ++j) {
            const uint32_t d = threadIdx.x + (uint32_t)j * kThr;
            tc[j] = 0;
            if (d < nb) {
#pragma unroll
                for (int w = 0; w < NW; ++w) tc[j] += base[w][d];
                if (ntile == 1) gst[d] = tc[j];
            }
        }
        if (ntile == 1) {                           // one tile: positions from its own counts
            __syncthreads();
            if (wv == 0) {
                uint32_t carry = s0;
                for (uint32_t d0 = 0; d0 < nb; d0 += 64) {
                    const uint32_t d = d0 + (uint32_t)lane;
                    const uint32_t x = d < nb ? gst[d] : 0u;
                    const uint32_t inc = wave_incl_scan(x);
                    if (d < nb) gst[d] = carry + inc - x;
                    carry += __builtin_amdgcn_readlane(inc, 63);
                }
            }
        }
        __syncthreads();
        rs_tile_scatter<R, NW>(k, v, i0, t_end, 0, lbits, base, gst, kout, vout, rw);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kDPT; ++j) {
            const uint32_t d = threadIdx.x + (uint32_t)j * kThr;
            if (d < nb) gst[d] += tc[j];
        }
    }
}

// ---- one-sweep slot sort (ina_set_tuning key 12 = 1; measured slower, kept for the lab)
// The same stable LSD digit passes, without the per-pass histogram and column-scan
// launches: the key pass also counts every pass's digits (one global histogram per pass,
// LDS counts then one atomic per nonzero bin and block), and each digit pass is ONE
// kernel whose blocks take tiles in ticket order (an atomic counter, so every tile a block
// waits for has already started) and find their tile's offset per digit by decoupled
// look-back over the earlier tiles' published counts.  Status word per (tile, digit):
// bits 31..30 = 1 aggregate of the tile alone, 2 inclusive prefix through the tile; bits
// 29..0 the count.  A word is self-contained (one 4-byte store), so the hand-off needs no
// ordering: agent-scope stores (write-through) and agent-scope relaxed loads polled by the
// waiting lanes (MI355X_MICROARCH.md, inter-workgroup visibility).  Launches per batch:
// memset + keys + one per digit pass (2 at <= 2^18 slots) -- 4 instead of 6.  Measured at
// 819,200 NGA-256 packets (profiles/r02/lab): each pass 26.5-27.8 us at 4,096-item tiles
// (44 us at 1,024) against 17-18 us per scatter + 5-6 us per histogram / column scan:
// 512 digits per tile make every tile's look-back a chain of dependent agent-scope polls,
// so the launches it saves cost more than they did.
constexpr uint32_t kOsAgg = 1u << 30, kOsInc = 2u << 30, kOsCnt = (1u << 30) - 1u;
constexpr int kOsMaxPasses = 4;

__device__ __forceinline__ void os_publish(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t os_poll(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// keys (slot, foreign sentinel, PS-ack bit 31) + every pass's global digit histogram, from
// the packet headers or from the batch's descriptors (header bytes 4..11, include/ina.h)
template <bool kDesc>
__global__ __launch_bounds__(kRsBlock) void k_switch_keys_os(const uint8_t* __restrict__ pkts,
                                                             const uint2* __restrict__ desc,
                                                             size_t npk, size_t stride,
                                                             uint32_t num_slots, int switch_id,
                                                             uint32_t* __restrict__ keys,
                                                             uint8_t* __restrict__ actions,
                                                             int passes, int bits,
                                                             uint32_t* __restrict__ ghist,
                                                             int ack_hint) {
    __shared__ uint32_t h[kOsMaxPasses * kRsBins];
    const uint32_t nb = 1u << bits;
    for (uint32_t d = threadIdx.x; d < (uint32_t)passes * nb; d += kRsBlock) h[d] = 0;
    __syncthreads();
    const bool al4 = (stride & 3) == 0 && ((uintptr_t)pkts & 3u) == 0;
    const size_t gs = (size_t)gridDim.x * kRsBlock;
    const size_t tid = (size_t)blockIdx.x * kRsBlock + threadIdx.x;
    for (size_t w0 = tid & ~(size_t)63; w0 < npk; w0 += gs) {       // wave-uniform trip count
        const size_t p = w0 + (threadIdx.x & 63);
        const bool valid = p < npk;
        uint32_t idx = 0, sid = 0, ack = 0;
        if (!valid) {
        } else if (kDesc) {
            const uint2 d = desc[p];
            idx = __builtin_bswap32((d.x >> 16) | (d.y << 16));
            sid = (d.y >> 16) & 0xFFu;
            ack = (d.x >> 14) & 1u;                                  // flags byte 5, bit 6
        } else if (al4) {
            const uint32_t* pk = reinterpret_cast<const uint32_t*>(pkts + p * stride);
            const uint32_t w1 = pk[1], w2 = pk[2];
            idx = __builtin_bswap32((w1 >> 16) | (w2 << 16));
            sid = (w2 >> 16) & 0xFFu;
            ack = (w1 >> 14) & 1u;
        } else {
            idx = rd_be32(pkts + p * stride + 6);
            sid = pkts[p * stride + 10];
            ack = (pkts[p * stride + 5] >> 6) & 1u;
        }
        const bool mine = switch_id >= 0 && sid == (uint32_t)(uint8_t)switch_id;
        const uint32_t key = mine ? idx % num_slots : num_slots;
        if (valid) {
            keys[p] = key | ((ack_hint && mine && ack) ? kAckBit : 0u);
            if (!mine) actions[p] = INA_ACT_FWD_OTHER;               // ngaa.p4:184-186
        }
        for (int q = 0; q < passes; ++q) lds_count(h + q * nb, (key >> (q * bits)) & (nb - 1), valid);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < (uint32_t)passes * nb; d += kRsBlock)
        if (h[d]) atomicAdd(&ghist[d], h[d]);
}

// one digit pass: tile = 4 waves x 64 x R items, wave w owns the tile's w-th quarter in
// rounds of 64 (the layout and in-round ballot ranks of k_rs_scatter)
template <bool kIds, int R>
__global__ __launch_bounds__(kRsBlock) void k_rs_onesweep(const uint32_t* __restrict__ kin,
                                                          const uint32_t* __restrict__ vin,
                                                          uint32_t* __restrict__ kout,
                                                          uint32_t* __restrict__ vout, size_t n,
                                                          int shift, int bits,
                                                          const uint32_t* __restrict__ ghist,
                                                          uint32_t* __restrict__ ticket,
                                                          uint32_t* __restrict__ status) {
    __shared__ uint32_t base[kRsWaves][kRsBins];   // per-wave counts, then per-wave bases
    __shared__ uint32_t dbase[kRsBins];            // global digit base (scan of ghist)
    __shared__ uint32_t tile_s;
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const uint32_t nb = 1u << bits;
    if (threadIdx.x == 0) tile_s = atomicAdd(ticket, 1u);
    for (uint32_t d = lane; d < nb; d += 64) base[wv][d] = 0;
    __syncthreads();
    const size_t c = __builtin_amdgcn_readfirstlane(tile_s);
    const size_t tile0 = c * (kRsWaves * 64 * R);
    const size_t i0 = tile0 + (size_t)wv * (64 * R) + (size_t)lane;
    uint32_t k[R], v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const size_t i = i0 + (size_t)r * 64;
        k[r] = i < n ? kin[i] : 0u;
        v[r] = kIds ? (i < n ? vin[i] : 0u) : (uint32_t)i;
    }
    constexpr int kDPT = kRsBins / kRsBlock;         // digits per thread
    uint32_t gh[kDPT];
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kRsBlock;
        gh[j] = d < nb ? ghist[d] : 0u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r)              // this wave's digit counts
        lds_count(base[wv], (k[r] >> shift) & (nb - 1), i0 + (size_t)r * 64 < n);
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kRsBlock;
        if (d < nb) dbase[d] = gh[j];
    }
    __syncthreads();
    // publish this tile's counts, then look back for its offsets (my digits)
    uint32_t cnt[kDPT], excl[kDPT];
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kRsBlock;
        cnt[j] = 0;
        if (d < nb) {
#pragma unroll
            for (int w = 0; w < kRsWaves; ++w) cnt[j] += base[w][d];
            os_publish(status + c * nb + d, (c == 0 ? kOsInc : kOsAgg) | cnt[j]);
        }
    }
    if (wv == 0) {                                   // digit bases: exclusive scan of ghist
        uint32_t carry = 0;
        for (uint32_t d0 = 0; d0 < nb; d0 += 64) {
            const uint32_t d = d0 + (uint32_t)lane;
            const uint32_t t = d < nb ? dbase[d] : 0u;
            const uint32_t inc = wave_incl_scan(t);
            if (d < nb) dbase[d] = carry + inc - t;
            carry += __builtin_amdgcn_readlane(inc, 63);
        }
    }
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kRsBlock;
        excl[j] = 0;
        if (d < nb && c > 0) {
            size_t t = c - 1;
            for (;;) {
                const uint32_t sv = os_poll(status + t * nb + d);
                if ((sv >> 30) == 0u) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl[j] += sv & kOsCnt;
                if ((sv >> 30) == 2u || t == 0) break;
                --t;
            }
            os_publish(status + c * nb + d, kOsInc | (excl[j] + cnt[j]));
        }
    }
    __syncthreads();                                  // dbase scanned, base[][] counts final
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {                 // the tile's first output position per digit
        const uint32_t d = threadIdx.x + (uint32_t)j * kRsBlock;
        if (d < nb) dbase[d] += excl[j];
    }
    __syncthreads();
    rs_tile_scatter<R>(k, v, i0, n, shift, bits, base, dbase, kout, vout);
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
    const int wv = wave_in_block();
    const size_t pos = (size_t)blockIdx.x * (kSwBlock / 64) + wv;
    if (pos >= npk) return;
    const uint32_t slot = keys[pos];
    if (slot >= st.num_slots) return;                      // not ours: already marked
    if (pos > 0 && keys[pos - 1] == slot) return;          // not the segment head
    const int V = st.V;
    uint8_t* lds = stage[wv];
    const bool vec = (stride % 16 == 0) && (((uintptr_t)pkts & 15u) == 0);
    // the program reads and rewrites header + payload only (15 + 4V <= 1039 bytes); row
    // padding past kMaxStride is never staged
    const size_t span = stride < (size_t)kMaxStride ? stride : (size_t)kMaxStride;

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
            for (size_t b = 16 * (size_t)lane; b < span; b += 64 * 16)
                *reinterpret_cast<u32x4s*>(lds + b) = *reinterpret_cast<const u32x4s*>(pk + b);
        } else {
            for (size_t b = lane; b < span; b += 64) lds[b] = pk[b];
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
                for (size_t b = 16 * (size_t)lane; b < span; b += 64 * 16)
                    *reinterpret_cast<u32x4s*>(pk + b) = *reinterpret_cast<const u32x4s*>(lds + b);
            } else {
                for (size_t b = lane; b < span; b += 64) pk[b] = lds[b];
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
#ifndef INA_SWITCH_BATCH
#define INA_SWITCH_BATCH 8
#endif
constexpr int kB = INA_SWITCH_BATCH;         // packets of a segment loaded at once
#ifndef INA_SWITCH_WIN_SMALL
#define INA_SWITCH_WIN_SMALL 8
#endif
#ifndef INA_SWITCH_WIN_LARGE
#define INA_SWITCH_WIN_LARGE 16
#endif
#ifndef INA_SWITCH_GRID
#define INA_SWITCH_GRID (1 << 20)
#endif
static_assert(INA_SWITCH_WIN_SMALL >= 1 && INA_SWITCH_WIN_SMALL <= 64 && INA_SWITCH_WIN_LARGE >= 1 &&
              INA_SWITCH_WIN_LARGE <= 64, "a window is at most one wave of keys");
// occupancy target of k_switch_run2 without the PS step (72 VGPRs -> 7 waves per SIMD)
#ifndef INA_SWITCH_WAVES_RUN
#define INA_SWITCH_WAVES_RUN 7
#endif
// occupancy floor of k_switch_run2<true> (waves per SIMD): the compiler then takes 75 VGPRs
// = 6 waves, no scratch; forcing 7 (72 VGPRs, 12 B/lane scratch) ran 1 % slower
// (profiles/r02/lab/fuse_lab_waves.log)
#ifndef INA_SWITCH_WAVES
#define INA_SWITCH_WAVES 4
#endif

// packet chunk loads of the run kernel carry the streaming (nt) hint: 294 -> 276 us for
// 819,200 NGA-256 packets (tools/lab/switch_lab.py, r01 session log switch_lab_nt.log);
// nt on the forwarded-packet stores or on the key pass's header loads cost 10 us each
#ifndef INA_SWITCH_NT
#define INA_SWITCH_NT 1
#endif
// the tail chunk (bytes 1024..1039 of an NGA-256 row) always lies in the 128-byte line
// the packet shares with the next row; loading it with the default policy keeps that line
// in L2 for the neighbour: run kernel HBM reads 975.7 -> 911.4 MB, switch 268 -> 265 us.
// A default-policy touch of each packet's head chunk as well read 870 MB but ran 288 us
// (profiles/r01/lab/switch_lab_tail.log)
#ifndef INA_SWITCH_TAIL_NT
#define INA_SWITCH_TAIL_NT 0
#endif
// the batch's action bytes leave in one store (lane b: packet b) instead of one per packet:
// 241.7 -> 234.9 us for the switch alone (profiles/r02/lab/switch_lab_actbatch.log); with
// the PS step fused, once that kernel sat at 75 VGPRs / 6 waves either way, 294.3 -> 291.0
// us (fuse_lab_actbatch_ps.log; at the time of the first lab it cost an occupancy step)
#ifndef INA_SWITCH_ACT_BATCH
#define INA_SWITCH_ACT_BATCH 1
#endif
__device__ __forceinline__ u32x4s sw_ld(const u32x4s* p) {
#if INA_SWITCH_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// byte shuffles of the NGA payload (values at byte 15 + 4j, big-endian) as one v_perm_b32
// each (selector byte k: 0-3 = second operand's bytes, 4-7 = first operand's):
//   dec_be(hi, lo) = the BE word at bytes {lo.b3, hi.b0, hi.b1, hi.b2}
//   enc_lo(prev, v) = LE dword of BE bytes 1..3 of prev followed by BE byte 0 of v
#ifndef INA_SWITCH_PERM
#define INA_SWITCH_PERM 1
#endif
__device__ __forceinline__ uint32_t dec_be(uint32_t hi, uint32_t lo) {
#if INA_SWITCH_PERM
    return __builtin_amdgcn_perm(hi, lo, 0x03040506u);
#else
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, 3));
#endif
}
__device__ __forceinline__ uint32_t enc_lo(uint32_t prev, uint32_t v) {
#if INA_SWITCH_PERM
    return __builtin_amdgcn_perm(v, prev, 0x07000102u);
#else
    return (__builtin_bswap32(prev) >> 8) | (v & 0xFF000000u);
#endif
}

// PS co-located with the switch (ina_switch_process_apply): a completed slot's sum goes
// straight from the VGPRs into the PS update out = local + ws * (sum * 2^-k) and the PS
// ack row -- exactly what ina_apply_completed_nga computes from the forwarded packet.
struct PsFuse {
    const float* local;
    float* out;
    size_t n;
    float inv, ws;
    uint32_t seq0, nslots;
    uint8_t* acks;
    size_t ack_stride;
    int on, keep_fwd;   // keep_fwd = 0: completed packets are consumed, not written back
};

// the run kernel's work for waves wave, wave + nwaves, ... (k_switch_run2: every wave of
// the grid; k_switch_tiny: the 16 waves of its one workgroup)
// kPs: PS update fused (ina_switch_process_apply); false costs nothing.  kLat (the
// one-launch tiny path, latency-bound): the slot's count and frag are read into SGPRs
// only after the first batch's packet loads are issued, so a segment waits for one memory
// round trip instead of three (no gain where the kernel is bandwidth-bound, and it costs
// registers there: profiles/r02/lab/switch_lab_state_late.log)
template <bool kPs, bool kLat = false>
__device__ __forceinline__ void switch_run2_body(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                 size_t npk, size_t stride,
                                                 const uint32_t* __restrict__ keys,
                                                 const uint32_t* __restrict__ ids,
                                                 uint8_t* __restrict__ actions, uint32_t win,
                                                 uint32_t kmask, const PsFuse& ps, size_t wave,
                                                 size_t nwaves) {
    constexpr bool kActBatch = INA_SWITCH_ACT_BATCH;
    const int lane = threadIdx.x & 63;
    const int V = st.V;
    const int L = V >> 2;                       // lanes holding values
    const bool vl = lane < L;
    const bool wide = L == 64;                  // tail chunk lives in lane 63's t[]
    const uint32_t NS = st.num_slots;
    // each wave takes windows of 64 sorted positions and processes the segments that
    // START in its window (a segment may run past the window's end)
    for (size_t w0 = wave * win; w0 < npk; w0 += nwaves * win) {
        const size_t i = w0 + (size_t)lane;
        const uint32_t kr = i < npk ? keys[i] : NS;
        const uint32_t ki = kr & kmask;                   // slot (bit 31: PS-ack hint)
        const uint32_t idw = i < npk ? ids[i] : 0u;     // packet ids of the window, one load
        const uint32_t kp = (i > 0 && i <= npk) ? (keys[i - 1] & kmask) : 0xFFFFFFFFu;
        const bool head = (uint32_t)lane < win && i < npk && ki < NS && (i == 0 || kp != ki);
        // a PS ack only clears the slot's frag register and is forwarded unchanged
        // (fragcheck.p4:26-31, ngaa.p4:130-132), so an ack at the HEAD of its segment is
        // done here for every such lane of the window at once, without reading the packet:
        // alone in its segment it also stores frag = 0; otherwise its segment runs below
        // from the next position with frag = 0 (lane 63 is never "alone": its successor is
        // unknown)
        const uint32_t kn = (uint32_t)__builtin_amdgcn_update_dpp((int)ki, (int)ki, 0x130, 0xF, 0xF, false);
        const bool head_ack = head && (kr & ~kmask) != 0u;
        const bool lone_ack = head_ack && kn != ki;
        if (head_ack) actions[idw] = INA_ACT_FWD_ACK;
        if (lone_ack) st.frag[ki] = 0u;
        unsigned long long hm = __ballot(head && !lone_ack);
        const unsigned long long am = __ballot(head_ack && !lone_ack);   // segments led by an ack
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
                    const bool diff = j >= npk || (keys[j] & kmask) != slot;
                    const unsigned long long m = __ballot(diff);
                    if (m) { end = j0 + (size_t)__builtin_ctzll(m); break; }
                    j0 += 64;
                }
            }
        }
        // slot state: count and frag are wave-uniform (SGPRs, scalar branches); the V
        // registers are loaded only if a packet adds to them before any overwrite
        // (count_reg == 1 overwrites, processor.p4:16-21), i.e. rarely
        const bool ack_led = (am >> hl) & 1ull;
        uint32_t cnt = 0, frag = 0, cnt_ld = 0, frag_ld = 0;
        bool st_ready = false;
        if constexpr (kLat) {
            cnt_ld = st.count[slot];
            frag_ld = st.frag[slot];
        } else {
            cnt = __builtin_amdgcn_readfirstlane((uint32_t)st.count[slot]);
            frag = ack_led ? 0u : __builtin_amdgcn_readfirstlane(st.frag[slot]);
        }
        u32x4s reg = {0u, 0u, 0u, 0u};
        bool have_reg = false;
        for (size_t q0 = pos + (ack_led ? 1 : 0); q0 < end; q0 += kB) {
            const int nb = (int)((end - q0) < (size_t)kB ? (end - q0) : (size_t)kB);
            u32x4s a[kB];
            uint32_t pid[kB];
            // packet ids first (no load in the common in-window case; one coalesced load
            // otherwise), so the kB packet loads below issue back to back with no
            // s_waitcnt between them
            if (q0 + (size_t)nb <= w0 + 64) {
                const int o = (int)(q0 - w0);
#pragma unroll
                for (int b = 0; b < kB; ++b)
                    pid[b] = b < nb ? __builtin_amdgcn_readlane(idw, o + b < 64 ? o + b : 63) : 0u;
            } else {
                const uint32_t my = lane < nb ? ids[q0 + (size_t)lane] : 0u;
#pragma unroll
                for (int b = 0; b < kB; ++b) pid[b] = __builtin_amdgcn_readlane(my, b);
            }
            // tail chunks 64 (V = 256 only): lane b holds packet b's, 4 VGPRs for the whole
            // batch instead of 4 per packet; lane 63 takes them by readlane when it needs
            // them.  Issued first, so packet 0 can start once its own load is back.
            // Every load is unconditional (slots past the batch re-read packet 0, lanes past
            // L re-read chunk 0) so no load sits in a branch: the compiler's wait counting
            // stays exact and packet b waits only for its own data.
#pragma unroll
            for (int b = 1; b < kB; ++b) pid[b] = b < nb ? pid[b] : pid[0];
            u32x4s tl = {0u, 0u, 0u, 0u};
            uint32_t mypid = pid[0];                 // lane b: packet b's id
#pragma unroll
            for (int b = 1; b < kB; ++b) mypid = lane == b ? pid[b] : mypid;
            uint32_t act_v = 0;                      // lane b: packet b's action (kActBatch)
            if (wide) {
#if INA_SWITCH_TAIL_NT
                tl = sw_ld(reinterpret_cast<const u32x4s*>(pkts + (size_t)mypid * stride) + 64);
#else
                tl = *(reinterpret_cast<const u32x4s*>(pkts + (size_t)mypid * stride) + 64);
#endif
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const u32x4s* pk = reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[b] * stride);
                a[b] = sw_ld(pk + (lane <= L ? lane : 0));
            }
            if constexpr (kLat) {
                if (!st_ready) {
                    cnt = __builtin_amdgcn_readfirstlane(cnt_ld);
                    frag = ack_led ? 0u : __builtin_amdgcn_readfirstlane(frag_ld);
                    st_ready = true;
                }
            }
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                if (b >= nb) break;
                const uint32_t h1 = __builtin_amdgcn_readlane(a[b].y, 0),
                               h2 = __builtin_amdgcn_readlane(a[b].z, 0),
                               h3 = __builtin_amdgcn_readlane(a[b].w, 0);
                const uint32_t hcount = h1 & 0xFFu, flags = (h1 >> 8) & 0xFFu;
                // keep the state machine scalar (SGPRs + scalar branches)
                const uint32_t frag_in =
                    __builtin_amdgcn_readfirstlane(__builtin_bswap32((h2 >> 24) | (h3 << 8)));
                uint8_t act;
                if ((flags >> 6) & 1u) {                     // ack: reset_id (fragcheck.p4:26-31)
                    frag = 0;
                    act = INA_ACT_FWD_ACK;
                } else {
                    if (frag == 0) frag = frag_in;           // write_read_id (fragcheck.p4:14-24)
                    if (frag != frag_in) {                   // collision (ngaa.p4:177-181):
                        act = INA_ACT_FWD_COLLISION;         // only the flag byte changes
                        if (lane == 0)
                            reinterpret_cast<uint32_t*>(pkts + (size_t)pid[b] * stride)[1] =
                                a[b].y | ((uint32_t)INA_FLAG_COLLISION << 8);
                    } else {
                        cnt = (cnt + 1u) & 0xFFu;            // read_add_count (ngaa.p4:66-78)
                        if (cnt == hcount) cnt = 0;
                        cnt = __builtin_amdgcn_readfirstlane(cnt);
                        const bool first = cnt == 1u;
                        u32x4s c;                            // chunk l+1
                        c.x = from_next_lane(a[b].x); c.y = from_next_lane(a[b].y);
                        c.z = from_next_lane(a[b].z); c.w = from_next_lane(a[b].w);
                        uint32_t tw = 0;                     // old byte 1039 (padding) for the tail
                        if (wide) {
                            const uint32_t tx = __builtin_amdgcn_readlane(tl.x, b);
                            const uint32_t ty = __builtin_amdgcn_readlane(tl.y, b);
                            const uint32_t tz = __builtin_amdgcn_readlane(tl.z, b);
                            tw = __builtin_amdgcn_readlane(tl.w, b);
                            if (lane == 63) c = u32x4s{tx, ty, tz, tw};
                        }
                        u32x4s v;                            // values 4l..4l+3
                        v.x = dec_be(c.x, a[b].w);
                        v.y = dec_be(c.y, c.x);
                        v.z = dec_be(c.z, c.y);
                        v.w = dec_be(c.w, c.z);
                        if (first) {                         // processor.p4:16-21
                            reg = v;
                        } else if (have_reg) {
                            reg += v;
                        } else {                             // adds to a stored register:
                            reg = vl ? *reinterpret_cast<const u32x4s*>(   // load it now
                                           st.regs + (size_t)slot * V + 4 * lane)
                                     : u32x4s{0u, 0u, 0u, 0u};
                            reg += v;
                        }
                        have_reg = true;
                        act = cnt == 0 ? INA_ACT_FWD_AGG : INA_ACT_DROP;   // ngaa.p4:170-175
                        // the PS consumes a completed packet of its bucket (ps_slot in range;
                        // wave-uniform); one outside the bucket is forwarded like the two-call
                        // path forwards it, whatever keep_fwd says
                        const uint32_t ps_slot = frag_in - ps.seq0;
                        const bool consumed = kPs && act == INA_ACT_FWD_AGG && ps_slot < ps.nslots;
                        if (consumed) {                      // launch.py:46-50 with the switch's sum
                            {
                                const size_t e0 = (size_t)ps_slot * (size_t)V + 4 * (size_t)lane;
                                if (vl && e0 + 4 <= ps.n) {
                                    const f32x4s l = *reinterpret_cast<const f32x4s*>(ps.local + e0);
                                    f32x4s r;
                                    r.x = __fadd_rn(l.x, __fmul_rn(__fmul_rn((float)(int32_t)reg.x, ps.inv), ps.ws));
                                    r.y = __fadd_rn(l.y, __fmul_rn(__fmul_rn((float)(int32_t)reg.y, ps.inv), ps.ws));
                                    r.z = __fadd_rn(l.z, __fmul_rn(__fmul_rn((float)(int32_t)reg.z, ps.inv), ps.ws));
                                    r.w = __fadd_rn(l.w, __fmul_rn(__fmul_rn((float)(int32_t)reg.w, ps.inv), ps.ws));
                                    *reinterpret_cast<f32x4s*>(ps.out + e0) = r;
                                } else if (vl) {
                                    const uint32_t rv[4] = {reg.x, reg.y, reg.z, reg.w};
                                    for (int t = 0; t < 4 && e0 + t < ps.n; ++t)
                                        ps.out[e0 + t] = __fadd_rn(ps.local[e0 + t],
                                            __fmul_rn(__fmul_rn((float)(int32_t)rv[t], ps.inv), ps.ws));
                                }
                                if (lane == 0 && ps.acks) {      // the PS ack (fragcheck.p4:26-31)
                                    u32x4s hd = a[b];
                                    hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                                    hd.w = (hd.w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                                    *reinterpret_cast<u32x4s*>(ps.acks + (size_t)ps_slot * ps.ack_stride) = hd;
                                }
                            }
                        }
                        if ((act != INA_ACT_DROP || st.write_dropped) && (!consumed || ps.keep_fwd)) {
                            // out_value -> payload (processor.p4:22): chunk c from lane c-1
                            u32x4s p;
                            p.x = from_prev_lane(reg.x); p.y = from_prev_lane(reg.y);
                            p.z = from_prev_lane(reg.z); p.w = from_prev_lane(reg.w);
                            u32x4s e = a[b];
                            if (lane == 0) {
                                e.w = (e.w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                            } else {
                                e.x = enc_lo(p.x, p.y);
                                e.y = enc_lo(p.y, p.z);
                                e.z = enc_lo(p.z, p.w);
                                e.w = enc_lo(p.w, lane < L ? reg.x : e.w);
                            }
                            if (lane <= L)
                                reinterpret_cast<u32x4s*>(pkts + (size_t)pid[b] * stride)[lane] = e;
                            if (wide && lane == 63) {        // tail chunk 64 from lane 63's values
                                u32x4s o;
                                o.x = enc_lo(reg.x, reg.y);
                                o.y = enc_lo(reg.y, reg.z);
                                o.z = enc_lo(reg.z, reg.w);
                                o.w = enc_lo(reg.w, tw);
                                reinterpret_cast<u32x4s*>(pkts + (size_t)pid[b] * stride)[64] = o;
                            }
                        }
                    }
                }
                if constexpr (kActBatch) act_v = lane == b ? (uint32_t)act : act_v;
                else if (lane == 0) actions[pid[b]] = act;
            }
            if constexpr (kActBatch)
                if (lane < nb) actions[mypid] = (uint8_t)act_v;   // one store for the batch
        }
        if (lane == 0) {
            st.count[slot] = (uint8_t)cnt;
            st.frag[slot] = frag;
        }
        if (have_reg && vl) *reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * lane) = reg;
        }
    }
}

// XCD-aware window map: blocks b and b + 8 share an XCD (and its L2), so logical block
// (b % 8) * G/8 + b / 8 gives each XCD one contiguous run of sorted positions -- a slot's
// neighbours, whose rows share their boundary 128-byte lines, are then gathered through
// the same L2 (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"; speed only)
#ifndef INA_SWITCH_XCD
#define INA_SWITCH_XCD 1
#endif
__device__ __forceinline__ size_t switch_block_index() {
#if INA_SWITCH_XCD
    const uint32_t G = gridDim.x, b = blockIdx.x, x = b & 7u;
    const uint32_t per = G >> 3, rem = G & 7u;
    return (size_t)x * per + (x < rem ? x : rem) + (b >> 3);
#else
    return blockIdx.x;
#endif
}

template <bool kPs>
__global__ __launch_bounds__(kSwBlock) __attribute__((amdgpu_waves_per_eu(kPs ? INA_SWITCH_WAVES : INA_SWITCH_WAVES_RUN, 8))) void k_switch_run2(ina_switch_state_t st,
                                                          uint8_t* __restrict__ pkts, size_t npk,
                                                          size_t stride,
                                                          const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ ids,
                                                          uint8_t* __restrict__ actions,
                                                          uint32_t win, uint32_t kmask, PsFuse ps,
                                                          const uint32_t* __restrict__ nforeign) {
    // bucket sort: the foreign packets' bucket was left unsorted at the END of the arrays;
    // the run kernel never processes foreign packets, so it stops before them
    if (nforeign) npk -= *nforeign;
    switch_run2_body<kPs>(st, pkts, npk, stride, keys, ids, actions, win, kmask, ps,
                          switch_block_index() * (kSwBlock / 64) + wave_in_block(),
                          ((size_t)gridDim.x * kSwBlock) >> 6);
}

// batches of at most INA_SWITCH_TINY_MAX packets (latency, not bandwidth): ONE launch of
// one 16-wave workgroup -- the bitonic (slot, packet id) sort in LDS, then the run
// kernel's work on the same 16 waves with the sorted arrays read from LDS.
template <bool kPs, typename T, int kIdBits>
__global__ __launch_bounds__(kSmallBlock) void k_switch_tiny(ina_switch_state_t st, uint8_t* __restrict__ pkts,
                                                             uint32_t npk, size_t stride,
                                                             uint8_t* __restrict__ actions, uint32_t win,
                                                             PsFuse ps) {
    // the sorted (slot, packet id) arrays stay in LDS: the run loop's window loads are LDS
    // reads, not a memory round trip
    __shared__ uint32_t keys_s[INA_SWITCH_SMALL_MAX], ids_s[INA_SWITCH_SMALL_MAX];
    switch_sort_small_body<T, kIdBits>(pkts, npk, stride, st.num_slots, st.switch_id, actions, keys_s, ids_s);
    __syncthreads();
    switch_run2_body<kPs, true>(st, pkts, npk, stride, keys_s, ids_s, actions, win, 0xFFFFFFFFu, ps,
                                wave_in_block(), kSmallBlock / 64);
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static int end_bit_for(uint32_t num_slots) {
    int b = 1;
    while (b < 32 && ((uint64_t)1 << b) <= (uint64_t)num_slots) ++b;
    return b;   // sentinel value num_slots fits
}

struct SortPlan {
    int passes, bits, rounds;   // rounds: 64-item rounds per wave (chunk = 4 waves x 64 x rounds)
    size_t nch, hist_elems;
};

static SortPlan sort_plan(size_t npk, uint32_t num_slots) {
    SortPlan p;
    const int eb = end_bit_for(num_slots);
    p.passes = (eb + kRsMaxBits - 1) / kRsMaxBits;
    p.bits = (eb + p.passes - 1) / p.passes;
    // chunk = 4 waves x 64 x rounds items: 1,024 up to 256 Ki packets (a batch of the PS's
    // acks still spreads over more than a few dozen CUs), 2,048 up to 512 Ki, 4,096 above
    // (switch_lab, profiles/r01/lab/switch_lab_rounds.log: 102,400 packets 77.7 -> 60.9 us,
    // 409,600 155.5 -> 146.1, 819,200 unchanged)
    p.rounds = npk <= (size_t)INA_RS_SMALL_ITEMS ? INA_RS_ROUNDS_SMALL
             : npk <= (size_t)INA_RS_MID_ITEMS   ? INA_RS_ROUNDS_MID
                                                 : kRsRounds;
    if (const int r = g_os_rounds.load()) p.rounds = r;   // ina_set_tuning key 13 (lab sweeps)
    const size_t chunk = (size_t)kRsWaves * 64 * (size_t)p.rounds;
    p.nch = (npk + chunk - 1) / chunk;
    p.hist_elems = ((size_t)1 << p.bits) * p.nch;
    return p;
}

static size_t sort_temp_bytes(size_t npk, uint32_t num_slots) {
    // sized for the SMALLEST chunk whatever tier npk falls in, so the scratch size is
    // monotonic in npk: a buffer sized for a batch serves every smaller batch too
    const SortPlan p = sort_plan(npk, num_slots);
    const size_t chunk = (size_t)kRsWaves * 64 * (size_t)INA_RS_ROUNDS_SMALL;
    const size_t hist = ((size_t)1 << p.bits) * ((npk + chunk - 1) / chunk);
    return align_up(hist * 4, 256) + align_up((size_t)kRsBins * 4, 256);
}

// one-sweep sort's auxiliary words, zeroed by one memset per batch: global digit
// histograms [kOsMaxPasses][512], tickets (one per pass), status [passes][tiles][2^bits]
constexpr size_t kOsHistBytes = (size_t)kOsMaxPasses * kRsBins * 4;
constexpr int kOsMinRounds = 4;
static size_t os_tiles(size_t npk, int rounds) {
    const size_t tile = (size_t)kRsWaves * 64 * (size_t)rounds;
    return (npk + tile - 1) / tile;
}
static size_t os_aux_bytes(size_t npk, const SortPlan& p, int rounds) {
    return kOsHistBytes + 256 + (size_t)p.passes * os_tiles(npk, rounds) * ((size_t)1 << p.bits) * 4;
}
static int os_rounds_for(size_t npk) {
    if (const int r = g_os_rounds.load()) return r;
    return npk <= (size_t)INA_RS_MID_ITEMS ? 4 : 8;
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
    const size_t aux = std::max(sort_temp_bytes(npkts, num_slots),
                                os_aux_bytes(npkts, sort_plan(npkts, num_slots), kOsMinRounds));
    return 4 * align_up(npkts * 4, 256) + align_up(aux, 256) + 256;
}

static int switch_process_impl(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                               const uint64_t* desc, uint8_t* actions, void* scratch,
                               ina_stream_t stream, const PsFuse& ps, bool* fused_out) {
    *fused_out = false;
    if (!st || st->V <= 0 || st->V > kMaxV || st->num_slots == 0)
        return set_error(INA_EINVAL, "bad switch state (V in [1,256])%s", "");
    if (stride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)st->V)
        return set_error(INA_EINVAL, "stride must be >= 15+4V%s", "");
    if (stride > 0xFFFFFFFFu) return set_error(INA_EINVAL, "stride too large%s", "");
    if (npk == 0) return INA_OK;
    if (npk > 0x7FFFFFFFu) return set_error(INA_EINVAL, "too many packets%s", "");
    if (!pkts || !actions || !scratch || !st->count || !st->frag || !st->regs)
        return set_error(INA_EINVAL, "null pointer%s", "");
    if (desc && ((uintptr_t)desc & 7u))
        return set_error(INA_EINVAL, "descriptors must be 8-byte aligned%s", "");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint8_t* base = reinterpret_cast<uint8_t*>(align_up((uintptr_t)scratch, 256));
    size_t arr = align_up(npk * 4, 256);
    uint32_t* k_in = reinterpret_cast<uint32_t*>(base);
    uint32_t* k_out = reinterpret_cast<uint32_t*>(base + arr);
    uint32_t* v_in = reinterpret_cast<uint32_t*>(base + 2 * arr);
    uint32_t* v_out = reinterpret_cast<uint32_t*>(base + 3 * arr);
    const SortPlan sp = sort_plan(npk, st->num_slots);
    // sort chunk geometry (sort_plan): one instantiation per rounds-per-wave choice
    constexpr int kR0 = INA_RS_ROUNDS_SMALL, kR1 = INA_RS_ROUNDS_MID, kR2 = kRsRounds;
    static_assert(kR0 % 4 == 0 && kR1 % 4 == 0 && kR2 % 4 == 0, "bucket pass: 16 waves x rounds/4");
    const int ri = sp.rounds == kR0 ? 0 : sp.rounds == kR1 ? 1 : 2;
    auto* k_keys = desc ? (ri == 0 ? &k_switch_keys<kR0, true> : ri == 1 ? &k_switch_keys<kR1, true>
                                                                : &k_switch_keys<kR2, true>)
                        : (ri == 0 ? &k_switch_keys<kR0, false> : ri == 1 ? &k_switch_keys<kR1, false>
                                                                 : &k_switch_keys<kR2, false>);
    auto* k_hist = ri == 0 ? &k_rs_hist<kR0> : ri == 1 ? &k_rs_hist<kR1> : &k_rs_hist<kR2>;
    auto* k_sc0 = ri == 0 ? &k_rs_scatter<false, kR0>
                : ri == 1 ? &k_rs_scatter<false, kR1> : &k_rs_scatter<false, kR2>;
    auto* k_sc1 = ri == 0 ? &k_rs_scatter<true, kR0>
                : ri == 1 ? &k_rs_scatter<true, kR1> : &k_rs_scatter<true, kR2>;
    uint32_t* hist = reinterpret_cast<uint32_t*>(base + 4 * arr);
    uint32_t* totals = reinterpret_cast<uint32_t*>(base + 4 * arr + align_up(sp.hist_elems * 4, 256));
    const unsigned gc = (unsigned)sp.nch;
    const uint32_t nb = 1u << sp.bits;
    const unsigned gd = (nb + kRsWaves - 1) / kRsWaves;

    uint32_t *kc = k_in, *vc = v_in, *kn = k_out, *vn = v_out;
    const bool fast = stride % 16 == 0 && ((uintptr_t)pkts & 15u) == 0 && st->V % 4 == 0 &&
                      st->V <= kMaxV && ((uintptr_t)st->regs & 15u) == 0;
    // keys carry the PS-ack bit for the run kernel when bit 31 is outside every digit pass
    const bool ack_hint = fast && sp.passes * sp.bits <= 31 && g_ack_fast.load();
    const bool small = npk <= (size_t)g_small_sort.load();
    const bool onesweep = !small && g_sort_mode.load() == 1 && npk < ((size_t)1 << 30);
    // bucket + local sort: two-digit keys only (the low digit is one workgroup's LDS bins)
    const int mode = g_sort_mode.load();
    const bool hybrid = !small && (mode == 0 || mode == 2) && sp.passes == 2;
    uint32_t skip_bucket = 0xFFFFFFFFu;
    const uint32_t* nforeign = nullptr;
    if (onesweep) {
        // memset(aux) + keys/histograms + one kernel per digit pass
        const int R = os_rounds_for(npk);
        const size_t ntiles = os_tiles(npk, R);
        uint8_t* aux = base + 4 * arr;
        uint32_t* ghist = reinterpret_cast<uint32_t*>(aux);
        uint32_t* tickets = reinterpret_cast<uint32_t*>(aux + kOsHistBytes);
        uint32_t* status = reinterpret_cast<uint32_t*>(aux + kOsHistBytes + 256);
        if (hipMemsetAsync(aux, 0, os_aux_bytes(npk, sp, R), s) != hipSuccess)
            return set_error(INA_EHIP, "switch sort memset%s", "");
        const unsigned gk = (unsigned)std::min<size_t>((npk + kRsBlock * 8 - 1) / (kRsBlock * 8), 2048);
        if (desc)
            hipLaunchKernelGGL(k_switch_keys_os<true>, dim3(gk), dim3(kRsBlock), 0, s, pkts,
                               reinterpret_cast<const uint2*>(desc), npk, stride, st->num_slots,
                               st->switch_id, kc, actions, sp.passes, sp.bits, ghist, ack_hint ? 1 : 0);
        else
            hipLaunchKernelGGL(k_switch_keys_os<false>, dim3(gk), dim3(kRsBlock), 0, s, pkts,
                               static_cast<const uint2*>(nullptr), npk, stride, st->num_slots,
                               st->switch_id, kc, actions, sp.passes, sp.bits, ghist, ack_hint ? 1 : 0);
        for (int pass = 0; pass < sp.passes; ++pass) {
            const int shift = pass * sp.bits;
            const uint32_t* gh = ghist + (size_t)pass * nb;
            uint32_t* stp = status + (size_t)pass * ntiles * nb;
#define INA_OS_LAUNCH(IDS, RR)                                                                        \
            hipLaunchKernelGGL((k_rs_onesweep<IDS, RR>), dim3((unsigned)ntiles), dim3(kRsBlock), 0, s, \
                               kc, vc, kn, vn, npk, shift, sp.bits, gh, tickets + pass, stp)
            if (pass == 0) {
                if (R == 4) INA_OS_LAUNCH(false, 4); else if (R == 8) INA_OS_LAUNCH(false, 8); else INA_OS_LAUNCH(false, 16);
            } else {
                if (R == 4) INA_OS_LAUNCH(true, 4); else if (R == 8) INA_OS_LAUNCH(true, 8); else INA_OS_LAUNCH(true, 16);
            }
#undef INA_OS_LAUNCH
            if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
            std::swap(kc, kn);
            std::swap(vc, vn);
        }
    } else if (small && fast && npk <= (size_t)g_tiny_max.load()) {
        // sort and run in ONE launch of one workgroup (k_switch_tiny)
        uint32_t win = (uint32_t)INA_SWITCH_WIN_SMALL;
        if (const int wv = g_switch_win.load()) win = (uint32_t)wv;
        const bool narrow = (uint64_t)st->num_slots + 1 <= (1u << 20);
        if (ps.on) {
            if (narrow) hipLaunchKernelGGL((k_switch_tiny<true, uint32_t, 12>), dim3(1), dim3(kSmallBlock), 0, s, *st, pkts, (uint32_t)npk, stride, actions, win, ps);
            else hipLaunchKernelGGL((k_switch_tiny<true, unsigned long long, 32>), dim3(1), dim3(kSmallBlock), 0, s, *st, pkts, (uint32_t)npk, stride, actions, win, ps);
        } else {
            if (narrow) hipLaunchKernelGGL((k_switch_tiny<false, uint32_t, 12>), dim3(1), dim3(kSmallBlock), 0, s, *st, pkts, (uint32_t)npk, stride, actions, win, ps);
            else hipLaunchKernelGGL((k_switch_tiny<false, unsigned long long, 32>), dim3(1), dim3(kSmallBlock), 0, s, *st, pkts, (uint32_t)npk, stride, actions, win, ps);
        }
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch tiny launch%s", "");
        *fused_out = ps.on != 0;
        return INA_OK;
    } else if (small) {
        if ((uint64_t)st->num_slots + 1 <= (1u << 20))
            hipLaunchKernelGGL((k_switch_sort_small<uint32_t, 12>), dim3(1), dim3(kSmallBlock), 0, s, pkts,
                               (uint32_t)npk, stride, st->num_slots, st->switch_id, actions, kc, vc);
        else
            hipLaunchKernelGGL((k_switch_sort_small<unsigned long long, 32>), dim3(1), dim3(kSmallBlock), 0,
                               s, pkts, (uint32_t)npk, stride, st->num_slots, st->switch_id, actions, kc, vc);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
    } else if (hybrid) {
        // high digit (bits lb..eb-1) over the whole batch, then each bucket on its low digit.
        // The high pass's chunks (4 waves x 64 x rounds items) run as 16 waves x rounds/4,
        // so each wave's dependent LDS-count / rank rounds are 4x fewer
        const int lb = end_bit_for(st->num_slots) - sp.bits;
        constexpr int kHw = 16;
        const dim3 hb(kHw * 64);
        const uint2* dsc = reinterpret_cast<const uint2*>(desc);
        if (sp.rounds == kR2) {
            hipLaunchKernelGGL((desc ? &k_switch_keys<kR2 / 4, true, kHw> : &k_switch_keys<kR2 / 4, false, kHw>),
                               dim3(gc), hb, 0, s, pkts, dsc, npk, stride, st->num_slots, st->switch_id, kc,
                               actions, sp.bits, lb, hist, sp.nch, ack_hint ? 1 : 0);
        } else if (sp.rounds == kR1) {
            hipLaunchKernelGGL((desc ? &k_switch_keys<kR1 / 4, true, kHw> : &k_switch_keys<kR1 / 4, false, kHw>),
                               dim3(gc), hb, 0, s, pkts, dsc, npk, stride, st->num_slots, st->switch_id, kc,
                               actions, sp.bits, lb, hist, sp.nch, ack_hint ? 1 : 0);
        } else {
            hipLaunchKernelGGL((desc ? &k_switch_keys<kR0 / 4, true, kHw> : &k_switch_keys<kR0 / 4, false, kHw>),
                               dim3(gc), hb, 0, s, pkts, dsc, npk, stride, st->num_slots, st->switch_id, kc,
                               actions, sp.bits, lb, hist, sp.nch, ack_hint ? 1 : 0);
        }
        hipLaunchKernelGGL(k_rs_colscan, dim3(gd), dim3(kRsBlock), 0, s, hist, sp.nch, nb, totals);
        auto* k_hs = sp.rounds == kR2 ? &k_rs_scatter<false, kR2 / 4, kHw>
                   : sp.rounds == kR1 ? &k_rs_scatter<false, kR1 / 4, kHw> : &k_rs_scatter<false, kR0 / 4, kHw>;
        hipLaunchKernelGGL(k_hs, dim3(gc), hb, 0, s, kc, nullptr, kn, vn, npk, lb, sp.bits, hist, totals, sp.nch);
        // a bucket of foreign packets only (a pool of a multiple of 2^lb slots): left where the
        // high pass put them when the register-resident run kernel takes the batch (it stops
        // before them); the generic run kernel reads every position, so then it is sorted
        if (fast && (st->num_slots & ((1u << lb) - 1u)) == 0u) {
            skip_bucket = st->num_slots >> lb;
            nforeign = totals + skip_bucket;
        }
        hipLaunchKernelGGL((k_rs_local<kLcWaves, kLcRounds>), dim3(nb), dim3(kLcWaves * 64), 0, s, kn, vn, kc, vc, lb,
                           totals, skip_bucket);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
    } else {
        hipLaunchKernelGGL(k_keys, dim3(gc), dim3(kRsBlock), 0, s, pkts,
                           reinterpret_cast<const uint2*>(desc), npk, stride, st->num_slots,
                           st->switch_id, k_in, actions, sp.bits, 0, hist, sp.nch, ack_hint ? 1 : 0);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch keys launch%s", "");
    }
    // r01 digit passes: (k_in, ids) -> (k_out, v_out) -> (k_in, v_in) -> ...
    for (int pass = 0; pass < (small || onesweep || hybrid ? 0 : sp.passes); ++pass) {
        const int shift = pass * sp.bits;
        if (pass > 0)
            hipLaunchKernelGGL(k_hist, dim3(gc), dim3(kRsBlock), 0, s, kc, npk, shift, sp.bits, hist,
                               sp.nch);
        hipLaunchKernelGGL(k_rs_colscan, dim3(gd), dim3(kRsBlock), 0, s, hist, sp.nch, nb, totals);
        if (pass == 0)
            hipLaunchKernelGGL(k_sc0, dim3(gc), dim3(kRsBlock), 0, s, kc, nullptr, kn, vn, npk, shift,
                               sp.bits, hist, totals, sp.nch);
        else
            hipLaunchKernelGGL(k_sc1, dim3(gc), dim3(kRsBlock), 0, s, kc, vc, kn, vn, npk, shift,
                               sp.bits, hist, totals, sp.nch);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
        std::swap(kc, kn);
        std::swap(vc, vn);
    }
    if (fast) {
        // a wave runs the segments that start in its window of `win` sorted positions: a
        // segment is a chain of dependent round trips, so small windows (more waves) win
        // at every size -- tools/lab/switch_lab.py, profiles/r01/lab/switch_lab_win.log:
        // 1,024 packets 52.9 -> 27.7 us (64 -> 8 positions), 819,200 packets 277 -> 266 us
        // (64 -> 16 positions, one pass of the grid)
        uint32_t win = npk <= 65536 ? (uint32_t)INA_SWITCH_WIN_SMALL : (uint32_t)INA_SWITCH_WIN_LARGE;
        if (const int wv = g_switch_win.load()) win = (uint32_t)wv;
        const size_t per_block = (size_t)win * (kSwBlock / 64);
        unsigned gr = (unsigned)std::min<size_t>((npk + per_block - 1) / per_block, INA_SWITCH_GRID);
        auto* run = ps.on ? &k_switch_run2<true> : &k_switch_run2<false>;
        hipLaunchKernelGGL(run, dim3(gr), dim3(kSwBlock), 0, s, *st, pkts, npk, stride, kc, vc, actions,
                           win, ack_hint ? ~kAckBit : 0xFFFFFFFFu, ps, nforeign);
        *fused_out = ps.on != 0;
    } else {
        unsigned gw = (unsigned)((npk + (kSwBlock / 64) - 1) / (kSwBlock / 64));
        hipLaunchKernelGGL(k_switch_run, dim3(gw), dim3(kSwBlock), 0, s, *st, pkts, npk, stride, kc,
                           vc, actions);
    }
    if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch run launch%s", "");
    return INA_OK;
}

int ina_switch_process_desc(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                            const ina_nga_desc_t* desc, uint8_t* actions, void* scratch,
                            ina_stream_t stream) {
    PsFuse off{};
    bool fused = false;
    return switch_process_impl(st, pkts, npk, stride, desc, actions, scratch, stream, off, &fused);
}

int ina_switch_process(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                       uint8_t* actions, void* scratch, ina_stream_t stream) {
    return ina_switch_process_desc(st, pkts, npk, stride, nullptr, actions, scratch, stream);
}

int ina_switch_process_apply(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                             uint8_t* actions, void* scratch, uint32_t seq0, const float* local, int k,
                             double weight_step, float* out, size_t n, uint8_t* acks,
                             size_t ack_stride, int keep_forwarded, ina_stream_t stream) {
    return ina_switch_process_apply_desc(st, pkts, npk, stride, nullptr, actions, scratch, seq0, local, k,
                                         weight_step, out, n, acks, ack_stride, keep_forwarded, stream);
}

int ina_switch_process_apply_desc(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                                  const ina_nga_desc_t* desc, uint8_t* actions, void* scratch,
                                  uint32_t seq0, const float* local, int k, double weight_step,
                                  float* out, size_t n, uint8_t* acks, size_t ack_stride,
                                  int keep_forwarded, ina_stream_t stream) {
    if (k < -126 || k > 127) return set_error(INA_EINVAL, "k out of range [-126,127]%s", "");
    if (npk == 0) return INA_OK;
    if (!local || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    if (((uintptr_t)local & 15u) || ((uintptr_t)out & 15u))
        return set_error(INA_EINVAL, "local/out must be 16-byte aligned%s", "");
    if (acks && (((uintptr_t)acks & 15u) || ack_stride % 16))
        return set_error(INA_EINVAL, "ack rows must be 16-byte aligned%s", "");
    if (!st || st->V <= 0) return set_error(INA_EINVAL, "bad switch state (V in [1,256])%s", "");
    // the PS step needs the layout ina_apply_completed_nga and the fused run kernel take
    // (16-byte aligned rows and slot registers); refuse before the switch touches its state
    // rather than after, so keep_forwarded always means what include/ina.h says
    if (st->V % 4 || st->V > 256 || stride % 16 || ((uintptr_t)pkts & 15u) || ((uintptr_t)st->regs & 15u))
        return set_error(INA_EINVAL,
                         "process_apply needs V %% 4 == 0 <= 256 and 16-byte aligned rows and registers%s", "");
    const size_t nslots = (n + (size_t)st->V - 1) / (size_t)st->V;
    PsFuse ps{local, out, n, ldexpf(1.0f, -k), (float)weight_step, seq0,
              nslots > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)nslots, acks, ack_stride, 1,
              keep_forwarded ? 1 : 0};
    bool fused = false;
    if (int rc = switch_process_impl(st, pkts, npk, stride, desc, actions, scratch, stream, ps, &fused)) return rc;
    if (fused) return INA_OK;
    // layouts the register-resident run kernel does not take: the two steps one by one
    return ina_apply_completed_nga(pkts, npk, st->V, stride, actions, seq0, local, k, weight_step, out,
                                   n, acks, ack_stride, stream);
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
