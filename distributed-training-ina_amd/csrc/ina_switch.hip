// ina_switch.hip -- the packet-stream aggregator: ngaa.p4's Ingress.apply
// (ngaa.p4:120-196), its count register (64-82), frag check (fragcheck.p4:14-57)
// and the V Processor registers (processor.p4:14-24), restated on the device.
//
// A batch of NGA-V packets in arrival order is grouped by aggregator slot with a
// stable sort (slot, arrival) -- slots are independent in the P4 program, so per-slot
// arrival order is all that matters: by default each chunk sorted by the key's high digit
// (k_sort_chunks) and one workgroup per bucket of slots gathering its runs and sorting them
// on the low digit (k_sort_buckets), else LSD digit passes or a one-workgroup bitonic sort
// for small batches.  Each slot's packets are
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
#include <mutex>
#include <unordered_map>

#include "ina.h"
#include "ina_internal.h"
#include "ina_device.h"

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
// chunk + bucket sort of more than 2 Mi packets: 8,192-packet chunks (32 rounds), so a
// bucket's run in each chunk is twice as long and B gathers half as many of them
#ifndef INA_RS_ROUNDS_BIG
#define INA_RS_ROUNDS_BIG 32
#endif
#ifndef INA_RS_BIG_ITEMS
#define INA_RS_BIG_ITEMS 2097152
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
template <int R, int NW = kRsWaves, int BINS = kRsBins>
__device__ __forceinline__ void rs_tile_scatter(const uint32_t (&k)[R], const uint32_t (&v)[R],
                                                size_t i0, size_t n, int shift, int bits,
                                                uint32_t (*base)[BINS], const uint32_t* gst,
                                                uint32_t* __restrict__ kout,
                                                uint32_t* __restrict__ vout, int rw = R) {
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const uint32_t nb = 1u << bits;
    constexpr int kThr = NW * 64;
    constexpr int kDPT = (BINS + kThr - 1) / kThr;
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
// Bit 30 of a sorted key (round 6): a PLAIN packet, one whose header fields the run can make
// from its slot -- this switch's, flags byte 0, index == slot (< num_slots), count field == C and
// frag id == index + B, with B and C the call's constants (header row 0's frag id - index and
// count).  Senders that number fragments in sequence and index slots by them
// (DataManager.py:116-134: index = (seq + i) mod pool, frag id = seq + i) make every packet of a
// pass over the pool plain.  The digit pass of a shuffled narrow split-row batch reads the
// header rows in arrival order (coalesced) and sets the bit; the sorted run then reads no header
// row for a plain packet -- each such read was a random 16-byte gather costing a whole line.
// No digit covers the bit; the run masks it out of the slot.
constexpr uint32_t kPlainBit = 0x40000000u;

// A batch's slot keys as the detection pass makes them (slot = index % num_slots, num_slots for
// another switch's packets, bit 31 = PS ack when ack_hint): read from the detection pass's key
// array, or -- narrow batches with descriptors (round 6) -- made again from the descriptor, the
// same arithmetic (an index already below num_slots skips the division).  There the detection
// pass stores a wave's keys only when the wave found a descent (a wave of a batch in slot order
// or of a dense run stores none: 26 MB of stores left the pass in front of every NGA-32 C3 call)
// and tags the wave's entry of `flags` with the call's epoch; a reader takes the array where the
// tag matches and the descriptor elsewhere (the in-order run: always the descriptor).
#ifndef INA_SWITCH_PLAIN
#define INA_SWITCH_PLAIN 1
#endif
#ifndef INA_KEYS_FROM_DESC
#define INA_KEYS_FROM_DESC 1
#endif
constexpr uint32_t kKeysSpanMax = 65535;      // slots a storing detection wave may span
// ... and must span more than this: a wave of small local disorder leaves its keys to the
// descriptors, which the lists then read instead.  NGA-32 C3 split (profiles/r06/lab/
// keys_span_min_ab_v32.log): jitter 64 289-290 -> 285 us, jitter 512 296 -> 292, jitter 4096
// unchanged at 128 (its waves span 193-256 slots; a minimum of 256 lost it 13 us)
#ifndef INA_KEYS_SPAN_MIN
#define INA_KEYS_SPAN_MIN 128
#endif
constexpr uint32_t kKeysSpanMin = INA_KEYS_SPAN_MIN;
struct KeySrc {
    const uint32_t* keys;
    const uint2* desc;
    uint32_t num_slots;
    int switch_id;
    bool ack_hint;
    const uint32_t* flags = nullptr;   // per detection wave (64 R positions, 2^kb_shift): the epoch if stored
    uint32_t epoch = 0, kb_shift = 0;
    __device__ __forceinline__ uint32_t operator()(size_t p) const {
        if (!desc || (flags && flags[p >> kb_shift] == epoch)) return keys[p];
        const uint2 d = desc[p];
        const uint32_t idx = __builtin_bswap32((d.x >> 16) | (d.y << 16));
        const bool mine = switch_id >= 0 && ((d.y >> 16) & 0xFFu) == (uint32_t)(uint8_t)switch_id;
        if (!mine) return num_slots;
        const uint32_t slot = idx < num_slots ? idx : idx % num_slots;
        return slot | ((ack_hint && ((d.x >> 14) & 1u)) ? kAckBit : 0u);
    }
};
template <int R, bool kDesc, int NW = kRsWaves>
__global__ __launch_bounds__(NW * 64) void k_switch_keys(const uint8_t* __restrict__ pkts,
                                                          const uint2* __restrict__ desc,
                                                          size_t npk, size_t stride,
                                                          uint32_t num_slots, int switch_id,
                                                          uint32_t* __restrict__ keys,
                                                          uint8_t* __restrict__ actions, int bits,
                                                          int shift, uint32_t* __restrict__ hist,
                                                          size_t nch, int ack_hint,
                                                          uint32_t* __restrict__ ctl, uint32_t epoch) {
    __shared__ uint32_t h[kRsBins];
    // the control block's epochs say "sorted" for ina_switch_batch_path (the run kernel of the
    // digit passes never reads them)
    if (ctl && blockIdx.x == 0 && threadIdx.x == 0) {
        ctl[0] = epoch;
        ctl[1] = epoch;
        ctl[2] = 0u;
    }
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
// ina_set_tuning key 12, the slot sort: 0 auto (chunk + bucket sort for keys of one or two
// digits, else the LSD digit passes), 3 the digit passes for every batch (the cross-check the
// tests run both ways).  The one-sweep and round-2 bucket + local variants moved to tools/lab
// (DESIGN.md section 4).
static std::atomic<int> g_sort_mode{0};
static std::atomic<int> g_os_rounds{0};    // ina_set_tuning key 13: sort chunk rounds (0 auto, 4/8/16)
static std::atomic<uint32_t> g_sort_epoch{0};   // per-call tag of the chunk sort's "unsorted" flag
static std::atomic<int> g_runs{1};         // ina_set_tuning key 18: dense-run batches skip the sort (0: off)
int set_runs(int v) {
    g_runs = v ? 1 : 0;
    return INA_OK;
}
static std::atomic<int> g_local{1};        // ina_set_tuning key 20: near-sorted batches skip the sort (0: off)
int set_local(int v) {
    g_local = v ? 1 : 0;
    return INA_OK;
}
// ina_set_tuning key 21 (tests): block 0 of the decision pass waits this many microseconds
// before it decides, so every other block's bounded wait for the near-sorted verdict runs out
// and it sorts its chunk anyway -- the shape of a block 0 dispatched late (0: off, the default)
static std::atomic<int> g_decide_delay{0};
int set_decide_delay(int v) {
    if (v < 0 || v > 100000) return INA_EINVAL;
    g_decide_delay = v;
    return INA_OK;
}
// ina_set_tuning key 19: the split chunk pass (detection, decision, then digits) for every key
// width (1, default) or for keys of 19-22 bits only (0).  Interleaved over packed and split
// rows at 819,200 NGA-256 packets (tools/lab/switch_pre_lab.py, profiles/r04/lab): worker-
// major -3.8 / -3.2 us, round-robin -6.1 / -5.4 us, a shuffled batch +5.6 / +4.9 us (it pays
// the detection pass and one launch more); NIC arrival is structured, so split by default
#ifndef INA_SWITCH_PRE_ALL
#define INA_SWITCH_PRE_ALL 1
#endif
static std::atomic<int> g_pre_all{INA_SWITCH_PRE_ALL};
int set_pre_all(int v) {
    g_pre_all = v ? 1 : 0;
    return INA_OK;
}
int set_sort_mode(int v) {
    if (v != 0 && v != 3) return INA_EINVAL;
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

// ---- chunk + bucket slot sort (keys of one or two digits; the default) --------------------
// Two launches instead of the digit passes' keys / column scan / scatter / bucket-local four:
//   A  k_sort_chunks   one block per chunk of CH = 16 waves x 64 x R packets: the packets'
//                      keys, and the chunk sorted STABLY by the key's high digit inside its
//                      own range of the output (per-wave LDS digit counts, a block scan, the
//                      ballot-ranked tile scatter), publishing per (digit, chunk) the run
//                      length and the run's start inside the chunk (= the chunk's packets
//                      in lower buckets).
//   B  k_sort_buckets  one block per bucket (high digit): its row of run lengths gives where
//                      each chunk's run goes inside the bucket, its row of run starts sums
//                      to the bucket's place in the output (no block waits for another);
//                      it gathers its runs in chunk order -- arrival order -- and sorts them
//                      on the low digit in LDS (tile by tile after a counting sweep when
//                      the bucket is larger than one tile).
// The permutation equals the LSD passes' (stable by (high, low) digit, arrival order inside
// a slot), so the run kernel sees the same arrays.  The bucket of foreign packets only (a
// pool that is a multiple of 2^lb slots) is not gathered: B stores its size and the
// register-resident run kernel stops before it.  Keys of one digit (pools < 512 slots) are
// the same with lb = 0: B only gathers.
#ifndef INA_BK_WAVES
#define INA_BK_WAVES 16
#endif
constexpr int kBkWaves = INA_BK_WAVES;
constexpr int kBkThr = kBkWaves * 64;
constexpr int kBkMaxChunks = 2048;                  // B's LDS rows: up to 2048 x CH packets
// B's tile: 16 waves x 64 x R items.  R = 4 (4,096) by default; 8,192 (R = 8) takes the
// steady-state batch's 9 x 512-packet buckets in one pass (24.4 -> 18.8 us for B) but costs
// the plain 8-worker batch (3,200 per bucket) 1-3 us (profiles/r03/lab/bucket_tile_lab.log),
// so the launch picks R = 8 only when the average bucket exceeds 7/8 of the smaller tile
constexpr int kLcRounds = 4;
constexpr int kLcRoundsBig = 8;
constexpr size_t kBigTileAvg = (size_t)kBkWaves * 64 * kLcRounds * 7 / 8;   // 3,584 items
static std::atomic<int> g_bucket_tile{0};   // ina_set_tuning key 17: 0 auto, 4 or 8 rounds
int set_bucket_tile(int v) {
    if (v != 0 && v != kLcRounds && v != kLcRoundsBig) return INA_EINVAL;
    g_bucket_tile = v;
    return INA_OK;
}

// The switch keys one batch runs under, read ONCE per call.  A sort-only call (phase 1)
// records its snapshot with the scratch it filled (g_sorts), and the run over that scratch
// (phase 2) follows the record, never the live keys: a thread that tunes between another
// thread's sort and run changes nothing in that batch (the run used to re-read
// key 19 and pick arrays the sort never wrote).
struct SwitchTuning {
    int small_sort, tiny_max, sort_mode, os_rounds, runs, local, pre_all, ack_fast, win, bucket_tile,
        decide_delay;
};
static SwitchTuning switch_tuning() {
    return SwitchTuning{g_small_sort.load(), g_tiny_max.load(), g_sort_mode.load(), g_os_rounds.load(),
                        g_runs.load(),       g_local.load(),    g_pre_all.load(),   g_ack_fast.load(),
                        g_switch_win.load(), g_bucket_tile.load(), g_decide_delay.load()};
}

// key fields of R rounds of 64 packets (all loads issued first): slot index, switch id and
// the PS-ack flag, from the batch's descriptors (header bytes 4..11) or the headers
template <int R, bool kDesc>
__device__ __forceinline__ void load_key_fields(const uint8_t* __restrict__ pkts, const uint2* __restrict__ desc,
                                                size_t npk, size_t stride, size_t p0, uint32_t (&idx)[R],
                                                uint32_t (&sid)[R], uint32_t (&ack)[R]) {
    if (kDesc) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t p = p0 + (size_t)r * 64;
            const uint2 d = p < npk ? desc[p] : uint2{0u, 0u};
            idx[r] = __builtin_bswap32((d.x >> 16) | (d.y << 16));
            sid[r] = (d.y >> 16) & 0xFFu;
            ack[r] = (d.x >> 14) & 1u;                         // flags byte 5, bit 6
        }
    } else if ((stride & 3) == 0 && ((uintptr_t)pkts & 3u) == 0) {
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
            ack[r] = (w1 >> 14) & 1u;
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
}

// exclusive scan of one value per thread over the block (thread d = digit d; kRsBins <=
// kBkThr, so one digit per thread), plus `carry`: wave DPP scans and one LDS exchange of the
// wave totals instead of one wave walking the digits serially.  Call convergent.
static_assert(kRsBins <= kBkThr, "one digit per thread");
__device__ __forceinline__ uint32_t block_digit_scan(uint32_t x, uint32_t* wtot, uint32_t carry) {
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const uint32_t inc = wave_incl_scan(x);
    if (lane == 63) wtot[wv] = inc;
    __syncthreads();
    uint32_t pre = carry;
#pragma unroll
    for (int w = 0; w < kBkWaves; ++w) pre += w < wv ? wtot[w] : 0u;
    return pre + inc - x;
}

// The chunk + bucket sort's digits: 512 bins (keys of <= 18 bits: two 9-bit digits) or, for
// pools of 2^18 .. 2^21 slots (keys of 19-22 bits), 2,048 bins (digits of 10-11 bits; the
// bucket pass's LDS then holds 16 x 2,048 per-wave counts, 152 KiB of the CU's 160).  With
// 2,048 bins a thread owns kDigitsPerThread CONSECUTIVE digits d = t * DPT + j, so the
// block scan of their sums orders them.
constexpr int kBinsBig = 2048;
constexpr int kBitsBig = 11;
template <int BINS>
constexpr int kDigitsPerThread = BINS > kBkThr ? BINS / kBkThr : 1;
static_assert(kBinsBig % kBkThr == 0, "whole digits per thread");
// exclusive positions of the thread's DPT consecutive digits (counts x[]), after `carry`
template <int DPT>
__device__ __forceinline__ void block_digit_scan_n(const uint32_t (&x)[DPT], uint32_t (&ex)[DPT],
                                                   uint32_t* wtot, uint32_t carry) {
    uint32_t tsum = 0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) tsum += x[j];
    uint32_t e = block_digit_scan(tsum, wtot, carry);
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        ex[j] = e;
        e += x[j];
    }
}

// ---- structured batches: dense ascending runs --------------------------------------------
// A batch made of a few runs of consecutive slots -- each worker's packets for slots s, s+1,
// ... (worker-major arrival), the PS's acks for the previous step in front of them -- needs
// no sort: slot s's segment is, in arrival order, the one packet each run holds for s, at
// run_start + (s - run_first_slot).  A "break" is a packet that does not continue its
// predecessor's run (first packet, slot != predecessor's + 1, a change of the PS-ack flag,
// a foreign packet).  The chunk pass records each chunk's breaks (count + up to kRunsMax
// (position, key) entries); when the whole batch has at most kRunsMax of them the bucket
// pass builds the run table instead of sorting and the run kernel walks slots
// (switch_runs_body).  Slots are independent (ngaa.p4:87-168) and a slot's packets stay in
// arrival order (ngaa.p4:120-196), so the results are those of the sorted run.
constexpr int kRunsMax = 64;   // one run per lane of the run kernel's waves
// control block in the sort scratch (32-bit words): [0] foreign-bucket size, [1..3] epochs
// (descent found, chunk pass, run table valid), then the run table: R, start[kRunsMax + 1]
// (start[R] = npk), key[kRunsMax] (slot | ack bit of each run's first packet)
constexpr int kCtlForeign = 0, kCtlEpochs = 1, kCtlRuns = 4;
constexpr int kRunsStart = 1, kRunsKey = 2 + kRunsMax;
// then the near-sorted path's words (see "near-sorted batches" below): the epoch of the last
// call that chose it, the smallest slot key, the number of slots its table covers and the
// number of units
constexpr int kCtlLocal = kCtlRuns + kRunsKey + kRunsMax;
constexpr int kLocEpoch = kCtlLocal - kCtlEpochs;     // offsets from the epochs (`unsorted`)
constexpr int kLocKmin = kLocEpoch + 1, kLocSlots = kLocEpoch + 2, kLocUnits = kLocEpoch + 3;
// the sorted narrow run's plain-packet constants (see kPlainBit): frag id - index, count field
constexpr int kPlainB = kLocEpoch + 4, kPlainC = kLocEpoch + 5;
constexpr int kLocVerdict = kLocEpoch + 6;            // 2 words: the decision, (epoch << 1) | local
static_assert((kCtlEpochs + kLocVerdict) % 2 == 0, "the verdict is 8-byte aligned in the control block");
constexpr int kCtlWords = kCtlLocal + 8;
static_assert(kCtlWords * 4 <= 1024, "control block fits its 1 KiB");

// the run table from the chunks' break records (a structured batch, total <= kRunsMax breaks),
// by one block of kBkThr threads: thread t takes chunks 2t and 2t+1 (nch <= 2 x kBkThr), so the
// entries land in chunk order = position order
__device__ __forceinline__ void build_run_table(const uint32_t* __restrict__ brk_cnt, const uint2* __restrict__ brk_ent,
                                                uint32_t nch, uint32_t total, uint32_t npk,
                                                uint32_t* __restrict__ unsorted, uint32_t epoch, uint32_t* wtot) {
    const uint32_t c0 = 2u * threadIdx.x;
    const uint32_t n0 = c0 < nch ? brk_cnt[c0] : 0u, n1 = c0 + 1 < nch ? brk_cnt[c0 + 1] : 0u;
    const uint32_t ex = block_digit_scan(n0 + n1, wtot, 0u);
    uint32_t* runs = unsorted + (kCtlRuns - kCtlEpochs);
    for (uint32_t j = 0; j < n0; ++j) {
        const uint2 e = brk_ent[(size_t)c0 * kRunsMax + j];
        runs[kRunsStart + ex + j] = e.x;
        runs[kRunsKey + ex + j] = e.y;
    }
    for (uint32_t j = 0; j < n1; ++j) {
        const uint2 e = brk_ent[(size_t)(c0 + 1) * kRunsMax + j];
        runs[kRunsStart + ex + n0 + j] = e.x;
        runs[kRunsKey + ex + n0 + j] = e.y;
    }
    if (threadIdx.x == 0) {
        runs[0] = total;
        runs[kRunsStart + total] = npk;
        unsorted[2] = epoch;                          // the run table is this call's
    }
}

// lds_count with the count shifted into the wave's half (the partner wave adds to the other
// half of the same word, hence atomics)
__device__ __forceinline__ void lds_count_half(uint32_t* h, uint32_t d, bool valid, int sh) {
    const unsigned long long act = __ballot(valid);
    if (!act) return;
    const int first = __builtin_ctzll(act);
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, first);
    const unsigned long long same = __ballot(valid && d == d0);
    if (same == act) {
        if ((int)(threadIdx.x & 63) == first) atomicAdd(&h[d0], (uint32_t)__builtin_popcountll(act) << sh);
    } else if (valid) {
        atomicAdd(&h[d], 1u << sh);
    }
}

// ---- near-sorted batches: per-slot lists, no sort (round 5) ---------------------------------
// W senders each emit their packets in sequence order (DataManager.py:116-134); a NIC that
// interleaves them with local disorder delivers a batch whose every packet sits within some
// distance D of its place in slot order, yet with far more than kRunsMax descents: neither in
// order nor dense runs, so it used to take the full chunk + bucket sort.  Such a batch needs no
// global order -- slots are independent (ngaa.p4:87-168), so each slot only needs its own
// packets in arrival order (ngaa.p4:120-196):
//   * the detection pass records each GRANULE's (kGranWaves waves of a chunk: 1/8 of it)
//     smallest and largest slot key;
//   * the digit pass's block 0 (local_decide; the other blocks wait for its verdict) turns them
//     into PM[g] = max over granules <= g and SM[g] = min over granules >= g (both non-decreasing).
//     UNIT u (kLocU granules) takes the slots [SM(u kLocU), SM((u+1) kLocU)): every packet past
//     the unit's granules has a key >= the unit's upper bound, and every packet before granule
//     g_lo(u) = the first g with PM[g] >= its lower bound has a key below it, so the unit's
//     packets all lie in its WINDOW, granule g_lo(u) to its last granule, whatever the disorder
//     -- which only widens the windows.  The path is taken when the windows' total scan (x the
//     LDS passes a wide slot range needs) stays within kLocBeta times the batch and no window
//     exceeds 65,535 positions; it writes the unit table;
//   * a unit's place in the list area needs no global scan: A(u) = #packets with a key below
//     its slots + #foreign packets before its granules = g_lo(u)'s first position + the window's
//     packets before the unit's granules that are foreign or below its slots, and A(u+1) - A(u)
//     >= the unit's packets;
//   * k_local_lists builds the lists, a 4-wave block per unit: its waves scan the unit's window
//     in position order, per-wave LDS counts of its slots (16-bit halves: counts and cursors stay
//     inside the window), a block scan, then each packet to its slot's list at the wave's cursor
//     + its ballot rank among the round's lanes of the same slot -- a stable counting sort: ids[]
//     (the sort's idle k_out) holds each slot's packets in arrival order, tab[slot - kmin] its
//     (first entry, length);
//   * the run kernel's lane groups take 8 slots at a time and walk each list through
//     group_packet -- the run table's and the sorted run's per-packet code.
// No key array is sorted, the ids are written once, and the row gather is as local as the arrival.
constexpr int kGranWaves = 2;                                 // detection-pass waves per granule
constexpr int kGranPerChunk = kBkWaves / kGranWaves;          // 8 granules per chunk
constexpr int kLocMaxGran = 8 * kBkThr;                       // the decision: <= 8 granules a thread
constexpr uint32_t kLocBeta = 3;                              // the windows' scan <= 3 x the batch
constexpr uint32_t kLocMaxWindow = 65535;                     // 16-bit cursors
// how long a digit-pass block waits for block 0's near-sorted verdict before it sorts its chunk
// anyway (constant 100 MHz clock: 50 us; block 0's decision takes ~8 us, r05)
constexpr unsigned long long kLocPollTicks = 5000;
#ifndef INA_LOC_U
#define INA_LOC_U 4                                           // granules per unit (a half chunk)
#endif
constexpr uint32_t kLocU = INA_LOC_U;
#ifndef INA_LL_WAVES
#define INA_LL_WAVES 4
#endif
constexpr int kLlWaves = INA_LL_WAVES;                        // waves per unit in the list build
constexpr int kLlBins = 1024;                                 // slots one LDS pass counts
constexpr int kLlBits = 10;
#ifndef INA_LL_ROUNDS
#define INA_LL_ROUNDS 20      // a J = 64 unit window (5 granules) held: 310.1 -> 304.3 us (r05v)
#endif
constexpr int kLlRounds = INA_LL_ROUNDS;                      // key rounds a lane holds

// wave-wide inclusive max (lane i: max over lanes <= i) and suffix min (lane i: min over lanes >= i)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x = max(x, y);
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_suffix_min(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_down((int)x, o);
        if (lane + o < 64) x = min(x, y);
    }
    return x;
}

#ifndef INA_LOC_TIMING
#define INA_LOC_TIMING 0
#endif
#if INA_LOC_TIMING
// lab builds only: per-unit wall-clock stamps of k_local_lists' phases (tools/lab)
__device__ unsigned long long g_loc_t[8192][4];
#define LOC_STAMP(q) do { if (threadIdx.x == 0 && u < 8192) g_loc_t[u][q] = wall_clock64(); } while (0)
// the decision pass: rows 8191 (block 0: entry, breaks summed, decided) and 8190 (the last
// block: entry, verdict seen)
#define DEC_STAMP(row, q) do { if (threadIdx.x == 0) g_loc_t[row][q] = wall_clock64(); } while (0)
#else
#define LOC_STAMP(q) do { } while (0)
#define DEC_STAMP(row, q) do { } while (0)
#endif

// unit u: slots [lo, hi), window from granule g_lo to the unit's last granule
struct LocUnit {
    uint32_t g_lo, lo, hi, pad;
};

// The near-sorted decision (call convergent): true when the batch takes the path.  `writer`
// also writes the unit table and the control words.  s_pm / s_sm: G words each of the caller's LDS (its count array,
// free before the digits); s_a / s_b: kBkWaves words each.
__device__ __forceinline__ bool local_decide(const uint32_t* __restrict__ gmin, const uint32_t* __restrict__ gmax,
                                             uint32_t G, uint32_t gsize, size_t npk,
                                             uint32_t* __restrict__ unsorted, uint32_t epoch,
                                             LocUnit* __restrict__ units, bool writer, uint32_t* s_pm,
                                             uint32_t* s_sm, uint32_t* s_a, uint32_t* s_b) {
    __shared__ unsigned long long s_cost[kBkWaves];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    // thread t: granules [g0, g0 + kpt), in registers (every load in flight at once) -- prefix
    // max / suffix min inside the thread ...
    constexpr int kGpt = kLocMaxGran / kBkThr;
    const uint32_t kpt = (G + kBkThr - 1) / kBkThr;                   // <= kGpt
    const uint32_t g0 = threadIdx.x * kpt;
    uint32_t pm[kGpt], sm[kGpt];
#pragma unroll
    for (int j = 0; j < kGpt; ++j) {
        const uint32_t g = g0 + (uint32_t)j;
        const bool ok = (uint32_t)j < kpt && g < G;
        pm[j] = ok ? gmax[g] : 0u;
        sm[j] = ok ? gmin[g] : 0xFFFFFFFFu;
    }
    uint32_t tmax = 0, tmin = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < kGpt; ++j) pm[j] = tmax = max(tmax, pm[j]);
#pragma unroll
    for (int j = kGpt - 1; j >= 0; --j) sm[j] = tmin = min(tmin, sm[j]);
    // ... and over the threads: the max of the earlier ones, the min of the later ones
    const uint32_t imx = wave_incl_max(tmax), imn = wave_suffix_min(tmin);
    if (lane == 63) s_a[wv] = imx;
    if (lane == 0) s_b[wv] = imn;
    __syncthreads();
    uint32_t xmx = 0, xmn = 0xFFFFFFFFu, kmax = 0, kmin = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 0; w < kBkWaves; ++w) {
        const uint32_t a = s_a[w], b = s_b[w];
        xmx = w < wv ? max(xmx, a) : xmx;
        xmn = w > wv ? min(xmn, b) : xmn;
        kmax = max(kmax, a);
        kmin = min(kmin, b);
    }
    {
        const uint32_t up = (uint32_t)__shfl_up((int)imx, 1), dn = (uint32_t)__shfl_down((int)imn, 1);
        if (lane > 0) xmx = max(xmx, up);
        if (lane < 63) xmn = min(xmn, dn);
    }
#pragma unroll
    for (int j = 0; j < kGpt; ++j) {
        const uint32_t g = g0 + (uint32_t)j;
        if ((uint32_t)j < kpt && g < G) {
            s_pm[g] = max(pm[j], xmx);
            s_sm[g] = min(sm[j], xmn);
        }
    }
    __syncthreads();                                          // PM / SM final; s_a is reused
    if (kmin > kmax) return false;                            // no packet of this switch
    DEC_STAMP(8189, 0);
    // the units: slot range, window, scan cost (window x LDS passes).  Thread t takes units
    // [t upt, (t+1) upt) and keeps them in registers: one binary search for g_lo of its first
    // unit (PM is non-decreasing), then a short forward walk for the next (g_lo grows with u)
    constexpr uint32_t kUpt = (kLocMaxGran / kLocU + kBkThr - 1) / kBkThr;
    const uint32_t nu = (G + kLocU - 1) / kLocU;
    const uint32_t upt = (nu + kBkThr - 1) / kBkThr;                  // <= kUpt (G <= kLocMaxGran)
    LocUnit mu[kUpt];
    unsigned long long cost = 0;
    uint32_t maxwin = 0, glo = 0;
#pragma unroll
    for (uint32_t j = 0; j < kUpt; ++j) {
        const uint32_t u = threadIdx.x * upt + j;
        mu[j] = LocUnit{0u, 0u, 0u, 0u};
        if (j >= upt || u >= nu) continue;
        const uint32_t a = s_sm[u * kLocU];
        const uint32_t b = (u + 1) * kLocU < G ? s_sm[(u + 1) * kLocU] : 0xFFFFFFFFu;
        const uint32_t lo = a == 0xFFFFFFFFu ? kmax + 1u : a, hi = b == 0xFFFFFFFFu ? kmax + 1u : b;
        uint32_t l = glo, r = G;
        if (j > 0)
            for (int s = 0; s < 8 && l < r && s_pm[l] < lo; ++s) ++l;
        if (l < r && s_pm[l] < lo)
            while (l < r) {
                const uint32_t m = (l + r) >> 1;
                if (s_pm[m] >= lo) r = m; else l = m + 1;
            }
        glo = l;
        mu[j] = LocUnit{l, lo, hi, 0u};
        const size_t p0 = (size_t)l * gsize, p1 = min((size_t)(u + 1) * kLocU * gsize, npk);
        const uint32_t win = hi > lo && p1 > p0 ? (uint32_t)min(p1 - p0, (size_t)0xFFFFFFFFu) : 0u;
        cost += (unsigned long long)((hi - lo + kLlBins - 1) / kLlBins) * win;
        maxwin = max(maxwin, win);
    }
    DEC_STAMP(8189, 1);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cost += (unsigned long long)__shfl_xor((long long)cost, o);
        maxwin = max(maxwin, (uint32_t)__shfl_xor((int)maxwin, o));
    }
    if (lane == 0) {
        s_cost[wv] = cost;
        s_a[wv] = maxwin;
    }
    __syncthreads();
    unsigned long long total = 0;
    uint32_t mw = 0;
#pragma unroll
    for (int w = 0; w < kBkWaves; ++w) {
        total += s_cost[w];
        mw = max(mw, s_a[w]);
    }
    DEC_STAMP(8189, 2);
    if (mw > kLocMaxWindow || total > (unsigned long long)kLocBeta * npk) return false;   // the sort
    if (writer) {
#pragma unroll
        for (uint32_t j = 0; j < kUpt; ++j) {
            const uint32_t u = threadIdx.x * upt + j;
            if (j < upt && u < nu) units[u] = mu[j];
        }
        if (threadIdx.x == 0) {
            unsorted[kLocKmin] = kmin;
            unsorted[kLocSlots] = kmax + 1u - kmin;
            unsorted[kLocUnits] = nu;
            unsorted[kLocEpoch] = epoch;                      // the lists, no sort
        }
    }
    return true;
}


// The near-sorted path's lists (see local_decide): one kLlWaves-wave block per unit at a time
// (units u = the block's XCD-ordered index + k * grid: neighbouring units, whose windows share
// granules, through one L2).  Wave w takes its share of the unit's window, in position order,
// holding up to kLlRounds rounds of keys in registers; per pass over kLlBins of the unit's slots:
// per-wave LDS counts (two waves' 16-bit halves per word: counts and cursors stay inside the
// window), a block scan -> each slot's first entry and length (tab) and each wave's cursor; then
// every packet of those slots to its list at the cursor + its ballot rank among the round's
// lanes of the same slot (a stable counting sort).  ids[e] = packet | PS-ack bit 31 (by its sort
// key).
__device__ __forceinline__ size_t switch_block_index();
__device__ __forceinline__ size_t xcd_block_index();
#ifndef INA_LL_WAVES_PER_EU
#define INA_LL_WAVES_PER_EU 8
#endif
__global__ __launch_bounds__(kLlWaves * 64) __attribute__((amdgpu_waves_per_eu(INA_LL_WAVES_PER_EU, 8))) void k_local_lists(const KeySrc keys_in, size_t npk,
                                                               uint32_t num_slots, uint32_t kmask,
                                                               const uint32_t* __restrict__ unsorted,
                                                               const LocUnit* __restrict__ units, uint32_t gsize,
                                                               uint32_t* __restrict__ ids, uint2* __restrict__ tab) {
    constexpr int kThr = kLlWaves * 64;
    constexpr int DPT = kLlBins / kThr;                           // consecutive slots a thread scans
    __shared__ uint32_t cw[kLlWaves / 2][kLlBins];                // per-wave counts, then cursors
    __shared__ uint32_t s_ws[kLlWaves];
    const uint32_t ep = unsorted[1];
    if (unsorted[kLocEpoch] != ep) return;                        // not this path's batch
    KeySrc kall = keys_in;
    kall.epoch = ep;                                              // this call's stored waves
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const int sh = (wv & 1) * 16;
    uint32_t* crow = cw[wv >> 1];
    const unsigned long long below = (1ull << lane) - 1ull;
    const uint32_t kmin = unsorted[kLocKmin], nunits = unsorted[kLocUnits];
    for (uint32_t u = (uint32_t)xcd_block_index(); u < nunits; u += gridDim.x) {
        const LocUnit w = units[u];
        if (w.hi <= w.lo) continue;                               // no slot (block-uniform)
        LOC_STAMP(0);
        // positions fit 32 bits (npk <= 2^31 - 1)
        const uint32_t P0 = w.g_lo * gsize, Pu = u * kLocU * gsize;
        const uint32_t P1 = (uint32_t)min((size_t)Pu + (size_t)kLocU * gsize, npk);
        const uint32_t per = ((P1 - P0 + kLlWaves * 64 - 1) / (kLlWaves * 64)) * 64;
        const uint32_t b0 = min(P0 + (uint32_t)wv * per, P1), b1 = min(b0 + per, P1);
        const bool held = per <= 64u * kLlRounds;                 // the keys stay in registers
        // one source for the whole window: the stored keys when every detection wave of the
        // window stored its own (a near-sorted batch: each has a descent), else the descriptors
        // (the same values) -- no per-key tag test between a load and the next
        KeySrc keys = kall;
        if (kall.desc && kall.flags) {
            bool miss = false;
            for (uint32_t f = (P0 >> kall.kb_shift) + (uint32_t)lane; f <= ((P1 - 1u) >> kall.kb_shift); f += 64u)
                miss |= kall.flags[f] != ep;
            if (__ballot(miss)) keys.flags = nullptr;             // the descriptors throughout
            else keys.desc = nullptr;                             // the stored keys throughout
        }
        uint32_t kk[kLlRounds];
        if (held) {
#pragma unroll
            for (int r = 0; r < kLlRounds; ++r) {
                const uint32_t p = b0 + (uint32_t)(r * 64 + lane);
                kk[r] = p < b1 ? keys(p) : num_slots;
            }
        }
        uint32_t area = 0;
        for (uint32_t q = w.lo; q < w.hi; q += kLlBins) {
            const uint32_t qn = min((uint32_t)kLlBins, w.hi - q);
            for (uint32_t d = lane; d < (uint32_t)kLlBins; d += 64) crow[d] = 0u;
            __syncthreads();                                      // the partner wave zeroes too
            uint32_t before = 0;                                  // (first pass) the area's count
            for (uint32_t r0 = b0; r0 < b1; r0 += 64 * kLlRounds) {
                if (!held) {
#pragma unroll
                    for (int r = 0; r < kLlRounds; ++r) {
                        const uint32_t p = r0 + (uint32_t)(r * 64 + lane);
                        kk[r] = p < b1 ? keys(p) : num_slots;
                    }
                }
#pragma unroll
                for (int r = 0; r < kLlRounds; ++r) {
                    const uint32_t slot = kk[r] & kmask;
                    const uint32_t p = r0 + (uint32_t)(r * 64 + lane);
                    lds_count_half(crow, slot - q, slot < num_slots && slot - q < qn, sh);
                    before += (p < Pu && p < b1 && (slot < w.lo || slot >= num_slots)) ? 1u : 0u;
                }
            }
            if (q == w.lo) {
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) before += (uint32_t)__shfl_xor((int)before, o);
                if (lane == 0) s_ws[wv] = before;
            }
            __syncthreads();
            if (q == w.lo) {
                area = P0;
#pragma unroll
                for (int v = 0; v < kLlWaves; ++v) area += s_ws[v];
            }
            LOC_STAMP(1);
            // thread t: slots d = t*DPT + j -- totals, the block scan, then the per-wave cursors
            uint32_t tc[DPT], tt = 0;
#pragma unroll
            for (int j = 0; j < DPT; ++j) {
                const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
                uint32_t t = 0;
#pragma unroll
                for (int v2 = 0; v2 < kLlWaves / 2; ++v2) {
                    const uint32_t word = cw[v2][d];
                    t += (word & 0xFFFFu) + (word >> 16);
                }
                tc[j] = t;
                tt += t;
            }
            __syncthreads();                                      // s_ws is reused by the scan
            const uint32_t inc = wave_incl_scan(tt);
            if (lane == 63) s_ws[wv] = inc;
            __syncthreads();
            uint32_t e = inc - tt, passn = 0;
#pragma unroll
            for (int v = 0; v < kLlWaves; ++v) {
                const uint32_t x = s_ws[v];
                e += v < wv ? x : 0u;
                passn += x;
            }
#pragma unroll
            for (int j = 0; j < DPT; ++j) {
                const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
                if (d < qn) tab[q + d - kmin] = uint2{area + e, tc[j]};
                uint32_t b = e;
#pragma unroll
                for (int v2 = 0; v2 < kLlWaves / 2; ++v2) {
                    const uint32_t word = cw[v2][d];
                    const uint32_t lo16 = word & 0xFFFFu;
                    cw[v2][d] = b | ((b + lo16) << 16);           // cursors, relative to the area
                    b += lo16 + (word >> 16);
                }
                e += tc[j];
            }
            __syncthreads();
            LOC_STAMP(2);
            for (uint32_t r0 = b0; r0 < b1; r0 += 64 * kLlRounds) { // the lists, in arrival order
                if (!held) {
#pragma unroll
                    for (int r = 0; r < kLlRounds; ++r) {
                        const uint32_t p = r0 + (uint32_t)(r * 64 + lane);
                        kk[r] = p < b1 ? keys(p) : num_slots;
                    }
                }
#pragma unroll
                for (int r = 0; r < kLlRounds; ++r) {
                    if (r0 + (uint32_t)(r * 64) >= b1) break;     // wave-uniform
                    const uint32_t slot = kk[r] & kmask;
                    const uint32_t d = slot - q;
                    const bool valid = slot < num_slots && d < qn;
                    const unsigned long long pm = lanes_with_digit(d, kLlBits, valid);
                    if (valid) {
                        const uint32_t rank = (uint32_t)__builtin_popcountll(pm & below);
                        const uint32_t cur = (crow[d] >> sh) & 0xFFFFu;
                        ids[area + cur + rank] = (r0 + (uint32_t)(r * 64 + lane)) | (kk[r] & ~kmask);
                        if (rank == 0) atomicAdd(&crow[d], (uint32_t)__builtin_popcountll(pm) << sh);
                    }
                }
            }
            area += passn;
            __syncthreads();                                      // cw of the next pass or unit
        }
        LOC_STAMP(3);
    }
}

// the 2,048-bin chunk pass stages its sorted chunk in LDS and writes it out contiguously
// (interleaved A/B at NGA-32 C3 size, shuffled: 732.8 -> 709.2 us packed, 639.7 -> 615.9 us
// split, bytes equal; profiles/r04/lab/sort_stage_ab_v32.log).  The LDS (104 KiB) costs
// the second block per CU the packed counts bought; the contiguous stores win.
// (lab) the largest chunk rounds the staging takes: at 8,192-packet chunks it costs one block
// per CU (139 KiB) and still wins, NGA-32 shuffled 654 vs 691 us unstaged at two blocks per
// CU (profiles/r04/lab/stage_big_chunk_ab_v32.log)
// the staging reuses the digit-count LDS once the offsets are read (0: its own arrays)
#ifndef INA_SORT_STAGE_ALIAS
#define INA_SORT_STAGE_ALIAS 1
#endif
#ifndef INA_SORT_STAGE_MAX_R
#define INA_SORT_STAGE_MAX_R 8
#endif
#ifndef INA_SORT_STAGE
#define INA_SORT_STAGE 1
#endif
// The 2,048-bin chunk pass and the 1,024- / 2,048-bin bucket pass keep two waves' per-digit
// counts in one LDS word (16 bits each: a wave counts at most 64 x 8 items of a digit, and
// the offsets below stay inside one chunk or tile, <= 8,192): half the count array, so two
// chunk blocks or three bucket blocks (1,024 bins) share a CU instead of one.
// rs_tile_scatter over the packed counts: each wave's offset of digit d inside the digit's
// run in this chunk (16-bit halves), the run's first output position in gst[d]
// kPosOnly: no stores -- each item's place minus sbase into spos_out (~0u: none), for a caller
// that stages the output itself
template <int R, int BINS, bool kStage = false, bool kPosOnly = false>
__device__ __forceinline__ void rs_tile_scatter_half(const uint32_t (&k)[R], const uint32_t (&v)[R],
                                                     size_t i0, size_t n, int shift, int bits,
                                                     uint32_t (*base)[BINS], const uint32_t* gst,
                                                     uint32_t* __restrict__ kout,
                                                     uint32_t* __restrict__ vout, int rw = R,
                                                     uint32_t* sk = nullptr, uint32_t* sv = nullptr,
                                                     uint32_t sbase = 0u, uint32_t* spos_out = nullptr) {
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    const int sh = (wv & 1) * 16;
    uint32_t* row = base[wv >> 1];
    const uint32_t nb = 1u << bits;
    constexpr int kDPT = (BINS + kBkThr - 1) / kBkThr;
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
        const uint32_t d = threadIdx.x + (uint32_t)j * kBkThr;
        if (d >= nb) continue;
        uint32_t b = 0;
#pragma unroll
        for (int w2 = 0; w2 < kBkWaves / 2; ++w2) {
            const uint32_t word = base[w2][d];
            const uint32_t lo = word & 0xFFFFu, hi = word >> 16;
            base[w2][d] = b | ((b + lo) << 16);
            b += lo + hi;
        }
    }
    __syncthreads();
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t spos[R];                                 // staged: the items' chunk-local places
#pragma unroll
    for (int r = 0; r < R; ++r) spos[r] = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r >= rw || i0 - (size_t)lane + (size_t)r * 64 >= n) break;   // wave-uniform
        const bool valid = i0 + (size_t)r * 64 < n;
        const uint32_t d = (k[r] >> shift) & (nb - 1);
        const unsigned long long pm = lanes_with_digit(d, bits, valid);
        const uint32_t rank = (uint32_t)__builtin_popcountll(pm & below);
        const uint32_t b0 = (row[d] >> sh) & 0xFFFFu;
        if (valid) {
            const uint32_t pos = gst[d] + b0 + rank;
            if constexpr (kPosOnly) {
                spos[r] = pos - sbase;
            } else if constexpr (kStage) {            // the chunk's output staged in LDS
#if INA_SORT_STAGE_ALIAS
                spos[r] = pos - sbase;
#else
                sk[pos - sbase] = k[r];
                sv[pos - sbase] = v[r];
#endif
            } else {
                kout[pos] = k[r];
                vout[pos] = v[r];
            }
            if (rank == 0) atomicAdd(&row[d], (uint32_t)__builtin_popcountll(pm) << sh);
        }
    }
    if constexpr (kPosOnly) {
#pragma unroll
        for (int r = 0; r < R; ++r) spos_out[r] = spos[r];
        return;
    }
#if INA_SORT_STAGE_ALIAS
    if constexpr (kStage) {
        // the staging area is the count array itself (sk, sv alias base): every wave's
        // offsets are read before any item lands there
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (spos[r] != 0xFFFFFFFFu) {
                sk[spos[r]] = k[r];
                sv[spos[r]] = v[r];
            }
    }
#endif
}

// kMode: 0 the chunk pass (keys, detection, digits, scatter); split in two (tuning key 19, the
// default; always for keys of 19-22 bits, whose 2,048-bin chunk pass holds one block per CU)
// so a structured batch never pays the digits: 1 = detection only (the arrival-order keys into
// kout, the descent flag, the breaks; no digits, a small LDS footprint), then 2 = the decision
// (every block sums the break counts; dense runs: block 0 writes the run table) and, for a
// batch neither in slot order nor dense runs, the digits + scatter.
// lab builds only (timing what the detection pass's action stores cost; results then differ)
// The digit pass writes each chunk's (digit, chunk) run lengths and starts as COLUMNS (word c of
// row d): neighbouring chunks write neighbouring words, so a line of them is written by 32 chunk
// blocks.  Dispatched round-robin over the XCDs, those blocks sat on 8 L2s and each wrote the line
// back partly: 182 MB written against 59 MB of data at NGA-32 C3 size.  With neighbouring chunks
// on one XCD (switch_block_index) the line fills in one L2: 69 MB, shuffled split 436 -> 426 us
// (profiles/r06/lab/sort_stage_xcd_ab_v32.log)
#ifndef INA_CHUNK_XCD
#define INA_CHUNK_XCD 1
#endif
// A one-tile bucket's sorted keys and values leave through LDS as two contiguous runs instead of
// scattered 4-byte stores: the bucket pass wrote 214 MB for 52 MB of keys and values, now 52 MB;
// shuffled split 436 -> 404 us, with the chunk mapping 393 us (same log; NGA-256 neutral)
#ifndef INA_BUCKET_STAGE
#define INA_BUCKET_STAGE 1
#endif
#ifndef INA_BUCKET_XCD
#define INA_BUCKET_XCD 0
#endif
// Groups of 8 neighbouring buckets on one XCD: a bucket's run in a digit-pass chunk is ~6 items,
// so the runs of neighbouring buckets share lines, and round-robin dispatch read each line into
// up to eight L2s (218 MB read for ~60 MB at NGA-32 C3 size, shuffled).  Groups of 8: 79 MB, the
// shuffled split call 386 -> 378 us, packed 554 / 515 -> 538 / 506 us, NGA-256 -2 us.  All 128 of
// an XCD's buckets in one run (INA_BUCKET_XCD) reads 62 MB but costs 7 us: its in-flight blocks
// then share too few lines (profiles/r06/lab/bucket_group_ab_v32.log, bucket_xcd_ab_v32.log)
#ifndef INA_BUCKET_GROUP
#define INA_BUCKET_GROUP 8
#endif
#ifndef INA_LAB_DETECT_NOACT
#define INA_LAB_DETECT_NOACT 0
#endif
template <int R, bool kDesc, int BINS, int kMode = 0>
__global__ __launch_bounds__(kBkThr) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_sort_chunks(const uint8_t* __restrict__ pkts,
                                                        const uint2* __restrict__ desc, size_t npk,
                                                        size_t stride, uint32_t num_slots, int switch_id,
                                                        uint8_t* __restrict__ actions, int hbits, int lb,
                                                        uint32_t* __restrict__ rcnt, uint32_t* __restrict__ rst,
                                                        size_t nch, uint32_t* __restrict__ kout,
                                                        uint32_t* __restrict__ vout, int ack_hint,
                                                        uint32_t* __restrict__ unsorted, uint32_t epoch,
                                                        uint32_t* __restrict__ brk_cnt,
                                                        uint2* __restrict__ brk_ent,
                                                        uint32_t* __restrict__ gstat, LocUnit* __restrict__ units,
                                                        uint32_t decide_delay_ticks = 0,
                                                        uint32_t* __restrict__ kflags = nullptr,
                                                        const uint32_t* __restrict__ plain_hdr = nullptr) {
    // per-wave digit counts, then bases (2,048 bins: two waves' 16-bit halves per word)
    constexpr bool kHalf = BINS > kBkThr;
    __shared__ uint32_t base[kHalf ? kBkWaves / 2 : kBkWaves][BINS];
    __shared__ uint32_t gst[BINS];                    // the chunk's run starts (output positions)
    __shared__ uint32_t wtot[kBkWaves];
    __shared__ uint32_t wbrk[kBkWaves];               // per-wave break counts
    __shared__ uint32_t wgmn[kBkWaves], wgmx[kBkWaves];   // per-wave slot-key bounds (near-sorted path)
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    // (INA_CHUNK_XCD: neighbouring chunks on one XCD, so the (digit, chunk) columns they write share its L2)
    const size_t c = INA_CHUNK_XCD && kMode == 2 ? xcd_block_index() : blockIdx.x;
    // gstat (near-sorted path on): granule bounds, gmin[G] then gmax[G], G = 8 granules a chunk
    const uint32_t G = (uint32_t)nch * (uint32_t)kGranPerChunk;
    if constexpr (kMode == 2) {
        if (unsorted[0] != epoch) return;             // in slot order: no sort
        if (c == 0) DEC_STAMP(8191, 0);
        if (c == nch - 1) DEC_STAMP(8190, 0);
        if (brk_cnt) {
            // the decision after the detection pass: every block sums the chunks' break counts
            // (the same answer everywhere); a batch of at most kRunsMax dense runs gets its run
            // table from block 0 and nobody sorts
            uint32_t part = 0;
            for (uint32_t cc = threadIdx.x; cc < (uint32_t)nch; cc += kBkThr) part += brk_cnt[cc];
            const uint32_t inc = wave_incl_scan(part);
            if (lane == 63) wtot[wv] = inc;
            __syncthreads();
            uint32_t total = 0;
#pragma unroll
            for (int w = 0; w < kBkWaves; ++w) total += wtot[w];
            __syncthreads();                          // wtot is reused below
            if (total <= (uint32_t)kRunsMax) {
                if (c == 0) build_run_table(brk_cnt, brk_ent, (uint32_t)nch, total, (uint32_t)npk, unsorted, epoch, wtot);
                return;
            }
        }
        // local disorder within the scan budget: the near-sorted path (the bucket pass builds its
        // lists), no sort.  PM / SM live in the count array (the host takes the path only for G
        // <= half of it)
        // Block 0 decides and publishes the verdict (epoch-tagged, agent scope); the other blocks
        // poll it for at most kLocPollTicks of the constant 100 MHz clock, then do the digits
        // anyway.  No block's progress depends on when (or whether) block 0 is dispatched (ADVICE
        // r05): a verdict that comes late only costs the digits' time, never the results -- on a
        // near-sorted batch the digits land in k_out / v_out and the per-(digit, chunk) rows,
        // which k_local_lists then overwrites (its ids) or nobody reads (the bucket pass and the
        // run kernel follow the verdict's epoch, written before the verdict by block 0).  The
        // verdict itself is the only word shared inside this launch; nothing block 0 writes is
        // read by another block of it (the unit table and the control words are read by the
        // NEXT launches).  Round 5's faulting lab kernel broke exactly these two
        // rules.
        if (gstat) {
            __shared__ uint32_t s_loc;
            unsigned long long* verdict = reinterpret_cast<unsigned long long*>(unsorted + kLocVerdict);
            if (c == 0) {
                DEC_STAMP(8191, 1);
                if (decide_delay_ticks) {                 // (tests: key 21) a late block 0
                    const unsigned long long t0 = wall_clock64();
                    while (wall_clock64() - t0 < decide_delay_ticks) __builtin_amdgcn_s_sleep(64);
                }
                const bool loc = local_decide(gstat, gstat + G, G, (uint32_t)(kBkThr * R / kGranPerChunk), npk,
                                              unsorted, epoch, units, true, &base[0][0],
                                              &base[0][0] + sizeof(base) / 8, wtot, wbrk);
                if (threadIdx.x == 0) {
                    __hip_atomic_store(verdict, ((unsigned long long)epoch << 1) | (loc ? 1ull : 0ull),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_loc = loc ? 1u : 0u;
                }
                DEC_STAMP(8191, 2);
            } else if (threadIdx.x == 0) {
                unsigned long long v;
                uint32_t loc = 0u;
                const unsigned long long t0 = wall_clock64();
                for (;;) {
                    v = __hip_atomic_load(verdict, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((v >> 1) == epoch) {
                        loc = (uint32_t)(v & 1ull);
                        break;
                    }
                    if (wall_clock64() - t0 > kLocPollTicks) break;      // no verdict yet: sort
                    __builtin_amdgcn_s_sleep(8);
                }
                s_loc = loc;
                if (c == nch - 1) DEC_STAMP(8190, 1);
            }
            __syncthreads();
            if (s_loc) return;
        }
    }
    const uint32_t nb = 1u << hbits;
    if constexpr (kMode != 1)
        for (uint32_t d = lane; d < nb; d += 64) base[kHalf ? wv >> 1 : wv][d] = 0;
    const size_t i0 = c * (size_t)(kBkThr * R) + (size_t)wv * (64 * R) + (size_t)lane;
    uint32_t idx[R], sid[R], ack[R], k[R], v[R];
    uint32_t plainm = 0u;                                     // bit r: round r's packet is plain
    if (kMode == 2 && plain_hdr) {
        // (split header rows, 16 B each) the key fields and the plain test from one row read
        const uint32_t w01 = plain_hdr[1], w02 = plain_hdr[2], w03 = plain_hdr[3];
        const uint32_t C0 = w01 & 0xFFu;
        const uint32_t B0 = __builtin_bswap32((w02 >> 24) | (w03 << 8)) - __builtin_bswap32((w01 >> 16) | (w02 << 16));
        if (c == 0 && threadIdx.x == 0) {
            unsorted[kPlainB] = B0;
            unsorted[kPlainC] = C0;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t p = i0 + (size_t)r * 64;
            uint32_t w1 = 0, w2 = 0, w3 = 0;
            if (p < npk) {
                const uint32_t* pk = plain_hdr + p * 4;
                w1 = pk[1];
                w2 = pk[2];
                w3 = pk[3];
            }
            idx[r] = __builtin_bswap32((w1 >> 16) | (w2 << 16));
            sid[r] = (w2 >> 16) & 0xFFu;
            ack[r] = (w1 >> 14) & 1u;
            const uint32_t fr = __builtin_bswap32((w2 >> 24) | (w3 << 8));
            const bool pl = (w1 & 0xFFFFu) == C0 && idx[r] < num_slots && fr - idx[r] == B0;
            plainm |= pl ? 1u << r : 0u;
        }
    } else {
        load_key_fields<R, kDesc>(pkts, desc, npk, stride, i0, idx, sid, ack);
    }
    // the key before the wave's first item (the previous wave's or chunk's last): every lane
    // loads the same entry
    uint32_t pidx[1], psid[1], pack[1];
    const size_t pw = i0 - (size_t)lane;                      // the wave's first position
    load_key_fields<1, kDesc>(pkts, desc, pw > 0 ? npk : 0, stride, pw - 1, pidx, psid, pack);
    __syncthreads();
    const bool pmine = psid[0] == (uint32_t)(uint8_t)switch_id && switch_id >= 0;
    uint32_t prev = pmine ? pidx[0] % num_slots : num_slots;
    uint32_t prevf = prev | ((ack_hint && pmine && pack[0]) ? kAckBit : 0u);   // with the ack bit
    bool down = false;                                        // a key below its predecessor's
    unsigned long long bm[R];                                 // breaks of the dense runs
    uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;                     // this lane's slot-key bounds
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const size_t p = i0 + (size_t)r * 64;
        const bool mine = switch_id >= 0 && sid[r] == (uint32_t)(uint8_t)switch_id;
        const uint32_t key = mine ? idx[r] % num_slots : num_slots;
        if (kMode == 1 && mine && p < npk) {
            kmn = min(kmn, key);
            kmx = max(kmx, key);
        }
        // bit 31 carries "PS ack" through the sort (no digit reads it)
        k[r] = key | ((ack_hint && mine && ack[r]) ? kAckBit : 0u) | ((mine && ((plainm >> r) & 1u)) ? kPlainBit : 0u);
        v[r] = (uint32_t)p;
        if (kMode == 0 && p < npk && !mine) actions[p] = INA_ACT_FWD_OTHER;   // switch_check miss, ngaa.p4:184-186
        // the detection pass stores EVERY packet's action byte by position: foreign packets
        // forwarded, this switch's starting as drops -- so a sorted or near-sorted run stores only
        // the other actions (1 in W): scattered byte stores in slot / list order wrote back a line
        // each (shuffled NGA-32 run kernel: 440 MB written, r05e); the in-order and run-table
        // paths store every action anyway
        if (kMode == 1 && p < npk && !INA_LAB_DETECT_NOACT) actions[p] = mine ? INA_ACT_DROP : INA_ACT_FWD_OTHER;
        if constexpr (kMode != 1) {
            if constexpr (kHalf) lds_count_half(base[wv >> 1], (key >> lb) & (nb - 1), p < npk, (wv & 1) * 16);
            else lds_count(base[wv], (key >> lb) & (nb - 1), p < npk);
        }
        if constexpr (kMode == 1)
            if (p < npk && !kflags) kout[p] = k[r];   // arrival-order keys (kflags: after the loop, see KeySrc)
        // predecessor: lane l-1 of this round (DPP wave_shr:1), lane 0 the previous round's
        // lane 63 (or, in round 0, the key loaded above)
        const uint32_t pk = (uint32_t)__builtin_amdgcn_update_dpp((int)prev, (int)key, 0x138, 0xF, 0xF, false);
        down |= p < npk && p > 0 && pk > key;
        prev = (uint32_t)__builtin_amdgcn_readlane((int)key, 63);
        const uint32_t pkf = (uint32_t)__builtin_amdgcn_update_dpp((int)prevf, (int)k[r], 0x138, 0xF, 0xF, false);
        bm[r] = __ballot(p < npk && (p == 0 || !mine || (pkf & ~kAckBit) + 1u != key ||
                                     ((pkf ^ k[r]) & kAckBit) != 0u));
        prevf = (uint32_t)__builtin_amdgcn_readlane((int)k[r], 63);
    }
    // the batch is not in slot order: B sorts (else B only copies A's output, which is then
    // the identity permutation).  Tagged with the call's epoch, so nothing needs clearing.
    if constexpr (kMode != 2) {
        if (__ballot(down) && lane == 0) unsorted[0] = epoch;
        if (c == 0 && threadIdx.x == 0) unsorted[1] = epoch;     // this call's epoch, for the run kernel
    }
    uint32_t nbw = 0;                                         // this wave's breaks
#pragma unroll
    for (int r = 0; r < R; ++r) nbw += (uint32_t)__builtin_popcountll(bm[r]);
    if (lane == 0) wbrk[wv] = nbw;
    if (kMode == 1 && gstat) {                                // the wave's slot-key bounds
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            kmn = min(kmn, (uint32_t)__shfl_xor((int)kmn, o));
            kmx = max(kmx, (uint32_t)__shfl_xor((int)kmx, o));
        }
        if (lane == 0) {
            wgmn[wv] = kmn;
            wgmx[wv] = kmx;
        }
        // (kflags) only a wave the near-sorted lists may read stores its keys: one with a descent
        // (a wave in slot order is read from the descriptors) whose slots span at most
        // kKeysSpanMax (a shuffled batch's waves span the pool and take the sort, which reads the
        // descriptors itself)
        if (kflags && __ballot(down) && kmx >= kmn && kmx - kmn <= kKeysSpanMax && kmx - kmn > kKeysSpanMin) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (i0 + (size_t)r * 64 < npk) kout[i0 + (size_t)r * 64] = k[r];
            if (lane == 0) kflags[c * kBkWaves + wv] = epoch;
        }
    }
    __syncthreads();
    if (kMode == 1 && gstat && threadIdx.x < (unsigned)kGranPerChunk) {   // granule = kGranWaves waves
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
        for (int w = 0; w < kGranWaves; ++w) {
            mn = min(mn, wgmn[threadIdx.x * kGranWaves + w]);
            mx = max(mx, wgmx[threadIdx.x * kGranWaves + w]);
        }
        gstat[c * kGranPerChunk + threadIdx.x] = mn;
        gstat[G + c * kGranPerChunk + threadIdx.x] = mx;
    }
    if (kMode != 2 && brk_cnt) {                              // the chunk's breaks, in order
        uint32_t tot = 0, pre = 0;
#pragma unroll
        for (int w = 0; w < kBkWaves; ++w) {
            const uint32_t x = wbrk[w];
            tot += x;
            pre += w < wv ? x : 0u;
        }
        if (threadIdx.x == 0) brk_cnt[c] = tot;
        if (tot <= (uint32_t)kRunsMax && nbw) {
            const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if ((bm[r] >> lane) & 1ull)
                    brk_ent[c * kRunsMax + pre + (uint32_t)__builtin_popcountll(bm[r] & below)] =
                        uint2{(uint32_t)(i0 + (size_t)r * 64), k[r]};
                pre += (uint32_t)__builtin_popcountll(bm[r]);
            }
        }
    }
    if constexpr (kMode == 1) return;
    // thread t owns digits t*DPT .. t*DPT+DPT-1: the chunk's counts, their chunk-local run
    // starts (block scan)
    constexpr int DPT = kDigitsPerThread<BINS>;
    uint32_t tc[DPT], ex[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
        tc[j] = 0;
        if (d < nb) {
            if constexpr (kHalf) {
#pragma unroll
                for (int w2 = 0; w2 < kBkWaves / 2; ++w2) {
                    const uint32_t word = base[w2][d];
                    tc[j] += (word & 0xFFFFu) + (word >> 16);
                }
            } else {
#pragma unroll
                for (int w = 0; w < kBkWaves; ++w) tc[j] += base[w][d];
            }
        }
    }
    block_digit_scan_n<DPT>(tc, ex, wtot, 0u);
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
        if (d < nb) {
            rcnt[(size_t)d * nch + c] = tc[j];
            rst[(size_t)d * nch + c] = ex[j];
            gst[d] = (uint32_t)(c * (size_t)(kBkThr * R)) + ex[j];
        }
    }
    __syncthreads();
#if INA_SORT_STAGE
    if constexpr (kHalf && R <= INA_SORT_STAGE_MAX_R) {
        // the chunk's sorted output lands in LDS, then leaves as one contiguous stretch (the
        // 2,048-bin scatter writes runs of ~2 items: scattered 4-byte stores)
#if INA_SORT_STAGE_ALIAS
        // the chunk's 2 x 4 x kBkThr x R bytes fit the packed count array (8 x 2,048 words
        // at R = 8): 139 -> 74 KiB at 8,192-packet chunks, two blocks per CU
        static_assert(2 * kBkThr * R <= (kBkWaves / 2) * BINS, "staging fits the count array");
        uint32_t* s_k = &base[0][0];
        uint32_t* s_v = s_k + kBkThr * R;
#else
        __shared__ uint32_t s_k[kBkThr * R], s_v[kBkThr * R];
#endif
        const uint32_t cb = (uint32_t)(c * (size_t)(kBkThr * R));
        rs_tile_scatter_half<R, BINS, true>(k, v, i0, npk, lb, hbits, base, gst, kout, vout, R, s_k, s_v, cb);
        __syncthreads();
        const uint32_t nc = (uint32_t)min((size_t)(kBkThr * R), npk - (size_t)cb);
        for (uint32_t i = threadIdx.x; i < nc; i += kBkThr) {
            kout[cb + i] = s_k[i];
            vout[cb + i] = s_v[i];
        }
        return;
    }
#endif
    if constexpr (kHalf) rs_tile_scatter_half<R, BINS>(k, v, i0, npk, lb, hbits, base, gst, kout, vout);
    else rs_tile_scatter<R, kBkWaves, BINS>(k, v, i0, npk, lb, hbits, base, gst, kout, vout);
}

#ifndef INA_BK_TIMING
#define INA_BK_TIMING 0
#endif
#if INA_BK_TIMING
// lab builds only: per-block wall-clock stamps of k_sort_buckets' phases (tools/lab)
__device__ unsigned long long g_bk_t[kBkMaxChunks][6];   // one row per bucket (<= 2,048)
#define BK_STAMP(q) do { if (threadIdx.x == 0) g_bk_t[blockIdx.x][q] = wall_clock64(); } while (0)
#else
#define BK_STAMP(q) do { } while (0)
#endif

// positions of bucket items i[r] (0 <= i < the bucket's size) in A's output: the run of the
// last chunk whose bucket offset is <= i (s_dst: exclusive prefix of the run lengths over the
// nch chunks, then the bucket's size).  A branch-free binary search with a uniform step
// sequence (top = the largest power of two < nch), the R searches interleaved so their LDS
// reads are in flight together
template <int R>
__device__ __forceinline__ void bucket_src(const uint32_t* s_dst, const uint32_t* s_src, uint32_t nch,
                                           uint32_t top, const uint32_t (&i)[R], uint32_t (&src)[R]) {
    uint32_t lo[R];
#pragma unroll
    for (int r = 0; r < R; ++r) lo[r] = 0;
    for (uint32_t step = top; step > 0; step >>= 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = lo[r] + step;
            if (t < nch && s_dst[t] <= i[r]) lo[r] = t;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) src[r] = s_src[lo[r]] + (i[r] - s_dst[lo[r]]);
}

// two blocks per CU (8 waves per SIMD) where the LDS allows it (<= 1,024 bins, 53 KiB): the
// bound caps the scalar registers too -- at 106 SGPRs (R = 8) a SIMD held 7 waves, so one
// 16-wave block per CU ran (most blocks in flight at once: 256, tools/lab/bucket_phase_lab.py)
template <int R, int BINS>
__global__ __launch_bounds__(kBkThr, BINS <= 1024 ? 2 * kBkThr / 256 : kBkThr / 256) void k_sort_buckets(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout,
                                                         uint32_t* __restrict__ vout,
                                                         const uint32_t* __restrict__ rcnt,
                                                         const uint32_t* __restrict__ rst, uint32_t nch,
                                                         uint32_t CH, int lbits, uint32_t* __restrict__ nforeign,
                                                         uint32_t skip, uint32_t* __restrict__ unsorted,
                                                         uint32_t epoch, int sorted_copy,
                                                         const uint32_t* __restrict__ brk_cnt,
                                                         const uint2* __restrict__ brk_ent, uint32_t npk,
                                                         int pre) {
    __shared__ uint32_t s_dst[kBkMaxChunks + 1], s_src[kBkMaxChunks];
    constexpr bool kHalf = BINS >= 1024;              // two waves' 16-bit counts per word
    __shared__ uint32_t base[kHalf ? kBkWaves / 2 : kBkWaves][BINS];
    __shared__ uint32_t gst[BINS];                    // bucket digit counts, then output positions
    __shared__ uint32_t red[kBkWaves], red2[kBkWaves];
    const int lane = threadIdx.x & 63, wv = wave_in_block();
    // (INA_BUCKET_XCD: neighbouring buckets on one XCD: their runs in a chunk share lines, read through one L2)
    uint32_t b = INA_BUCKET_XCD ? (uint32_t)xcd_block_index() : blockIdx.x;
#if INA_BUCKET_GROUP > 1
    {   // groups of INA_BUCKET_GROUP neighbouring buckets on one XCD (blocks go to the XCDs
        // round-robin); the grid's tail past whole groups of 8 x G keeps its own index
        constexpr uint32_t G = INA_BUCKET_GROUP;
        const uint32_t p = blockIdx.x, full = (gridDim.x / (8u * G)) * (8u * G);
        if (p < full) {
            const uint32_t x = p & 7u, i = p >> 3;
            b = (i / G) * (8u * G) + x * G + (i % G);
        }
    }
#endif
    // keys already in slot order: A's output is the sorted order and the register-resident
    // run kernel reads it there (sorted_copy = 0), so only the foreign bucket's size is needed
    const bool in_order = unsorted[0] != epoch;
    // after the split chunk pass (pre): structured batches were decided, nothing to gather
    if (pre && (in_order || unsorted[2] == epoch || unsorted[kLocEpoch] == epoch)) return;
    if (in_order && !sorted_copy && b != skip) return;
    if (!in_order && brk_cnt) {
        // dense ascending runs (brk_cnt != NULL only for the register-resident run kernel):
        // every block sums the chunks' break counts (the same answer everywhere); at most
        // kRunsMax of them and block 0 writes the run table, nobody sorts
        uint32_t part = 0;
        for (uint32_t c = threadIdx.x; c < nch; c += kBkThr) part += brk_cnt[c];
        const uint32_t inc = wave_incl_scan(part);
        if (lane == 63) red[wv] = inc;
        __syncthreads();
        uint32_t total = 0;
#pragma unroll
        for (int w = 0; w < kBkWaves; ++w) total += red[w];
        if (total <= (uint32_t)kRunsMax) {
            if (b == 0) build_run_table(brk_cnt, brk_ent, nch, total, npk, unsorted, epoch, red2);
            return;
        }
        __syncthreads();                              // red[] is reused below
    }
    BK_STAMP(0);
    // this bucket's run in every chunk: thread t owns chunks [t*per, t*per + per).  A chunk's
    // run start rst[b][c] is the number of its packets in lower buckets, so the rst row also
    // sums to the bucket's place in the output: no look-back over the other buckets
    const uint32_t per = (nch + kBkThr - 1) / kBkThr;        // <= 4
    const uint32_t c0 = threadIdx.x * per;
    uint32_t part = 0, below = 0;
    for (uint32_t q = 0; q < per; ++q) {
        const uint32_t c = c0 + q;
        if (c < nch) {
            const uint32_t x = rcnt[(size_t)b * nch + c];
            const uint32_t st0 = rst[(size_t)b * nch + c];
            s_src[c] = c * CH + st0;
            s_dst[c] = x;
            part += x;
            below += st0;
        }
    }
    const uint32_t inc = wave_incl_scan(part);
    const uint32_t bsum = wave_incl_scan(below);
    if (lane == 63) {
        red[wv] = inc;
        red2[wv] = bsum;
    }
    __syncthreads();
    uint32_t wpre = 0, total = 0, s0 = 0;
#pragma unroll
    for (int w = 0; w < kBkWaves; ++w) {
        const uint32_t t = red[w];
        wpre += w < wv ? t : 0u;
        total += t;
        s0 += red2[w];
    }
    uint32_t run = wpre + inc - part;                         // bucket offset of chunk c0's run
    for (uint32_t q = 0; q < per; ++q) {
        const uint32_t c = c0 + q;
        if (c < nch) {
            const uint32_t x = s_dst[c];
            s_dst[c] = run;
            run += x;
        }
    }
    if (threadIdx.x == 0) s_dst[nch] = total;
    __syncthreads();
    BK_STAMP(1);
    const uint32_t cnt = total;
    if (b == skip) {                                  // foreign packets only: left out, counted
        if (threadIdx.x == 0) *nforeign = cnt;
        return;
    }
    if (cnt == 0) return;                             // block-uniform
    if (in_order) {                                   // (the generic run kernel reads B's
        for (uint32_t i = threadIdx.x; i < cnt; i += kBkThr) {   // output: the bucket is its
            kout[s0 + i] = kin[s0 + i];               // own run of A's output, copied)
            vout[s0 + i] = vin[s0 + i];
        }
        return;
    }
    uint32_t top = 1;                                 // search steps: powers of two below nch
    while (top * 2 < nch) top *= 2;
    if (nch == 1) top = 0;
    if (lbits == 0) {                                 // one-digit keys: the runs are the order
        for (uint32_t i0 = threadIdx.x; i0 - threadIdx.x < cnt; i0 += kBkThr) {
            const uint32_t ii[1] = {i0 < cnt ? i0 : 0u};
            uint32_t src[1];
            bucket_src<1>(s_dst, s_src, nch, top, ii, src);
            if (i0 < cnt) {
                kout[s0 + i0] = kin[src[0]];
                vout[s0 + i0] = vin[src[0]];
            }
        }
        return;
    }
    const uint32_t nb = 1u << lbits;
    constexpr int DPT = kDigitsPerThread<BINS>;       // thread t owns low digits t*DPT + j
    for (uint32_t d = threadIdx.x; d < nb; d += kBkThr) gst[d] = 0;
    __syncthreads();
    constexpr uint32_t kTile = (uint32_t)kBkThr * (uint32_t)R;
    const uint32_t ntile = (cnt + kTile - 1) / kTile;
    if (ntile > 1) {                                  // bucket digit totals -> output positions
        for (uint32_t i = (uint32_t)wv * 64 + (uint32_t)lane; i - (uint32_t)lane < cnt; i += kBkThr) {
            const bool ok = i < cnt;
            const uint32_t ii[1] = {ok ? i : 0u};
            uint32_t src[1];
            bucket_src<1>(s_dst, s_src, nch, top, ii, src);
            lds_count(gst, ok ? kin[src[0]] & (nb - 1) : 0u, ok);
        }
        __syncthreads();
        uint32_t x[DPT], ex[DPT];
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
            x[j] = d < nb ? gst[d] : 0u;
        }
        block_digit_scan_n<DPT>(x, ex, red, s0);
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
            if (d < nb) gst[d] = ex[j];
        }
    }
    for (uint32_t t = 0; t < ntile; ++t) {
        // the tile's items split evenly over the waves in order (wave w: rw rounds of 64)
        const uint32_t tn = min(kTile, cnt - t * kTile);
        const int rw = (int)((tn + (uint32_t)kBkThr - 1) / (uint32_t)kBkThr);
        const uint32_t i0 = t * kTile + (uint32_t)wv * 64u * (uint32_t)rw + (uint32_t)lane;
        const uint32_t t_end = t * kTile + tn;
        uint32_t ii[R], src[R], k[R], v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = i0 + (uint32_t)r * 64u;
            ii[r] = (r < rw && i < t_end) ? i : 0u;
        }
        bucket_src<R>(s_dst, s_src, nch, top, ii, src);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool ok = r < rw && i0 + (uint32_t)r * 64u < t_end;
            k[r] = ok ? kin[src[r]] : 0u;
            v[r] = ok ? vin[src[r]] : 0u;
        }
        for (uint32_t dd = lane; dd < nb; dd += 64) base[kHalf ? wv >> 1 : wv][dd] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r < rw) {
                if constexpr (kHalf)
                    lds_count_half(base[wv >> 1], k[r] & (nb - 1), i0 + (uint32_t)r * 64u < t_end, (wv & 1) * 16);
                else
                    lds_count(base[wv], k[r] & (nb - 1), i0 + (uint32_t)r * 64u < t_end);
            }
        __syncthreads();
        BK_STAMP(2);
        uint32_t tc[DPT];                             // this tile's counts of the thread's digits
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
            tc[j] = 0;
            if (d < nb) {
                if constexpr (kHalf) {
#pragma unroll
                    for (int w2 = 0; w2 < kBkWaves / 2; ++w2) {
                        const uint32_t word = base[w2][d];
                        tc[j] += (word & 0xFFFFu) + (word >> 16);
                    }
                } else {
#pragma unroll
                    for (int w = 0; w < kBkWaves; ++w) tc[j] += base[w][d];
                }
            }
        }
        if (ntile == 1) {                             // one tile: positions from its own counts
            uint32_t ex[DPT];
            block_digit_scan_n<DPT>(tc, ex, red, s0);
#pragma unroll
            for (int j = 0; j < DPT; ++j) {
                const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
                if (d < nb) gst[d] = ex[j];
            }
        }
        __syncthreads();
        BK_STAMP(3);
        // (staging a one-tile bucket's output in LDS: round 3 measured it neutral at NGA-256,
        // profiles/r03/lab/bucket_stage_lab.log; at NGA-32 it cuts the pass's writes 4x, see
        // INA_BUCKET_STAGE)
#if INA_BUCKET_STAGE
        if constexpr (kHalf) {
            if (ntile == 1) {
                // a one-tile bucket leaves as two contiguous runs: keys, then values, each staged in
                // the count array once every wave has read its offsets (8 x BINS words >= a tile)
                static_assert((kBkWaves / 2) * BINS >= (int)kTile, "a tile fits the count array");
                uint32_t sp[R];
                rs_tile_scatter_half<R, BINS, false, true>(k, v, i0, t_end, 0, lbits, base, gst, kout, vout, rw,
                                                           nullptr, nullptr, s0, sp);
                uint32_t* stg = &base[0][0];
                __syncthreads();
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (sp[r] != 0xFFFFFFFFu) stg[sp[r]] = k[r];
                __syncthreads();
                for (uint32_t i = threadIdx.x; i < cnt; i += kBkThr) kout[s0 + i] = stg[i];
                __syncthreads();
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (sp[r] != 0xFFFFFFFFu) stg[sp[r]] = v[r];
                __syncthreads();
                for (uint32_t i = threadIdx.x; i < cnt; i += kBkThr) vout[s0 + i] = stg[i];
                return;
            }
        }
#endif
        if constexpr (kHalf) rs_tile_scatter_half<R, BINS>(k, v, i0, t_end, 0, lbits, base, gst, kout, vout, rw);
        else rs_tile_scatter<R, kBkWaves, BINS>(k, v, i0, t_end, 0, lbits, base, gst, kout, vout, rw);
        __syncthreads();
        BK_STAMP(4);
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = threadIdx.x * DPT + (uint32_t)j;
            if (d < nb) gst[d] += tc[j];
        }
    }
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
#ifndef INA_SWITCH_WIN_NARROW
#define INA_SWITCH_WIN_NARROW 64
#endif
static_assert(INA_SWITCH_WIN_NARROW >= 1 && INA_SWITCH_WIN_NARROW <= 64, "a narrow window's heads are one wave's lanes");
#ifndef INA_SWITCH_WIN_LARGE
#define INA_SWITCH_WIN_LARGE 16
#endif
#ifndef INA_SWITCH_GRID
#define INA_SWITCH_GRID (1 << 20)
#endif
// the narrow (V <= 32) run over a run table: 8 slots side by side per wave, the runs walked in
// order (1), or one slot's 8 packets side by side (0; a lab build's A/B switch)
#ifndef INA_SWITCH_NARROW_SLOTS
#define INA_SWITCH_NARROW_SLOTS 1
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
// forwarded packets: written once per call, never read back by it (lab knob: nt).  Not
// stream_store: its buffer resource starts at the wave's first active lane, and the lists and
// sorted paths scatter a wave's rows below it too -- a write-through build of sw_st lost those
// stores (jitter 64 and shuffled differed from the default build; it was also no faster on the
// structured orders: profiles/r06/lab/switch_store_sc1_ab.log)
__device__ __forceinline__ void sw_st(u32x4s v, u32x4s* p) {
#if INA_SWITCH_FWD_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
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

// PS co-located with the switch (ina_switch with a PS step): a completed slot's sum goes
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
    uint2* ack_desc;    // the ack rows' descriptors (header bytes 4..11), or NULL
};

// the run kernel's work for waves wave, wave + nwaves, ... (k_switch_run2: every wave of
// the grid; k_switch_tiny: the 16 waves of its one workgroup)
// kPs: PS update fused (ina_switch with a PS step); false costs nothing.  kLat (the
// one-launch tiny path, latency-bound): the slot's count and frag are read into SGPRs
// only after the first batch's packet loads are issued, so a segment waits for one memory
// round trip instead of three (no gain where the kernel is bandwidth-bound, and it costs
// registers there: profiles/r02/lab/switch_lab_state_late.log)
// One slot segment -- packets q_begin .. q_end-1 of slot `slot`, in arrival order (after the
// PS ack that leads it, when ack_led) -- through count (ngaa.p4:64-82), frag (fragcheck.p4:14-57) and
// the V Processor registers (processor.p4:14-24) with the slot's state in registers.
// pid_batch(q0, nb, pid) gives the packet ids of the segment's packets q0 .. q0+nb-1 (wave-
// uniform): the sorted run reads them from its window, the structured run (a batch of
// dense ascending runs) from its run table.
// kSplit: split rows (include/ina.h) -- pkts holds 16-byte header rows (stride 16) and pay the
// 4V-byte payload rows: lane l loads payload chunk l (values 4l..4l+3, one byte swap each,
// no neighbour lane), lane b < kB the header row of packet b, and a forwarded packet
// rewrites only its payload row.
template <bool kPs, bool kLat, bool kSplit, typename PidFn>
__device__ __forceinline__ void run_segment(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                            size_t stride, uint8_t* __restrict__ pay,
                                            uint8_t* __restrict__ actions, const PsFuse& ps,
                                            uint32_t slot, bool ack_led, size_t q_begin, size_t q_end,
                                            PidFn&& pid_batch, bool drop_written = false) {
    // (drop_written: the detection pass stored every packet's drop by position)
    constexpr bool kActBatch = INA_SWITCH_ACT_BATCH;
    const int lane = threadIdx.x & 63;
    const int V = st.V;
    const int L = V >> 2;                       // lanes holding values
    const bool vl = lane < L;
    const bool wide = L == 64;                  // tail chunk lives in lane 63's t[]
    // slot state: count and frag are wave-uniform (SGPRs, scalar branches); the V
    // registers are loaded only if a packet adds to them before any overwrite
    // (count_reg == 1 overwrites, processor.p4:16-21), i.e. rarely
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
    for (size_t q0 = q_begin; q0 < q_end; q0 += kB) {
        const int nb = (int)((q_end - q0) < (size_t)kB ? (q_end - q0) : (size_t)kB);
        u32x4s a[kB];
        uint32_t pid[kB];
        pid_batch(q0, nb, pid);
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
        if constexpr (kSplit) {                  // lane b: packet b's header row
            tl = *reinterpret_cast<const u32x4s*>(pkts + (size_t)mypid * 16);
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const u32x4s* pk = reinterpret_cast<const u32x4s*>(pay + (size_t)pid[b] * (size_t)(4 * V));
                a[b] = sw_ld(pk + (vl ? lane : 0));
            }
        } else {
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
            const uint32_t h1 = kSplit ? __builtin_amdgcn_readlane(tl.y, b) : __builtin_amdgcn_readlane(a[b].y, 0),
                           h2 = kSplit ? __builtin_amdgcn_readlane(tl.z, b) : __builtin_amdgcn_readlane(a[b].z, 0),
                           h3 = kSplit ? __builtin_amdgcn_readlane(tl.w, b) : __builtin_amdgcn_readlane(a[b].w, 0);
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
                        reinterpret_cast<uint32_t*>(pkts + (size_t)pid[b] * (kSplit ? 16 : stride))[1] =
                            h1 | ((uint32_t)INA_FLAG_COLLISION << 8);
                } else {
                    cnt = (cnt + 1u) & 0xFFu;            // read_add_count (ngaa.p4:66-78)
                    if (cnt == hcount) cnt = 0;
                    cnt = __builtin_amdgcn_readfirstlane(cnt);
                    const bool first = cnt == 1u;
                    u32x4s v;                            // values 4l..4l+3
                    uint32_t tw = 0;                     // old byte 1039 (padding) for the tail
                    if constexpr (kSplit) {
                        v.x = __builtin_bswap32(a[b].x); v.y = __builtin_bswap32(a[b].y);
                        v.z = __builtin_bswap32(a[b].z); v.w = __builtin_bswap32(a[b].w);
                    } else {
                    u32x4s c;                            // chunk l+1
                    c.x = from_next_lane(a[b].x); c.y = from_next_lane(a[b].y);
                    c.z = from_next_lane(a[b].z); c.w = from_next_lane(a[b].w);
                    if (wide) {
                        const uint32_t tx = __builtin_amdgcn_readlane(tl.x, b);
                        const uint32_t ty = __builtin_amdgcn_readlane(tl.y, b);
                        const uint32_t tz = __builtin_amdgcn_readlane(tl.z, b);
                        tw = __builtin_amdgcn_readlane(tl.w, b);
                        if (lane == 63) c = u32x4s{tx, ty, tz, tw};
                    }
                    v.x = dec_be(c.x, a[b].w);
                    v.y = dec_be(c.y, c.x);
                    v.z = dec_be(c.z, c.y);
                    v.w = dec_be(c.w, c.z);
                    }
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
                                // nt: 249.9 -> 241.3 us for the fused pass, the
                                // steady-state step 0.71 -> 0.70 ms (default policy;
                                // write-through 247.8; profiles/r03/lab/psout_lab.log)
                                __builtin_nontemporal_store(r, reinterpret_cast<f32x4s*>(ps.out + e0));
                            } else if (vl) {
                                const uint32_t rv[4] = {reg.x, reg.y, reg.z, reg.w};
                                for (int t = 0; t < 4 && e0 + t < ps.n; ++t)
                                    ps.out[e0 + t] = __fadd_rn(ps.local[e0 + t],
                                        __fmul_rn(__fmul_rn((float)(int32_t)rv[t], ps.inv), ps.ws));
                            }
                            if (lane == 0 && ps.acks) {      // the PS ack (fragcheck.p4:26-31)
                                u32x4s hd = a[b];
                                if constexpr (kSplit) hd = u32x4s{(uint32_t)__builtin_amdgcn_readlane(tl.x, b), h1, h2, h3};
                                hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                                if constexpr (!kSplit) hd.w = (hd.w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                                *reinterpret_cast<u32x4s*>(ps.acks + (size_t)ps_slot * ps.ack_stride) = hd;
                                // its descriptor, so the next switch batch (these acks in
                                // front of the next step's packets) needs no gather pass
                                if (ps.ack_desc) ps.ack_desc[ps_slot] = uint2{hd.y, hd.z};
                            }
                        }
                    }
                    if (kSplit && (act != INA_ACT_DROP || st.write_dropped) && (!consumed || ps.keep_fwd)) {
                        // out_value -> payload (processor.p4:22): the payload row, word for word
                        const u32x4s e{__builtin_bswap32(reg.x), __builtin_bswap32(reg.y),
                                       __builtin_bswap32(reg.z), __builtin_bswap32(reg.w)};
                        if (vl) sw_st(e, reinterpret_cast<u32x4s*>(pay + (size_t)pid[b] * (size_t)(4 * V)) + lane);
                    } else if ((act != INA_ACT_DROP || st.write_dropped) && (!consumed || ps.keep_fwd)) {
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
                            sw_st(e, reinterpret_cast<u32x4s*>(pkts + (size_t)pid[b] * stride) + lane);
                        if (wide && lane == 63) {        // tail chunk 64 from lane 63's values
                            u32x4s o;
                            o.x = enc_lo(reg.x, reg.y);
                            o.y = enc_lo(reg.y, reg.z);
                            o.z = enc_lo(reg.z, reg.w);
                            o.w = enc_lo(reg.w, tw);
                            sw_st(o, reinterpret_cast<u32x4s*>(pkts + (size_t)pid[b] * stride) + 64);
                        }
                    }
                }
            }
            if constexpr (kActBatch) act_v = lane == b ? (uint32_t)act : act_v;
            else if (lane == 0 && !(drop_written && act == INA_ACT_DROP)) actions[pid[b]] = act;
        }
        if constexpr (kActBatch)                      // one store for the batch
            if (lane < nb && !(drop_written && act_v == INA_ACT_DROP)) actions[mypid] = (uint8_t)act_v;
    }
    if (lane == 0) {
        st.count[slot] = (uint8_t)cnt;
        st.frag[slot] = frag;
    }
    // the slot registers are written once per call and read back only by a later batch
    // (and then rarely: the first packet of a fresh segment overwrites them), so they
    // are stored nt and do not displace the packet lines the gather shares in L2:
    // bench.py's switch leg 228.4 -> 213.9 us worker-major, 217.2 -> 195.1 round-robin
    // (tools/lab/psout_ab.sh, profiles/r03/lab/switch_reg_nt_lab.log)
    if (have_reg && vl) __builtin_nontemporal_store(reg, reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * lane));
}

// Narrow packets (V <= 32: NGA-32, the P4 program's own format, headers.p4:40-73): run_segment
// above gives each packet the whole wave, so only V/4 + 1 of its 64 lanes work and a batch's
// packets go one after another -- at 6.5 M NGA-32 packets the kernel was instruction-bound
// (0.19 of the HBM roofline).  Here the wave takes a batch's 8 packets side by side: lane
// group g = lane / 8 holds packet g, its lane l = lane % 8 chunk l (values 4l..4l+3; the
// group's last value lane also loads the tail chunk V/4).  The count / frag state machine
// still runs packet by packet in arrival order, in SGPRs (8 x 3 header words by readlane),
// and leaves per-packet masks (adds, overwrites, forwards, collisions, PS consumption); the
// Processor adds become ONE segmented inclusive scan over the 8 groups (resets at the
// count_reg == 1 overwrites, processor.p4:16-21) -- 3 shuffle steps -- so each packet's
// running sum, the value the P4 program writes into it (processor.p4:22), is in its group's
// lanes at once.  Same results as run_segment, packet for packet.
__device__ __forceinline__ uint32_t from_lane(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)x);
}
// DPP row_shl:1 / row_shr:1: lane i reads lane i+1 / i-1 inside its 16-lane row (a group of 8
// never needs its neighbour group: chunk l+1 of the group's last lane is the loaded tail, and
// lane 0 of a group encodes the header chunk without its predecessor)
__device__ __forceinline__ uint32_t from_next_in_row(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x101, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_prev_in_row(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x111, 0xF, 0xF, false);
}
constexpr int kNarrowMaxV = 32;
static_assert(kB == 8, "the narrow run puts a batch of 8 packets in 8 lane groups");

// packet group g's row loads (lanes past L re-read chunk 0; the tail chunk is one request per
// group); the caller's mypid is packet g's id
template <bool kSplit>
__device__ __forceinline__ void narrow_load(const uint8_t* __restrict__ pkts, size_t stride,
                                            const uint8_t* __restrict__ pay, int V, uint32_t mypid,
                                            u32x4s& a, u32x4s& tl) {
    const int l = threadIdx.x & 7, L = V >> 2;
    const bool vl = l < L;
    if constexpr (kSplit) {                           // payload chunk l; the group's header row
        a = sw_ld(reinterpret_cast<const u32x4s*>(pay + (size_t)mypid * (size_t)(4 * V)) + (vl ? l : 0));
        tl = *reinterpret_cast<const u32x4s*>(pkts + (size_t)mypid * 16);
    } else {
        const u32x4s* pk = reinterpret_cast<const u32x4s*>(pkts + (size_t)mypid * stride);
        a = sw_ld(pk + (vl ? l : 0));
        tl = *(pk + L);
    }
}

template <bool kPs, bool kSplit, typename PidFn>
__device__ __forceinline__ void run_segment_narrow(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                   size_t stride, uint8_t* __restrict__ pay,
                                                   uint8_t* __restrict__ actions,
                                                   const PsFuse& ps, uint32_t slot, bool ack_led,
                                                   size_t q_begin, size_t q_end, PidFn&& pid_batch) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, l = lane & 7;      // packet group, value lane
    const int V = st.V;
    const int L = V >> 2;                       // value lanes per group (<= 8)
    const bool vl = l < L;
    uint32_t cnt = __builtin_amdgcn_readfirstlane((uint32_t)st.count[slot]);
    uint32_t frag = ack_led ? 0u : __builtin_amdgcn_readfirstlane(st.frag[slot]);
    u32x4s reg = {0u, 0u, 0u, 0u};              // the slot's running registers, in every group
    bool have_reg = false;
    for (size_t q0 = q_begin; q0 < q_end; q0 += kB) {
        const int nb = (int)((q_end - q0) < (size_t)kB ? (q_end - q0) : (size_t)kB);
        uint32_t pid[kB];
        pid_batch(q0, nb, pid);
#pragma unroll
        for (int b = 1; b < kB; ++b) pid[b] = b < nb ? pid[b] : pid[0];
        uint32_t mypid = pid[0], lanepid = pid[0];   // group g's packet; lane b's (actions)
#pragma unroll
        for (int b = 1; b < kB; ++b) {
            mypid = g == b ? pid[b] : mypid;
            lanepid = lane == b ? pid[b] : lanepid;
        }
        u32x4s a, tl;
        narrow_load<kSplit>(pkts, stride, pay, V, mypid, a, tl);
        const u32x4s hw = kSplit ? tl : a;            // header words (lane 8b: packet b's)
        // per-group outcome of the state machine: adds, overwrites, forwards, PS consumption,
        // collisions (group g's packet, in every lane of the group)
        bool add_g, first_g, fwd_g, ps_g, coll_g;
        uint32_t act_v = 0, ps_slot_v = 0;
        int lastb;                                    // the batch's last adding packet (-1: none)
        bool before;                                  // an add before the batch's first overwrite
        // header words of packet g in every lane of its group; lane b also packet b's
        const uint32_t g1 = kSplit ? hw.y : from_lane(hw.y, 8 * g), g2 = kSplit ? hw.z : from_lane(hw.z, 8 * g),
                       g3 = kSplit ? hw.w : from_lane(hw.w, 8 * g);
        const uint32_t gfin = __builtin_bswap32((g2 >> 24) | (g3 << 8)), ghc = g1 & 0xFFu;
        // the common batch -- no PS ack, every frag id the slot's (or the first packet's when
        // the slot is free), one degree H with count < H -- needs no packet-by-packet walk:
        // packet b's count is (count + b + 1) mod H (ngaa.p4:66-78), it completes the slot when
        // that is 0 and overwrites the registers when it is 1
        const uint32_t F = frag ? frag : (uint32_t)__builtin_amdgcn_readlane(gfin, 0);
        const uint32_t H = (uint32_t)__builtin_amdgcn_readlane(ghc, 0);
        const bool odd = g < nb && (((g1 >> 14) & 1u) || gfin != F || ghc != H);
        if (__ballot(odd) == 0 && H >= 1u && cnt < H) {
            frag = F;
            const uint32_t cg = (cnt + (uint32_t)g + 1u) % H;
            const uint32_t cl = (cnt + (uint32_t)lane + 1u) % H;   // lane b as packet b
            const bool cons = kPs && F - ps.seq0 < ps.nslots;       // the PS takes this slot
            add_g = g < nb;
            first_g = add_g && cg == 1u;
            ps_g = add_g && cons && cg == 0u;
            fwd_g = add_g && (cg == 0u || st.write_dropped) && (!ps_g || ps.keep_fwd);
            coll_g = false;
            if (cons) ps_slot_v = F - ps.seq0;
            act_v = cl == 0u ? INA_ACT_FWD_AGG : INA_ACT_DROP;
            lastb = nb - 1;
            before = !(H > 1u && cnt == 0u);          // count 0: packet 0 overwrites
            cnt = __builtin_amdgcn_readfirstlane((cnt + (uint32_t)nb) % H);
        } else {
        // the state machine, packet by packet in arrival order (SGPRs, scalar branches)
        uint32_t m_add = 0, m_first = 0, m_fwd = 0, m_coll = 0, m_ps = 0;
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            if (b >= nb) break;
            const uint32_t h1 = __builtin_amdgcn_readlane(hw.y, 8 * b),
                           h2 = __builtin_amdgcn_readlane(hw.z, 8 * b),
                           h3 = __builtin_amdgcn_readlane(hw.w, 8 * b);
            const uint32_t hcount = h1 & 0xFFu, flags = (h1 >> 8) & 0xFFu;
            const uint32_t frag_in =
                __builtin_amdgcn_readfirstlane(__builtin_bswap32((h2 >> 24) | (h3 << 8)));
            uint32_t act;
            if ((flags >> 6) & 1u) {                     // ack: reset_id (fragcheck.p4:26-31)
                frag = 0;
                act = INA_ACT_FWD_ACK;
            } else {
                if (frag == 0) frag = frag_in;           // write_read_id (fragcheck.p4:14-24)
                if (frag != frag_in) {                   // collision (ngaa.p4:177-181)
                    act = INA_ACT_FWD_COLLISION;
                    m_coll |= 1u << b;
                } else {
                    cnt = (cnt + 1u) & 0xFFu;            // read_add_count (ngaa.p4:66-78)
                    if (cnt == hcount) cnt = 0;
                    cnt = __builtin_amdgcn_readfirstlane(cnt);
                    m_add |= 1u << b;
                    if (cnt == 1u) m_first |= 1u << b;   // processor.p4:16-21 overwrite
                    act = cnt == 0 ? INA_ACT_FWD_AGG : INA_ACT_DROP;   // ngaa.p4:170-175
                    const uint32_t ps_slot = frag_in - ps.seq0;
                    const bool consumed = kPs && act == INA_ACT_FWD_AGG && ps_slot < ps.nslots;
                    if (consumed) {
                        m_ps |= 1u << b;
                        ps_slot_v = g == b ? ps_slot : ps_slot_v;
                    }
                    if ((act != INA_ACT_DROP || st.write_dropped) && (!consumed || ps.keep_fwd))
                        m_fwd |= 1u << b;
                }
            }
            act_v = lane == b ? act : act_v;
        }
        add_g = (m_add >> g) & 1u;
        first_g = (m_first >> g) & 1u;
        fwd_g = (m_fwd >> g) & 1u;
        ps_g = (m_ps >> g) & 1u;
        coll_g = (m_coll >> g) & 1u;
        lastb = m_add ? 31 - __builtin_clz(m_add) : -1;
        // the stored registers count only before the batch's first overwrite
        before = (m_first ? m_add & ((m_first & (0u - m_first)) - 1u) : m_add) != 0u;
        }
        if (lane < nb) actions[lanepid] = (uint8_t)act_v;   // one store for the batch
        if (coll_g && l == 0)                              // only the flag byte changes
            reinterpret_cast<uint32_t*>(pkts + (size_t)mypid * (kSplit ? 16 : stride))[1] =
                g1 | ((uint32_t)INA_FLAG_COLLISION << 8);
        if (lastb >= 0) {
            // values 4l..4l+3 of packet g: chunk l and chunk l+1 (the neighbour lane, or the
            // tail for the group's last value lane)
            u32x4s x;
            if constexpr (kSplit) {
                x.x = __builtin_bswap32(a.x); x.y = __builtin_bswap32(a.y);
                x.z = __builtin_bswap32(a.z); x.w = __builtin_bswap32(a.w);
            } else {
                u32x4s c;
                c.x = from_next_in_row(a.x); c.y = from_next_in_row(a.y);
                c.z = from_next_in_row(a.z); c.w = from_next_in_row(a.w);
                if (l == L - 1) c = tl;
                x.x = dec_be(c.x, a.w); x.y = dec_be(c.y, c.x); x.z = dec_be(c.z, c.y); x.w = dec_be(c.w, c.z);
            }
            uint32_t f = first_g ? 1u : 0u;
            if (!add_g) x = u32x4s{0u, 0u, 0u, 0u};
            // segmented inclusive scan over the groups (a reset at each overwrite)
#pragma unroll
            for (int d = 1; d < kB; d <<= 1) {
                const int src = lane - 8 * d;
                u32x4s y;
                y.x = from_lane(x.x, src); y.y = from_lane(x.y, src);
                y.z = from_lane(x.z, src); y.w = from_lane(x.w, src);
                const uint32_t fy = from_lane(f, src);
                if (g >= d && !f) {
                    x += y;
                    f |= fy;
                }
            }
            // the stored registers count only before the batch's first overwrite; load them
            // if an add comes before it and no earlier batch left them in registers
            if (before && !have_reg)
                reg = vl ? *reinterpret_cast<const u32x4s*>(st.regs + (size_t)slot * V + 4 * l)
                         : u32x4s{0u, 0u, 0u, 0u};
            const u32x4s S = f ? x : x + reg;        // packet g's running sum
            // the registers after the batch: the last adding packet's running sum
            const int src = 8 * lastb + l;
            reg.x = from_lane(S.x, src); reg.y = from_lane(S.y, src);
            reg.z = from_lane(S.z, src); reg.w = from_lane(S.w, src);
            have_reg = true;
            if (kPs && ps_g) {                       // launch.py:46-50 with the switch's sum
                const size_t e0 = (size_t)ps_slot_v * (size_t)V + 4 * (size_t)l;
                if (vl && e0 + 4 <= ps.n) {
                    const f32x4s lo = *reinterpret_cast<const f32x4s*>(ps.local + e0);
                    f32x4s r;
                    r.x = __fadd_rn(lo.x, __fmul_rn(__fmul_rn((float)(int32_t)S.x, ps.inv), ps.ws));
                    r.y = __fadd_rn(lo.y, __fmul_rn(__fmul_rn((float)(int32_t)S.y, ps.inv), ps.ws));
                    r.z = __fadd_rn(lo.z, __fmul_rn(__fmul_rn((float)(int32_t)S.z, ps.inv), ps.ws));
                    r.w = __fadd_rn(lo.w, __fmul_rn(__fmul_rn((float)(int32_t)S.w, ps.inv), ps.ws));
                    __builtin_nontemporal_store(r, reinterpret_cast<f32x4s*>(ps.out + e0));
                } else if (vl) {
                    const uint32_t rv[4] = {S.x, S.y, S.z, S.w};
                    for (int t = 0; t < 4 && e0 + t < ps.n; ++t)
                        ps.out[e0 + t] = __fadd_rn(ps.local[e0 + t],
                                                   __fmul_rn(__fmul_rn((float)(int32_t)rv[t], ps.inv), ps.ws));
                }
                if (l == 0 && ps.acks) {             // the PS ack (fragcheck.p4:26-31)
                    u32x4s hd = hw;
                    hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                    if constexpr (!kSplit) hd.w = (hd.w & 0x00FFFFFFu) | (S.x & 0xFF000000u);
                    *reinterpret_cast<u32x4s*>(ps.acks + (size_t)ps_slot_v * ps.ack_stride) = hd;
                    if (ps.ack_desc) ps.ack_desc[ps_slot_v] = uint2{hd.y, hd.z};
                }
            }
            if (kSplit && fwd_g) {                   // out_value -> the payload row (processor.p4:22)
                const u32x4s e{__builtin_bswap32(S.x), __builtin_bswap32(S.y), __builtin_bswap32(S.z),
                               __builtin_bswap32(S.w)};
                if (vl) sw_st(e, reinterpret_cast<u32x4s*>(pay + (size_t)mypid * (size_t)(4 * V)) + l);
            } else if (fwd_g) {                      // out_value -> payload (processor.p4:22)
                u32x4s p;                            // values of lane l-1
                p.x = from_prev_in_row(S.x); p.y = from_prev_in_row(S.y);
                p.z = from_prev_in_row(S.z); p.w = from_prev_in_row(S.w);
                u32x4s e = a;
                if (l == 0) {
                    e.w = (e.w & 0x00FFFFFFu) | (S.x & 0xFF000000u);
                } else {
                    e.x = enc_lo(p.x, p.y);
                    e.y = enc_lo(p.y, p.z);
                    e.z = enc_lo(p.z, p.w);
                    e.w = enc_lo(p.w, S.x);
                }
                u32x4s* dst = reinterpret_cast<u32x4s*>(pkts + (size_t)mypid * stride);
                if (vl) sw_st(e, dst + l);
                if (l == L - 1) {                    // the tail chunk from the last value lane
                    u32x4s o;
                    o.x = enc_lo(S.x, S.y);
                    o.y = enc_lo(S.y, S.z);
                    o.z = enc_lo(S.z, S.w);
                    o.w = enc_lo(S.w, tl.w);
                    sw_st(o, dst + L);
                }
            }
        }
    }
    if (lane == 0) {
        st.count[slot] = (uint8_t)cnt;
        st.frag[slot] = frag;
    }
    if (have_reg && g == 0 && vl)
        __builtin_nontemporal_store(reg, reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * l));
}

// packets' loads in flight per lane group (the VGPRs buy occupancy): 1 for packed and for split
// rows.  Interleaved A/Bs at NGA-32 C3 size (profiles/r04/lab/slot_inflight_ab_v32_*.log):
// 2 against 4 -- worker-major split 274.6 -> 260.7 us, round-robin packed 390.8 -> 374.7,
// shuffled 757.9 -> 734.8, the rest equal (8 spills: 2-3x slower); 1 against 2 -- split rows
// worker-major 258.6 -> 220.8, round-robin 285.9 -> 252.1, shuffled 646 -> 642, packed rows
// 4-7 % slower (3: no better than 2)
// (round 5: packed rows read as one unaligned 16-byte access per lane, no LDS exchange -- 1 in
// flight at 8 waves per SIMD: round-robin 337.2 -> 329.5 us, jitter 64 398.4 -> 365.5 us,
// worker-major and shuffled equal; 2 at 8 waves spills, profiles/r05/lab/packed_inflight_waves_ab_v32.log)
#ifndef INA_SWITCH_SLOT_INFLIGHT
#define INA_SWITCH_SLOT_INFLIGHT 1
#endif
#ifndef INA_PACKED_UNALIGNED
#define INA_PACKED_UNALIGNED 1
#endif
#ifndef INA_SWITCH_SLOT_INFLIGHT_SPLIT
#define INA_SWITCH_SLOT_INFLIGHT_SPLIT 1
#endif
template <bool kSplit>
constexpr int kSlotInFlight = kSplit ? INA_SWITCH_SLOT_INFLIGHT_SPLIT : INA_SWITCH_SLOT_INFLIGHT;
// Packed rows (the payload at byte 15 of the row): a lane's four values are one 16-byte access at
// byte 15 + 16 l -- an unaligned global load / store (gfx950 runs HSA code in unaligned access
// mode; the compiler emits one dwordx4 with offset 15) instead of the aligned chunk l + 1 and the
// neighbour lane's word through LDS
__device__ __forceinline__ u32x4s ld_row16(const uint8_t* p) {
    u32x4s v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st_row16(uint8_t* p, const u32x4s& v) { __builtin_memcpy(p, &v, 16); }

// one packet of a lane group's slot (group-uniform: every lane of the group runs it with the
// same header): ack / collision / count / Processor add, the PS step, the rewritten packet
// and its action byte.  m: this lane's payload chunk (packed rows: row chunk l + 1), h: the
// header chunk / header row; ack_known: a PS ack by its sort key (then m and h are unread)
template <bool kPs, bool kSplit, int kThr = kSwBlock>
__device__ __forceinline__ void group_packet(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                             size_t stride, uint8_t* __restrict__ pay,
                                             uint8_t* __restrict__ actions, const PsFuse& ps, uint32_t slot,
                                             uint32_t pid, const u32x4s& m, const u32x4s& h, bool ack_known,
                                             uint32_t& cnt, uint32_t& frag, u32x4s& reg, bool& have_reg,
                                             bool drop_written = false) {
    // neighbour lanes' words go through LDS, not DPP: a DPP move whose source lane is disabled
    // returns its fallback, and the compiler may narrow EXEC around a DPP that feeds a per-lane
    // select (it did: l == 0 ? h3 : row_shr(m.w) became a branch on l != 0).  Every lane of the
    // group stores, then reads its neighbour's word (LDS executes one wave's ops in order)
    __shared__ uint32_t s_xch[kThr];
    const int l = threadIdx.x & 7;
    const int V = st.V, L = V >> 2;
    const bool vl = l < L;
    const uint32_t h1 = h.y, h2 = h.z, h3 = h.w;
    const bool is_ack = ack_known || ((h1 >> 14) & 1u);
    uint8_t act;
    if (is_ack) {                            // reset_id (fragcheck.p4:26-31)
        frag = 0;
        act = INA_ACT_FWD_ACK;
    } else {
        const uint32_t hcount = h1 & 0xFFu;
        const uint32_t frag_in = __builtin_bswap32((h2 >> 24) | (h3 << 8));
        if (frag == 0) frag = frag_in;       // write_read_id (fragcheck.p4:14-24)
        if (frag != frag_in) {               // collision (ngaa.p4:177-181): the flag byte
            act = INA_ACT_FWD_COLLISION;
            if (l == 0)
                reinterpret_cast<uint32_t*>(pkts + (size_t)pid * (kSplit ? 16 : stride))[1] =
                    h1 | ((uint32_t)INA_FLAG_COLLISION << 8);
        } else {
            cnt = (cnt + 1u) & 0xFFu;        // read_add_count (ngaa.p4:66-78)
            if (cnt == hcount) cnt = 0;
            const bool first = cnt == 1u;
            u32x4s v;                        // values 4l..4l+3
            if constexpr (kSplit || INA_PACKED_UNALIGNED) {
                v.x = __builtin_bswap32(m.x); v.y = __builtin_bswap32(m.y);
                v.z = __builtin_bswap32(m.z); v.w = __builtin_bswap32(m.w);
            } else {
                // value 4l starts at the last byte of chunk l: the previous lane's
                // chunk, or the header chunk for the group's lane 0
                s_xch[threadIdx.x] = m.w;
                __builtin_amdgcn_wave_barrier();
                const uint32_t pw = l == 0 ? h3 : s_xch[threadIdx.x - 1];
                __builtin_amdgcn_wave_barrier();
                v.x = dec_be(m.x, pw);
                v.y = dec_be(m.y, m.x);
                v.z = dec_be(m.z, m.y);
                v.w = dec_be(m.w, m.z);
            }
            if (first) {                     // processor.p4:16-21
                reg = v;
            } else {
                if (!have_reg)               // adds to a stored register: load it now
                    reg = vl ? *reinterpret_cast<const u32x4s*>(st.regs + (size_t)slot * V + 4 * l)
                             : u32x4s{0u, 0u, 0u, 0u};
                reg += v;
            }
            have_reg = true;
            act = cnt == 0 ? INA_ACT_FWD_AGG : INA_ACT_DROP;   // ngaa.p4:170-175
            const uint32_t ps_slot = frag_in - ps.seq0;
            const bool consumed = kPs && act == INA_ACT_FWD_AGG && ps_slot < ps.nslots;
            if (kPs && consumed) {           // launch.py:46-50 with the switch's sum
                const size_t e0 = (size_t)ps_slot * (size_t)V + 4 * (size_t)l;
                if (vl && e0 + 4 <= ps.n) {
                    const f32x4s lc = *reinterpret_cast<const f32x4s*>(ps.local + e0);
                    f32x4s o;
                    o.x = __fadd_rn(lc.x, __fmul_rn(__fmul_rn((float)(int32_t)reg.x, ps.inv), ps.ws));
                    o.y = __fadd_rn(lc.y, __fmul_rn(__fmul_rn((float)(int32_t)reg.y, ps.inv), ps.ws));
                    o.z = __fadd_rn(lc.z, __fmul_rn(__fmul_rn((float)(int32_t)reg.z, ps.inv), ps.ws));
                    o.w = __fadd_rn(lc.w, __fmul_rn(__fmul_rn((float)(int32_t)reg.w, ps.inv), ps.ws));
                    __builtin_nontemporal_store(o, reinterpret_cast<f32x4s*>(ps.out + e0));
                } else if (vl) {
                    const uint32_t rv[4] = {reg.x, reg.y, reg.z, reg.w};
                    for (int t = 0; t < 4 && e0 + t < ps.n; ++t)
                        ps.out[e0 + t] = __fadd_rn(ps.local[e0 + t],
                                                   __fmul_rn(__fmul_rn((float)(int32_t)rv[t], ps.inv), ps.ws));
                }
                if (l == 0 && ps.acks) {     // the PS ack (fragcheck.p4:26-31)
                    u32x4s hd = h;
                    hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                    if constexpr (!kSplit) hd.w = (hd.w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                    *reinterpret_cast<u32x4s*>(ps.acks + (size_t)ps_slot * ps.ack_stride) = hd;
                    if (ps.ack_desc) ps.ack_desc[ps_slot] = uint2{hd.y, hd.z};
                }
            }
            if ((act != INA_ACT_DROP || st.write_dropped) && (!consumed || ps.keep_fwd)) {
                // out_value -> the packet (processor.p4:22)
                if constexpr (kSplit) {
                    const u32x4s e{__builtin_bswap32(reg.x), __builtin_bswap32(reg.y),
                                   __builtin_bswap32(reg.z), __builtin_bswap32(reg.w)};
                    if (vl) sw_st(e, reinterpret_cast<u32x4s*>(pay + (size_t)pid * (size_t)(4 * V)) + l);
                } else if constexpr (INA_PACKED_UNALIGNED) {
                    const u32x4s e{__builtin_bswap32(reg.x), __builtin_bswap32(reg.y),
                                   __builtin_bswap32(reg.z), __builtin_bswap32(reg.w)};
                    if (vl) st_row16(pkts + (size_t)pid * stride + 15 + 16 * l, e);
                } else {
                    // chunk l + 1: bytes 1..3 of values 4l..4l+3, then byte 0 of value
                    // 4l + 4 (the next lane's; the group's last value lane keeps the
                    // padding byte); lane 0 also rewrites the header chunk's byte 15
                    u32x4s* dst = reinterpret_cast<u32x4s*>(pkts + (size_t)pid * stride);
                    s_xch[threadIdx.x] = reg.x;
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t nx = l < L - 1 ? s_xch[threadIdx.x + 1] : m.w;
                    __builtin_amdgcn_wave_barrier();
                    u32x4s e;
                    e.x = enc_lo(reg.x, reg.y);
                    e.y = enc_lo(reg.y, reg.z);
                    e.z = enc_lo(reg.z, reg.w);
                    e.w = enc_lo(reg.w, nx);
                    if (vl) sw_st(e, dst + l + 1);
                    if (l == 0) {
                        u32x4s c0 = h;
                        c0.w = (c0.w & 0x00FFFFFFu) | (reg.x & 0xFF000000u);
                        sw_st(c0, dst);
                    }
                }
            }
        }
    }
    // (drop_written: the detection pass stored the drops by position)
    if (l == 0 && !(drop_written && act == INA_ACT_DROP)) actions[pid] = act;
}

// ---- whole segments of 8 (round 6) ---------------------------------------------------------
// The common narrow segment is one slot's W = 8 packets of one step: no PS ack, every frag id the
// slot's (or, the slot free, the first packet's), count field 8 and the slot's count at 0.  Then
// ngaa.p4:66-78 / processor.p4:14-24 reduce to: packet 0 overwrites the registers, packets 1..7
// add, packet 7 completes the slot (count back to 0) and is forwarded with the sum, packets 0..6
// are dropped.  The per-packet walk (group_packet) pays a dependent round trip and the state
// machine's branches per packet; here a wave whose 8 lane groups each hold such a segment (or
// none) reads every header row and the slots' count / frag in ONE round trip, checks the
// conditions, then issues all 8 payload loads per lane at once and adds them in registers.  Any
// other segment in the wave -> false, and the caller walks the wave's segments packet by packet
// (the rows it reads then come from L2).  Lane l of group g: pidl = the id of packet l of group
// g's segment, ackl its PS-ack hint (sort key bit 31); has = the group holds a segment.
#ifndef INA_SWITCH_SEG8
#define INA_SWITCH_SEG8 1
#endif
#ifndef INA_SEG8_FLIGHT
#define INA_SEG8_FLIGHT 4
#endif
constexpr int kSeg8Flight = INA_SEG8_FLIGHT;
static_assert(8 % kSeg8Flight == 0, "whole rounds of payload loads");
// kPs: the completing packet's sum goes straight into the PS update and its ack row (as
// group_packet does).  ack_pid != ~0u (group-uniform): a PS ack leads the segment (the steady
// state: step t's ack in front of step t+1's packets) -- it clears the slot's frag register
// (fragcheck.p4:26-31), so the first packet's frag id is the slot's, and it is forwarded as is.
template <bool kPs, bool kSplit>
__device__ __forceinline__ bool seg8_fast(const ina_switch_state_t& st, uint8_t* __restrict__ pkts, size_t stride,
                                          uint8_t* __restrict__ pay, uint8_t* __restrict__ actions,
                                          const PsFuse& ps, bool has, uint32_t slot, uint32_t pidl, bool ackl,
                                          bool drop_written, uint32_t ack_pid = ~0u, bool plainl = false,
                                          uint32_t plB = 0u, uint32_t plC = 0u) {
    const int lane = threadIdx.x & 63, l = lane & 7, g0 = lane & ~7;
    const int V = st.V, L = V >> 2;
    const bool vl = l < L;
    u32x4s h = {0u, 0u, 0u, 0u};
    uint32_t cnt = 0u, frag = 0u;
    // a plain packet (kPlainBit, sorted window path without the PS step): no header row read
    const bool pl = !kPs && plainl;
    if (has) {
        if (!pl) h = *reinterpret_cast<const u32x4s*>(pkts + (size_t)pidl * (kSplit ? 16 : stride));
        cnt = st.count[slot];
        if (ack_pid == ~0u) frag = st.frag[slot];
    }
    const uint32_t fin = pl ? slot + plB : __builtin_bswap32((h.z >> 24) | (h.w << 8));
    const uint32_t F = frag ? frag : (uint32_t)__shfl((int)fin, g0);
    const bool hok = pl ? plC == 8u : (!ackl && ((h.y >> 14) & 1u) == 0u && (h.y & 0xFFu) == 8u);
    const bool ok = !has || (hok && fin == F && cnt == 0u);
    if (__ballot(!ok)) return false;
    // the PS step (launch.py:46-50): this slot's update row, when the PS takes it
    const uint32_t ps_slot = F - ps.seq0;
    const bool consumed = kPs && has && ps_slot < ps.nslots;
    // the payload loads in flight together: kSeg8Flight at a time (the VGPRs they hold)
    constexpr int kF = kSeg8Flight;
    u32x4s run = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k0 = 0; k0 < 8; k0 += kF) {
    u32x4s m[kF];
#pragma unroll
    for (int j = 0; j < kF; ++j) {
        const uint32_t pk = (uint32_t)__shfl((int)pidl, g0 + k0 + j);
        m[j] = u32x4s{0u, 0u, 0u, 0u};
        if (has && vl) {
            if constexpr (kSplit)
                m[j] = sw_ld(reinterpret_cast<const u32x4s*>(pay + (size_t)pk * (size_t)(4 * V)) + l);
            else
                m[j] = ld_row16(pkts + (size_t)pk * stride + 15 + 16 * l);
        }
    }
#pragma unroll
    for (int j = 0; j < kF; ++j) {
        const int k = k0 + j;
        const u32x4s v{__builtin_bswap32(m[j].x), __builtin_bswap32(m[j].y), __builtin_bswap32(m[j].z),
                       __builtin_bswap32(m[j].w)};
        run = k == 0 ? v : run + v;
        // out_value -> the packet (processor.p4:22): the completing packet 7 (unless the PS
        // consumed it), and with write_dropped the dropped ones' running sums too (the id moved
        // with every lane active: lanes past V/4 sit out the store, and a moved value from an
        // inactive lane is undefined)
        const uint32_t pk = (uint32_t)__shfl((int)pidl, g0 + k);
        if (has && vl && (k == 7 ? (!consumed || ps.keep_fwd) : st.write_dropped)) {
            const u32x4s e{__builtin_bswap32(run.x), __builtin_bswap32(run.y), __builtin_bswap32(run.z),
                           __builtin_bswap32(run.w)};
            if constexpr (kSplit) sw_st(e, reinterpret_cast<u32x4s*>(pay + (size_t)pk * (size_t)(4 * V)) + l);
            else st_row16(pkts + (size_t)pk * stride + 15 + 16 * l, e);
        }
    }
    }
    if (has) {
        if (vl) __builtin_nontemporal_store(run, reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * l));
        if (l == 0) {
            st.count[slot] = 0u;                                  // 8 adds of count 8: back to 0
            st.frag[slot] = F;
            if (ack_pid != ~0u) actions[ack_pid] = INA_ACT_FWD_ACK;
        }
        if (l == 7 || !drop_written) actions[pidl] = l == 7 ? INA_ACT_FWD_AGG : INA_ACT_DROP;
        if constexpr (kPs) {
            if (consumed) {                                       // launch.py:46-50 with the switch's sum
                const size_t e0 = (size_t)ps_slot * (size_t)V + 4 * (size_t)l;
                if (vl && e0 + 4 <= ps.n) {
                    const f32x4s lc = *reinterpret_cast<const f32x4s*>(ps.local + e0);
                    f32x4s o;
                    o.x = __fadd_rn(lc.x, __fmul_rn(__fmul_rn((float)(int32_t)run.x, ps.inv), ps.ws));
                    o.y = __fadd_rn(lc.y, __fmul_rn(__fmul_rn((float)(int32_t)run.y, ps.inv), ps.ws));
                    o.z = __fadd_rn(lc.z, __fmul_rn(__fmul_rn((float)(int32_t)run.z, ps.inv), ps.ws));
                    o.w = __fadd_rn(lc.w, __fmul_rn(__fmul_rn((float)(int32_t)run.w, ps.inv), ps.ws));
                    __builtin_nontemporal_store(o, reinterpret_cast<f32x4s*>(ps.out + e0));
                } else if (vl) {
                    const uint32_t rv[4] = {run.x, run.y, run.z, run.w};
                    for (int t = 0; t < 4 && e0 + t < ps.n; ++t)
                        ps.out[e0 + t] = __fadd_rn(ps.local[e0 + t],
                                                   __fmul_rn(__fmul_rn((float)(int32_t)rv[t], ps.inv), ps.ws));
                }
                if (l == 7 && ps.acks) {                          // the PS ack (fragcheck.p4:26-31): packet 7's header
                    static_assert(kSplit || !kPs, "packed rows' ack rows also carry value 0's first byte");
                    u32x4s hd = h;
                    hd.y = (hd.y & ~0xFF00u) | ((uint32_t)INA_FLAG_ACK << 8);
                    *reinterpret_cast<u32x4s*>(ps.acks + (size_t)ps_slot * ps.ack_stride) = hd;
                    if (ps.ack_desc) ps.ack_desc[ps_slot] = uint2{hd.y, hd.z};
                }
            }
        }
    }
    return true;
}

// Narrow packets (V <= 32) in sorted order (the bucket sort's arrays, or a batch already in
// slot order read in place), segment-parallel: each wave takes windows of `win` sorted
// positions, and its 8 lane groups take the segments that START in the window, 8 at a time
// (group g: the g-th head), walking each segment's packets in position order (= arrival
// order inside the slot, ngaa.p4:120-196) with kP positions' loads in flight.  Per packet the
// same group_packet as the run-table path; a segment may run past the window's end.
template <bool kPs, bool kSplit>
__device__ __forceinline__ void window_slots_narrow(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                    uint8_t* __restrict__ pay, size_t npk, size_t stride,
                                                    const KeySrc keys, const uint32_t* __restrict__ ids,
                                                    uint8_t* __restrict__ actions, uint32_t win, uint32_t kmask,
                                                    const PsFuse& ps, size_t wave, size_t nwaves,
                                                    bool drop_written = false, uint32_t plB = 0u,
                                                    uint32_t plC = 0u) {
    constexpr int kP = kSlotInFlight<kSplit>;
    // plain packets (kPlainBit: set only for split rows without the PS step) read no header row
    constexpr bool kPlain = kSplit && !kPs;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, l = lane & 7;
    const int V = st.V, L = V >> 2;
    const bool vl = l < L;
    const uint32_t NS = st.num_slots;
    const uint32_t xm = ~kmask;                           // the hint bits: PS ack, plain
    // the window's packet ids and ack hints, for the lane groups to pick from (through LDS,
    // written by every lane of the wave: see group_packet on DPP / permutes and EXEC)
    __shared__ uint32_t s_wid[kSwBlock], s_wack[kSwBlock];
    const int wb = (int)threadIdx.x & ~63;
    for (size_t w0 = wave * win; w0 < npk; w0 += nwaves * win) {
        const size_t i = w0 + (size_t)lane;
        const uint32_t kr = i < npk ? keys(i) : NS;
        const uint32_t ki = kr & kmask;                   // slot (bit 31: PS-ack hint)
        const uint32_t idw = i < npk ? (ids ? ids[i] : (uint32_t)i) : 0u;
        const uint32_t kp = (i > 0 && i <= npk) ? (keys(i - 1) & kmask) : 0xFFFFFFFFu;
        const bool head = (uint32_t)lane < win && i < npk && ki < NS && (i == 0 || kp != ki);
        __builtin_amdgcn_wave_barrier();
        s_wid[threadIdx.x] = idw;
        // bit 0: a PS ack by its key (with the hint); bit 1: a plain packet
        s_wack[threadIdx.x] = ((kr & xm & kAckBit) ? 1u : 0u) | ((kr & xm & kPlainBit) ? 2u : 0u);
        __builtin_amdgcn_wave_barrier();
        unsigned long long hm = __ballot(head);
        while (hm) {
            // up to 8 segments: group g takes the g-th head's [start, end)
            uint32_t hslot = 0, hst = 0, hlen = 0, maxlen = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if (!hm) break;
                const int hl = __builtin_ctzll(hm);
                hm &= hm - 1;
                const uint32_t slot_b = __builtin_amdgcn_readlane(ki, hl);
                size_t end;
                const unsigned long long dm = __ballot(ki != slot_b) & ~((2ull << hl) - 1ull);
                if (dm) {
                    end = w0 + (size_t)__builtin_ctzll(dm);
                } else {
                    size_t j0 = w0 + 64;
                    for (;;) {
                        const size_t j = j0 + (size_t)lane;
                        const bool diff = j >= npk || (keys(j) & kmask) != slot_b;
                        const unsigned long long mm = __ballot(diff);
                        if (mm) { end = j0 + (size_t)__builtin_ctzll(mm); break; }
                        j0 += 64;
                    }
                }
                const uint32_t len_b = (uint32_t)(end - (w0 + (size_t)hl));
                maxlen = len_b > maxlen ? len_b : maxlen;
                if (g == b) {
                    hslot = slot_b;
                    hst = (uint32_t)hl;                   // window-relative start
                    hlen = len_b;
                }
            }
            const bool has = hlen != 0;
#if INA_SWITCH_SEG8
            if constexpr (kSplit && !kPs) {
                // every segment of these heads 8 packets long: the whole-segment path
                if (maxlen == 8u && !__ballot(has && hlen != 8u)) {
                    const uint32_t q = hst + (uint32_t)l;
                    uint32_t pidl = 0u, hint = 0u;
                    if (has) {
                        if (q < 64u) {
                            pidl = s_wid[wb + (int)q];
                            hint = s_wack[wb + (int)q];
                        } else {
                            const size_t qa = w0 + (size_t)q;
                            pidl = ids ? ids[qa] : (uint32_t)qa;
                            const uint32_t kq = keys(qa) & xm;
                            hint = ((kq & kAckBit) ? 1u : 0u) | ((kq & kPlainBit) ? 2u : 0u);
                        }
                    }
                    if (seg8_fast<kPs, kSplit>(st, pkts, stride, pay, actions, ps, has, hslot, pidl, (hint & 1u) != 0u,
                                               drop_written, ~0u, (hint & 2u) != 0u, plB, plC))
                        continue;
                }
            }
#endif
            uint32_t cnt = 0, frag = 0;
            if (has) {
                cnt = st.count[hslot];
                frag = st.frag[hslot];
            }
            u32x4s reg = {0u, 0u, 0u, 0u};
            bool have_reg = false;
            for (uint32_t k0 = 0; k0 < maxlen; k0 += kP) {
                u32x4s m[kP], h[kP];
                uint32_t pid[kP];
                bool in[kP], acq[kP];
#pragma unroll
                for (int j = 0; j < kP; ++j) {
                    const uint32_t k = k0 + (uint32_t)j;
                    const uint32_t q = hst + k;           // window-relative position
                    in[j] = has && k < hlen;
                    // id and hints: the window's (LDS), past the window from memory
                    pid[j] = 0u;
                    uint32_t hint = 0u;
                    if (in[j]) {
                        if (q < 64u) {
                            pid[j] = s_wid[wb + (int)q];
                            hint = s_wack[wb + (int)q];
                        } else {
                            const size_t qa = w0 + (size_t)q;
                            pid[j] = ids ? ids[qa] : (uint32_t)qa;
                            const uint32_t kq = keys(qa) & xm;
                            hint = ((kq & kAckBit) ? 1u : 0u) | ((kq & kPlainBit) ? 2u : 0u);
                        }
                    }
                    acq[j] = (hint & 1u) != 0u;
                    if (in[j] && !acq[j]) {
                        if constexpr (kSplit) {
                            m[j] = sw_ld(reinterpret_cast<const u32x4s*>(pay + (size_t)pid[j] * (size_t)(4 * V)) +
                                         (vl ? l : 0));
                            if (kPlain && (hint & 2u)) {
                                // the header fields group_packet reads, made from the slot: words 1-3
                                // of the row (count, flags 0, index = slot, switch id, frag id, pad 0)
                                const uint32_t fr = hslot + plB;
                                h[j] = u32x4s{0u, plC | (__builtin_bswap32(hslot) & 0xFFFFu) << 16,
                                              (__builtin_bswap32(hslot) >> 16) | ((uint32_t)(uint8_t)st.switch_id << 16) |
                                                  (fr & 0xFF000000u),
                                              (__builtin_bswap32(fr) >> 8)};
                            } else {
                                h[j] = *reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[j] * 16);
                            }
                        } else {
                            const u32x4s* pk = reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[j] * stride);
                            if constexpr (INA_PACKED_UNALIGNED)
                                m[j] = ld_row16(pkts + (size_t)pid[j] * stride + 15 + 16 * (vl ? l : 0));
                            else
                                m[j] = sw_ld(pk + (vl ? l + 1 : 1));
                            h[j] = *pk;
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < kP; ++j) {
                    if (!__ballot(in[j])) continue;
                    if (!in[j]) continue;
                    group_packet<kPs, kSplit>(st, pkts, stride, pay, actions, ps, hslot, pid[j], m[j], h[j], acq[j],
                                              cnt, frag, reg, have_reg, drop_written);
                }
            }
            if (has && l == 0) {
                st.count[hslot] = (uint8_t)cnt;
                st.frag[hslot] = frag;
            }
            if (have_reg && vl)
                __builtin_nontemporal_store(reg, reinterpret_cast<u32x4s*>(st.regs + (size_t)hslot * V + 4 * l));
        }
    }
}

// Narrow packets (V <= 32) from the near-sorted path's per-slot lists (local_lists): each wave
// takes 8 consecutive slots at a time (grid-stride; consecutive waves of an XCD take neighbouring
// slots), lane group g slot s8 + g: its (first entry, length) from the slot table, its list's
// first 8 packet ids one per lane (loaded beside the slot's count and frag), then the packets in
// list order = arrival order (ngaa.p4:120-196) through group_packet, kP loads in flight.
template <bool kPs, bool kSplit>
__device__ __forceinline__ void lists_slots_narrow(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                   size_t stride, uint8_t* __restrict__ pay,
                                                   uint8_t* __restrict__ actions, const PsFuse& ps,
                                                   const uint32_t* __restrict__ ids, const uint2* __restrict__ tab,
                                                   uint32_t kmin, uint32_t nslot, size_t wave, size_t nwaves) {
    constexpr int kP = kSlotInFlight<kSplit>;
    static_assert(8 % kP == 0, "a batch of list entries never crosses a group of 8 ids");
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, l = lane & 7;
    const int V = st.V, L = V >> 2;
    const bool vl = l < L;
    // the next 8 slots' table entries and first ids are loaded one step ahead (the table ->
    // ids -> rows chain would otherwise cost two round trips per step more than an in-order batch)
    const size_t step = nwaves * 8;
    size_t s8 = wave * 8;
    uint2 e_nx = s8 + (size_t)g < nslot ? tab[s8 + (size_t)g] : uint2{0u, 0u};
    uint32_t id_nx = (uint32_t)l < e_nx.y ? ids[e_nx.x + (uint32_t)l] : 0u;
    for (; s8 < nslot; s8 += step) {
        const uint32_t hst = e_nx.x, hlen = e_nx.y;
        uint32_t idl = id_nx;                                      // entries 0..7 of the list
        const size_t sn = s8 + step + (size_t)g;
        e_nx = sn < nslot ? tab[sn] : uint2{0u, 0u};
        uint32_t maxlen = hlen;
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) maxlen = max(maxlen, (uint32_t)__shfl_xor((int)maxlen, o));
        maxlen = __builtin_amdgcn_readfirstlane(maxlen);
        if (maxlen == 0) {
            id_nx = (uint32_t)l < e_nx.y ? ids[e_nx.x + (uint32_t)l] : 0u;
            continue;
        }
        const uint32_t slot = kmin + (uint32_t)s8 + (uint32_t)g;
        const bool has = hlen != 0;
#if INA_SWITCH_SEG8
        if constexpr (kSplit && !kPs) {
            // every list of these 8 slots 8 packets long: the whole-segment path
            if (maxlen == 8u && !__ballot(has && hlen != 8u) &&
                seg8_fast<kPs, kSplit>(st, pkts, stride, pay, actions, ps, has, slot, idl & ~kAckBit,
                                       (idl & kAckBit) != 0u, true)) {
                id_nx = (uint32_t)l < e_nx.y ? ids[e_nx.x + (uint32_t)l] : 0u;   // the next step's first ids
                continue;
            }
        }
#endif
        uint32_t cnt = 0, frag = 0;
        if (has) {
            cnt = st.count[slot];
            frag = st.frag[slot];
        }
        u32x4s reg = {0u, 0u, 0u, 0u};
        bool have_reg = false;
        for (uint32_t k0 = 0; k0 < maxlen; k0 += kP) {
            if (k0 && (k0 & 7u) == 0)                              // entries k0..k0+7
                idl = k0 + (uint32_t)l < hlen ? ids[hst + k0 + (uint32_t)l] : 0u;
            u32x4s m[kP], h[kP];
            uint32_t pid[kP];
            bool in[kP], acq[kP];
#pragma unroll
            for (int j = 0; j < kP; ++j) {
                const uint32_t k = k0 + (uint32_t)j;
                in[j] = k < hlen;
                const uint32_t en = (uint32_t)__shfl((int)idl, 8 * g + (int)(k & 7u));   // every lane active
                pid[j] = en & ~kAckBit;
                acq[j] = (en & kAckBit) != 0u;                     // a PS ack by its sort key
                if (in[j] && !acq[j]) {
                    if constexpr (kSplit) {
                        m[j] = sw_ld(reinterpret_cast<const u32x4s*>(pay + (size_t)pid[j] * (size_t)(4 * V)) + (vl ? l : 0));
                        h[j] = *reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[j] * 16);
                    } else {
                        const u32x4s* pk = reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[j] * stride);
                        if constexpr (INA_PACKED_UNALIGNED)
                            m[j] = ld_row16(pkts + (size_t)pid[j] * stride + 15 + 16 * (vl ? l : 0));
                        else
                            m[j] = sw_ld(pk + (vl ? l + 1 : 1));
                        h[j] = *pk;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kP; ++j) {
                if (!__ballot(in[j])) continue;
                if (!in[j]) continue;
                group_packet<kPs, kSplit>(st, pkts, stride, pay, actions, ps, slot, pid[j], m[j], h[j], acq[j], cnt,
                                          frag, reg, have_reg, true);
            }
        }
        id_nx = (uint32_t)l < e_nx.y ? ids[e_nx.x + (uint32_t)l] : 0u;   // the next step's first ids
        if (has && l == 0) {
            st.count[slot] = (uint8_t)cnt;
            st.frag[slot] = frag;
        }
        if (have_reg && vl)
            __builtin_nontemporal_store(reg, reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * l));
    }
}

template <bool kPs, bool kLat = false, bool kNarrow = false, bool kSplit = false>
__device__ __forceinline__ void switch_run2_body(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                 uint8_t* __restrict__ pay, size_t npk, size_t stride,
                                                 const uint32_t* __restrict__ keys,
                                                 const uint32_t* __restrict__ ids,
                                                 uint8_t* __restrict__ actions, uint32_t win,
                                                 uint32_t kmask, const PsFuse& ps, size_t wave,
                                                 size_t nwaves, bool drop_written = false,
                                                 const uint2* __restrict__ kdesc = nullptr,
                                                 uint32_t plB = 0u, uint32_t plC = 0u) {
#if INA_SWITCH_NARROW_SLOTS
    if constexpr (kNarrow) {
        // (kdesc: a batch in slot order whose keys come from its descriptors, see KeySrc)
        const KeySrc ks{keys, kdesc, st.num_slots, st.switch_id, kmask != 0xFFFFFFFFu};
        window_slots_narrow<kPs, kSplit>(st, pkts, pay, npk, stride, ks, ids, actions, win, kmask, ps, wave,
                                         nwaves, drop_written, plB, plC);
        return;
    }
#endif
    const int lane = threadIdx.x & 63;
    const uint32_t NS = st.num_slots;
    // each wave takes windows of 64 sorted positions and processes the segments that
    // START in its window (a segment may run past the window's end)
    for (size_t w0 = wave * win; w0 < npk; w0 += nwaves * win) {
        const size_t i = w0 + (size_t)lane;
        const uint32_t kr = i < npk ? keys[i] : NS;
        const uint32_t ki = kr & kmask;                   // slot (bit 31: PS-ack hint)
        // packet ids of the window, one load (no ids: a batch in slot order read in place)
        const uint32_t idw = i < npk ? (ids ? ids[i] : (uint32_t)i) : 0u;
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
        const bool ack_led = (am >> hl) & 1ull;
        auto pids = [&](size_t q0, int nb, uint32_t (&pid)[kB]) {
            // packet ids first (no load in the common in-window case; one coalesced load
            // otherwise), so the kB packet loads below issue back to back with no
            // s_waitcnt between them
            if (q0 + (size_t)nb <= w0 + 64) {
                const int o = (int)(q0 - w0);
#pragma unroll
                for (int b = 0; b < kB; ++b)
                    pid[b] = b < nb ? __builtin_amdgcn_readlane(idw, o + b < 64 ? o + b : 63) : 0u;
            } else {
                const uint32_t my = lane < nb ? (ids ? ids[q0 + (size_t)lane] : (uint32_t)(q0 + (size_t)lane)) : 0u;
#pragma unroll
                for (int b = 0; b < kB; ++b) pid[b] = __builtin_amdgcn_readlane(my, b);
            }
        };
        if constexpr (kNarrow)
            run_segment_narrow<kPs, kSplit>(st, pkts, stride, pay, actions, ps, slot, ack_led,
                                            pos + (ack_led ? 1 : 0), end, pids);
        else
            run_segment<kPs, kLat, kSplit>(st, pkts, stride, pay, actions, ps, slot, ack_led,
                                           pos + (ack_led ? 1 : 0), end, pids, drop_written);
        }
    }
}

// Narrow packets (V <= 32) over a run table, slot-parallel: lane group g = lane / 8 owns slot
// s0 + g of the wave's range, and the wave walks the runs in order (= each slot's arrival
// order, ngaa.p4:120-196): run r's packets for slots s0 .. s0+7 are neighbouring rows, so one
// wave instruction reads them contiguously (lane l: payload chunk l; packed rows: row chunk
// l + 1, the header chunk 0 for every lane of the group).  The count / frag state machine
// (ngaa.p4:64-82, fragcheck.p4:14-57) and the Processor add (processor.p4:14-24) run in every
// group at once on group-uniform VGPRs -- no per-packet scalar walk and no cross-group scan,
// about a tenth of run_segment_narrow's instructions per packet.  kP runs' loads are in
// flight together.  Same results as the per-slot walk, packet for packet.
template <bool kPs, bool kSplit>
__device__ __forceinline__ void runs_slots_narrow(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                  size_t stride, uint8_t* __restrict__ pay,
                                                  uint8_t* __restrict__ actions, const PsFuse& ps,
                                                  uint32_t R, uint32_t rpos, uint32_t rlen, uint32_t rslot,
                                                  bool rack, uint32_t lo, uint32_t hi, size_t wave,
                                                  size_t nwaves, bool drop_written = false) {
    constexpr int kP = kSlotInFlight<kSplit>;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, l = lane & 7;
    const int V = st.V, L = V >> 2;
    const bool vl = l < L;
    // whole groups of 8 slots per wave
    size_t per = ((size_t)(hi - lo) + nwaves - 1) / nwaves;
    per = (per + 7) & ~(size_t)7;
    const size_t s_begin = (size_t)lo + wave * per;
    const size_t s_end = s_begin + per < (size_t)hi ? s_begin + per : (size_t)hi;
    const uint32_t rack_u = rack ? 1u : 0u;
    // packed rows: run r's rows for the wave's 8 slots are neighbours, 8 x (L + 1) chunks of 16
    // bytes; lane c loads chunk c (and chunk 64 + c) of that stretch, so each wave instruction
    // reads contiguous lines, and the chunks reach their group's lanes through LDS (each
    // group reading its own row straight from memory issued ~24 line requests per 8 rows
    // instead of ~10)
    const int cpr = L + 1;                            // chunks per packed row
    const int gg0 = lane / cpr, cc0 = lane - gg0 * cpr;
    const int gg1 = (64 + lane) / cpr, cc1 = 64 + lane - gg1 * cpr;
    const bool has1 = 64 + lane < 8 * cpr;
    for (size_t s8 = s_begin; s8 < s_end; s8 += 8) {
        const uint32_t slot = (uint32_t)(s8 + (size_t)g);
        const bool sv = s8 + (size_t)g < s_end;
#if INA_SWITCH_SEG8
        if constexpr (kSplit) {
            // 8 runs, each holding every slot of this group once -- or a run of PS acks and then
            // 8 such runs (the packet path's steady state): the whole-segment path (lane l of a
            // group: run l's (l + 1's) packet of the group's slot, in run order = arrival order)
            const uint32_t a = R == 9u ? 1u : 0u;         // a leading run of acks
            if (R - a == 8u && (a == 0u || (__builtin_amdgcn_readfirstlane(rack_u) != 0u &&
                                            __builtin_amdgcn_readlane(rack_u, 1) == 0u))) {
                const uint32_t rsl = (uint32_t)__shfl((int)rslot, l + (int)a), rll = (uint32_t)__shfl((int)rlen, l + (int)a),
                               rpl = (uint32_t)__shfl((int)rpos, l + (int)a);
                const bool ackl = __shfl((int)rack_u, l + (int)a) != 0;
                const uint32_t off = slot - rsl;
                // the ack run's packet of this slot (a: every slot of the wave must have one)
                const uint32_t r0s = __builtin_amdgcn_readfirstlane(rslot), r0l = __builtin_amdgcn_readfirstlane(rlen),
                               r0p = __builtin_amdgcn_readfirstlane(rpos);
                const uint32_t aoff = slot - r0s;
                if (!__ballot(sv && (off >= rll || (a && aoff >= r0l))) &&
                    seg8_fast<kPs, kSplit>(st, pkts, stride, pay, actions, ps, sv, slot, rpl + off, ackl, drop_written,
                                           a ? r0p + aoff : ~0u))
                    continue;
            }
        }
#endif
        uint32_t cnt = 0, frag = 0;
        if (sv) {
            cnt = st.count[slot];
            frag = st.frag[slot];
        }
        u32x4s reg = {0u, 0u, 0u, 0u};
        bool have_reg = false, touched = false;
        for (uint32_t r0 = 0; r0 < R; r0 += kP) {
            // issue kP runs' loads: the group's packet of run r (if the run holds the slot)
            u32x4s m[kP], h[kP];
            uint32_t pid[kP];
            bool in[kP], ackr[kP];
#pragma unroll
            for (int j = 0; j < kP; ++j) {
                const uint32_t r = r0 + (uint32_t)j;
                const uint32_t rr = r < R ? r : 0u;
                const uint32_t rs = __builtin_amdgcn_readlane(rslot, rr);
                const uint32_t rl = r < R ? __builtin_amdgcn_readlane(rlen, rr) : 0u;
                const uint32_t rp = __builtin_amdgcn_readlane(rpos, rr);
                ackr[j] = __builtin_amdgcn_readlane(rack_u, rr) != 0u;
                const uint32_t off = slot - rs;
                in[j] = sv && off < rl;
                pid[j] = rp + off;
                if constexpr (kSplit) {
                    if (in[j] && !ackr[j]) {              // a run of PS acks needs no read
                        m[j] = sw_ld(reinterpret_cast<const u32x4s*>(pay + (size_t)pid[j] * (size_t)(4 * V)) +
                                     (vl ? l : 0));
                        h[j] = *reinterpret_cast<const u32x4s*>(pkts + (size_t)pid[j] * 16);
                    }
                } else {
                    // the stretch of run r holding group gg's row: rows rp + (slot - rs)
                    const uint32_t sg0 = (uint32_t)s8 + (uint32_t)gg0, sg1 = (uint32_t)s8 + (uint32_t)gg1;
                    const bool ok0 = !ackr[j] && gg0 < 8 && sg0 < s_end && sg0 - rs < rl;
                    const bool ok1 = !ackr[j] && has1 && sg1 < s_end && sg1 - rs < rl;
                    if (ok0)
                        m[j] = sw_ld(reinterpret_cast<const u32x4s*>(pkts + (size_t)(rp + (sg0 - rs)) * stride) + cc0);
                    if (ok1)
                        h[j] = sw_ld(reinterpret_cast<const u32x4s*>(pkts + (size_t)(rp + (sg1 - rs)) * stride) + cc1);
                }
            }
            if constexpr (!kSplit) {
                // the stretches to LDS, then each group's chunks back: chunk l + 1 of its row
                // (value lanes) and chunk 0 (the header chunk) for every lane of the group
                __shared__ u32x4s s_stage[kSwBlock / 64][kP][64 + 8];
                const int wb = (int)(threadIdx.x >> 6);
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int j = 0; j < kP; ++j) {
                    s_stage[wb][j][lane] = m[j];
                    if (has1) s_stage[wb][j][64 + lane] = h[j];
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int j = 0; j < kP; ++j) {
                    if (in[j] && !ackr[j]) {
                        if constexpr (INA_PACKED_UNALIGNED) {
                            // the lane's bytes 15 + 16 l .. 30 + 16 l (group_packet's packed-row
                            // form): chunk l's last byte, then chunk l + 1's first fifteen
                            const u32x4s c0 = s_stage[wb][j][g * cpr + (vl ? l : 0)];
                            const u32x4s c1 = s_stage[wb][j][g * cpr + (vl ? l + 1 : 1)];
                            m[j] = u32x4s{__builtin_amdgcn_alignbyte(c1.x, c0.w, 3), __builtin_amdgcn_alignbyte(c1.y, c1.x, 3),
                                          __builtin_amdgcn_alignbyte(c1.z, c1.y, 3), __builtin_amdgcn_alignbyte(c1.w, c1.z, 3)};
                        } else {
                            m[j] = s_stage[wb][j][g * cpr + (vl ? l + 1 : 1)];
                        }
                        h[j] = s_stage[wb][j][g * cpr];
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int j = 0; j < kP; ++j) {
                if (!__ballot(in[j])) continue;          // no slot of this wave in run r0 + j
                if (!in[j]) continue;
                touched = true;
                group_packet<kPs, kSplit>(st, pkts, stride, pay, actions, ps, slot, pid[j], m[j], h[j], ackr[j],
                                          cnt, frag, reg, have_reg, drop_written);
            }
        }
        if (touched && l == 0) {
            st.count[slot] = (uint8_t)cnt;
            st.frag[slot] = frag;
        }
        if (have_reg && vl)
            __builtin_nontemporal_store(reg, reinterpret_cast<u32x4s*>(st.regs + (size_t)slot * V + 4 * l));
    }
}

// The run kernel's work over a batch of dense ascending runs (the run table the bucket
// pass wrote, see kRunsMax): lane r holds run r; each wave takes one contiguous range of
// slots (one pass of the grid) and runs slot s's segment -- the packets start_r + s -
// first_r of the runs that hold s, in run order = arrival order -- through run_segment.
// A PS ack leading its segment is done without reading it, as in switch_run2_body.
template <bool kPs, bool kNarrow, bool kSplit>
__device__ __forceinline__ void switch_runs_body(const ina_switch_state_t& st, uint8_t* __restrict__ pkts,
                                                 size_t stride, uint8_t* __restrict__ pay,
                                                 uint8_t* __restrict__ actions,
                                                 uint32_t kmask, const PsFuse& ps,
                                                 const uint32_t* __restrict__ runs, size_t wave,
                                                 size_t nwaves, bool drop_written = false) {
    const int lane = threadIdx.x & 63;
    const uint32_t NS = st.num_slots;
    const uint32_t R = __builtin_amdgcn_readfirstlane(runs[0]);
    uint32_t rpos = 0, rslot = 0, rlen = 0;
    bool rack = false;
    if ((uint32_t)lane < R) {
        rpos = runs[kRunsStart + lane];
        rlen = runs[kRunsStart + lane + 1] - rpos;
        const uint32_t rk = runs[kRunsKey + lane];
        rslot = rk & kmask;
        rack = (rk & ~kmask & kAckBit) != 0u;
        if (rslot >= NS) rlen = 0;                    // foreign packets: A set their action
    }
    // the slots the runs cover: [lo, hi)
    uint32_t lo = rlen ? rslot : 0xFFFFFFFFu, hi = rlen ? rslot + rlen : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    if (lo >= hi) return;
    const size_t per = ((size_t)(hi - lo) + nwaves - 1) / nwaves;
    const size_t s_begin = (size_t)lo + wave * per;
    const size_t s_end = s_begin + per < (size_t)hi ? s_begin + per : (size_t)hi;
#if INA_SWITCH_NARROW_SLOTS
    if constexpr (kNarrow) {
        runs_slots_narrow<kPs, kSplit>(st, pkts, stride, pay, actions, ps, R, rpos, rlen, rslot, rack, lo, hi,
                                       wave, nwaves, drop_written);
        return;
    }
#endif
    for (size_t s = s_begin; s < s_end; ++s) {
        const uint32_t slot = (uint32_t)s;
        const uint32_t off = slot - rslot;
        const bool in = off < rlen;                   // wraps above for slots below the run
        unsigned long long m = __ballot(in);
        if (!m) continue;
        const uint32_t pidv = rpos + off;
        const int l0 = __builtin_ctzll(m);
        const bool ack_led = (__ballot(in && rack) >> l0) & 1ull;
        if (ack_led) {                                // reset_id (fragcheck.p4:26-31), unread
            const uint32_t p0 = __builtin_amdgcn_readlane(pidv, l0);
            m &= m - 1;
            if (lane == 0) {
                actions[p0] = INA_ACT_FWD_ACK;
                if (!m) st.frag[slot] = 0u;           // a lone ack
            }
            if (!m) continue;
        }
        const size_t nseg = (size_t)__builtin_popcountll(m);
        auto pids = [&](size_t, int nb, uint32_t (&pid)[kB]) {
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                if (b < nb) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    pid[b] = __builtin_amdgcn_readlane(pidv, l);
                } else {
                    pid[b] = 0u;
                }
            }
        };
        if constexpr (kNarrow)
            run_segment_narrow<kPs, kSplit>(st, pkts, stride, pay, actions, ps, slot, ack_led, 0, nseg, pids);
        else
            run_segment<kPs, false, kSplit>(st, pkts, stride, pay, actions, ps, slot, ack_led, 0, nseg, pids,
                                            drop_written);
    }
}

// XCD-contiguous block map: blocks b and b + 8 share an XCD (and its L2), so logical block
// (b % 8) * G/8 + b / 8 gives each XCD one contiguous run of the logical index
// (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"; speed only).  The digit pass's
// chunks and the near-sorted lists' units use it (their neighbours share lines and windows);
// the run kernel's windows and slot ranges do NOT since round 6 (INA_SWITCH_XCD = 0): each XCD
// then streams from every part of the batch instead of one eighth of it, and every order ran
// faster -- NGA-32 split worker-major 207.8 -> 202.5 us, round-robin 232.8 -> 228.0, jitter 64
// 286.4 -> 281.5, shuffled 384.5 -> 374.8, packed worker-major 259.3 -> 236.2; NGA-256 packed
// 4-7 us, split worker-major 195.3 -> 180.0; the NGA-256 packet path's switch + PS 219.4 ->
// 204.1 us (profiles/r06/lab/run_block_map_ab.log).  The near-sorted lists keep the map, in
// their build and in the run's walk of them: plain, jitter 4096 lost 15-16 us.
#ifndef INA_SWITCH_XCD
#define INA_SWITCH_XCD 0
#endif
__device__ __forceinline__ size_t xcd_block_index() {
    const uint32_t G = gridDim.x, b = blockIdx.x, x = b & 7u;
    const uint32_t per = G >> 3, rem = G & 7u;
    return (size_t)x * per + (x < rem ? x : rem) + (b >> 3);
}
__device__ __forceinline__ size_t switch_block_index() {
#if INA_SWITCH_XCD
    return xcd_block_index();
#else
    return blockIdx.x;
#endif
}

// occupancy target of the narrow split-row run without the PS step: 8 waves per SIMD takes its
// SGPRs to the 80 that admit 8 blocks per CU (8 spilled to VGPR lanes; 86 admitted 7)
#ifndef INA_SWITCH_WAVES_RUN_NS
#define INA_SWITCH_WAVES_RUN_NS 8     // NGA-32 C3 split: worker-major 232.2 -> 223.0, round-robin 259.2 -> 252.6 us (r05x)
#endif
#ifndef INA_SWITCH_WAVES_PS_NS
#define INA_SWITCH_WAVES_PS_NS 8      // NGA-32 packet path: switch + PS 329.3 -> 297.6 us, step 636.9 -> 608.9 (r05y)
#endif
template <bool kPs, bool kNarrow, bool kSplit>
#ifndef INA_SWITCH_WAVES_RUN_NP
#define INA_SWITCH_WAVES_RUN_NP 8     // narrow packed rows (with 1 packet in flight, see kSlotInFlight)
#endif
__global__ __launch_bounds__(kSwBlock) __attribute__((amdgpu_waves_per_eu(kPs ? ((kNarrow && kSplit) ? INA_SWITCH_WAVES_PS_NS : INA_SWITCH_WAVES) : (kNarrow && kSplit) ? INA_SWITCH_WAVES_RUN_NS : kNarrow ? INA_SWITCH_WAVES_RUN_NP : INA_SWITCH_WAVES_RUN, 8))) void k_switch_run2(ina_switch_state_t st,
                                                          uint8_t* __restrict__ pkts,
                                                          uint8_t* __restrict__ pay, size_t npk,
                                                          size_t stride,
                                                          const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ ids,
                                                          uint8_t* __restrict__ actions,
                                                          uint32_t win, uint32_t kmask, PsFuse ps,
                                                          const uint32_t* __restrict__ nforeign,
                                                          const uint32_t* __restrict__ keys_a,
                                                          const uint32_t* __restrict__ ids_a,
                                                          const uint32_t* __restrict__ unsorted,
                                                          const uint32_t* __restrict__ loc_ids,
                                                          const uint2* __restrict__ loc_tab, int drop_prefill,
                                                          const uint2* __restrict__ kdesc) {
    const size_t wave = switch_block_index() * (kSwBlock / 64) + wave_in_block();
    // (drop_prefill: the detection pass stored every packet's drop, so no path stores drops again)
    const size_t nwaves = ((size_t)gridDim.x * kSwBlock) >> 6;
    // (unsorted[1]: the epoch of the sort that filled the scratch, written by its chunk pass,
    // so a run queued apart from its sort needs no host-side state)
    uint32_t plB = 0u, plC = 0u;                            // (sorted keys with kPlainBit)
    if (unsorted) {
        const uint32_t ep = unsorted[1];
        if (unsorted[kLocEpoch] == ep) {                   // a near-sorted batch: its per-slot lists
            if constexpr (kNarrow)
                // (the lists' slots XCD-contiguous: neighbouring slots' lists point into the same
                // arrival windows, whose rows then come through one L2 -- the plain map cost
                // jitter 4096 16 us)
                lists_slots_narrow<kPs, kSplit>(st, pkts, stride, pay, actions, ps, loc_ids, loc_tab,
                                                unsorted[kLocKmin], unsorted[kLocSlots],
                                                xcd_block_index() * (kSwBlock / 64) + wave_in_block(), nwaves);
            return;
        }
        if (unsorted[2] == ep) {
            // a batch of dense ascending runs: the decision wrote the run table, not a sort
            switch_runs_body<kPs, kNarrow, kSplit>(st, pkts, stride, pay, actions, kmask, ps,
                                                   unsorted + (kCtlRuns - kCtlEpochs), wave, nwaves,
                                                   drop_prefill != 0);
            return;
        }
        if (unsorted[0] != ep) {
            // a batch already in slot order: the chunk sort's own output is the sorted order
            // (after the split chunk pass of wide keys: the arrival-order keys, ids_a NULL --
            // the packets in place, the foreign ones last with key num_slots, never a head)
            keys = keys_a;
            ids = ids_a;
            if (!ids_a) nforeign = nullptr;
        } else {
            kdesc = nullptr;                                // only an in-order batch reads them
            if constexpr (kNarrow && kSplit && !kPs) {
                plB = unsorted[kPlainB];
                plC = unsorted[kPlainC];
            }
        }
    } else {
        kdesc = nullptr;
    }
    // bucket sort: the foreign packets' bucket was left unsorted at the END of the arrays;
    // the run kernel never processes foreign packets, so it stops before them
    if (nforeign) npk -= *nforeign;
    switch_run2_body<kPs, false, kNarrow, kSplit>(st, pkts, pay, npk, stride, keys, ids, actions, win, kmask, ps,
                                                  wave, nwaves, drop_prefill != 0, kdesc, plB, plC);
}

// batches of at most INA_SWITCH_TINY_MAX packets (latency, not bandwidth): ONE launch of
// one 16-wave workgroup -- the bitonic (slot, packet id) sort in LDS, then the run
// kernel's work on the same 16 waves with the sorted arrays read from LDS.
template <bool kPs, typename T, int kIdBits, bool kSplit>
__global__ __launch_bounds__(kSmallBlock) void k_switch_tiny(ina_switch_state_t st, uint8_t* __restrict__ pkts,
                                                             uint8_t* __restrict__ pay, uint32_t npk, size_t stride,
                                                             uint8_t* __restrict__ actions, uint32_t win,
                                                             PsFuse ps) {
    // the sorted (slot, packet id) arrays stay in LDS: the run loop's window loads are LDS
    // reads, not a memory round trip
    __shared__ uint32_t keys_s[INA_SWITCH_SMALL_MAX], ids_s[INA_SWITCH_SMALL_MAX];
    switch_sort_small_body<T, kIdBits>(pkts, npk, stride, st.num_slots, st.switch_id, actions, keys_s, ids_s);
    __syncthreads();
    switch_run2_body<kPs, true, false, kSplit>(st, pkts, pay, npk, stride, keys_s, ids_s, actions, win,
                                               0xFFFFFFFFu, ps, wave_in_block(), kSmallBlock / 64);
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
    // the chunk + bucket sort: A's high digit and B's low digit (hbits + lbits = the key's
    // bits); wide = 2,048-bin kernels (keys of 19-22 bits); bucket_ok = keys of <= 22 bits
    int hbits, lbits;
    bool wide, bucket_ok;
};

static SortPlan sort_plan(size_t npk, uint32_t num_slots, const SwitchTuning& t) {
    SortPlan p;
    const int eb = end_bit_for(num_slots);
    p.passes = (eb + kRsMaxBits - 1) / kRsMaxBits;
    p.bits = (eb + p.passes - 1) / p.passes;
    // chunk + bucket split: the digit passes' two digits up to 18 bits (512 bins); 19-22 bits
    // (pools of 2^18 .. 2^21 slots) in two digits of 10-11 bits (2,048 bins) instead of the
    // three LSD passes
    p.wide = eb > 2 * kRsMaxBits;
    p.bucket_ok = eb <= 2 * kBitsBig;
    p.hbits = p.wide ? (eb + 1) / 2 : p.bits;
    p.lbits = eb - p.hbits;
    // chunk = 4 waves x 64 x rounds items: 1,024 up to 256 Ki packets (a batch of the PS's
    // acks still spreads over more than a few dozen CUs), 2,048 up to 512 Ki, 4,096 above
    // (switch_lab, profiles/r01/lab/switch_lab_rounds.log: 102,400 packets 77.7 -> 60.9 us,
    // 409,600 155.5 -> 146.1, 819,200 unchanged).  With the chunk + bucket sort, 819,200
    // packets: 4,096-packet chunks (200 A blocks) 234.6 us worker-major, 2,048 235.8, 1,024
    // 241.3 (profiles/r03/lab/sort_rounds_lab.log)
    p.rounds = npk <= (size_t)INA_RS_SMALL_ITEMS ? INA_RS_ROUNDS_SMALL
             : npk <= (size_t)INA_RS_MID_ITEMS   ? INA_RS_ROUNDS_MID
                                                 : kRsRounds;
    // more than 2 Mi packets through the chunk + bucket sort: 8,192-packet chunks.  NGA-32
    // at C3 size (6,553,600 packets, 2^20 slots: 1,025 buckets of 6,400, i.e. runs of 4
    // packets per 4,096-packet chunk) shuffled 709 -> 676 us packed, 616 -> 583 us split;
    // structured arrival unchanged; at 819,200 NGA-256 packets (100 chunks) +2 %, so not
    // there (interleaved A/B, bytes equal, profiles/r04/lab/chunk_rounds32_ab_v*.log).  The
    // digit passes keep 4,096 (they never see this tier: bucket_ok, mode 0, <= 2,048 chunks)
    if (npk > (size_t)INA_RS_BIG_ITEMS && p.bucket_ok && t.sort_mode == 0 &&
        npk <= (size_t)kBkMaxChunks * kRsWaves * 64 * INA_RS_ROUNDS_BIG)
        p.rounds = INA_RS_ROUNDS_BIG;
    if (const int r = t.os_rounds) p.rounds = r;   // ina_set_tuning key 13 (the tests' tier cover)
    const size_t chunk = (size_t)kRsWaves * 64 * (size_t)p.rounds;
    p.nch = (npk + chunk - 1) / chunk;
    p.hist_elems = ((size_t)1 << std::max(p.bits, p.hbits)) * p.nch;
    return p;
}

// sort scratch after the four key / id arrays, sized for the SMALLEST chunk whatever tier
// npk falls in (so the size is monotonic in npk: a buffer sized for a batch serves every
// smaller batch): per (digit, chunk) counts -- the digit passes' histogram, or A's run
// lengths -- and A's run starts, the digit passes' digit totals, the control block (the
// size of the foreign-only bucket B leaves out, the epochs, the run table) and A's per-chunk
// breaks of the dense runs (count + kRunsMax entries per chunk)
struct SortAux {
    uint32_t* hist;               // [2^bits][nch]
    uint32_t* rst;                // [2^bits][nch]
    uint32_t* totals;             // [512]
    uint32_t* nforeign;           // control block word kCtlForeign
    uint32_t* unsorted;           // [3]: the epoch of the last call whose keys were out of order,
                                  // the epoch of the last chunk pass, the epoch of the last run
                                  // table; the run table follows
    uint32_t* brk_cnt;            // [nch]
    uint2* brk_ent;               // [nch][kRunsMax]
    uint32_t* gstat;              // near-sorted path: granule key bounds, gmin[G] then gmax[G]
    LocUnit* units;               // near-sorted path: per unit (>= 2 granules) its slot range and window
    uint2* tab;                   // near-sorted path: per slot (first list entry, length)
    uint32_t* kflags;             // per detection wave: the epoch of the call whose keys it stored
};

static size_t sort_nch_cap(size_t npk) {
    const size_t chunk = (size_t)kRsWaves * 64 * (size_t)INA_RS_ROUNDS_SMALL;
    return (npk + chunk - 1) / chunk;
}

static size_t sort_hist_cap(size_t npk, uint32_t num_slots) {
    const SortPlan p = sort_plan(npk, num_slots, SwitchTuning{});     // bits: no key changes them
    return ((size_t)1 << std::max(p.bits, p.hbits)) * sort_nch_cap(npk);
}

static size_t sort_temp_bytes(size_t npk, uint32_t num_slots) {
    const size_t hist = align_up(sort_hist_cap(npk, num_slots) * 4, 256);
    const size_t nc = sort_nch_cap(npk);
    return 2 * hist + align_up((size_t)kRsBins * 4, 256) + 1024 + align_up(nc * 4, 256) +
           align_up(nc * (size_t)kRunsMax * 8, 256) + align_up(2 * nc * kGranPerChunk * 4, 256) +
           align_up(nc * (kGranPerChunk / 2) * sizeof(LocUnit), 256) + align_up((size_t)num_slots * 8, 256) +
           nc * kBkWaves * 4;
}

static SortAux sort_aux(uint8_t* aux, size_t npk, uint32_t num_slots) {
    const size_t hist = align_up(sort_hist_cap(npk, num_slots) * 4, 256);
    const size_t nc = sort_nch_cap(npk);
    SortAux a;
    a.hist = reinterpret_cast<uint32_t*>(aux);
    a.rst = reinterpret_cast<uint32_t*>(aux + hist);
    a.totals = reinterpret_cast<uint32_t*>(aux + 2 * hist);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(aux + 2 * hist + align_up((size_t)kRsBins * 4, 256));
    a.nforeign = ctl + kCtlForeign;
    a.unsorted = ctl + kCtlEpochs;
    a.brk_cnt = ctl + 256;
    a.brk_ent = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(a.brk_cnt) + align_up(nc * 4, 256));
    a.gstat = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.brk_ent) + align_up(nc * (size_t)kRunsMax * 8, 256));
    a.units = reinterpret_cast<LocUnit*>(reinterpret_cast<uint8_t*>(a.gstat) + align_up(2 * nc * kGranPerChunk * 4, 256));
    a.tab = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(a.units) + align_up(nc * (kGranPerChunk / 2) * sizeof(LocUnit), 256));
    a.kflags = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.tab) + align_up((size_t)num_slots * 8, 256));
    return a;
}

// The sorts queued alone (phase 1), by scratch: the switch keys they ran under and the batch
// they sorted -- its shape, its rows, its actions (the detection pass stored every packet's drop
// / foreign action there, and the run stores only the others) and the switch id its keys were
// made for.  The run over that scratch (phase 2) takes its keys from here, refuses a scratch no
// sort of exactly this batch filled, and consumes the record.  Every sort or sort + run call
// drops the scratch's record before it launches anything (it overwrites what an earlier sort
// left), and a sort alone records only once all its launches succeeded.
struct SortRecord {
    SwitchTuning t;
    size_t npk, stride;
    uint32_t num_slots;
    int V;
    bool split;
    const void *rows, *pay, *actions;
    int switch_id;
};
static std::mutex g_sorts_mu;
static std::unordered_map<const void*, SortRecord> g_sorts;
static std::atomic<size_t> g_sorts_n{0};

static void sort_record_set(const void* scratch, bool keep, const SortRecord& r) {
    if (!keep && g_sorts_n.load() == 0) return;               // nothing recorded anywhere
    std::lock_guard<std::mutex> lk(g_sorts_mu);
    if (keep) g_sorts[scratch] = r;
    else g_sorts.erase(scratch);
    g_sorts_n = g_sorts.size();
}

static bool sort_record_find(const void* scratch, const SortRecord& want, SwitchTuning* t) {
    std::lock_guard<std::mutex> lk(g_sorts_mu);
    const auto it = g_sorts.find(scratch);
    if (it == g_sorts.end()) return false;
    const SortRecord& r = it->second;
    if (r.npk != want.npk || r.stride != want.stride || r.num_slots != want.num_slots || r.V != want.V ||
        r.split != want.split || r.rows != want.rows || r.pay != want.pay || r.actions != want.actions ||
        r.switch_id != want.switch_id)
        return false;
    *t = r.t;
    return true;
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

#if INA_LOC_TIMING
int ina_lab_loc_times(unsigned long long* host_out) {  // lab builds only
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_loc_t), sizeof(g_loc_t)) == hipSuccess ? 0 : -1;
}
#endif
#if INA_BK_TIMING
int ina_lab_bk_times(unsigned long long* host_out) {   // lab builds only
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_bk_t), sizeof(g_bk_t)) == hipSuccess ? 0 : -1;
}
#endif

size_t ina_switch_scratch_bytes(size_t npkts, uint32_t num_slots) {
    if (npkts == 0 || npkts > 0x7FFFFFFFu || num_slots == 0) return 256;
    return 4 * align_up(npkts * 4, 256) + align_up(sort_temp_bytes(npkts, num_slots), 256) + 256;
}

// phase: 0 sort + run; 1 the slot sort alone (descriptor batches: it reads only the
// descriptors, so it may run before or beside the kernels that fill the payload); 2 the run
// alone over a scratch a phase-1 call filled for the same batch (paths whose sort reads the
// packets -- the one-workgroup small-batch paths -- sort in phase 2 instead)
// pay != NULL: split rows -- pkts are the 16-byte header rows (stride 16), pay the 4V-byte
// payload rows (include/ina.h "split NGA rows"); only the register-resident run kernels
// take them
static int switch_process_impl(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                               const uint64_t* desc, uint8_t* actions, void* scratch,
                               ina_stream_t stream, const PsFuse& ps, bool* fused_out, int phase = 0,
                               uint8_t* pay = nullptr) {
    *fused_out = false;
    const bool split = pay != nullptr;
    if (split && (!st || st->V % 4 || st->V <= 0 || st->V > kMaxV || stride != 16 || ((uintptr_t)pay & 15u)))
        return set_error(INA_EINVAL, "split rows need V a multiple of 4 <= 256 and 16-byte aligned rows%s", "");
    if (phase == 1 && !desc && npk)
        return set_error(INA_EINVAL, "the separate slot sort needs the batch's descriptors%s", "");
    const bool do_sort = phase != 2, do_run = phase != 1;
    if (!st || st->V <= 0 || st->V > kMaxV || st->num_slots == 0)
        return set_error(INA_EINVAL, "bad switch state (V in [1,256])%s", "");
    if (!split && stride < (size_t)INA_NGA_HDR_BYTES + 4u * (size_t)st->V)
        return set_error(INA_EINVAL, "stride must be >= 15+4V%s", "");
    if (stride > 0xFFFFFFFFu) return set_error(INA_EINVAL, "stride too large%s", "");
    if (npk == 0) return INA_OK;
    if (npk > 0x7FFFFFFFu) return set_error(INA_EINVAL, "too many packets%s", "");
    if (!pkts || !actions || !scratch || !st->count || !st->frag || !st->regs)
        return set_error(INA_EINVAL, "null pointer%s", "");
    if (desc && ((uintptr_t)desc & 7u))
        return set_error(INA_EINVAL, "descriptors must be 8-byte aligned%s", "");
    // the switch keys of this batch: read once here, or (a run alone) its sort's record
    SwitchTuning t;
    SortRecord rec{SwitchTuning{}, npk, stride, st->num_slots, st->V, split, pkts, pay, actions, st->switch_id};
    if (phase == 2) {
        if (!sort_record_find(scratch, rec, &t))
            return set_error(INA_EINVAL,
                             "run alone: no sort of this batch (rows, actions, shape, switch id) was queued into "
                             "this scratch%s", "");
    } else {
        t = switch_tuning();
        rec.t = t;
        sort_record_set(scratch, false, rec);                  // this call overwrites the scratch
    }
    // a sort alone records its batch once every launch succeeded; a run alone consumes the record
    auto sorted_ok = [&]() {
        if (phase == 1) sort_record_set(scratch, true, rec);
        return INA_OK;
    };
    auto run_ok = [&]() {
        if (phase == 2) sort_record_set(scratch, false, rec);
        return INA_OK;
    };
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint8_t* base = reinterpret_cast<uint8_t*>(align_up((uintptr_t)scratch, 256));
    size_t arr = align_up(npk * 4, 256);
    uint32_t* k_in = reinterpret_cast<uint32_t*>(base);
    uint32_t* k_out = reinterpret_cast<uint32_t*>(base + arr);
    uint32_t* v_in = reinterpret_cast<uint32_t*>(base + 2 * arr);
    uint32_t* v_out = reinterpret_cast<uint32_t*>(base + 3 * arr);
    const SortPlan sp = sort_plan(npk, st->num_slots, t);
    const SortAux ax = sort_aux(base + 4 * arr, npk, st->num_slots);
    // sort chunk geometry (sort_plan): one instantiation per rounds-per-wave choice
    constexpr int kR0 = INA_RS_ROUNDS_SMALL, kR1 = INA_RS_ROUNDS_MID, kR2 = kRsRounds, kR3 = INA_RS_ROUNDS_BIG;
    static_assert(kR0 % 4 == 0 && kR1 % 4 == 0 && kR2 % 4 == 0 && kR3 % 4 == 0, "chunk sort: 16 waves x rounds/4");
    const int ri = sp.rounds == kR0 ? 0 : sp.rounds == kR1 ? 1 : sp.rounds == kR2 ? 2 : 3;
    const unsigned gc = (unsigned)sp.nch;
    const uint32_t nb = 1u << sp.bits;

    uint32_t *kc = k_in, *vc = v_in, *kn = k_out, *vn = v_out;
    const bool fast = stride % 16 == 0 && ((uintptr_t)pkts & 15u) == 0 && st->V % 4 == 0 &&
                      st->V <= kMaxV && ((uintptr_t)st->regs & 15u) == 0;
    if (split && !fast) return set_error(INA_EINVAL, "split rows need 16-byte aligned rows and registers%s", "");
    // keys carry the PS-ack bit for the run kernel when bit 31 is outside every digit
    const bool ack_hint = fast && sp.passes * sp.bits <= 31 && t.ack_fast;
    const bool small = npk <= (size_t)t.small_sort;
    // chunk + bucket sort: keys of one or two digits (the low digit is one workgroup's LDS
    // bins) and at most kBkMaxChunks chunks (B's LDS rows); else the digit passes
    const bool bucket = !small && t.sort_mode == 0 && sp.bucket_ok && sp.nch <= (size_t)kBkMaxChunks;
    const uint32_t* nforeign = nullptr;
    const uint32_t* unsorted = nullptr;     // bucket sort: the run kernel may read A's output
    uint32_t epoch = 0;
    uint32_t loc_gsize = 0;                 // the near-sorted path's granule: 1/8 of a sort chunk
    bool drop_prefill = false;              // the detection pass (mode 1) stores every packet's drop
    bool keys_from_desc = false;            // narrow + descriptors, one call: no arrival-order key array
    bool plain = false;                     // the digit pass marks plain packets (kPlainBit)
    if (small && fast && npk <= (size_t)t.tiny_max) {
        // sort and run in ONE launch of one workgroup (k_switch_tiny)
        if (!do_run) return sorted_ok();
        uint32_t win = (uint32_t)INA_SWITCH_WIN_SMALL;
        if (const int wv = t.win) win = (uint32_t)wv;
        const bool narrow = (uint64_t)st->num_slots + 1 <= (1u << 20);
#define INA_TINY(P_, T_, B_, S_) hipLaunchKernelGGL((k_switch_tiny<P_, T_, B_, S_>), dim3(1), dim3(kSmallBlock), 0, s, \
                                                   *st, pkts, pay, (uint32_t)npk, stride, actions, win, ps)
        if (ps.on) {
            if (narrow) { if (split) INA_TINY(true, uint32_t, 12, true); else INA_TINY(true, uint32_t, 12, false); }
            else { if (split) INA_TINY(true, unsigned long long, 32, true); else INA_TINY(true, unsigned long long, 32, false); }
        } else {
            if (narrow) { if (split) INA_TINY(false, uint32_t, 12, true); else INA_TINY(false, uint32_t, 12, false); }
            else { if (split) INA_TINY(false, unsigned long long, 32, true); else INA_TINY(false, unsigned long long, 32, false); }
        }
#undef INA_TINY
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch tiny launch%s", "");
        *fused_out = ps.on != 0;
        return run_ok();
    } else if (small) {
        if (!do_run) return sorted_ok();                         // this sort reads the packets
        if ((uint64_t)st->num_slots + 1 <= (1u << 20))
            hipLaunchKernelGGL((k_switch_sort_small<uint32_t, 12>), dim3(1), dim3(kSmallBlock), 0, s, pkts,
                               (uint32_t)npk, stride, st->num_slots, st->switch_id, actions, kc, vc);
        else
            hipLaunchKernelGGL((k_switch_sort_small<unsigned long long, 32>), dim3(1), dim3(kSmallBlock), 0,
                               s, pkts, (uint32_t)npk, stride, st->num_slots, st->switch_id, actions, kc, vc);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
    } else if (bucket) {
        // A: keys + each chunk sorted by the high digit (bits lb..eb-1) -> (kn, vn) and the
        // per (digit, chunk) run lengths / starts; B: each bucket gathered in chunk order and
        // sorted on its low digit -> (kc, vc)
        const int lb = sp.lbits;                           // low digit bits (0: one-digit keys)
        const uint2* dsc = reinterpret_cast<const uint2*>(desc);
        const int ah = ack_hint ? 1 : 0;
        // dense ascending runs skip the sort (run table, switch_runs_body): the register-
        // resident run kernel only (ina_set_tuning key 18 = 0 turns it off)
        const bool runs_on = fast && t.runs != 0;
        // near-sorted batches (local disorder) skip the sort and run from per-slot lists: the
        // narrow run (V <= 32) after the split chunk pass, <= kLocMaxGran granules
        // (the decision keeps PM and SM in the digit pass's count array: G <= 8,192 granules for the
        // 2,048-bin pass, <= 4,096 for the 512-bin one)
        const bool loc = fast && st->V <= kNarrowMaxV && (sp.wide || t.pre_all) && t.local != 0 &&
                         sp.nch * kGranPerChunk <= (size_t)(sp.wide ? kLocMaxGran : kLocMaxGran / 2);
        loc_gsize = (uint32_t)((size_t)kRsWaves * 64u * (size_t)sp.rounds / kGranPerChunk);
        // never 0 (fresh scratch reads as "unsorted": the safe side); a stale epoch equal to
        // this one (2^32 calls later) also only costs the full sort
        // keys of 19-22 bits (2,048-bin digits) with the register-resident run kernel: the
        // chunk pass split in two (detection, then decision + digits), so structured batches skip the digits
        const bool pre = (sp.wide || t.pre_all) && fast;
        drop_prefill = pre;
        // the detection pass's arrival-order keys are read only by the in-order narrow run and the
        // near-sorted lists; with descriptors the pass stores only the waves that found a descent
        // (a batch in slot order or of dense runs: none of its 26 MB at NGA-32 C3 size), the lists
        // read those and make the rest from the descriptors, the in-order run makes all (KeySrc).
        // A sort queued alone still writes every key (its run may come without the descriptors).
        keys_from_desc = INA_KEYS_FROM_DESC && pre && desc && phase == 0 && st->V <= kNarrowMaxV;
        // plain packets (kPlainBit): the digit pass of a narrow split-row batch reads its header rows
        // and marks them, so the sorted run reads no header row for them.  One call only (a sort
        // queued alone reads nothing but the descriptors), no PS step, and the ack hint on (both
        // hint bits outside the digits, masked out of the slot by the run)
        plain = INA_SWITCH_PLAIN && pre && split && phase == 0 && !ps.on && ack_hint && st->V <= kNarrowMaxV &&
                sp.passes * sp.bits <= 30 && st->num_slots < kPlainBit;
        if (do_sort) {
        epoch = g_sort_epoch.fetch_add(1u) + 1u;
        if (epoch == 0u) epoch = g_sort_epoch.fetch_add(1u) + 1u;
        if (pre) {
#define INA_A_DETECT(RR)                                                                              \
            hipLaunchKernelGGL((desc ? &k_sort_chunks<RR, true, 64, 1> : &k_sort_chunks<RR, false, 64, 1>),      \
                               dim3(gc), dim3(kBkThr), 0, s, pkts, dsc, npk, stride, st->num_slots,       \
                               st->switch_id, actions, sp.hbits, lb, ax.hist, ax.rst, sp.nch, kc, vc, ah, \
                               ax.unsorted, epoch, runs_on ? ax.brk_cnt : nullptr, ax.brk_ent, loc ? ax.gstat : nullptr, ax.units, 0u, \
                               keys_from_desc ? ax.kflags : nullptr, nullptr)
            if (ri == 3) INA_A_DETECT(kR3 / 4);
            else if (ri == 2) INA_A_DETECT(kR2 / 4);
            else if (ri == 1) INA_A_DETECT(kR1 / 4);
            else INA_A_DETECT(kR0 / 4);
#undef INA_A_DETECT

#define INA_A_SORT(RR)                                                                                \
            hipLaunchKernelGGL((sp.wide ? (desc ? &k_sort_chunks<RR, true, kBinsBig, 2> : &k_sort_chunks<RR, false, kBinsBig, 2>) \
                                        : (desc ? &k_sort_chunks<RR, true, kRsBins, 2> : &k_sort_chunks<RR, false, kRsBins, 2>)), \
                               dim3(gc), dim3(kBkThr), 0, s, pkts, dsc, npk, stride, st->num_slots,       \
                               st->switch_id, actions, sp.hbits, lb, ax.hist, ax.rst, sp.nch, kn, vn, ah, \
                               ax.unsorted, epoch, runs_on ? ax.brk_cnt : nullptr, ax.brk_ent, loc ? ax.gstat : nullptr, ax.units, \
                               (uint32_t)t.decide_delay * 100u, nullptr,                                  \
                               plain ? reinterpret_cast<const uint32_t*>(pkts) : nullptr)
            if (ri == 3) INA_A_SORT(kR3 / 4);
            else if (ri == 2) INA_A_SORT(kR2 / 4);
            else if (ri == 1) INA_A_SORT(kR1 / 4);
            else INA_A_SORT(kR0 / 4);
#undef INA_A_SORT
        } else {
#define INA_A_LAUNCH(RR)                                                                              \
        hipLaunchKernelGGL((sp.wide ? (desc ? &k_sort_chunks<RR, true, kBinsBig> : &k_sort_chunks<RR, false, kBinsBig>) \
                                    : (desc ? &k_sort_chunks<RR, true, kRsBins> : &k_sort_chunks<RR, false, kRsBins>)), \
                           dim3(gc), dim3(kBkThr), 0, s, pkts, dsc, npk, stride, st->num_slots,       \
                           st->switch_id, actions, sp.hbits, lb, ax.hist, ax.rst, sp.nch, kn, vn, ah,  \
                           ax.unsorted, epoch, runs_on ? ax.brk_cnt : nullptr, ax.brk_ent, loc ? ax.gstat : nullptr, ax.units, 0u, nullptr, \
                           nullptr)
        if (ri == 3) INA_A_LAUNCH(kR3 / 4);
        else if (ri == 2) INA_A_LAUNCH(kR2 / 4);
        else if (ri == 1) INA_A_LAUNCH(kR1 / 4);
        else INA_A_LAUNCH(kR0 / 4);
#undef INA_A_LAUNCH
        }
        }
        // the bucket of foreign packets only (a pool of a multiple of 2^lb slots) is left out
        // when the register-resident run kernel takes the batch (it stops before them); the
        // generic run kernel reads every position, so then it is gathered like the others
        uint32_t skip = 0xFFFFFFFFu;
        if (fast && (st->num_slots & ((1u << lb) - 1u)) == 0u) {
            skip = st->num_slots >> lb;
            nforeign = ax.nforeign;
        }
        const uint32_t CH = (uint32_t)kRsWaves * 64u * (uint32_t)sp.rounds;
        // buckets past the sentinel's (num_slots >> lb) are always empty: no block for them,
        // so at 2^17 slots 257 blocks (one per CU, one generation) instead of 512
        const unsigned gb = std::min<unsigned>(1u << sp.hbits, (st->num_slots >> lb) + 1u);
        const int tile = t.bucket_tile;
        const bool big = tile == kLcRoundsBig || (tile == 0 && npk > (size_t)gb * kBigTileAvg);
        if (do_sort)
            // the bucket pass's bins follow the low digit: 1,024 for keys of 19-21 bits (three
            // blocks per CU with the packed counts), 2,048 for 22 bits
            hipLaunchKernelGGL((sp.wide ? (lb <= 10 ? (big ? &k_sort_buckets<kLcRoundsBig, 1024> : &k_sort_buckets<kLcRounds, 1024>)
                                                    : (big ? &k_sort_buckets<kLcRoundsBig, kBinsBig> : &k_sort_buckets<kLcRounds, kBinsBig>))
                                        : (big ? &k_sort_buckets<kLcRoundsBig, kRsBins> : &k_sort_buckets<kLcRounds, kRsBins>)),
                               dim3(gb),
                               dim3(kBkThr), 0, s, kn, vn, kc, vc, ax.hist, ax.rst, (uint32_t)sp.nch, CH, lb,
                               ax.nforeign, skip, ax.unsorted, epoch, fast ? 0 : 1,
                               (runs_on && !pre) ? ax.brk_cnt : nullptr, ax.brk_ent, (uint32_t)npk, pre ? 1 : 0);
        if (do_sort && loc)
            // the near-sorted path's per-slot lists into the idle k_out (exits at once unless the
            // decision chose the path)
            hipLaunchKernelGGL(k_local_lists, dim3((unsigned)std::min<size_t>(sp.nch * kGranPerChunk / kLocU, 2048)),
                               dim3(kLlWaves * 64), 0, s,
                               KeySrc{kc, keys_from_desc ? dsc : nullptr, st->num_slots, st->switch_id, ack_hint,
                                      ax.kflags, 0u, 6u + (uint32_t)__builtin_ctz((unsigned)(sp.rounds / 4))},
                               npk, st->num_slots, ack_hint ? ~kAckBit : 0xFFFFFFFFu,
                               ax.unsorted, ax.units, loc_gsize, k_out, ax.tab);
        if (pre) {                                 // the in-order run reads the arrival-order keys
            kn = kc;
            vn = nullptr;
        }
        if (fast) unsorted = ax.unsorted;
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
    } else {
        // LSD digit passes (keys of three digits, batches beyond B's rows, or key 12 = 3):
        // keys + pass-0 histogram, then per pass a column scan and a scatter
        if (ri == 3) return set_error(INA_EINVAL, "8,192-packet chunks are the bucket sort's only%s", "");
        auto* k_keys = desc ? (ri == 0 ? &k_switch_keys<kR0, true> : ri == 1 ? &k_switch_keys<kR1, true>
                                                                    : &k_switch_keys<kR2, true>)
                            : (ri == 0 ? &k_switch_keys<kR0, false> : ri == 1 ? &k_switch_keys<kR1, false>
                                                                     : &k_switch_keys<kR2, false>);
        auto* k_hist = ri == 0 ? &k_rs_hist<kR0> : ri == 1 ? &k_rs_hist<kR1> : &k_rs_hist<kR2>;
        auto* k_sc0 = ri == 0 ? &k_rs_scatter<false, kR0>
                    : ri == 1 ? &k_rs_scatter<false, kR1> : &k_rs_scatter<false, kR2>;
        auto* k_sc1 = ri == 0 ? &k_rs_scatter<true, kR0>
                    : ri == 1 ? &k_rs_scatter<true, kR1> : &k_rs_scatter<true, kR2>;
        const unsigned gd = (nb + kRsWaves - 1) / kRsWaves;
        if (do_sort) {
        uint32_t lsd_epoch = g_sort_epoch.fetch_add(1u) + 1u;
        if (lsd_epoch == 0u) lsd_epoch = g_sort_epoch.fetch_add(1u) + 1u;
        hipLaunchKernelGGL(k_keys, dim3(gc), dim3(kRsBlock), 0, s, pkts,
                           reinterpret_cast<const uint2*>(desc), npk, stride, st->num_slots,
                           st->switch_id, k_in, actions, sp.bits, 0, ax.hist, sp.nch, ack_hint ? 1 : 0,
                           ax.unsorted, lsd_epoch);
        if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch keys launch%s", "");
        // (k_in, ids) -> (k_out, v_out) -> (k_in, v_in) -> ...
        for (int pass = 0; pass < sp.passes; ++pass) {
            const int shift = pass * sp.bits;
            if (pass > 0)
                hipLaunchKernelGGL(k_hist, dim3(gc), dim3(kRsBlock), 0, s, kc, npk, shift, sp.bits, ax.hist,
                                   sp.nch);
            hipLaunchKernelGGL(k_rs_colscan, dim3(gd), dim3(kRsBlock), 0, s, ax.hist, sp.nch, nb, ax.totals);
            if (pass == 0)
                hipLaunchKernelGGL(k_sc0, dim3(gc), dim3(kRsBlock), 0, s, kc, nullptr, kn, vn, npk, shift,
                                   sp.bits, ax.hist, ax.totals, sp.nch);
            else
                hipLaunchKernelGGL(k_sc1, dim3(gc), dim3(kRsBlock), 0, s, kc, vc, kn, vn, npk, shift,
                                   sp.bits, ax.hist, ax.totals, sp.nch);
            if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch sort launch%s", "");
            std::swap(kc, kn);
            std::swap(vc, vn);
        }
        } else {
            for (int pass = 0; pass < sp.passes; ++pass) {    // where the passes left the keys
                std::swap(kc, kn);
                std::swap(vc, vn);
            }
        }
    }
    if (!do_run) return sorted_ok();
    if (fast) {
        // a wave runs the segments that start in its window of `win` sorted positions: a
        // segment is a chain of dependent round trips, so small windows (more waves) win
        // at every size -- tools/lab/switch_lab.py, profiles/r01/lab/switch_lab_win.log:
        // 1,024 packets 52.9 -> 27.7 us (64 -> 8 positions), 819,200 packets 277 -> 266 us
        // (64 -> 16 positions, one pass of the grid)
        // V <= 32 (NGA-32, the P4 program's format): 8 packets of a segment side by side per
        // wave (run_segment_narrow); wider packets: a packet per wave instruction
        const bool narrow = st->V <= kNarrowMaxV;
        uint32_t win = npk <= 65536 ? (uint32_t)INA_SWITCH_WIN_SMALL : (uint32_t)INA_SWITCH_WIN_LARGE;
        // a narrow wave moves a whole segment per batch: a window of 64 sorted positions
        // (about 8 segments) keeps the grid at npk / 256 workgroups
        if (narrow && (INA_SWITCH_NARROW_SLOTS || npk > 65536)) win = INA_SWITCH_WIN_NARROW;   // 8 lane groups: ~8 segments
        if (const int wv = t.win) win = (uint32_t)wv;
        const size_t per_block = (size_t)win * (kSwBlock / 64);
        unsigned gr = (unsigned)std::min<size_t>((npk + per_block - 1) / per_block, INA_SWITCH_GRID);
        auto* run = split ? (ps.on ? (narrow ? &k_switch_run2<true, true, true> : &k_switch_run2<true, false, true>)
                                   : (narrow ? &k_switch_run2<false, true, true> : &k_switch_run2<false, false, true>))
                          : (ps.on ? (narrow ? &k_switch_run2<true, true, false> : &k_switch_run2<true, false, false>)
                                   : (narrow ? &k_switch_run2<false, true, false> : &k_switch_run2<false, false, false>));
        hipLaunchKernelGGL(run, dim3(gr), dim3(kSwBlock), 0, s, *st, pkts, pay, npk, stride, kc, vc, actions,
                           win, plain ? ~(kAckBit | kPlainBit) : ack_hint ? ~kAckBit : 0xFFFFFFFFu, ps, nforeign, kn, vn,
                           unsorted, k_out, ax.tab,
                           drop_prefill ? 1 : 0, keys_from_desc ? reinterpret_cast<const uint2*>(desc) : nullptr);
        *fused_out = ps.on != 0;
    } else {
        unsigned gw = (unsigned)((npk + (kSwBlock / 64) - 1) / (kSwBlock / 64));
        hipLaunchKernelGGL(k_switch_run, dim3(gw), dim3(kSwBlock), 0, s, *st, pkts, npk, stride, kc,
                           vc, actions);
    }
    if (hipGetLastError() != hipSuccess) return set_error(INA_EHIP, "switch run launch%s", "");
    return run_ok();
}

static int switch_apply_impl(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                             const ina_nga_desc_t* desc, uint8_t* actions, void* scratch,
                             uint32_t seq0, const float* local, int k, double weight_step,
                             float* out, size_t n, uint8_t* acks, size_t ack_stride,
                             ina_nga_desc_t* ack_desc, int keep_forwarded, ina_stream_t stream, int phase,
                             uint8_t* pay) {
    if (k < -126 || k > 127) return set_error(INA_EINVAL, "k out of range [-126,127]%s", "");
    if (npk == 0) return INA_OK;
    if (!local || !out) return set_error(INA_EINVAL, "null pointer%s", "");
    if (((uintptr_t)local & 15u) || ((uintptr_t)out & 15u))
        return set_error(INA_EINVAL, "local/out must be 16-byte aligned%s", "");
    if (acks && (((uintptr_t)acks & 15u) || ack_stride % 16))
        return set_error(INA_EINVAL, "ack rows must be 16-byte aligned%s", "");
    if (ack_desc && (!acks || ((uintptr_t)ack_desc & 7u)))
        return set_error(INA_EINVAL, "ack descriptors need ack rows and 8-byte alignment%s", "");
    if (!st || st->V <= 0) return set_error(INA_EINVAL, "bad switch state (V in [1,256])%s", "");
    // the PS step needs the layout ina_apply_completed_nga and the fused run kernel take
    // (16-byte aligned rows and slot registers); refuse before the switch touches its state
    // rather than after, so keep_forwarded always means what include/ina.h says
    if (st->V % 4 || st->V > 256 || stride % 16 || ((uintptr_t)pkts & 15u) || ((uintptr_t)st->regs & 15u))
        return set_error(INA_EINVAL,
                         "the PS step needs V %% 4 == 0 <= 256 and 16-byte aligned rows and registers%s", "");
    const size_t nslots = (n + (size_t)st->V - 1) / (size_t)st->V;
    PsFuse ps{local, out, n, ldexpf(1.0f, -k), (float)weight_step, seq0,
              nslots > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)nslots, acks, ack_stride, 1,
              keep_forwarded ? 1 : 0, reinterpret_cast<uint2*>(ack_desc)};
    bool fused = false;
    if (int rc = switch_process_impl(st, pkts, npk, stride, desc, actions, scratch, stream, ps, &fused, phase, pay))
        return rc;
    // the checks above admit only the layouts the register-resident run kernels take, so the
    // PS step always runs fused (ack_desc: exactly the rows the call writes, in every layout)
    if (fused || phase == INA_SWITCH_SORT) return INA_OK;         // (a sort alone: the PS step runs with the run)
    return set_error(INA_EHIP, "internal: the PS step was not fused%s", "");
}

int ina_switch(const ina_switch_state_t* st, const ina_switch_batch_t* b, const ina_switch_ps_t* ps, int phase,
               ina_stream_t stream) {
    if (!b) return set_error(INA_EINVAL, "null batch%s", "");
    if (phase != INA_SWITCH_ALL && phase != INA_SWITCH_SORT && phase != INA_SWITCH_RUN)
        return set_error(INA_EINVAL, "phase must be INA_SWITCH_ALL, _SORT or _RUN%s", "");
    const bool split = b->pay != nullptr;
    const size_t stride = split ? 16 : b->stride;
    if (ps) {
        if (split && ps->ack_stride != 16 && ps->ack_stride != 0)
            return set_error(INA_EINVAL, "split rows: the ack rows are header rows (ack_stride 16)%s", "");
        return switch_apply_impl(st, b->rows, b->npkts, stride, b->desc, b->actions, b->scratch, ps->seq0,
                                 ps->local, ps->k, ps->weight_step, ps->out, ps->n, ps->acks,
                                 split ? 16 : ps->ack_stride, ps->ack_desc, ps->keep_forwarded, stream, phase,
                                 b->pay);
    }
    PsFuse off{};
    bool fused = false;
    return switch_process_impl(st, b->rows, b->npkts, stride, b->desc, b->actions, b->scratch, stream, off, &fused,
                               phase, b->pay);
}

int ina_switch_process(const ina_switch_state_t* st, uint8_t* pkts, size_t npk, size_t stride,
                       uint8_t* actions, void* scratch, ina_stream_t stream) {
    const ina_switch_batch_t b{pkts, nullptr, npk, stride, nullptr, actions, scratch};
    return ina_switch(st, &b, nullptr, INA_SWITCH_ALL, stream);
}

int ina_switch_batch_path(const void* scratch, size_t npk, uint32_t num_slots, int* path) {
    if (!scratch || !path || npk == 0 || npk > 0x7FFFFFFFu || num_slots == 0)
        return set_error(INA_EINVAL, "bad arguments%s", "");
    const uint8_t* base = reinterpret_cast<const uint8_t*>(align_up((uintptr_t)scratch, 256));
    const SortAux ax = sort_aux(const_cast<uint8_t*>(base) + 4 * align_up(npk * 4, 256), npk, num_slots);
    uint32_t e[kLocEpoch + 1];
    // the caller's stream may be a non-blocking one: wait for the whole device first
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(e, ax.unsorted, sizeof(e), hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(INA_EHIP, "reading the control block%s", "");
    *path = e[kLocEpoch] == e[1] ? INA_PATH_LOCAL
          : e[0] != e[1]        ? INA_PATH_IN_ORDER
          : e[2] == e[1]        ? INA_PATH_RUNS
                                : INA_PATH_SORTED;
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

#if INA_STORE_CHECK
namespace ina {
unsigned long long store_violations_switch() {
    unsigned long long v = 0, z = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_store_violations), sizeof(v)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_store_violations), &z, sizeof(z)) != hipSuccess)
        return ~0ull;                                  // unreadable: report as a violation
    return v;
}
}  // namespace ina
#endif
