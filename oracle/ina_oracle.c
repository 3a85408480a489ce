/*
 * ina_oracle.c -- CPU restatement of the reference's gradient-aggregation path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the
 * cpu_baseline ("port") of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (libina.so, built from
 * distributed-training-ina_amd/csrc) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repo root, Fangjin98/distributed-training-INA).
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - C-128 packetiser  : pinned byte-for-byte by tests/golden/c128_*.bin, captured
 *                         from the reference's own communicator.cc compiled here.
 *   - NGA-32 header     : pinned by tests/golden/nga_*.bin, captured from the
 *                         reference's DataManager._send_data imported here.
 *   - PS float combine  : pinned by tests/golden/ps_aggregate_*.npz, produced by the
 *                         reference's launch.py / launch_async.py aggregate().
 *   - P4 aggregator     : the P4 program cannot run here (no Tofino toolchain);
 *                         known-answer tests are hand-derived from the P4 source.
 *   - quantiser         : float_to_int / int_to_float are ABSENT from the reference
 *                         (imported at DataManager.py:9, NGAPacket.py:5 from a module
 *                         that is not in the repo).  "Parity unpinned": the build
 *                         defines the quantiser (power-of-two scale, RNE, saturate).
 */
#include "ina_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* byte order helpers (communicator.cc:54-63 uses htonl; P4 bit<32> is BE)    */
/* ------------------------------------------------------------------------- */
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
static inline void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);  p[3] = (uint8_t)v;
}
static inline uint32_t get_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* ------------------------------------------------------------------------- */
/* a1/a2: quantise / dequantise (build-defined; reference's is missing:       */
/*        DataManager.py:9,37,168, NGAPacket.py:5,118, intent types.p4:10)    */
/* ------------------------------------------------------------------------- */
static inline float pow2f(int k) { return ldexpf(1.0f, k); }

int32_t orc_q_i32(float x, float scale) {
    if (isnan(x)) return 0;
    float y = nearbyintf(x * scale);           /* x*2^k exact; RNE to integer */
    if (y >= 2147483648.0f) return INT32_MAX;
    if (y < -2147483648.0f) return INT32_MIN;
    return (int32_t)y;
}

/* returns saturated value; *sat = 1 if clamped (or NaN) */
int16_t orc_q_i16(float x, float scale, int* sat) {
    if (isnan(x)) { *sat = 1; return 0; }
    float y = nearbyintf(x * scale);
    if (y > 32767.0f) { *sat = 1; return INT16_MAX; }
    if (y < -32768.0f) { *sat = 1; return INT16_MIN; }
    *sat = 0;
    return (int16_t)y;
}

int orc_quantize_f32_i32(const float* x, int32_t* q, size_t n, int k) {
    if (k < -126 || k > 127) return ORC_EINVAL;
    float s = pow2f(k);
    for (size_t i = 0; i < n; ++i) q[i] = orc_q_i32(x[i], s);
    return 0;
}

int orc_quantize_f32_i16_sat(const float* x, int16_t* q, size_t n, int k, int V,
                             uint8_t* ovf) {
    if (k < -126 || k > 127 || V <= 0) return ORC_EINVAL;
    float s = pow2f(k);
    size_t slots = (n + (size_t)V - 1) / (size_t)V;
    if (ovf) memset(ovf, 0, slots);
    for (size_t i = 0; i < n; ++i) {
        int sat = 0;
        q[i] = orc_q_i16(x[i], s, &sat);
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
    return 0;
}

int orc_dequantize_i32_f32(const int32_t* s, float* y, size_t n, int k) {
    if (k < -126 || k > 127) return ORC_EINVAL;
    float inv = pow2f(-k);
    for (size_t i = 0; i < n; ++i) y[i] = (float)s[i] * inv;   /* RNE cvt, exact scale */
    return 0;
}

int orc_dequantize_i16_f32(const int16_t* s, float* y, size_t n, int k) {
    if (k < -126 || k > 127) return ORC_EINVAL;
    float inv = pow2f(-k);
    for (size_t i = 0; i < n; ++i) y[i] = (float)s[i] * inv;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a10: Processor add, bulk form. processor.p4:14-24: reg = reg + value_in on */
/* bit<32> (wraps mod 2^32) summed over the W workers of one slot.            */
/* ------------------------------------------------------------------------- */
int orc_sum_reduce_i32(const int32_t* const* bufs, int W, int32_t* out, size_t n) {
    if (W <= 0) return ORC_EINVAL;
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = (uint32_t)bufs[0][i];
        for (int w = 1; w < W; ++w) acc += (uint32_t)bufs[w][i];
        out[i] = (int32_t)acc;
    }
    return 0;
}

/* int16 narrow path (config 4; overflow bit headers.p4:30): exact int32
 * accumulation, one saturation at the end, per-slot overflow flag. */
int orc_sum_reduce_i16_sat(const int16_t* const* bufs, int W, int16_t* out, size_t n,
                           int V, uint8_t* ovf) {
    if (W <= 0 || V <= 0) return ORC_EINVAL;
    size_t slots = (n + (size_t)V - 1) / (size_t)V;
    if (ovf) memset(ovf, 0, slots);
    for (size_t i = 0; i < n; ++i) {
        int32_t acc = 0;
        for (int w = 0; w < W; ++w) acc += bufs[w][i];
        int16_t r;
        int sat = 0;
        if (acc > INT16_MAX) { r = INT16_MAX; sat = 1; }
        else if (acc < INT16_MIN) { r = INT16_MIN; sat = 1; }
        else r = (int16_t)acc;
        out[i] = r;
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
    return 0;
}

/* fused: W fp32 worker buffers -> quantise -> int32 wrapping sum */
int orc_quantize_reduce_f32_i32(const float* const* bufs, int W, int32_t* out, size_t n,
                                int k) {
    if (W <= 0 || k < -126 || k > 127) return ORC_EINVAL;
    float s = pow2f(k);
    for (size_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (int w = 0; w < W; ++w) acc += (uint32_t)orc_q_i32(bufs[w][i], s);
        out[i] = (int32_t)acc;
    }
    return 0;
}

/* fused int16: each worker's value saturates to int16 at quantisation (the
 * wire width), the sum is accumulated exactly and saturated once; a slot's
 * overflow flag is set when either saturation happened in that slot. */
int orc_quantize_reduce_f32_i16_sat(const float* const* bufs, int W, int16_t* out,
                                    size_t n, int k, int V, uint8_t* ovf) {
    if (W <= 0 || V <= 0 || k < -126 || k > 127) return ORC_EINVAL;
    float s = pow2f(k);
    size_t slots = (n + (size_t)V - 1) / (size_t)V;
    if (ovf) memset(ovf, 0, slots);
    for (size_t i = 0; i < n; ++i) {
        int32_t acc = 0;
        int any = 0;
        for (int w = 0; w < W; ++w) {
            int sat = 0;
            acc += orc_q_i16(bufs[w][i], s, &sat);
            any |= sat;
        }
        int16_t r;
        if (acc > INT16_MAX) { r = INT16_MAX; any = 1; }
        else if (acc < INT16_MIN) { r = INT16_MIN; any = 1; }
        else r = (int16_t)acc;
        out[i] = r;
        if (any && ovf) ovf[i / (size_t)V] = 1;
    }
    return 0;
}

/* int16 wire under sharding (build-defined; include/ina.h): a rank
 * sends q16 widened to int32 plus its saturation bit at 2^22, the ranks' wires are
 * summed in int32, and the owner decodes sum q16 and the saturation count.  Written
 * here with 64-bit floor division (the device uses shifts), so the check is not a copy
 * of the kernel.  End to end it must equal orc_quantize_reduce_f32_i16_sat. */
int orc_quantize_f32_i16_wire(const float* x, int32_t* wire, size_t n, int k) {
    if (k < -126 || k > 127) return ORC_EINVAL;
    float s = pow2f(k);
    for (size_t i = 0; i < n; ++i) {
        int sat = 0;
        int32_t v = orc_q_i16(x[i], s, &sat);
        wire[i] = (int32_t)((int64_t)v + (int64_t)sat * (1 << 22));
    }
    return 0;
}

int orc_i16_wire_finish(const int32_t* wsum, size_t n, int k, int V, int16_t* out16, float* y,
                        uint8_t* ovf) {
    if (k < -126 || k > 127 || V <= 0) return ORC_EINVAL;
    float inv = pow2f(-k);
    size_t slots = (n + (size_t)V - 1) / (size_t)V;
    if (ovf) memset(ovf, 0, slots);
    for (size_t i = 0; i < n; ++i) {
        int64_t t = (int64_t)wsum[i] + (1 << 21);
        int64_t c = t >= 0 ? t / (1 << 22) : -((-t + (1 << 22) - 1) / (1 << 22));   /* floor */
        int64_t v = (int64_t)wsum[i] - c * (1 << 22);
        int sat = c != 0;
        int16_t r;
        if (v > INT16_MAX) { r = INT16_MAX; sat = 1; }
        else if (v < INT16_MIN) { r = INT16_MIN; sat = 1; }
        else r = (int16_t)v;
        if (out16) out16[i] = r;
        if (y) y[i] = (float)r * inv;
        if (sat && ovf) ovf[i / (size_t)V] = 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a13: PS float combine, launch.py:42-52 (and launch_async.py:42-57):         */
/*   local += (w * step) * sum([p_w - local for w])                            */
/* torch evaluates: acc = 0 + d_0 (python sum starts at int 0), acc += d_i     */
/* in list order, t = acc * float(w*step), local + t -- every op fp32 RNE.     */
/* ------------------------------------------------------------------------- */
int orc_ps_combine_f32(const float* local, const float* const* paras, int W,
                       double weight_step, float* out, size_t n) {
    if (W <= 0) return ORC_EINVAL;
    float ws = (float)weight_step;
    for (size_t i = 0; i < n; ++i) {
        float l = local[i];
        float acc = 0.0f;
        for (int w = 0; w < W; ++w) {
            float d = paras[w][i] - l;   /* built with -ffp-contract=off */
            acc = acc + d;
        }
        float t = acc * ws;
        out[i] = l + t;
    }
    return 0;
}

/* INA form of the same update (build-defined: the reference never wires its
 * quantiser into aggregate()): workers quantise their deltas d_w = p_w - local,
 * the switch sums the integers mod 2^32, the PS dequantises and applies
 * out = local + float(w*step) * ((float)sum * 2^-k). */
int orc_ps_combine_ina_f32(const float* local, const float* const* paras, int W, int k,
                           double weight_step, float* out, size_t n) {
    if (W <= 0 || k < -126 || k > 127) return ORC_EINVAL;
    float s = pow2f(k), inv = pow2f(-k), ws = (float)weight_step;
    for (size_t i = 0; i < n; ++i) {
        float l = local[i];
        uint32_t acc = 0;
        for (int w = 0; w < W; ++w) acc += (uint32_t)orc_q_i32(paras[w][i] - l, s);
        float y = (float)(int32_t)acc * inv;
        float t = y * ws;
        out[i] = l + t;
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a3: NGA-V packetiser.  DataManager._send_data (DataManager.py:111-165):     */
/*   header struct.pack('!IbbIbI', worker_id, degree, 0, seq%16384, switch_id, */
/*   seq) (122-130) == ngaa_h (headers.p4:27-38) 15 bytes; payload V words     */
/*   (131-133, BE as P4 bit<32>); tail zero-padded (135-153).                  */
/* ------------------------------------------------------------------------- */
void orc_nga_write_header(uint8_t* p, uint32_t bitmap, uint8_t count, uint8_t flags,
                          uint32_t index, uint8_t switch_id, uint32_t frag_id) {
    put_be32(p + 0, bitmap);
    p[4] = count;
    p[5] = flags;
    put_be32(p + 6, index);
    p[10] = switch_id;
    put_be32(p + 11, frag_id);
}

int orc_pack_nga(const int32_t* vals, size_t n, const orc_nga_params_t* prm,
                 const uint8_t* ovf, uint8_t* pkts, size_t stride) {
    int V = prm->V;
    if (V <= 0 || prm->num_slots == 0 || stride < (size_t)ORC_NGA_HDR + 4u * (size_t)V)
        return ORC_EINVAL;
    size_t np = (n + (size_t)V - 1) / (size_t)V;
    for (size_t p = 0; p < np; ++p) {
        uint8_t* pk = pkts + p * stride;
        uint32_t seq = prm->seq0 + (uint32_t)p;
        uint8_t flags = prm->flags;
        if (ovf && ovf[p]) flags |= ORC_FLAG_OVERFLOW;
        orc_nga_write_header(pk, prm->bitmap, prm->count, flags, seq % prm->num_slots,
                             prm->switch_id, seq);
        for (int j = 0; j < V; ++j) {
            size_t i = p * (size_t)V + (size_t)j;
            uint32_t v = i < n ? (uint32_t)vals[i] : 0u;   /* tail pad: 135-153 */
            put_be32(pk + ORC_NGA_HDR + 4 * j, v);
        }
        for (size_t b = ORC_NGA_HDR + 4u * (size_t)V; b < stride; ++b) pk[b] = 0;
    }
    return 0;
}

/* a12: PS-side parse (NGAPacket.py:62-143).  Follows headers.p4 (payload at
 * offset 15 after IP, big-endian), not the ctypes struct's padded offset 36. */
int orc_unpack_nga(const uint8_t* pkts, size_t np, int V, size_t stride,
                   orc_nga_fields_t* f, int32_t* vals) {
    if (V <= 0 || stride < (size_t)ORC_NGA_HDR + 4u * (size_t)V) return ORC_EINVAL;
    for (size_t p = 0; p < np; ++p) {
        const uint8_t* pk = pkts + p * stride;
        if (f) {
            if (f->bitmap) f->bitmap[p] = get_be32(pk + 0);
            if (f->count) f->count[p] = pk[4];
            if (f->flags) f->flags[p] = pk[5];
            if (f->index) f->index[p] = get_be32(pk + 6);
            if (f->switch_id) f->switch_id[p] = pk[10];
            if (f->frag_id) f->frag_id[p] = get_be32(pk + 11);
        }
        if (vals)
            for (int j = 0; j < V; ++j)
                vals[p * (size_t)V + (size_t)j] = (int32_t)get_be32(pk + ORC_NGA_HDR + 4 * j);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a5: C-128 packetiser, send_gradients (communicator.cc:3-47,                 */
/*     communicator.h:18-27): packet_t = {htonl(1<<(worker_id-1)),             */
/*     htonl(aggregator_index), htonl(tensor_index+i), htonl(g[i*128+j])}.     */
/*     The shift is UB for worker_id 0 in C; x86 masks the count to 5 bits     */
/*     (measured 0x80000000), restated explicitly here.                        */
/* ------------------------------------------------------------------------- */
uint32_t orc_c128_bitmap(int worker_id) {
    return (uint32_t)1u << ((unsigned)(worker_id - 1) & 31u);
}

int orc_pack_c128(const uint32_t* g, int packet_num, int worker_id,
                  uint32_t aggregator_index, int tensor_index, uint8_t* out) {
    if (packet_num < 0) return ORC_EINVAL;
    uint32_t bm = orc_c128_bitmap(worker_id);
    for (int i = 0; i < packet_num; ++i) {
        uint32_t* pk = (uint32_t*)(out + (size_t)i * ORC_C128_BYTES);
        uint32_t hdr[3] = {bswap32(bm), bswap32(aggregator_index),
                           bswap32((uint32_t)(tensor_index + i))};
        memcpy(pk, hdr, sizeof hdr);
        /* memcpy 512 B then htonl x128 (communicator.cc:57-63) */
        uint32_t body[ORC_C128_V];
        memcpy(body, g + (size_t)i * ORC_C128_V, sizeof body);
        for (int j = 0; j < ORC_C128_V; ++j) body[j] = bswap32(body[j]);
        memcpy(pk + 3, body, sizeof body);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a8-a11: the stateful P4 aggregator, one packet at a time (ngaa.p4:120-196)  */
/* ------------------------------------------------------------------------- */
int orc_switch_init(orc_switch_t* sw, uint32_t num_slots, int V, int switch_id) {
    if (num_slots == 0 || V <= 0) return ORC_EINVAL;
    sw->num_slots = num_slots;
    sw->V = V;
    sw->switch_id = switch_id;
    sw->count = (uint8_t*)calloc(num_slots, 1);                     /* ngaa.p4:64 (init 0) */
    sw->frag = (uint32_t*)calloc(num_slots, sizeof(uint32_t));       /* fragcheck.p4:12 */
    sw->regs = (uint32_t*)calloc((size_t)num_slots * (size_t)V, sizeof(uint32_t)); /* processor.p4:12 */
    if (!sw->count || !sw->frag || !sw->regs) { orc_switch_free(sw); return ORC_ENOMEM; }
    return 0;
}

void orc_switch_free(orc_switch_t* sw) {
    free(sw->count); free(sw->frag); free(sw->regs);
    sw->count = NULL; sw->frag = NULL; sw->regs = NULL;
}

/* Processes one NGA packet in place (header flags / payload rewritten exactly
 * as the switch's deparser would emit them) and returns the forwarding action. */
int orc_switch_packet(orc_switch_t* sw, uint8_t* pk) {
    /* switch_check (ngaa.p4:27-37,122): exact match on switch_id -> set_agg */
    if (sw->switch_id < 0 || pk[10] != (uint8_t)sw->switch_id) return ORC_ACT_FWD_OTHER;
    uint32_t idx = get_be32(pk + 6) % sw->num_slots;     /* ig_md.index (125) */
    int is_ack = (pk[5] >> 6) & 1;                       /* headers.p4:31 */
    uint32_t frag_in = get_be32(pk + 11);
    /* frag_check (fragcheck.p4:14-57, applied ngaa.p4:128) */
    uint32_t frag_out;
    if (is_ack) {                                        /* reset_id (26-31) */
        sw->frag[idx] = 0;
        frag_out = frag_in;
    } else {                                             /* write_read_id (14-24) */
        if (sw->frag[idx] == 0) sw->frag[idx] = frag_in;
        frag_out = sw->frag[idx];
    }
    if (is_ack) return ORC_ACT_FWD_ACK;                  /* ngaa.p4:130-132 */
    if (frag_out != frag_in) {                           /* collision (177-181) */
        pk[5] |= ORC_FLAG_COLLISION;
        return ORC_ACT_FWD_COLLISION;
    }
    /* read_add_count (ngaa.p4:66-78) on bit<8> */
    uint8_t c = (uint8_t)(sw->count[idx] + 1);
    if (c == pk[4]) c = 0;
    sw->count[idx] = c;
    /* Processor x V (processor.p4:14-24) */
    uint32_t* reg = sw->regs + (size_t)idx * (size_t)sw->V;
    for (int j = 0; j < sw->V; ++j) {
        uint8_t* q = pk + ORC_NGA_HDR + 4 * j;
        uint32_t v = get_be32(q);
        if (c == 1) reg[j] = v;
        else reg[j] = reg[j] + v;
        put_be32(q, reg[j]);
    }
    return c == 0 ? ORC_ACT_FWD_AGG : ORC_ACT_DROP;      /* ngaa.p4:170-175 */
}

/* ------------------------------------------------------------------------- */
/* CPU baseline: the reference's CPU packetise + aggregate path, end to end.   */
/* Per slot and worker: build the packet the way communicator.cc:23-37 does    */
/* (header + memcpy + htonl) into a per-packet buffer that stands in for the   */
/* sendto() sink, run it through the P4 aggregator restated above; the PS      */
/* unpacks the completed packet (ntohl) and acks the slot (fragcheck.p4:26).   */
/* Threads split slots floor(S/P) each, remainder to the last                  */
/* (communicator.py:133-157); each thread drives its own switch pipe.          */
/* ------------------------------------------------------------------------- */
typedef struct {
    const int32_t* const* bufs;
    int W;
    size_t n;
    int V;
    size_t slot_lo, slot_hi;
    int32_t* out;
    uint32_t num_slots;
    int rc;
} cpu_job_t;

static void* cpu_job(void* arg) {
    cpu_job_t* jb = (cpu_job_t*)arg;
    int V = jb->V;
    orc_switch_t sw;
    jb->rc = orc_switch_init(&sw, jb->num_slots, V, 1);
    if (jb->rc) return NULL;
    size_t plen = (size_t)ORC_NGA_HDR + 4u * (size_t)V;
    uint8_t* pk = (uint8_t*)malloc(plen);
    uint32_t* body = (uint32_t*)malloc(4u * (size_t)V);
    for (size_t s = jb->slot_lo; s < jb->slot_hi; ++s) {
        size_t base = s * (size_t)V;
        size_t cnt = jb->n - base < (size_t)V ? jb->n - base : (size_t)V;
        uint32_t seq = (uint32_t)s + 1u;        /* send_data starts at 1 (DataManager.py:106) */
        for (int w = 0; w < jb->W; ++w) {
            orc_nga_write_header(pk, (uint32_t)(w + 1), (uint8_t)jb->W, 0,
                                 seq % jb->num_slots, 1, seq);
            memcpy(body, jb->bufs[w] + base, cnt * 4u);
            if (cnt < (size_t)V) memset(body + cnt, 0, ((size_t)V - cnt) * 4u);
            for (int j = 0; j < V; ++j) body[j] = bswap32(body[j]);
            memcpy(pk + ORC_NGA_HDR, body, 4u * (size_t)V);
            int act = orc_switch_packet(&sw, pk);
            if (act == ORC_ACT_FWD_AGG) {
                for (size_t j = 0; j < cnt; ++j)
                    jb->out[base + j] = (int32_t)get_be32(pk + ORC_NGA_HDR + 4 * j);
                pk[5] = ORC_FLAG_ACK;            /* PS ack clears the slot */
                orc_switch_packet(&sw, pk);
            } else if (act != ORC_ACT_DROP) {
                jb->rc = ORC_ESTATE;
            }
        }
    }
    free(body);
    free(pk);
    orc_switch_free(&sw);
    return NULL;
}

int orc_cpu_packetise_aggregate(const int32_t* const* bufs, int W, size_t n, int V,
                                int threads, int32_t* out, double* seconds) {
    if (W <= 0 || W > 255 || V <= 0 || threads <= 0) return ORC_EINVAL;
    size_t slots = (n + (size_t)V - 1) / (size_t)V;
    size_t per = slots / (size_t)threads, rem = slots % (size_t)threads;
    cpu_job_t* jobs = (cpu_job_t*)calloc((size_t)threads, sizeof(cpu_job_t));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    size_t lo = 0;
    for (int t = 0; t < threads; ++t) {
        size_t cnt = per + (t == threads - 1 ? rem : 0);
        jobs[t] = (cpu_job_t){bufs, W, n, V, lo, lo + cnt, out, ORC_NUM_REGISTER, 0};
        lo += cnt;
        if (threads == 1) cpu_job(&jobs[t]);
        else pthread_create(&tids[t], NULL, cpu_job, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    int rc = 0;
    for (int t = 0; t < threads; ++t) if (jobs[t].rc) rc = jobs[t].rc;
    free(jobs);
    free(tids);
    return rc;
}

/* linear checksum mod 2^32 used by full-size property tests:
 * c(x) = sum_i x_i * (2i+1) mod 2^32, so c(sum_w x_w) = sum_w c(x_w). */
uint32_t orc_checksum_i32(const int32_t* x, size_t n) {
    uint32_t acc = 0;
    for (size_t i = 0; i < n; ++i) acc += (uint32_t)x[i] * (uint32_t)(2u * (uint32_t)i + 1u);
    return acc;
}

/* batch form of orc_switch_packet: packets in arrival order, in place */
int orc_switch_run(orc_switch_t* sw, uint8_t* pkts, size_t np, size_t stride, uint8_t* actions) {
    for (size_t p = 0; p < np; ++p) {
        int a = orc_switch_packet(sw, pkts + p * stride);
        if (actions) actions[p] = (uint8_t)a;
    }
    return 0;
}

/* ipRoute (ngaa.p4:39-61): every packet the ingress forwards -- aggregation done
 * (170-172), ack (130-131), collision (177-180), other switch (184-186) -- is
 * matched exactly on hdr.ipv4.dst_addr; ipv4_forward sets the egress port (46-51),
 * a drop entry or a table miss (default_action = drop, 60) drops it, NoAction
 * leaves the port unset.  Ingress drops (175) never reach the table. */
void orc_route_ipv4(const uint8_t* actions, const uint32_t* dst_ip, uint32_t dst_default,
                    size_t np, const uint32_t* keys, const int32_t* ports, int nent,
                    int32_t* egress) {
    for (size_t p = 0; p < np; ++p) {
        int32_t port = ORC_PORT_DROP;
        if (actions[p] != ORC_ACT_DROP) {
            uint32_t d = dst_ip ? dst_ip[p] : dst_default;
            for (int i = 0; i < nent; ++i)
                if (keys[i] == d) { port = ports[i]; break; }
        }
        egress[p] = port;
    }
}
