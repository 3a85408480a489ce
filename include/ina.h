/*
 * ina.h -- C ABI of libina.so, the MI355X-native gradient-aggregation path.
 *
 * Drop-in boundary for the reference Fangjin98/distributed-training-INA:
 *   - the in-switch aggregator (src/p4/p4src/ngaa.p4, processor.p4, fragcheck.p4)
 *     becomes device kernels (sum-reduce, packet-stream switch);
 *   - the worker-side quantise/packetise code (src/common/DataManager.py,
 *     communicator.{h,cc,py}, NGAPacket.py) becomes device quantise/pack/unpack;
 *   - the legacy C symbol send_gradients (communicator.h:27) keeps its exact
 *     signature so the reference's ctypes loader (communicator.py:15-24) binds it.
 *
 * Conventions (all ina_* entry points):
 *   - plain pointers and sizes; every data pointer is a DEVICE pointer (hipMalloc /
 *     torch CUDA tensor) owned by the caller, borrowed for the call;
 *   - arrays of worker buffers (`bufs`) are HOST arrays of W device pointers; the
 *     array itself is copied into the kernel arguments, so it may live on the stack;
 *   - `stream` is a hipStream_t (NULL = the legacy default stream); device calls are
 *     asynchronous on that stream and never synchronise, allocate or free (the host
 *     paths -- send_gradients, ina_*_fd, ina_sum_reduce_host_i32 -- are synchronous);
 *   - return 0 on success, a negative INA_E* code otherwise (no exit(), unlike
 *     communicator.cc:11-12,38-39); ina_last_error_string() describes the last error.
 * Vector fast paths need 16-byte aligned pointers; other alignments take a slower
 * scalar path with identical results.
 */
#ifndef INA_H
#define INA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INA_OK 0
#define INA_EINVAL (-1)   /* bad argument */
#define INA_EHIP (-2)     /* HIP runtime / launch error */
#define INA_ESOCK (-3)    /* socket error (host send path) */
#define INA_ENOMEM (-4)

#define INA_MAX_WORKERS 64      /* W per launch */
#define INA_NGA_HDR_BYTES 15    /* ngaa_h, headers.p4:27-38 */
#define INA_NUM_REGISTER 16384u /* aggregator slots, config.p4:5 */
#define INA_C128_VALUES 128     /* TENSOR_NUM, communicator.h:18 */
#define INA_C128_BYTES 524      /* sizeof(packet_t), communicator.h:20-25 */

/* ngaa_h flag byte: overflow|is_ack|collision|resend|timestamp[3:0] (headers.p4:30-34) */
#define INA_FLAG_OVERFLOW 0x80u
#define INA_FLAG_ACK 0x40u
#define INA_FLAG_COLLISION 0x20u
#define INA_FLAG_RESEND 0x10u

/* forwarding decision per packet of the switch (ngaa.p4:120-196) */
#define INA_ACT_DROP 0
#define INA_ACT_FWD_AGG 1        /* aggregation complete: payload = slot sum */
#define INA_ACT_FWD_COLLISION 2  /* frag mismatch: collision=1, payload untouched */
#define INA_ACT_FWD_ACK 3        /* PS ack: frag register cleared */
#define INA_ACT_FWD_OTHER 4      /* switch_id not ours */

typedef void* ina_stream_t; /* hipStream_t */

/* "ina-mi355x 0.2 (gfx950)".  0.2 broke the 0.1 ABI: the switch is the one struct-taking call
 * ina_switch (+ ina_switch_process); 0.1's ina_switch_process_desc / _apply / _apply_desc /
 * _apply_ackdesc / _split / _apply_split, ina_switch_sort_desc and ina_switch_run_sorted* are
 * gone ("ABI 0.2"). */
const char* ina_version(void);
const char* ina_last_error_string(void);

/* Launch-geometry knobs (process-wide; results never change, only speed; every switch batch
 * reads the switch keys once, and a run alone follows what its sort recorded).  Keys:
 * 0 elementwise grid cap, 1 reduce chunks per worker per thread (0 = per-W auto, 1/2/4), 2 reduce
 * non-temporal loads/stores (0/1), 3 reduce grid (0 = 64*W rule), 7 host-ingest H2D streams
 * (1/2), 8 16-byte chunks per flat packet-kernel launch, 9 largest switch batch for the
 * one-workgroup sort (0 never, 1 default 768, 2..2048), 11 switch lane-parallel path for PS
 * acks alone in their slot's segment (0/1), 12 switch slot sort (0 auto = chunk + bucket sort
 * for keys of one or two digits, else the LSD digit passes; 3 the digit passes for every
 * batch), 13 slot-sort chunk rounds per wave (0 auto, 4, 8, 16), 15 largest switch batch
 * sorted and run in ONE launch of one workgroup (0 = off, <= 2048; it applies only to batches
 * that also take key 9's one-workgroup path, so it is capped by key 9's threshold), 16 host
 * reduce on pinned device-mapped buffers in place over PCIe (1, default) or through the
 * chunked copy pipeline (0), 17 the slot sort's bucket tile in 64-item rounds per wave (0
 * auto: 8 when the average bucket exceeds 3,584 packets, else 4; or 4, 8), 18 switch batches
 * made of at most 64 runs of consecutive slots (worker-major arrival, PS acks in front) skip
 * the slot sort and run from a table of the runs (1, default; 0 = always sort), 19 the slot
 * sort's first pass split into detection + decision + digits for every key width (1, default:
 * structured batches then skip the digits) or only for keys of 19-22 bits (0), 20 near-sorted
 * batches (V <= 32, local disorder) skip the sort and run from per-slot lists (1, default; 0 =
 * sort), 21 (tests) microseconds the near-sorted decision waits before deciding, 0..100000
 * (0, default): the other blocks' bounded wait for it then runs out and they sort their chunks
 * anyway -- results unchanged.  (Keys 4, 5, 6, 10 and 14, grid-cap sweeps, exist in lab builds
 * only.)
 * Returns INA_EINVAL for an unknown key or value.                                 */
int ina_set_tuning(int key, int value);

/* ---- quantise / dequantise ---------------------------------------------------
 * Replaces float_to_int / int_to_float, imported at DataManager.py:9 and
 * NGAPacket.py:5 (used DataManager.py:37,168, NGAPacket.py:118) but absent from
 * the reference repo.  Build-defined: q = sat(round_half_even(x * 2^k)), NaN -> 0,
 * k in [-126, 127]; dequantise y = (float)q * 2^-k (exact scaling).            */
int ina_quantize_f32_i32(const float* x, int32_t* q, size_t n, int k, ina_stream_t stream);
/* int16 saturating (config 4): overflow_per_slot[s] = 1 iff an element of slot s
 * (V consecutive values) saturated or was NaN, else 0 (every slot written). May be NULL. */
int ina_quantize_f32_i16_sat(const float* x, int16_t* q, size_t n, int k, int V,
                             uint8_t* overflow_per_slot, ina_stream_t stream);
int ina_dequantize_i32_f32(const int32_t* s, float* y, size_t n, int k, ina_stream_t stream);
int ina_dequantize_i16_f32(const int16_t* s, float* y, size_t n, int k, ina_stream_t stream);

/* Dynamic scale (build-defined, like the quantiser): *out_dev (device float) =
 * max_i |x[i] - base[i]| (base may be NULL; NaN ignored, as the quantiser maps it to 0).
 * ina_scale_for turns the max over all W workers into the largest k in [-126, 127] with
 * W * (absmax * 2^k + 1/2) <= 2^(bits-1) - 1, so neither a worker value nor the W-way
 * sum saturates (bits = 32, or 16 for the int16 wire); absmax 0 gives 127.  *k_out gets
 * k; INA_EINVAL for absmax negative, NaN or infinite, W < 1, or W too large for the width. */
int ina_absmax_f32(const float* x, const float* base, size_t n, float* out_dev, ina_stream_t stream);
/* The same over W (1..64) worker buckets in ONE pass: *out_dev = max_w,i |xs[w][i] - base[i]|
 * (each base chunk read once for all W workers) -- what ina_scale_for takes for W workers. */
int ina_absmax_multi_f32(const float* const* xs, int W, const float* base, size_t n, float* out_dev,
                         ina_stream_t stream);
int ina_scale_for(float absmax, int W, int bits, int* k_out);

/* ---- the aggregator ------------------------------------------------------------
 * Replaces the switch's per-slot Processor add (processor.p4:14-24, x32 at
 * ngaa.p4:87-168): out[i] = sum_w bufs[w][i] mod 2^32, bit-identical to the
 * switch for any arrival order.  1 <= W <= INA_MAX_WORKERS.  out may alias bufs[0]. */
int ina_sum_reduce_i32(const int32_t* const* bufs, int W, int32_t* out, size_t n,
                       ina_stream_t stream);
/* int16 narrow path: exact int32 accumulation, one saturation to int16; overflow
 * flag per slot of V values as above. */
int ina_sum_reduce_i16_sat(const int16_t* const* bufs, int W, int16_t* out, size_t n, int V,
                           uint8_t* overflow_per_slot, ina_stream_t stream);
/* fused quantise + reduce from W fp32 worker buffers (configs 2 and 4) */
int ina_quantize_reduce_f32_i32(const float* const* bufs, int W, int32_t* out, size_t n, int k,
                                ina_stream_t stream);
int ina_quantize_reduce_f32_i16_sat(const float* const* bufs, int W, int16_t* out, size_t n,
                                    int k, int V, uint8_t* overflow_per_slot,
                                    ina_stream_t stream);

/* ---- int16 wire under slot-range sharding (config-4 semantics across GPUs)
 * Saturation is not associative, so sharded ranks never reduce int16 through the
 * collective.  Each rank widens its int16-saturated quantisation (the quantiser of
 * ina_quantize_f32_i16_sat) into an int32 wire word
 *     wire[i] = q16(x[i]) + (sat_i << INA_I16_WIRE_SHIFT)     (sat_i: clamped or NaN)
 * and the wires are summed with an ordinary int32 SUM (RCCL reduce-scatter, any order).
 * For <= INA_I16_WIRE_MAX_RANKS ranks the low 22 bits hold sum q16 exactly and the high
 * bits count the ranks that saturated.  ina_i16_wire_finish decodes a summed shard:
 * out16[i] = sat16(sum q16), y[i] = out16[i] * 2^-k, overflow_per_slot[s] = 1 iff a rank
 * saturated an element of slot s (V values) or its sum saturated (the ngaa_h overflow
 * bit, headers.p4:30) -- bit-identical to ina_quantize_reduce_f32_i16_sat over the same
 * buckets.  out16, y, overflow_per_slot may each be NULL; every slot flag is written.  */
#define INA_I16_WIRE_SHIFT 22
#define INA_I16_WIRE_MAX_RANKS 64
int ina_quantize_f32_i16_wire(const float* x, int32_t* wire, size_t n, int k, ina_stream_t stream);
int ina_i16_wire_finish(const int32_t* wire_sum, size_t n, int k, int V, int16_t* out16, float* y,
                        uint8_t* overflow_per_slot, ina_stream_t stream);

/* ---- PS combine ------------------------------------------------------------------
 * launch.py:42-52 / launch_async.py:42-57 aggregate(), fused, bit-exact to the
 * torch fp32 sequence: out = local + float(weight_step) * (0 + sum_w (paras[w] - local)).
 * out may alias local. */
int ina_ps_combine_f32(const float* local, const float* const* paras, int W, double weight_step,
                       float* out, size_t n, ina_stream_t stream);
/* INA form of the same update: out = local + float(weight_step) * dequant(sum_int) */
int ina_ps_apply_i32(const float* local, const int32_t* sum_int, int k, double weight_step,
                     float* out, size_t n, ina_stream_t stream);

/* INA-semantics update in one pass (what the switch path computes end to end):
 * out = local + float(weight_step) * ((float)(sum_w q(paras[w] - local)) * 2^-k),
 * q = the quantiser above, integer sum mod 2^32. */
int ina_ps_combine_ina_f32(const float* local, const float* const* paras, int W, int k,
                           double weight_step, float* out, size_t n, ina_stream_t stream);

/* ---- packets ------------------------------------------------------------------- */
typedef struct ina_nga_params {
    uint32_t bitmap;    /* header word 0; DataManager passes worker_id raw (DataManager.py:124) */
    uint8_t count;      /* aggregation degree (ngaa_h.count) */
    uint8_t flags;      /* flag byte; INA_FLAG_OVERFLOW is OR-ed per slot from overflow_per_slot */
    uint8_t switch_id;
    uint8_t pad;
    uint32_t seq0;      /* packet p: frag_id = seq0 + p, index = (seq0 + p) % num_slots */
    uint32_t num_slots; /* INA_NUM_REGISTER (DataManager.py:119 uses 16384) */
    int32_t V;          /* payload words per packet (32 = the P4 program; 128, 256, ...) */
} ina_nga_params_t;

typedef struct ina_nga_fields { /* SoA header fields; any pointer may be NULL */
    uint32_t* bitmap;
    uint8_t* count;
    uint8_t* flags;
    uint32_t* index;
    uint8_t* switch_id;
    uint32_t* frag_id;
} ina_nga_fields_t;

/* NGA-V pack (DataManager._send_data, DataManager.py:111-165 / headers.p4:27-80):
 * ceil(n/V) packets at `stride` bytes (>= 15 + 4V): 15-byte big-endian header,
 * V big-endian 32-bit words, zero-padded tail.  stride % 16 == 0 with 16-byte
 * aligned buffers takes the vector path (the recommended layout; each packet is a
 * sendmmsg iovec of 15 + 4V bytes).  overflow_per_slot may be NULL. */
int ina_pack_nga(const int32_t* vals, size_t n, const ina_nga_params_t* prm,
                 const uint8_t* overflow_per_slot, uint8_t* pkts, size_t stride,
                 ina_stream_t stream);
/* Fused worker side: quantise fp32 gradients (x - base when base != NULL: the
 * worker's delta against the global parameters) and packetise in one pass, with
 * exactly the bytes of ina_quantize_f32_i32 (+ fp32 subtraction) then ina_pack_nga. */
int ina_quantize_pack_nga(const float* x, const float* base, size_t n, int k,
                          const ina_nga_params_t* prm, uint8_t* pkts, size_t stride,
                          ina_stream_t stream);
/* Packet descriptors: desc[p] holds bytes 4..11 of packet p's NGA header (count, flags,
 * index, switch_id and frag_id's first byte) in wire order, byte 4 lowest -- all the
 * fields the switch reads to order a batch by slot (ngaa.p4:27-37 switch_check,
 * headers.p4:27-38).  They play the part of a NIC's receive descriptors: the producer of
 * the packets hands them over beside the payload, so the switch sorts a batch from 8 bytes
 * per packet instead of fetching one 128-byte line of every packet's header
 * (ina_switch, batch.desc).  The pack entry points write them as they write each header
 * (desc may be NULL); ina_nga_descriptors gathers them from packets that arrive without.
 * desc: device memory, 8-byte aligned, npkts entries. */
typedef uint64_t ina_nga_desc_t;
int ina_pack_nga_desc(const int32_t* vals, size_t n, const ina_nga_params_t* prm,
                      const uint8_t* overflow_per_slot, uint8_t* pkts, size_t stride,
                      ina_nga_desc_t* desc, ina_stream_t stream);
int ina_quantize_pack_nga_desc(const float* x, const float* base, size_t n, int k,
                               const ina_nga_params_t* prm, uint8_t* pkts, size_t stride,
                               ina_nga_desc_t* desc, ina_stream_t stream);
int ina_nga_descriptors(const uint8_t* pkts, size_t npkts, size_t stride, ina_nga_desc_t* desc,
                        ina_stream_t stream);
/* Descriptors from the header parameters alone (nothing read): W workers x npkts packets,
 * desc[w][p] = what the pack entry points write for packet p of worker w (prm[w]'s count,
 * flags, switch_id, sequence; the overflow bit is not known without the values).  desc is a
 * host array of W device pointers; every prm[w] has the same num_slots. */
int ina_nga_make_descriptors(const ina_nga_params_t* prm, int W, size_t npkts,
                             ina_nga_desc_t* const* desc, ina_stream_t stream);
/* W workers' fused quantise + pack in one launch (a GPU hosting a group of the job's
 * workers): worker w's x[w] - base (base shared, may be NULL) into pkts[w] with header
 * prm[w] and descriptors desc[w] (desc itself may be NULL) -- exactly the bytes of W calls
 * of ina_quantize_pack_nga_desc (DataManager.py:37 + 111-165 per worker), with the base
 * read once for every 8 workers.  Every prm[w] has the same V and num_slots; W <= 64;
 * x, pkts and desc are host arrays of W device pointers. */
int ina_quantize_pack_nga_multi(const float* const* x, int W, const float* base, size_t n, int k,
                                const ina_nga_params_t* prm, uint8_t* const* pkts, size_t stride,
                                ina_nga_desc_t* const* desc, ina_stream_t stream);
/* PS-side parse (NGAPacket.py:62-143 / get_data_from_nic, utils.py:61-64), following
 * headers.p4: payload at byte 15, big-endian.  vals gets npkts*V int32 (may be NULL). */
int ina_unpack_nga(const uint8_t* pkts, size_t npkts, int V, size_t stride,
                   const ina_nga_fields_t* fields, int32_t* vals, ina_stream_t stream);
/* PS side, fused, after ina_switch_process: for each packet with actions[p] ==
 * INA_ACT_FWD_AGG, slot = frag_id - seq0; out[slot*V + j] = local[..] +
 * float(weight_step) * ((float)payload_j * 2^-k) for slot*V + j < n, and (acks !=
 * NULL) row `slot` of acks (ack_stride bytes apart) gets the packet's header with
 * is_ack = 1 -- the PS acknowledgement that frees the slot (fragcheck.p4:26-31).
 * V = 4 x a power of two <= 256; 16-byte aligned rows. */
int ina_apply_completed_nga(const uint8_t* pkts, size_t npkts, int V, size_t stride,
                            const uint8_t* actions, uint32_t seq0, const float* local, int k,
                            double weight_step, float* out, size_t n, uint8_t* acks,
                            size_t ack_stride, ina_stream_t stream);
/* ---- split NGA rows -------------------------------------------------------------
 * The same datagrams (header || payload on the wire, DataManager.py:111-165 /
 * headers.p4:27-80) stored as two arrays: hdr = npkts rows of 16 bytes (the 15-byte
 * header + one zero byte), pay = npkts rows of 4V bytes (the V big-endian payload words).
 * Every payload row is 16-byte aligned and covers whole cache lines (the packed NGA-256 row
 * of 15 + 1024 bytes straddles them), so packs, the switch and the PS move aligned 16-byte
 * chunks with no byte shifting.  sendmmsg / recvmmsg take two iovecs per datagram
 * (ina_send_packets_split_fd / ina_recv_packets_split_fd), so the bytes on the socket are
 * identical.  V is a multiple of 4 in [4, 256]; hdr, pay and value buffers 16-byte aligned.
 * Packet p's payload row is pay + p * 4V, so a bucket's payload stream is its values in
 * order, byte-swapped, zero-padded to whole packets. */
int ina_pack_nga_split(const int32_t* vals, size_t n, const ina_nga_params_t* prm,
                       const uint8_t* overflow_per_slot, uint8_t* hdr, uint8_t* pay,
                       ina_nga_desc_t* desc, ina_stream_t stream);
int ina_quantize_pack_nga_multi_split(const float* const* x, int W, const float* base, size_t n, int k,
                                      const ina_nga_params_t* prm, uint8_t* const* hdr,
                                      uint8_t* const* pay, ina_nga_desc_t* const* desc,
                                      ina_stream_t stream);
int ina_unpack_nga_split(const uint8_t* hdr, const uint8_t* pay, size_t npkts, int V,
                         const ina_nga_fields_t* fields, int32_t* vals, ina_stream_t stream);
/* C-128 pack (communicator.cc:23-37): npkts x 524-byte packet_t, all words htonl. */
int ina_pack_c128(const uint32_t* gradient, int packet_num, int worker_id,
                  uint32_t aggregator_index, int tensor_index, uint8_t* pkts,
                  ina_stream_t stream);

/* ---- packet-stream switch (ngaa.p4:120-196 restated on the device) -------------
 * State lives in device memory: count[num_slots] u8, frag[num_slots] u32,
 * regs[num_slots*V] u32 (zero-initialise once, like the P4 registers).  Packets are
 * processed in array order per slot (different slots are independent); forwarded
 * packets are rewritten in place (slot sum, collision bit; dropped ones too when
 * write_dropped) and actions[p] gets INA_ACT_*.
 * scratch: device buffer of ina_switch_scratch_bytes(npkts, num_slots) bytes; the size
 * is monotonic in npkts, so one buffer sized for the largest batch serves them all. */
typedef struct ina_switch_state {
    uint32_t num_slots;
    int32_t V;
    int32_t switch_id;  /* the switch_check entry (ngaa.p4:27-37); -1 = none */
    int32_t write_dropped; /* 1: also rewrite packets that are dropped (their running sums,
                              as the P4 deparser would); 0: leave them -- a dropped packet
                              is never observed, and skipping saves (W-1)/W of the writes */
    uint8_t* count;
    uint32_t* frag;
    uint32_t* regs;
} ina_switch_state_t;
size_t ina_switch_scratch_bytes(size_t npkts, uint32_t num_slots);

/* One batch through the switch (every layout and option in one call).
 *   rows     packed rows (stride bytes apart, stride >= 15 + 4V), or -- pay != NULL -- the
 *            split header rows (16 bytes apart; stride is ignored), see "split NGA rows";
 *   pay      split payload rows (4V bytes apart), NULL for packed rows;
 *   desc     the packets' descriptors (ina_pack_nga_desc / ina_nga_descriptors; desc[p] must
 *            equal bytes 4..11 of packet p): the slot sort reads them instead of the headers,
 *            results identical; NULL: the sort reads the headers;
 *   actions  npkts INA_ACT_* out;  scratch  ina_switch_scratch_bytes(npkts, num_slots) bytes. */
typedef struct ina_switch_batch {
    uint8_t* rows;
    uint8_t* pay;
    size_t npkts;
    size_t stride;
    const ina_nga_desc_t* desc;
    uint8_t* actions;
    void* scratch;
} ina_switch_batch_t;

/* The PS co-located with the switch on one GPU, fused into the switch's pass: a completed
 * slot's sum goes from the switch's registers straight into out[slot*V + j] = local +
 * float(weight_step) * (sum * 2^-k) (slot = frag_id - seq0, slot*V + j < n) and its PS ack row
 * (the packet's header with is_ack = 1, fragcheck.p4:26-31) -- the same results as the switch
 * followed by ina_apply_completed_nga.  acks: ack rows ack_stride bytes apart (NULL: none;
 * split rows: header rows, ack_stride 16 or 0); ack_desc (may be NULL; needs acks): each ack
 * row's descriptor beside it, for exactly the rows the call writes, so the next batch -- these
 * acks in front of the next step's packets -- is sorted without a gather pass.  The step always
 * runs fused in the switch's run kernel (the layouts below are the ones it takes; others are
 * refused before the switch touches its state).  keep_forwarded = 0: completed packets are
 * consumed and their buffers left as they arrived.  Replaces the Tofino -> PS hop of ngaa.p4:170-175 +
 * NGAPacket.py:62-143 + launch.py:42-52 when both live on the GPU.  16-byte aligned local,
 * out, rows and registers; V % 4 == 0. */
typedef struct ina_switch_ps {
    uint32_t seq0;
    int k;
    double weight_step;
    const float* local;
    float* out;
    size_t n;
    uint8_t* acks;
    size_t ack_stride;
    ina_nga_desc_t* ack_desc;
    int keep_forwarded;
} ina_switch_ps_t;

/* phase: the whole call, or its two halves.  With descriptors the slot sort reads nothing but
 * them, so INA_SWITCH_SORT can be queued as soon as they exist -- before, or on another stream
 * beside, the kernels that still fill the payload (descriptors from the header parameters
 * alone: ina_nga_make_descriptors); rows must already be the batch's final address.
 * INA_SWITCH_RUN then runs the batch over that scratch (the caller orders the two: same stream
 * or an event) under the switch tuning keys the sort recorded -- ina_set_tuning between them,
 * from any thread, changes nothing in this batch.  The run must name the SAME batch: rows, pay,
 * actions (the sort already stored every dropped and foreign packet's action byte there; the run
 * stores only the others), npkts, stride, V, num_slots and switch_id.  A run over a scratch that
 * no sort of that batch filled is refused (INA_EINVAL), and a run consumes its sort's record (a
 * second run needs a second sort).  A sort that fails leaves no record.  (Batches the
 * small-batch paths take, which sort from the headers, are sorted inside the run.) */
#define INA_SWITCH_ALL 0
#define INA_SWITCH_SORT 1
#define INA_SWITCH_RUN 2
/* ps may be NULL (the switch alone).  Same semantics, actions, registers and forwarded bytes
 * in every layout (a collision rewrites the header row's flag byte, a forwarded packet its
 * payload row). */
int ina_switch(const ina_switch_state_t* st, const ina_switch_batch_t* batch, const ina_switch_ps_t* ps,
               int phase, ina_stream_t stream);
/* The common case in one line: packed rows, headers read by the sort, no PS step. */
int ina_switch_process(const ina_switch_state_t* st, uint8_t* pkts, size_t npkts, size_t stride,
                       uint8_t* actions, void* scratch, ina_stream_t stream);

/* Diagnostic: which slot-sort path the last call over `scratch` took (a batch of npkts
 * packets, more than 768 of them; the one-workgroup small-batch paths do not record one; the
 * LSD digit passes report INA_PATH_SORTED).  Synchronous (reads 12 bytes of the scratch). */
#define INA_PATH_IN_ORDER 1   /* already in slot order: no sort */
#define INA_PATH_RUNS 2       /* at most 64 runs of consecutive slots: a run table, no sort */
#define INA_PATH_SORTED 3     /* the bucket sort (or the LSD digit passes) */
#define INA_PATH_LOCAL 4      /* near-sorted (local disorder, V <= 32): per-slot lists, no sort */
int ina_switch_batch_path(const void* scratch, size_t npkts, uint32_t num_slots, int* path);

/* ---- ipRoute (ngaa.p4:39-61, entries as bfrt/setup.py:85-95 installs them) -------
 * Every packet the ingress does not drop (actions FWD_AGG, FWD_COLLISION, FWD_ACK,
 * FWD_OTHER) leaves through ipRoute: an exact match on the IPv4 destination.
 * The table is n_entries <= INA_ROUTE_MAX rows (keys[i] = IPv4 address, host order;
 * ports[i] = egress port >= 0 for ipv4_forward, INA_PORT_DROP for the drop action,
 * INA_PORT_NONE for NoAction); the first matching row wins and a miss takes the
 * default action, drop.  egress[p] = the port, INA_PORT_DROP for packets the ingress
 * or the table dropped, INA_PORT_NONE for NoAction.  dst_ip is a per-packet device
 * array, or NULL for dst_default on every packet (a stand-in without IP headers).
 * keys, ports, actions, egress: device memory. */
#define INA_ROUTE_MAX 256        /* ipRoute size = 1<<8, ngaa.p4:59 */
#define INA_PORT_DROP (-1)
#define INA_PORT_NONE (-2)
int ina_route_ipv4(const uint8_t* actions, const uint32_t* dst_ip, uint32_t dst_default,
                   size_t npkts, const uint32_t* keys, const int32_t* ports, int n_entries,
                   int32_t* egress, ina_stream_t stream);

/* ---- PCIe-inclusive aggregation (PS ingest) ----------------------------------------
 * The PS side of the reference receives each worker's gradients over a socket into host
 * memory and sums them on the CPU (worker.py:63-79, launch.py:111-130, 42-52).  When all
 * W HOST buckets and host_out are pinned, device-mapped memory (hipHostMalloc,
 * hipHostRegister, torch pin_memory), ONE launch of the W-way sum-reduce on `stream`
 * reads the buckets and writes the aggregate across PCIe directly (zero copy; tuning key
 * 16 = 0 turns this off).  Otherwise the buckets move through HBM in chunks of
 * chunk_values values (0 = 4 Mi; rounded up to a multiple of 64): H2D copies, the
 * reduce, D2H of the aggregate into host_out, pipelined over a ring of 3 device slots on
 * internal copy streams so both copy directions overlap the reduce.  Bit-identical to
 * ina_sum_reduce_i32 either way.  dev_scratch: device memory (256-byte aligned) of
 * ina_host_reduce_scratch_bytes(W, chunk_values) bytes (the pipeline's ring).
 * Synchronous: returns once host_out holds the aggregate (the PS sends it next). */
size_t ina_host_reduce_scratch_bytes(int W, size_t chunk_values);
int ina_sum_reduce_host_i32(const int32_t* const* host_bufs, int W, int32_t* host_out, size_t n,
                            size_t chunk_values, void* dev_scratch, ina_stream_t stream);

/* ---- integrity ------------------------------------------------------------------
 * *out_dev (device u32) = sum_i x[i]*(2i+1) mod 2^32 (linear in x, so the checksum
 * of a reduce equals the wrapped sum of the input checksums). */
int ina_checksum_i32(const int32_t* x, size_t n, uint32_t* out_dev, ina_stream_t stream);

/* ---- host send path --------------------------------------------------------------
 * Legacy symbol, exact reference signature and behaviour (communicator.h:27,
 * communicator.cc:3-47): gradient_array is a HOST pointer to packet_num*128 u32;
 * packets are built on the GPU (ina_pack_c128) and sent with sendmmsg on a raw
 * IPPROTO_UDP socket to dst_ip (host order).  Like the reference, a socket
 * failure prints perror and exits the process with -1. */
void send_gradients(uint32_t* gradient_array, int packet_num, uint32_t dst_ip, int worker_id,
                    uint32_t aggregator_index, int tensor_index);
/* Same as send_gradients but returns a status instead of exiting, and sends on a
 * caller-provided datagram socket fd (connected, or dst_ip used as AF_INET dest
 * when dst_ip != 0).  Returns packets sent (>= 0) or INA_E*. */
int ina_send_gradients_fd(int fd, const uint32_t* gradient_array, int packet_num,
                          uint32_t dst_ip, int worker_id, uint32_t aggregator_index,
                          int tensor_index);

/* Batched datagram egress for packets already in HOST memory (e.g. copied back
 * from ina_pack_nga): sends npkts datagrams of pkt_len bytes found at `stride`
 * apart with sendmmsg() on fd (to dst_ip, host order, when != 0).  Replaces the
 * per-packet sendto() loops of DataManager.py:134,153 and communicator.cc:37.
 * Returns packets sent or INA_E*. */
int ina_send_packets_fd(int fd, const uint8_t* host_pkts, size_t npkts, size_t stride,
                        size_t pkt_len, uint32_t dst_ip);

/* Split rows on the socket: datagram p = hdr row p's 15 bytes || pay row p's 4V bytes (two
 * iovecs), the same bytes ina_send_packets_fd sends from packed rows.  host_hdr / host_pay:
 * host memory, rows 16 / 4V bytes apart. */
int ina_send_packets_split_fd(int fd, const uint8_t* host_hdr, const uint8_t* host_pay, size_t npkts,
                              int V, uint32_t dst_ip);
/* ... and into them: each datagram's first 15 bytes (after `skip`) land in its header row,
 * the next 4V in its payload row (header byte 15 is left as it was).  lens as below. */
int ina_recv_packets_split_fd(int fd, uint8_t* host_hdr, uint8_t* host_pay, size_t max_pkts, int V,
                              size_t skip, int timeout_ms, uint32_t* lens);
/* Batched datagram ingest, the counterpart of get_data_from_nic (utils.py:61-64,
 * one recvfrom per packet): up to max_pkts datagrams land in host_pkts at `stride`
 * apart via recvmmsg(); the first `skip` bytes of each datagram (20 for the IPv4
 * header a raw socket delivers) are discarded.  Returns once max_pkts datagrams have
 * arrived or timeout_ms has passed (0 = drain what is queued).  lens (may be NULL)
 * receives each packet's length after `skip`.  Returns packets received. */
int ina_recv_packets_fd(int fd, uint8_t* host_pkts, size_t max_pkts, size_t stride, size_t skip,
                        int timeout_ms, uint32_t* lens);

#ifdef __cplusplus
}
#endif
#endif /* INA_H */
