/* ina_oracle.h -- TEST INFRASTRUCTURE ONLY (see ina_oracle.c header). */
#ifndef INA_ORACLE_H
#define INA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_EINVAL (-1)
#define ORC_ENOMEM (-2)
#define ORC_ESTATE (-3)

#define ORC_NGA_HDR 15          /* ngaa_h, headers.p4:27-38 */
#define ORC_NUM_REGISTER 16384u /* config.p4:5 */
#define ORC_C128_V 128          /* communicator.h:18 */
#define ORC_C128_BYTES 524      /* sizeof(packet_t), communicator.h:20-25 */

/* flags byte of ngaa_h: overflow|is_ack|collision|resend|timestamp[4] (headers.p4:30-34) */
#define ORC_FLAG_OVERFLOW 0x80u
#define ORC_FLAG_ACK 0x40u
#define ORC_FLAG_COLLISION 0x20u
#define ORC_FLAG_RESEND 0x10u

/* forwarding decisions of Ingress.apply (ngaa.p4:120-196) */
#define ORC_ACT_DROP 0
#define ORC_ACT_FWD_AGG 1
#define ORC_ACT_FWD_COLLISION 2
#define ORC_ACT_FWD_ACK 3
#define ORC_ACT_FWD_OTHER 4

typedef struct {
    uint32_t bitmap;    /* DataManager passes worker_id raw (DataManager.py:124) */
    uint8_t count;      /* degree */
    uint8_t flags;
    uint8_t switch_id;
    uint8_t pad;
    uint32_t seq0;      /* frag_id of packet p = seq0 + p; index = frag_id mod num_slots */
    uint32_t num_slots; /* 16384 */
    int32_t V;          /* payload words per packet */
} orc_nga_params_t;

typedef struct {
    uint32_t* bitmap;
    uint8_t* count;
    uint8_t* flags;
    uint32_t* index;
    uint8_t* switch_id;
    uint32_t* frag_id;
} orc_nga_fields_t;

typedef struct {
    uint32_t num_slots;
    int V;
    int switch_id;      /* the one switch_check entry; -1 = none */
    uint8_t* count;
    uint32_t* frag;
    uint32_t* regs;
} orc_switch_t;

int32_t orc_q_i32(float x, float scale);
int16_t orc_q_i16(float x, float scale, int* sat);
int orc_quantize_f32_i32(const float* x, int32_t* q, size_t n, int k);
int orc_quantize_f32_i16_sat(const float* x, int16_t* q, size_t n, int k, int V, uint8_t* ovf);
int orc_dequantize_i32_f32(const int32_t* s, float* y, size_t n, int k);
int orc_dequantize_i16_f32(const int16_t* s, float* y, size_t n, int k);
int orc_sum_reduce_i32(const int32_t* const* bufs, int W, int32_t* out, size_t n);
int orc_sum_reduce_i16_sat(const int16_t* const* bufs, int W, int16_t* out, size_t n, int V,
                           uint8_t* ovf);
int orc_quantize_reduce_f32_i32(const float* const* bufs, int W, int32_t* out, size_t n, int k);
int orc_quantize_reduce_f32_i16_sat(const float* const* bufs, int W, int16_t* out, size_t n,
                                    int k, int V, uint8_t* ovf);
int orc_quantize_f32_i16_wire(const float* x, int32_t* wire, size_t n, int k);
int orc_i16_wire_finish(const int32_t* wsum, size_t n, int k, int V, int16_t* out16, float* y,
                        uint8_t* ovf);
int orc_ps_combine_f32(const float* local, const float* const* paras, int W,
                       double weight_step, float* out, size_t n);
int orc_ps_combine_ina_f32(const float* local, const float* const* paras, int W, int k,
                           double weight_step, float* out, size_t n);
void orc_nga_write_header(uint8_t* p, uint32_t bitmap, uint8_t count, uint8_t flags,
                          uint32_t index, uint8_t switch_id, uint32_t frag_id);
int orc_pack_nga(const int32_t* vals, size_t n, const orc_nga_params_t* prm, const uint8_t* ovf,
                 uint8_t* pkts, size_t stride);
int orc_unpack_nga(const uint8_t* pkts, size_t np, int V, size_t stride, orc_nga_fields_t* f,
                   int32_t* vals);
uint32_t orc_c128_bitmap(int worker_id);
int orc_pack_c128(const uint32_t* g, int packet_num, int worker_id, uint32_t aggregator_index,
                  int tensor_index, uint8_t* out);
int orc_switch_init(orc_switch_t* sw, uint32_t num_slots, int V, int switch_id);
void orc_switch_free(orc_switch_t* sw);
int orc_switch_packet(orc_switch_t* sw, uint8_t* pk);
int orc_cpu_packetise_aggregate(const int32_t* const* bufs, int W, size_t n, int V, int threads,
                                int32_t* out, double* seconds);
uint32_t orc_checksum_i32(const int32_t* x, size_t n);
int orc_switch_run(orc_switch_t* sw, uint8_t* pkts, size_t np, size_t stride, uint8_t* actions);
#define ORC_PORT_DROP (-1)
#define ORC_PORT_NONE (-2)
void orc_route_ipv4(const uint8_t* actions, const uint32_t* dst_ip, uint32_t dst_default,
                    size_t np, const uint32_t* keys, const int32_t* ports, int nent,
                    int32_t* egress);

#ifdef __cplusplus
}
#endif
#endif
