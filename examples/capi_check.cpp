// capi_check.cpp -- a C/C++ caller of libina.so with no Python and no torch: links the
// library through include/ina.h only, allocates device memory with the HIP runtime,
// runs quantise -> W-way sum-reduce -> NGA-256 pack -> unpack -> dequantise, then the
// workers' packets through the device switch with the PS step fused, and checks every
// step against a host computation.  Built by `make -C examples`; run by
// tests/test_gpu_capi_binary.py on the GPU box.  Exit status 0 = all checks passed.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ina.h"

#define CK(x)                                                                    \
    do {                                                                         \
        int rc_ = (x);                                                           \
        if (rc_ != 0) {                                                          \
            std::fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, ina_last_error_string()); \
            return 1;                                                            \
        }                                                                        \
    } while (0)
#define HK(x)                                                                    \
    do {                                                                         \
        if ((x) != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s failed\n", #x);                             \
            return 1;                                                            \
        }                                                                        \
    } while (0)

static int32_t q_host(float x, int k) {   // the build-defined quantiser (include/ina.h)
    if (x != x) return 0;
    const double y = std::nearbyint((double)x * std::ldexp(1.0, k));   // RNE (default mode)
    if (y >= 2147483647.0) return INT32_MAX;
    if (y <= -2147483648.0) return INT32_MIN;
    return (int32_t)y;
}

int main() {
    const int W = 8, k = 16, V = 256;
    const size_t n = 1000003;
    std::printf("%s\n", ina_version());
    std::vector<std::vector<float>> g(W, std::vector<float>(n));
    uint32_t seed = 12345;
    for (int w = 0; w < W; ++w)
        for (size_t i = 0; i < n; ++i) {
            seed = seed * 1664525u + 1013904223u;
            g[w][i] = ((int32_t)seed >> 8) * 1e-9f;
        }
    float* d_g[W];
    int32_t* d_q[W];
    for (int w = 0; w < W; ++w) {
        HK(hipMalloc(&d_g[w], n * 4));
        HK(hipMalloc(&d_q[w], n * 4));
        HK(hipMemcpy(d_g[w], g[w].data(), n * 4, hipMemcpyHostToDevice));
    }
    int32_t* d_sum;
    HK(hipMalloc(&d_sum, n * 4));
    hipStream_t s;
    HK(hipStreamCreate(&s));
    for (int w = 0; w < W; ++w) CK(ina_quantize_f32_i32(d_g[w], d_q[w], n, k, s));
    CK(ina_sum_reduce_i32((const int32_t* const*)d_q, W, d_sum, n, s));

    const size_t stride = (15 + 4 * V + 15) / 16 * 16, npk = (n + V - 1) / V;
    uint8_t* d_pk;
    HK(hipMalloc(&d_pk, npk * stride));
    ina_nga_params_t prm;
    std::memset(&prm, 0, sizeof prm);
    prm.bitmap = 1; prm.count = W; prm.switch_id = 1; prm.seq0 = 1;
    prm.num_slots = INA_NUM_REGISTER; prm.V = V;
    CK(ina_pack_nga(d_sum, n, &prm, nullptr, d_pk, stride, s));
    int32_t* d_back;
    HK(hipMalloc(&d_back, npk * V * 4));
    CK(ina_unpack_nga(d_pk, npk, V, stride, nullptr, d_back, s));
    float* d_f;
    HK(hipMalloc(&d_f, n * 4));
    CK(ina_dequantize_i32_f32(d_back, d_f, n, k, s));
    HK(hipStreamSynchronize(s));

    std::vector<int32_t> sum(n), back(npk * V);
    std::vector<float> f(n);
    std::vector<uint8_t> pk(npk * stride);
    HK(hipMemcpy(sum.data(), d_sum, n * 4, hipMemcpyDeviceToHost));
    HK(hipMemcpy(back.data(), d_back, npk * V * 4, hipMemcpyDeviceToHost));
    HK(hipMemcpy(f.data(), d_f, n * 4, hipMemcpyDeviceToHost));
    HK(hipMemcpy(pk.data(), d_pk, npk * stride, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t want = 0;
        for (int w = 0; w < W; ++w) want += (uint32_t)q_host(g[w][i], k);
        if ((uint32_t)sum[i] != want || back[i] != sum[i] ||
            f[i] != (float)sum[i] * std::ldexp(1.0f, -k))
            ++bad;
        // wire bytes: value i of packet i / V at 15 + 4 (i % V), big-endian
        const uint8_t* b = &pk[(i / V) * stride + 15 + 4 * (i % V)];
        const uint32_t be = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
        if (be != want) ++bad;
    }
    for (size_t i = n; i < npk * V; ++i) bad += back[i] != 0;   // zero-padded tail

    // the packet path: every worker's quantised bucket as NGA-256 packets through the
    // device switch with the PS update fused (local = 0, weight 1 -> out = dequantised sum)
    const uint32_t slots = 1u << 13;
    uint8_t* d_stream;
    HK(hipMalloc(&d_stream, (size_t)W * npk * stride));
    for (int w = 0; w < W; ++w) {
        prm.bitmap = 1u << w; prm.num_slots = slots;
        CK(ina_pack_nga(d_q[w], n, &prm, nullptr, d_stream + (size_t)w * npk * stride, stride, s));
    }
    // the same packets from the fp32 gradients, every worker quantised and packed in ONE
    // launch (ina_quantize_pack_nga_multi): byte-identical to quantise, then pack
    {
        uint8_t* d_stream2;
        HK(hipMalloc(&d_stream2, (size_t)W * npk * stride));
        std::vector<ina_nga_params_t> prms(W, prm);
        std::vector<uint8_t*> outs(W);
        for (int w = 0; w < W; ++w) {
            prms[w].bitmap = 1u << w;
            outs[w] = d_stream2 + (size_t)w * npk * stride;
        }
        CK(ina_quantize_pack_nga_multi((const float* const*)d_g, W, nullptr, n, k, prms.data(), outs.data(),
                                       stride, nullptr, s));
        HK(hipStreamSynchronize(s));
        std::vector<uint8_t> a((size_t)W * npk * stride), b(a.size());
        HK(hipMemcpy(a.data(), d_stream, a.size(), hipMemcpyDeviceToHost));
        HK(hipMemcpy(b.data(), d_stream2, b.size(), hipMemcpyDeviceToHost));
        if (a != b) ++bad;
        HK(hipFree(d_stream2));
    }
    uint8_t *d_count, *d_act;
    uint32_t *d_frag, *d_regs;
    float *d_zero, *d_out;
    HK(hipMalloc(&d_count, slots));
    HK(hipMalloc(&d_frag, slots * 4));
    HK(hipMalloc(&d_regs, (size_t)slots * V * 4));
    HK(hipMalloc(&d_act, (size_t)W * npk));
    HK(hipMalloc(&d_zero, n * 4));
    HK(hipMalloc(&d_out, n * 4));
    HK(hipMemset(d_count, 0, slots));
    HK(hipMemset(d_frag, 0, slots * 4));
    HK(hipMemset(d_regs, 0, (size_t)slots * V * 4));
    HK(hipMemset(d_zero, 0, n * 4));
    ina_switch_state_t st = {slots, V, 1, 0, d_count, d_frag, d_regs};
    void* d_scratch;
    HK(hipMalloc(&d_scratch, ina_switch_scratch_bytes((size_t)W * npk, slots)));
    // one call: the packed batch, the PS step fused (ina_switch_ps_t), sort + run
    const ina_switch_batch_t batch{d_stream, nullptr, (size_t)W * npk, stride, nullptr, d_act, d_scratch};
    const ina_switch_ps_t ps{1, k, 1.0, d_zero, d_out, n, nullptr, 0, nullptr, 0};
    CK(ina_switch(&st, &batch, &ps, INA_SWITCH_ALL, s));
    HK(hipStreamSynchronize(s));
    std::vector<float> out(n);
    std::vector<uint8_t> act((size_t)W * npk);
    HK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
    HK(hipMemcpy(act.data(), d_act, act.size(), hipMemcpyDeviceToHost));
    size_t done = 0;
    for (uint8_t a : act) done += a == INA_ACT_FWD_AGG;
    if (done != npk) ++bad;
    for (size_t i = 0; i < n; ++i) bad += std::memcmp(&out[i], &f[i], 4) != 0;

    // the same step over split rows (16-byte headers + 4V-byte payloads): fresh switch
    // state, same dequantised sum, same actions
    {
        uint8_t *d_hdr, *d_pay;
        HK(hipMalloc(&d_hdr, (size_t)W * npk * 16));
        HK(hipMalloc(&d_pay, (size_t)W * npk * 4 * V));
        for (int w = 0; w < W; ++w) {
            prm.bitmap = 1u << w;
            CK(ina_pack_nga_split(d_q[w], n, &prm, nullptr, d_hdr + (size_t)w * npk * 16,
                                  d_pay + (size_t)w * npk * 4 * V, nullptr, s));
        }
        HK(hipMemsetAsync(d_count, 0, slots, s));
        HK(hipMemsetAsync(d_frag, 0, slots * 4, s));
        HK(hipMemsetAsync(d_regs, 0, (size_t)slots * V * 4, s));
        HK(hipMemsetAsync(d_out, 0xff, n * 4, s));
        const ina_switch_batch_t sb{d_hdr, d_pay, (size_t)W * npk, 0, nullptr, d_act, d_scratch};
        CK(ina_switch(&st, &sb, &ps, INA_SWITCH_ALL, s));
        HK(hipStreamSynchronize(s));
        std::vector<uint8_t> act2(act.size());
        HK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(act2.data(), d_act, act2.size(), hipMemcpyDeviceToHost));
        if (act2 != act) ++bad;
        for (size_t i = 0; i < n; ++i) bad += std::memcmp(&out[i], &f[i], 4) != 0;
        HK(hipFree(d_hdr));
        HK(hipFree(d_pay));
    }
    // the same step in two phases: the slot sort from the packets' descriptors, the switch
    // tuning flipped in between (the run follows what its sort recorded), then the run
    {
        ina_nga_desc_t* d_desc;
        HK(hipMalloc(&d_desc, (size_t)W * npk * 8));
        // the packed rows were consumed (keep_forwarded = 0 leaves them as they arrived)
        CK(ina_nga_descriptors(d_stream, (size_t)W * npk, stride, d_desc, s));
        HK(hipMemsetAsync(d_count, 0, slots, s));
        HK(hipMemsetAsync(d_frag, 0, slots * 4, s));
        HK(hipMemsetAsync(d_regs, 0, (size_t)slots * V * 4, s));
        HK(hipMemsetAsync(d_out, 0xff, n * 4, s));
        const ina_switch_batch_t tb{d_stream, nullptr, (size_t)W * npk, stride, d_desc, d_act, d_scratch};
        CK(ina_switch(&st, &tb, nullptr, INA_SWITCH_SORT, s));
        CK(ina_set_tuning(18, 0));                 // runs off, digits for every width, LSD passes
        CK(ina_set_tuning(19, 0));
        CK(ina_set_tuning(12, 3));
        CK(ina_switch(&st, &tb, &ps, INA_SWITCH_RUN, s));
        CK(ina_set_tuning(18, 1));
        CK(ina_set_tuning(19, 1));
        CK(ina_set_tuning(12, 0));
        HK(hipStreamSynchronize(s));
        std::vector<uint8_t> act3(act.size());
        HK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(act3.data(), d_act, act3.size(), hipMemcpyDeviceToHost));
        if (act3 != act) ++bad;
        for (size_t i = 0; i < n; ++i) bad += std::memcmp(&out[i], &f[i], 4) != 0;
        // a run with no sort of its batch in the scratch is refused: the run above consumed the
        // sort; a fresh sort, then runs that name another batch length, another actions buffer
        // (the sort stored the drops in d_act) or another switch id are refused too
        const ina_switch_batch_t other{d_stream, nullptr, (size_t)W * npk - 1, stride, nullptr, d_act, d_scratch};
        if (ina_switch(&st, &tb, nullptr, INA_SWITCH_RUN, s) != INA_EINVAL) ++bad;
        CK(ina_switch(&st, &tb, nullptr, INA_SWITCH_SORT, s));
        if (ina_switch(&st, &other, nullptr, INA_SWITCH_RUN, s) != INA_EINVAL) ++bad;
        uint8_t* d_act2;
        HK(hipMalloc(&d_act2, (size_t)W * npk));
        const ina_switch_batch_t other_act{d_stream, nullptr, (size_t)W * npk, stride, nullptr, d_act2, d_scratch};
        if (ina_switch(&st, &other_act, nullptr, INA_SWITCH_RUN, s) != INA_EINVAL) ++bad;
        ina_switch_state_t st2 = st;
        st2.switch_id = st.switch_id + 1;
        if (ina_switch(&st2, &tb, nullptr, INA_SWITCH_RUN, s) != INA_EINVAL) ++bad;
        HK(hipStreamSynchronize(s));
        HK(hipFree(d_act2));
        HK(hipFree(d_desc));
    }
    // the error path: a bad argument returns a code, sets a message, never exits
    const int rc = ina_sum_reduce_i32((const int32_t* const*)d_q, 0, d_sum, n, s);
    if (rc != INA_EINVAL || std::strlen(ina_last_error_string()) == 0) ++bad;
    std::printf("capi_check: %zu values x %d workers (bulk reduce, NGA-256 pack/unpack, one-launch worker packs, switch + fused PS step, packed and split rows, two-phase sort/run across a tuning change), %zu mismatches\n", n, W, bad);
    return bad ? 1 : 0;
}
