// ina_host.cpp -- PCIe-inclusive aggregation path of libina.so.
//
// At the PS, worker gradients arrive from sockets into host memory and the aggregate
// leaves on a socket (north star; the reference's PS receives pickled tensors,
// worker.py:63-79 / launch.py:111-130, and sums them on the CPU, launch.py:42-52).
// ina_sum_reduce_host_i32: when every bucket and the output are pinned, device-mapped host
// memory, ONE launch of the W-way reduce reads the buckets over PCIe and writes the
// aggregate back over PCIe (zero copy); otherwise it moves the buckets through HBM in
// chunks: H2D copies on one or two copy streams (workers alternate), the W-way sum-reduce
// on the caller's stream, D2H of the aggregate on another, over a ring of kSlots device
// slots, so the two copy directions and the reduce overlap and the run approaches the
// PCIe link rate instead of the sum of the three phases.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "ina.h"
#include "ina_internal.h"

namespace {

constexpr int kSlots = 3;                     // ring depth: copy-in, reduce, copy-out in flight
// values per worker per chunk: 16 MiB copies (MI355X, 8 x 100 MiB: 1 Mi-value chunks
// 15.3 ms, 4 Mi 15.1 ms, 256 Ki 21.8 ms -- each hipMemcpyAsync carries tens of us of
// fixed cost), bench_extra 'end-to-end pipelined' rows
constexpr size_t kDefaultChunk = 1u << 22;
constexpr size_t kChunkAlign = 64;            // values: device sub-buffers stay 256-byte aligned

struct HostPipe {   // per host thread: copy streams and ring events, created once per device
    int device = -1;
    int n_h2d = 0;
    hipStream_t h2d[2] = {nullptr, nullptr};
    hipStream_t d2h = nullptr;
    hipEvent_t start = nullptr;
    hipEvent_t in_done[kSlots][2] = {};
    hipEvent_t red_done[kSlots] = {};
    hipEvent_t out_done[kSlots] = {};

    void release() {
        for (int s = 0; s < kSlots; ++s) {
            for (auto& e : in_done[s])
                if (e) (void)hipEventDestroy(e), e = nullptr;
            if (red_done[s]) (void)hipEventDestroy(red_done[s]), red_done[s] = nullptr;
            if (out_done[s]) (void)hipEventDestroy(out_done[s]), out_done[s] = nullptr;
        }
        if (start) (void)hipEventDestroy(start), start = nullptr;
        for (auto& s : h2d)
            if (s) (void)hipStreamDestroy(s), s = nullptr;
        if (d2h) (void)hipStreamDestroy(d2h), d2h = nullptr;
        device = -1;
        n_h2d = 0;
    }
    ~HostPipe() { release(); }

    bool ready(int dev, int want_h2d) {
        if (device == dev && n_h2d == want_h2d) return true;
        release();
        const unsigned ef = hipEventDisableTiming;
        for (int i = 0; i < want_h2d; ++i)
            if (hipStreamCreateWithFlags(&h2d[i], hipStreamNonBlocking) != hipSuccess) return false;
        if (hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&start, ef) != hipSuccess) return false;
        for (int s = 0; s < kSlots; ++s) {
            for (int i = 0; i < want_h2d; ++i)
                if (hipEventCreateWithFlags(&in_done[s][i], ef) != hipSuccess) return false;
            if (hipEventCreateWithFlags(&red_done[s], ef) != hipSuccess) return false;
            if (hipEventCreateWithFlags(&out_done[s], ef) != hipSuccess) return false;
        }
        device = dev;
        n_h2d = want_h2d;
        return true;
    }
};

thread_local HostPipe t_pipe;
// ina_set_tuning key 7: H2D copy streams; two (workers alternate) measured faster at
// every chunk size (15.1 vs 16.0 ms at 4 Mi values: the link, ~55.6 GB/s H2D, is the bound)
int g_h2d_streams = 2;
// ina_set_tuning key 16: 1 (default) reduce device-mapped pinned buffers in place over PCIe,
// 0 always the chunked copy pipeline (tests run both)
int g_zero_copy = 1;

size_t chunk_for(size_t chunk_values) {
    size_t c = chunk_values ? chunk_values : kDefaultChunk;
    return (c + kChunkAlign - 1) / kChunkAlign * kChunkAlign;
}

}  // namespace

namespace ina {
int set_zero_copy(int v) {
    if (v != 0 && v != 1) return INA_EINVAL;
    g_zero_copy = v;
    return INA_OK;
}
int set_h2d_streams(int v) {
    if (v != 1 && v != 2) return INA_EINVAL;
    g_h2d_streams = v;
    return INA_OK;
}
}  // namespace ina

extern "C" {

size_t ina_host_reduce_scratch_bytes(int W, size_t chunk_values) {
    if (W < 1 || W > INA_MAX_WORKERS) return 0;
    return (size_t)kSlots * (size_t)(W + 1) * chunk_for(chunk_values) * sizeof(int32_t);
}

int ina_sum_reduce_host_i32(const int32_t* const* host_bufs, int W, int32_t* host_out, size_t n,
                            size_t chunk_values, void* dev_scratch, ina_stream_t stream) {
    using ina::set_error;
    if (W < 1 || W > INA_MAX_WORKERS) return set_error(INA_EINVAL, "W must be in [1, 64]%s", "");
    if (n == 0) return INA_OK;
    if (!host_bufs || !host_out || !dev_scratch) return set_error(INA_EINVAL, "null pointer%s", "");
    for (int w = 0; w < W; ++w)
        if (!host_bufs[w]) return set_error(INA_EINVAL, "null worker buffer%s", "");
    if ((uintptr_t)dev_scratch & 255u) return set_error(INA_EINVAL, "scratch must be 256-byte aligned%s", "");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return set_error(INA_EHIP, "hipGetDevice%s", "");
    HostPipe& P = t_pipe;
    if (!P.ready(dev, g_h2d_streams)) {
        P.release();
        return set_error(INA_EHIP, "copy stream/event creation%s", "");
    }
    hipStream_t cs = reinterpret_cast<hipStream_t>(stream);
    // pinned (device-mapped) host buckets and output: no staging at all -- the reduce
    // kernel's loads and stores cross PCIe themselves (GPU-initiated reads of the workers'
    // buckets, writes of the aggregate), one launch; 55.7-56.5 GB/s against 54.2 GB/s for
    // the chunked copy pipeline and 56.4 GB/s for plain H2D copies of the same 8 x 100 MiB
    // (tools/lab/zerocopy_lab.py, profiles/r03/lab).  Pageable memory takes the pipeline.
    if (g_zero_copy) {
        const int32_t* dptr[INA_MAX_WORKERS];
        void* dout = nullptr;
        bool mapped = hipHostGetDevicePointer(&dout, host_out, 0) == hipSuccess;
        for (int w = 0; w < W && mapped; ++w) {
            void* p = nullptr;
            mapped = hipHostGetDevicePointer(&p, const_cast<int32_t*>(host_bufs[w]), 0) == hipSuccess;
            dptr[w] = static_cast<const int32_t*>(p);
        }
        if (mapped) {
            if (int rc = ina::sum_reduce_i32_impl(dptr, W, static_cast<int32_t*>(dout), n, stream, true))
                return rc;
            if (hipStreamSynchronize(cs) != hipSuccess) return set_error(INA_EHIP, "zero-copy reduce sync%s", "");
            return INA_OK;
        }
        (void)hipGetLastError();               // a refused query is not an error of this call
    }
    const size_t c = chunk_for(chunk_values);
    const size_t nchunks = (n + c - 1) / c;
    int32_t* base = reinterpret_cast<int32_t*>(dev_scratch);
    auto in_buf = [&](int slot, int w) { return base + ((size_t)slot * (W + 1) + (size_t)w) * c; };
    auto out_buf = [&](int slot) { return base + ((size_t)slot * (W + 1) + (size_t)W) * c; };
    bool ok = true;
    auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
    // on an error return, copies already enqueued still read host_bufs / write host_out:
    // drain every stream first so the caller may free them
    auto drain = [&]() {
        for (int i = 0; i < P.n_h2d; ++i) (void)hipStreamSynchronize(P.h2d[i]);
        (void)hipStreamSynchronize(P.d2h);
        (void)hipStreamSynchronize(cs);
    };

    // earlier work of the caller's stream on the scratch finishes before the first copy
    chk(hipEventRecord(P.start, cs));
    for (int i = 0; i < P.n_h2d; ++i) chk(hipStreamWaitEvent(P.h2d[i], P.start, 0));
    chk(hipStreamWaitEvent(P.d2h, P.start, 0));
    for (size_t k = 0; k < nchunks && ok; ++k) {
        const int slot = (int)(k % kSlots);
        const size_t off = k * c, len = (n - off < c) ? n - off : c;
        // copy in: the slot's inputs are free once chunk k - kSlots was reduced
        for (int i = 0; i < P.n_h2d; ++i) {
            if (k >= (size_t)kSlots) chk(hipStreamWaitEvent(P.h2d[i], P.red_done[slot], 0));
            for (int w = i; w < W; w += P.n_h2d)
                chk(hipMemcpyAsync(in_buf(slot, w), host_bufs[w] + off, len * sizeof(int32_t),
                                   hipMemcpyHostToDevice, P.h2d[i]));
            chk(hipEventRecord(P.in_done[slot][i], P.h2d[i]));
            chk(hipStreamWaitEvent(cs, P.in_done[slot][i], 0));
        }
        // reduce: the slot's output is free once chunk k - kSlots was copied out
        if (k >= (size_t)kSlots) chk(hipStreamWaitEvent(cs, P.out_done[slot], 0));
        const int32_t* ptrs[INA_MAX_WORKERS];
        for (int w = 0; w < W; ++w) ptrs[w] = in_buf(slot, w);
        if (int rc = ina::sum_reduce_i32_impl(ptrs, W, out_buf(slot), len, stream, true)) {
            drain();
            return rc;
        }
        chk(hipEventRecord(P.red_done[slot], cs));
        // copy out
        chk(hipStreamWaitEvent(P.d2h, P.red_done[slot], 0));
        chk(hipMemcpyAsync(host_out + off, out_buf(slot), len * sizeof(int32_t),
                           hipMemcpyDeviceToHost, P.d2h));
        chk(hipEventRecord(P.out_done[slot], P.d2h));
    }
    if (!ok) {
        drain();
        return set_error(INA_EHIP, "host pipeline enqueue%s", "");
    }
    // synchronous: the aggregate is in host_out when this returns (the PS sends it next)
    if (hipStreamSynchronize(P.d2h) != hipSuccess || hipStreamSynchronize(cs) != hipSuccess)
        return set_error(INA_EHIP, "host pipeline sync%s", "");
    return INA_OK;
}

}  // extern "C"
