// Lab (experiment only): can a switch call hide the passes that exit at once on structured
// batches behind the run kernel?  The NGA-32 call is detection -> decision/digits -> buckets ->
// lists -> run, and on an in-order batch the middle three exit at once (~4.6 us each,
// profiles/r05/lab/detect_tail_v32.log).  Variants, each timed with HIP events on the main
// stream over K back-to-back calls:
//   serial    detection -> 3 exit-at-once passes -> run                   (the shipped order)
//   floor     detection -> run                                             (nothing in between)
//   forkjoin  main: detection, record e1, run, wait e2;
//             side: wait e1, 3 exit-at-once passes + an exit-at-once run, record e2
//   graph_*   the same captured once into a hipGraph and replayed
// The "detection" and "run" kernels are streaming stand-ins of the real kernels' bytes (85 MB and
// ~1.1 GB at NGA-32 C3 size), so the side stream's launches compete with a busy chip.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/forkjoin_lab tools/lab/forkjoin_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr size_t kNpk = 6553600;            // NGA-32 C3 packets

// detection stand-in: 8-byte descriptor in, 4-byte key + 1-byte action out per packet
__global__ __launch_bounds__(1024) void k_detect(const uint2* __restrict__ d, uint32_t* __restrict__ keys,
                                                 uint8_t* __restrict__ act, uint32_t* flag, uint32_t ep) {
    const size_t i0 = (size_t)blockIdx.x * 8192 + threadIdx.x;
    uint2 v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const size_t p = i0 + (size_t)r * 1024;
        v[r] = p < kNpk ? d[p] : uint2{0u, 0u};
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const size_t p = i0 + (size_t)r * 1024;
        if (p < kNpk) {
            keys[p] = v[r].x ^ v[r].y;
            act[p] = (uint8_t)v[r].x;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) flag[0] = ep;
}

// an exit-at-once pass: reads the control word, leaves (flag never equals want)
template <int kLdsWords>
__global__ __launch_bounds__(1024) void k_exit_1024(const uint32_t* flag, uint32_t want, uint32_t* sink) {
    __shared__ uint32_t s[kLdsWords];
    if (flag[0] != want) return;
    s[threadIdx.x % kLdsWords] = threadIdx.x;
    __syncthreads();
    sink[blockIdx.x] = s[(threadIdx.x + 1) % kLdsWords];
}
__global__ __launch_bounds__(256) void k_exit_256(const uint32_t* flag, uint32_t want, uint32_t* sink) {
    if (flag[0] != want) return;
    sink[blockIdx.x] = threadIdx.x;
}

// run stand-in: 144 B read per packet (header row + payload row), 1/8 of the payloads and the
// keys' words written back
__global__ __launch_bounds__(256) void k_run(const uint4* __restrict__ hdr, uint4* __restrict__ pay,
                                             const uint32_t* __restrict__ keys, uint32_t* flag, uint32_t want) {
    if (flag[0] == want + 1u) return;       // never
    const size_t p = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3);   // 8 lanes per packet
    const int l = threadIdx.x & 7;
    if (p >= kNpk) return;
    const uint4 h = hdr[p];
    uint4 a = pay[p * 8 + l];
    a.x += h.x + keys[p];
    if ((p & 7) == 7) pay[p * 8 + l] = a;
}

int main() {
    uint2* d;
    uint32_t *keys, *flag, *sink;
    uint8_t* act;
    uint4 *hdr, *pay;
    HK(hipMalloc(&d, kNpk * 8));
    HK(hipMalloc(&keys, kNpk * 4));
    HK(hipMalloc(&act, kNpk));
    HK(hipMalloc(&hdr, kNpk * 16));
    HK(hipMalloc(&pay, kNpk * 128));
    HK(hipMalloc(&flag, 256));
    HK(hipMalloc(&sink, 1 << 20));
    HK(hipMemset(d, 1, kNpk * 8));
    HK(hipMemset(hdr, 2, kNpk * 16));
    HK(hipMemset(pay, 3, kNpk * 128));
    HK(hipMemset(flag, 0, 256));
    hipStream_t s, side;
    HK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    hipEvent_t a, b, e1, e2;
    HK(hipEventCreate(&a));
    HK(hipEventCreate(&b));
    HK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    HK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    const unsigned gd = (unsigned)((kNpk + 8191) / 8192), gr = (unsigned)((kNpk + 31) / 32);
    const int K = 50;
    auto mids = [&](hipStream_t st) {
        hipLaunchKernelGGL(k_exit_1024<18432>, dim3(gd), dim3(1024), 0, st, flag, 0xFFFFFFFFu, sink);
        hipLaunchKernelGGL(k_exit_1024<13568>, dim3(1025), dim3(1024), 0, st, flag, 0xFFFFFFFFu, sink);
        hipLaunchKernelGGL(k_exit_256, dim3(1600), dim3(256), 0, st, flag, 0xFFFFFFFFu, sink);
    };
    auto call = [&](int mode, uint32_t i) -> hipError_t {
        hipLaunchKernelGGL(k_detect, dim3(gd), dim3(1024), 0, s, d, keys, act, flag, i);
        if (mode == 0) {                 // serial
            mids(s);
            hipLaunchKernelGGL(k_run, dim3(gr), dim3(256), 0, s, hdr, pay, keys, flag, 0u);
        } else if (mode == 1) {          // floor
            hipLaunchKernelGGL(k_run, dim3(gr), dim3(256), 0, s, hdr, pay, keys, flag, 0u);
        } else if (mode == 2) {          // fork / join
            hipError_t e;
            if ((e = hipEventRecord(e1, s)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(side, e1, 0)) != hipSuccess) return e;
            hipLaunchKernelGGL(k_run, dim3(gr), dim3(256), 0, s, hdr, pay, keys, flag, 0u);
            mids(side);
            hipLaunchKernelGGL(k_exit_256, dim3(gr), dim3(256), 0, side, flag, 0xFFFFFFFFu, sink);
            if ((e = hipEventRecord(e2, side)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(s, e2, 0)) != hipSuccess) return e;
        } else if (mode == 3) {          // run, then the passes after it on the same stream
            hipLaunchKernelGGL(k_run, dim3(gr), dim3(256), 0, s, hdr, pay, keys, flag, 0u);
            mids(s);
        }
        return hipGetLastError();
    };
    const char* names[] = {"serial", "floor", "forkjoin", "run_then_passes"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 4; ++mode) {
            for (int i = 0; i < 10; ++i) HK(call(mode, (uint32_t)i + 1));
            HK(hipEventRecord(a, s));
            for (int i = 0; i < K; ++i) HK(call(mode, (uint32_t)i + 1));
            HK(hipEventRecord(b, s));
            HK(hipEventSynchronize(b));
            float ms = 0;
            HK(hipEventElapsedTime(&ms, a, b));
            std::printf("rep %d %-16s %8.2f us per call\n", rep, names[mode], ms * 1e3f / K);
        }
        // the same calls captured into graphs (K calls per graph), replayed
        for (int mode = 0; mode < 3; ++mode) {
            hipGraph_t g;
            hipGraphExec_t ge;
            HK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < K; ++i) HK(call(mode, (uint32_t)i + 1));
            HK(hipStreamEndCapture(s, &g));
            HK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            HK(hipGraphLaunch(ge, s));
            HK(hipStreamSynchronize(s));
            HK(hipEventRecord(a, s));
            HK(hipGraphLaunch(ge, s));
            HK(hipEventRecord(b, s));
            HK(hipEventSynchronize(b));
            float ms = 0;
            HK(hipEventElapsedTime(&ms, a, b));
            std::printf("rep %d graph_%-10s %8.2f us per call\n", rep, names[mode], ms * 1e3f / K);
            HK(hipGraphExecDestroy(ge));
            HK(hipGraphDestroy(g));
        }
    }
    HK(hipDeviceSynchronize());
    std::printf("done\n");
    return 0;
}
