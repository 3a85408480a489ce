// Lab (experiment only): what an early-exit launch costs on gfx950.  The switch launches its
// decision and bucket passes on every batch and they exit at once on structured arrival, so
// their cost is paid by every in-order / run-table batch.  Each variant: a producer launch
// that writes a flag (like the detection pass writing the control block), then K consumer
// launches that read it and exit, back to back on one stream; HIP events, per consumer launch.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/empty_lab tools/lab/empty_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_produce(uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) flag[0] = v;
}

// exits when flag[0] != want (the structured batch's case)
template <int kLds>
__global__ __launch_bounds__(1024) void k_exit_1024(const uint32_t* flag, uint32_t want, uint32_t* sink) {
    __shared__ uint32_t s[kLds / 4 > 0 ? kLds / 4 : 1];
    if (flag[0] != want) return;
    s[threadIdx.x % (kLds / 4 > 0 ? kLds / 4 : 1)] = threadIdx.x;
    __syncthreads();
    sink[blockIdx.x] = s[(threadIdx.x + 1) % (kLds / 4 > 0 ? kLds / 4 : 1)];
}

__global__ __launch_bounds__(256) void k_exit_256(const uint32_t* flag, uint32_t want, uint32_t* sink) {
    if (flag[0] != want) return;
    sink[blockIdx.x] = threadIdx.x;
}

__global__ __launch_bounds__(256) void k_noread_256(uint32_t* sink, int never) {
    if (never) sink[blockIdx.x] = threadIdx.x;
}

int main() {
    uint32_t *flag, *sink;
    HK(hipMalloc(&flag, 256));
    HK(hipMalloc(&sink, 1 << 20));
    hipStream_t s;
    HK(hipStreamCreate(&s));
    hipEvent_t a, b;
    HK(hipEventCreate(&a));
    HK(hipEventCreate(&b));
    const int K = 200;
    struct V { const char* name; int kind; unsigned grid; };
    std::vector<V> vs = {
        {"produce only (1 block)", 0, 1},
        {"exit_1024 grid 257, LDS 0", 1, 257},
        {"exit_1024 grid 257, LDS 64 KiB", 2, 257},
        {"exit_1024 grid 800, LDS 72 KiB", 3, 800},
        {"exit_256 grid 1600", 4, 1600},
        {"exit_256 grid 256", 5, 256},
        {"noread_256 grid 1600", 6, 1600},
        {"noread_256 grid 1", 7, 1},
    };
    for (int rep = 0; rep < 2; ++rep) {
        for (const V& v : vs) {
            auto launch = [&](int i) {
                hipLaunchKernelGGL(k_produce, dim3(1), dim3(64), 0, s, flag, (uint32_t)i);
                switch (v.kind) {
                    case 1: hipLaunchKernelGGL(k_exit_1024<0>, dim3(v.grid), dim3(1024), 0, s, flag, 0xFFFFFFFFu, sink); break;
                    case 2: hipLaunchKernelGGL(k_exit_1024<65536>, dim3(v.grid), dim3(1024), 0, s, flag, 0xFFFFFFFFu, sink); break;
                    case 3: hipLaunchKernelGGL(k_exit_1024<73728>, dim3(v.grid), dim3(1024), 0, s, flag, 0xFFFFFFFFu, sink); break;
                    case 4: case 5: hipLaunchKernelGGL(k_exit_256, dim3(v.grid), dim3(256), 0, s, flag, 0xFFFFFFFFu, sink); break;
                    case 6: case 7: hipLaunchKernelGGL(k_noread_256, dim3(v.grid), dim3(256), 0, s, sink, 0); break;
                    default: break;
                }
            };
            for (int i = 0; i < 20; ++i) launch(i);
            HK(hipEventRecord(a, s));
            for (int i = 0; i < K; ++i) launch(i);
            HK(hipEventRecord(b, s));
            HK(hipEventSynchronize(b));
            float ms = 0;
            HK(hipEventElapsedTime(&ms, a, b));
            if (rep == 1) std::printf("%-34s %7.2f us per (producer + consumer)\n", v.name, ms * 1e3f / K);
        }
    }
    return 0;
}
