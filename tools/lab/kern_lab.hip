// kern_lab.hip -- experiment harness (NOT product code): compiles the product kernels
// (csrc/ina_kernels.hip, included as-is) and exposes a launcher that runs a chosen
// kernel at a chosen grid so tools/lab/kern_lab.py can A/B geometries and variants in
// one process with interleaved timing.
#include "../../distributed-training-ina_amd/csrc/ina_kernels.hip"

extern "C" int lab_kern(int which, int grid, const void* const* bufs, int W, void* out,
                        size_t n, int V, void* ovf, void* stream) {
    using namespace ina;
    hipStream_t s = (hipStream_t)stream;
    float sc = 8192.0f;
    PtrPack<float> pk;
    for (int w = 0; w < INA_MAX_WORKERS; ++w) pk.p[w] = w < W ? (const float*)bufs[w] : nullptr;
    if (which == 0) {                                     // C4 int16 fused (row form), W = 16
        hipLaunchKernelGGL(k_quant_reduce_i16<16>, dim3(grid), dim3(kBlock), 0, s, pk, W,
                           (int16_t*)out, n, sc, V, V / 8, (uint8_t*)ovf);
    } else if (which == 2) {                              // C2 int32 fused, W = 4
        hipLaunchKernelGGL(k_quant_reduce_i32<4>, dim3(grid), dim3(kBlock), 0, s, pk, W,
                           (int32_t*)out, n, 65536.0f, 1);
    } else if (which == 3) {                              // quantise
        hipLaunchKernelGGL(k_quantize_i32, dim3(grid), dim3(kBlock), 0, s, (const float*)bufs[0],
                           (int32_t*)out, n, 65536.0f, 1);
    } else {
        return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
