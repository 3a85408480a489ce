// ina_internal.h -- shared between the libina.so translation units (not installed).
#pragma once
#include <cstddef>
#include <cstdint>

#include "ina.h"

namespace ina {

// W device pointers passed by value in the kernel arguments (512 B at W_max = 64)
template <typename T>
struct PtrPack {
    const T* p[INA_MAX_WORKERS];
};

int set_error(int code, const char* fmt, const char* detail);
int set_h2d_streams(int v);   // ina_host.cpp
int set_zero_copy(int v);     // ina_host.cpp
int sum_reduce_i32_impl(const int32_t* const* bufs, int W, int32_t* out, size_t n, ina_stream_t stream,
                        bool host);   // ina_kernels.hip
int set_small_sort(int v);    // ina_switch.hip
int set_switch_win(int v);    // ina_switch.hip
int set_ack_fast(int v);      // ina_switch.hip
int set_sort_mode(int v);     // ina_switch.hip
int set_os_rounds(int v);     // ina_switch.hip
int set_tiny_max(int v);      // ina_switch.hip
int set_bucket_tile(int v);   // ina_switch.hip
int set_runs(int v);          // ina_switch.hip
int set_pre_all(int v);       // ina_switch.hip
int set_local(int v);         // ina_switch.hip
int set_decide_delay(int v);  // ina_switch.hip
int ew_grid_cap();            // ina_kernels.hip: grid cap of the elementwise kernels (tuning key 14)
// checked builds (INA_STORE_CHECK, ina_device.h): each source's stream_store contract
// violations since the last read, cleared by the read
unsigned long long store_violations_kernels();   // ina_kernels.hip
unsigned long long store_violations_shard();     // ina_shard.hip
unsigned long long store_violations_switch();    // ina_switch.hip

}  // namespace ina

extern "C" int ina_set_tuning(int key, int value);
