// Fused DQ kernels: runtime code generation of Project/Filter chains (see dqvm.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace dq4ml {

// Compile HIP source (one extern "C" kernel named `entry`) for gfx950 with hipRTC; returns an
// opaque handle.  Compiled code objects are cached by source text for the life of the process.
int64_t rtc_compile(const std::string& src, const std::string& entry, std::string* log);
// the module function of a compiled handle (launched by a typed host wrapper, e.g. gram_stream_rtc)
void* rtc_function(int64_t handle);
// kernel signature (void* const* ptrs, long long n): a device pointer table
void rtc_launch(int64_t handle, int grid, int block, void* const* ptrs_dev, int64_t n, hipStream_t st);
// kernel signature (DqPtrs ptrs, long long n), DqPtrs = { void* v[nptr]; } passed BY VALUE in the
// kernel-argument segment: the host array is copied into it at the launch (no device table)
void rtc_launch_args(int64_t handle, int grid, int block, const int64_t* ptrs_host, int nptr, int64_t n, hipStream_t st);

}  // namespace dq4ml
