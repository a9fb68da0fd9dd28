// K5-wide: LDS-tiled MFMA SYRK for d > 64 (see gram_wide.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

int64_t gram_wide_workspace(int mode, int d, int64_t n);
void gram_wide(int mode, const void* X, int64_t ld, int d, int64_t n, int xdt, const float* scales, void* ws,
               int64_t ws_bytes, double* out_full, hipStream_t st);

}  // namespace dq4ml
