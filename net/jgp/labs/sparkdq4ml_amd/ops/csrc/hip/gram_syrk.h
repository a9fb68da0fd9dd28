// K5-wide exact: LDS-tiled f64 / exact-f32 MFMA SYRK for d > 64 (see gram_syrk.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

struct SyrkArgs {
  const void* X;       // feature-major [d, ld] (f64 / f32 / bf16), 16-byte aligned feature rows
  int64_t ld;
  int d;
  int64_t n;
  int xdt;             // DType of X
  const double* y;     // label [n] f64
  const double* w;     // w_eff = weight * selection [n] f64, or null (all rows, unit weight)
  const int* pairs;    // [npair][2] upper panel pairs over the augmented [X | 1 | y]
  int npair;
  int splitk;
  double* part;        // [npair][splitk][128][128] f64 partial tiles
};

int syrk_panels(int d);                  // ceil((d + 2) / 128)
int64_t syrk_partials(int d, int splitk);
int64_t syrk_stages(int64_t n);          // 16-row stages
// compute_f64 = 1: v_mfma_f64_16x16x4_f64; 0: exact-f32 v_mfma_f32_32x32x2_f32.  Writes every
// entry of the flat WLS layout except out[0] (count) and out[2] (wwSum).
void gram_syrk(int compute_f64, SyrkArgs s, double* out, hipStream_t st);

}  // namespace dq4ml
