// K5 Gram / WLS-statistics kernels (see gram.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

enum GramMode : int { GRAM_F64 = 0, GRAM_F32 = 1, GRAM_BF16 = 2, GRAM_FP8 = 3 };

struct GramArgs {
  const void* X;       // feature-major [d, ld]
  int64_t ld;          // elements between consecutive features
  int d;
  int64_t n;
  int xdt;             // DType of X
  const void* y;       // label [n]
  int ydt;
  const void* w;       // weights [n] or null
  int wdt;
  const uint8_t* sel;  // selection [n] (bool) or null
  double* partials;    // [blocks][P]
  int P;
  int64_t spw;         // supersteps (64 rows) per wave
  int64_t nsuper;      // n / 64
};

int64_t gram_partial_stride(int mode, int d);
int gram_default_blocks(int64_t n);
// grid that exactly fills the chip for the kernel instantiation (occupancy-sized, persistent-style)
int gram_plan_blocks(int mode, int d, int64_t n, int xdt, int xmode);
// xmode: 0 = X already zero on dead rows (or no sel/w), 1 = binary mask from sel, 2 = general weights
void gram_tall(int mode, GramArgs a, int xmode, int blocks, double* out, hipStream_t st);

}  // namespace dq4ml
