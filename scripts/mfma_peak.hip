// Sustained MFMA rate probe for the config-5 ceiling (BASELINE.md prices 1e7 x 4096 fp8 at
// 5 PF/s block-scaled, i.e. 2.4 GHz).  Every wave issues back-to-back MFMAs on register
// operands (4 independent accumulator chains, no memory traffic in the loop), one block of
// 8 waves per CU, and the kernel is timed with hipEvents: the FLOP/s it reaches is the chip's
// sustained rate for that instruction under its own power limit — the ceiling a memory-fed
// SYRK can approach, not exceed.
//
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak scripts/mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// RND: operands re-drawn every iteration (an LCG step per 32-bit word on the VALU, which
// co-issues with the MFMAs) — random fp8 bit patterns like real data toggle far more of the
// multiplier array than constant operands, and the power limit sees that
template <int KIND, bool RND = false>
__global__ __launch_bounds__(512) void mfma_loop(float* out, int iters, int seed) {
  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x16{};
  const int t = threadIdx.x + seed;
  if constexpr (KIND == 0) {  // block-scaled fp8 e4m3, K = 64 (the config-5 instruction)
    i32x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = 0x38383838 ^ (t * (i + 1)), b[i] = 0x30303030 ^ (t * (i + 3));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[c], 0, 0, 0, 127, 0, 127);
      if constexpr (RND) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          // keep every byte a finite e4m3 value (exponent field != 1111 with mantissa 111)
          a[i] = (int)(((unsigned)a[i] * 1664525u + 1013904223u) & 0x77777777u);
          b[i] = (int)(((unsigned)b[i] * 22695477u + 1u) & 0x77777777u);
        }
      }
    }
  } else {  // bf16, K = 16 (the headline / wide-bf16 instruction)
    bf16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (__bf16)(0.001f * (t + i)), b[i] = (__bf16)(0.002f * (t - i));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  if (s == 12345.678f) out[threadIdx.x] = s;  // keep the chains live
}

template <int KIND, bool RND = false>
static void run(const char* name, double flop_per_mfma, int cus, float* out) {
  const int iters = KIND == 0 ? 20000 : 40000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((mfma_loop<KIND, RND>), dim3(cus), dim3(512), 0, 0, out, 100, 0);  // warm
  CHECK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((mfma_loop<KIND, RND>), dim3(cus), dim3(512), 0, 0, out, iters, rep);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double mfmas = (double)cus * 8 /*waves*/ * iters * 4 /*chains*/;
    const double pf = mfmas * flop_per_mfma / (ms * 1e-3) / 1e15;
    printf("{\"instr\": \"%s\", \"ms\": %.3f, \"pflops\": %.3f, \"blocks\": %d}\n", name, ms, pf, cus);
    fflush(stdout);
  }
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  float* out;
  CHECK(hipMalloc(&out, 4096));
  run<0>("v_mfma_scale_f32_32x32x64_f8f6f4", 2.0 * 32 * 32 * 64, cus, out);
  run<0, true>("v_mfma_scale_f32_32x32x64_f8f6f4 random operands", 2.0 * 32 * 32 * 64, cus, out);
  run<1>("v_mfma_f32_32x32x16_bf16", 2.0 * 32 * 32 * 16, cus, out);
  CHECK(hipFree(out));
  return 0;
}
