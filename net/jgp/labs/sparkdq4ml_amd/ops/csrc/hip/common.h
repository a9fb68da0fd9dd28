// Shared helpers for the dq4ml gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace dq4ml {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((ext_vector_type(2))) double f64x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int kWave = 64;  // CDNA wavefront

#define DQ_HIP_CHECK(expr)                                                                          \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// dtype codes shared with the python side (ops/device.py)
enum DType : int { DT_F64 = 0, DT_F32 = 1, DT_BF16 = 2, DT_I32 = 3, DT_I64 = 4, DT_U8 = 5, DT_F16 = 6, DT_FP8 = 7 };

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) { return __uint_as_float(uint32_t(b) << 16); }

// 32x32 MFMA accumulator (f32, 16 regs): element reg of lane -> (row, col)
__device__ __forceinline__ int mfma32_row(int lane, int reg) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ int mfma32_col(int lane) { return lane & 31; }
// f64 16x16x4 accumulator (4 regs)
__device__ __forceinline__ int mfma16d_row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
__device__ __forceinline__ int mfma16d_col(int lane) { return lane & 15; }

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace dq4ml
