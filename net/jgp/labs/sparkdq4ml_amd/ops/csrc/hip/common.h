// Shared helpers for the dq4ml gfx950 kernels.
#pragma once
#ifndef __HIPCC_RTC__  // (hipRTC builds of the kernels take only the device parts below)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#endif

namespace dq4ml {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((ext_vector_type(2))) double f64x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;

constexpr int kWave = 64;  // CDNA wavefront

#ifndef __HIPCC_RTC__
#define DQ_HIP_CHECK(expr)                                                                          \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
#endif

// dtype codes shared with the python side (ops/device.py)
enum DType : int { DT_F64 = 0, DT_F32 = 1, DT_BF16 = 2, DT_I32 = 3, DT_I64 = 4, DT_U8 = 5, DT_F16 = 6, DT_FP8 = 7 };

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) { return __uint_as_float(uint32_t(b) << 16); }

// Generic pointers that reach a kernel through a descriptor table compile to FLAT loads, which
// count on lgkmcnt too — every LDS wait/barrier would then drain the prefetch.  All descriptor
// pointers point at device global memory: load through the global address space.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gptr(const void* p) {
  return (const __attribute__((address_space(1))) T*)(p);
}

// 8 consecutive elements [r0, r0+8) of a typed column as f32 (zero past n); 16-byte vector loads
// when the run is complete and aligned (r0 is a multiple of 8 in every caller)
__device__ __forceinline__ void load8_f32(const void* p, int dt, int64_t r0, int64_t n, float x[8]) {
  const bool full = r0 + 8 <= n && ((reinterpret_cast<uintptr_t>(p) & 15) == 0);
  if (full && dt == DT_F32) {
    const f32x4 a = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0);
    const f32x4 b = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = a[j], x[4 + j] = b[j];
    return;
  }
  if (full && dt == DT_F64) {
    const double* q = reinterpret_cast<const double*>(p) + r0;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f64x2 v = *gptr<f64x2>(q + j);
      x[j] = (float)v[0], x[j + 1] = (float)v[1];
    }
    return;
  }
  if (full && dt == DT_BF16) {
    const u32x4 v = *gptr<u32x4>(reinterpret_cast<const uint16_t*>(p) + r0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = __uint_as_float(v[j] << 16);
      x[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t r = r0 + j;
    float v = 0.0f;
    if (r < n) {
      switch (dt) {
        case DT_F64: v = (float)gptr<double>(p)[r]; break;
        case DT_F32: v = gptr<float>(p)[r]; break;
        case DT_BF16: v = bf16_bits_to_f32(gptr<uint16_t>(p)[r]); break;
        case DT_I32: v = (float)gptr<int32_t>(p)[r]; break;
        case DT_I64: v = (float)gptr<int64_t>(p)[r]; break;
        case DT_U8: v = (float)gptr<uint8_t>(p)[r]; break;
        default: v = 0.0f;
      }
    }
    x[j] = v;
  }
}

// Typed variant for kernels specialized on one source dtype (no per-element switch, no alignment
// test: the host guarantees 16-byte aligned columns).  Only the ragged last 8 rows take the
// guarded scalar path.
template <int SDT, bool FULL = false>
__device__ __forceinline__ void load8_typed(const void* p, int64_t r0, int64_t n, float x[8]) {
  if (FULL || r0 + 8 <= n) {
    if constexpr (SDT == DT_F32) {
      const f32x4 a = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0);
      const f32x4 b = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = a[j], x[4 + j] = b[j];
    } else if constexpr (SDT == DT_F64) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f64x2 v = *gptr<f64x2>(reinterpret_cast<const double*>(p) + r0 + j);
        x[j] = (float)v[0], x[j + 1] = (float)v[1];
      }
    } else {
      const u32x4 v = *gptr<u32x4>(reinterpret_cast<const uint16_t*>(p) + r0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = __uint_as_float(v[j] << 16);
        x[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t r = r0 + j;
    float v = 0.0f;
    if (r < n) {
      if constexpr (SDT == DT_F32) v = gptr<float>(p)[r];
      else if constexpr (SDT == DT_F64) v = (float)gptr<double>(p)[r];
      else v = bf16_bits_to_f32(gptr<uint16_t>(p)[r]);
    }
    x[j] = v;
  }
}

// x[j] -= s for the rows r0 + j < n (rows past the end stay exactly 0): the per-feature shift
// applied before a low-precision cast (GramArgs::xshift)
__device__ __forceinline__ void sub_shift8(float x[8], float s, int64_t r0, int64_t n) {
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (r0 + j < n) x[j] -= s;
}

// zero the elements of x whose row is dead in the 0/1 selection (one 8-byte load when possible)
__device__ __forceinline__ void mask8(const uint8_t* sel, int64_t r0, int64_t n, float x[8]) {
  if (sel == nullptr) return;
  if (r0 + 8 <= n && ((reinterpret_cast<uintptr_t>(sel + r0) & 7) == 0)) {
    const uint64_t m = *gptr<uint64_t>(sel + r0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (((m >> (8 * j)) & 0xff) == 0) x[j] = 0.0f;
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (r0 + j >= n || gptr<uint8_t>(sel)[r0 + j] == 0) x[j] = 0.0f;
}

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

// Grid-wide barrier of a plain launch whose blocks are co-resident (at most one block per CU, as
// the launchers size it).  bar = [arrivals, abandoned], zeroed by a stream-ordered memset before
// the launch; gen counts the barriers this block has passed (thread 0's copy).  Writes before the
// barrier are released at agent scope (L2 write-back across the XCDs) and acquired after it.  A
// wait longer than kGridSpin polls (seconds) marks the barrier abandoned: every later barrier of
// the launch passes at once, the kernel drains, and the launcher's status word reports it.
// (hipLaunchCooperativeKernel gave the same guarantee through a dedicated runtime queue whose
// teardown crashed rocprofv3 at process exit: profiles/r6_coop_exit.md.)
constexpr unsigned kGridSpin = 1u << 22;

__device__ __forceinline__ void grid_barrier(unsigned* bar, unsigned& gen, unsigned nblocks) {
  __threadfence();  // release: every thread's writes (the fence's L2 write-back), then the arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned target = ++gen * nblocks;
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // relaxed polls: an acquiring load would invalidate the XCD's L2 on every poll, under the
    // blocks of that XCD still re-reading their tiles from it (the l-bfgs pass: 9.30 ms per
    // evaluation with acquiring polls)
    for (unsigned it = 0; __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++it) {
      if (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
      if (it >= kGridSpin) {
        __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // once, after the wait
}

__device__ __forceinline__ bool grid_abandoned(const unsigned* bar) {
  return __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

}  // namespace dq4ml
