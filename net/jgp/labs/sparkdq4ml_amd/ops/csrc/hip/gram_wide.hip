// K5-wide: LDS-tiled MFMA SYRK for d > 64 (BASELINE config 5: 1e7 rows x 4096 features, fp8).
//
// G = Xᵀ X over rows, upper 256x256 panel pairs only, split-K over row ranges.  MI355X design:
//  * storage is the MFMA-fragment-ordered tiling (ops/layout.py): for superstep s (64 rows),
//    32-feature tile t, k-step ki (16 rows) the 64 lanes' fragments are contiguous (16 B/lane for
//    bf16, 8 B/lane for fp8 e4m3 OCP).  A 256-feature panel of one superstep is therefore ONE
//    contiguous 32 KiB (bf16) / 16 KiB (fp8) block;
//  * each stage streams the A and B panels HBM -> LDS with global_load_lds (16 B per lane,
//    lane-linear — no VGPR staging, no swizzle needed because the image is already in fragment
//    order and every ds_read is lane-linear, i.e. conflict-free), double buffered;
//  * 8 waves (2 x 4) per 256x256 block, 128 x 64 per wave: 4 x 2 accumulators of
//    v_mfma_f32_32x32x16_{bf16,fp8_fp8}; per k-step 6 fragment reads feed 8 MFMAs;
//  * the label and the intercept column ride along as an "augmentation" panel [1, y_hi, y_lo]
//    (a 32-feature tile of its own), so count, Σy, Σy², Σx, Σxy all fall out of the same SYRK —
//    the augmented [X | 1 | y] Gram of SURVEY.md K5, without re-streaming X;
//  * per-column fp8 scales are applied in the f64 slab reduction (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include "common.h"
#include "gram_wide.h"

namespace dq4ml {

namespace {

constexpr int kWBlock = 512;
constexpr int kPanel = 256;        // features per panel
constexpr int kTilesPerPanel = 8;  // 32-feature tiles

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

template <int EB>
struct WideTraits;

template <>
struct WideTraits<16> {  // bf16
  typedef bf16x8 frag;
  static __device__ __forceinline__ frag read(const unsigned char* p) { return *reinterpret_cast<const frag*>(p); }
  static __device__ __forceinline__ f32x16 mfma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

template <>
struct WideTraits<8> {  // fp8 e4m3 (OCP)
  typedef long frag;
  static __device__ __forceinline__ frag read(const unsigned char* p) { return *reinterpret_cast<const long*>(p); }
  static __device__ __forceinline__ f32x16 mfma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
  }
};

// bytes of one (tile, k-step) chunk and of one panel per superstep
template <int EB>
constexpr int chunk_bytes() { return 64 * EB; }
template <int EB>
constexpr int panel_bytes() { return kTilesPerPanel * 4 * chunk_bytes<EB>(); }

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g),
                                   (__attribute__((address_space(3))) void*)(l), 16, 0, 0);
}

template <int EB>
__global__ __launch_bounds__(kWBlock, 1) void gram_wide_kernel(WideArgs a) {
  typedef WideTraits<EB> Tr;
  constexpr int PB = panel_bytes<EB>();
  constexpr int CB = chunk_bytes<EB>();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // 2 x 4 waves
  const int pair = blockIdx.x / a.splitk, split = blockIdx.x % a.splitk;
  const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
  const bool diag = I == J;
  const bool aug_a = I == a.npanels, aug_b = J == a.npanels;  // augmentation tile [1, y_hi, y_lo]
  const int64_t s0 = a.nsup * split / a.splitk, s1 = a.nsup * (split + 1) / a.splitk;

  // LDS images: A[b] at (2b) * PB, B[b] at (2b + 1) * PB
  auto bufA = [&](int b) { return smem + (size_t)(2 * b) * PB; };
  auto bufB = [&](int b) { return smem + (size_t)(2 * b + 1) * PB; };

  // stage loader: a data panel (8 tiles x 4 k-steps, contiguous) or the single augmentation tile
  auto issue_panel = [&](unsigned char* dst, int pidx, int64_t s) {
    if (pidx == a.npanels) {  // [1, y_hi, y_lo]: 1 tile x 4 k-steps; the other tiles stay zero
      const unsigned char* g = a.Xaug + (s * 4) * CB;
      if (tid * 16 < 4 * CB) glds16(g + tid * 16, dst + (wave * 64) * 16);
      return;
    }
    const unsigned char* g = a.X + ((s * a.NT + (int64_t)pidx * kTilesPerPanel) * 4) * CB;
#pragma unroll
    for (int r = 0; r < PB / (kWBlock * 16); ++r) glds16(g + (r * kWBlock + tid) * 16, dst + (r * kWBlock + wave * 64) * 16);
  };
  auto issue = [&](int64_t s, int b) {
    issue_panel(bufA(b), I, s);
    if (!diag) issue_panel(bufB(b), J, s);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // augmentation images: only tile 0 is ever loaded, zero the rest once
  for (int i = tid * 16; i < 2 * PB; i += kWBlock * 16) {
    if (aug_a) *reinterpret_cast<u32x4*>(bufA(i / PB) + (i % PB)) = u32x4{0u, 0u, 0u, 0u};
    if (aug_b && !diag) *reinterpret_cast<u32x4*>(bufB(i / PB) + (i % PB)) = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  const bool wave_active = (!aug_a || wm == 0) && (!aug_b || wn == 0);

  if (s0 < s1) {
    issue(s0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    for (int64_t s = s0; s < s1; ++s) {
      if (s + 1 < s1) issue(s + 1, cur ^ 1);
      const unsigned char* A = bufA(cur);
      const unsigned char* B = diag ? bufA(cur) : bufB(cur);
      if (wave_active) {
#pragma unroll
        for (int ki = 0; ki < 4; ++ki) {
          typename Tr::frag fa[4], fb[2];
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[i] = Tr::read(A + ((wm * 4 + i) * 4 + ki) * CB + lane * EB);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[j] = Tr::read(B + ((wn * 2 + j) * 4 + ki) * CB + lane * EB);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = Tr::mfma(fa[i], fb[j], acc[i][j]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      cur ^= 1;
    }
  }
  // f32 partial tile [256][256] of this (pair, split)
  float* out = a.part + (int64_t)blockIdx.x * kPanel * kPanel;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 128 + i * 32 + mfma32_row(lane, r);
        const int col = wn * 64 + j * 32 + mfma32_col(lane);
        out[row * kPanel + col] = acc[i][j][r];
      }
}

// f64 reduction of the split-K slabs, fp8 scales applied, straight into the flat WLS layout:
// [count, wSum, wwSum, bSum, bbSum, aSum(d), abSum(d), aa packed-upper(d)]
__device__ __forceinline__ double slab_sum(const WideArgs& a, int pair, int r, int c) {
  double s = 0.0;
  const float* p = a.part + (int64_t)pair * a.splitk * kPanel * kPanel + r * kPanel + c;
  for (int k = 0; k < a.splitk; ++k) s += (double)p[(int64_t)k * kPanel * kPanel];
  return s;
}

__device__ __forceinline__ int pair_index(int I, int J, int P) {
  // pairs listed row-major over I <= J in [0, P] (P = augmentation panel)
  return I * (P + 1) - I * (I - 1) / 2 + (J - I);
}

__global__ __launch_bounds__(256) void gram_wide_reduce_kernel(WideArgs a, const float* __restrict__ scales,
                                                              double* __restrict__ out) {
  const int d = a.d, P = a.npanels;
  const int64_t K = 5 + 2 * (int64_t)d + (int64_t)d * (d + 1) / 2;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += (int64_t)gridDim.x * blockDim.x) {
    const int pa = pair_index(P, P, P);
    const double s1 = a.aug_scale[0], syh = a.aug_scale[1], syl = a.aug_scale[2];
    double v;
    if (k < 5) {
      const double g11 = slab_sum(a, pa, 0, 0) * s1 * s1;
      const double g1h = slab_sum(a, pa, 0, 1) * s1 * syh, g1l = slab_sum(a, pa, 0, 2) * s1 * syl;
      const double ghh = slab_sum(a, pa, 1, 1) * syh * syh, ghl = slab_sum(a, pa, 1, 2) * syh * syl;
      const double gll = slab_sum(a, pa, 2, 2) * syl * syl;
      if (k <= 2) v = g11;                       // count, wSum, wwSum (unit weights; dead rows are zero)
      else if (k == 3) v = g1h + g1l;            // Σy
      else v = ghh + 2.0 * ghl + gll;            // Σy²
    } else if (k < 5 + 2 * (int64_t)d) {
      const int i = (int)((k - 5) % d);
      const bool xy = (k - 5) >= d;
      const int pi = pair_index(i / kPanel, P, P);
      const double si = scales ? (double)scales[i] : 1.0;
      if (!xy) v = slab_sum(a, pi, i % kPanel, 0) * si * s1;
      else v = slab_sum(a, pi, i % kPanel, 1) * si * syh + slab_sum(a, pi, i % kPanel, 2) * si * syl;
    } else {
      const int64_t kk = k - (5 + 2 * (int64_t)d);
      int64_t j = (int64_t)((sqrt(8.0 * (double)kk + 1.0) - 1.0) * 0.5);
      while (j * (j + 1) / 2 > kk) --j;
      while ((j + 1) * (j + 2) / 2 <= kk) ++j;
      const int64_t i = kk - j * (j + 1) / 2;
      const int pij = pair_index((int)(i / kPanel), (int)(j / kPanel), P);
      const double sc = scales ? (double)scales[i] * (double)scales[j] : 1.0;
      v = slab_sum(a, pij, (int)(i % kPanel), (int)(j % kPanel)) * sc;
    }
    out[k] = v;
  }
}

// ---- packing into the wide tiled layouts ----------------------------------------------------
// per-feature amax (for fp8 scales): one block per feature
__global__ __launch_bounds__(256) void amax_kernel(const PackSrcW* __restrict__ srcs, int64_t n,
                                                  const uint8_t* __restrict__ sel, float* __restrict__ amax) {
  const PackSrcW s = srcs[blockIdx.x];
  float m = 0.0f;
  for (int64_t r = threadIdx.x; r < n; r += blockDim.x) {
    if (sel && !sel[r]) continue;
    float v;
    switch (s.dt) {
      case DT_F64: v = (float)reinterpret_cast<const double*>(s.ptr)[r]; break;
      case DT_F32: v = reinterpret_cast<const float*>(s.ptr)[r]; break;
      case DT_BF16: v = bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(s.ptr)[r]); break;
      case DT_I32: v = (float)reinterpret_cast<const int32_t*>(s.ptr)[r]; break;
      default: v = 0.0f;
    }
    m = fmaxf(m, fabsf(v));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__device__ __forceinline__ float load_src(const PackSrcW& s, int64_t r) {
  switch (s.dt) {
    case DT_F64: return (float)reinterpret_cast<const double*>(s.ptr)[r];
    case DT_F32: return reinterpret_cast<const float*>(s.ptr)[r];
    case DT_BF16: return bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(s.ptr)[r]);
    case DT_I32: return (float)reinterpret_cast<const int32_t*>(s.ptr)[r];
    case DT_I64: return (float)reinterpret_cast<const int64_t*>(s.ptr)[r];
    default: return 0.0f;
  }
}

// columns -> fragment-ordered tiles (EB = 16: bf16, EB = 8: fp8 with 1/scale pre-multiplied)
template <int EB>
__global__ __launch_bounds__(256) void pack_wide_kernel(const PackSrcW* __restrict__ srcs, int d, int64_t n, int NT,
                                                       int64_t nsup, const uint8_t* __restrict__ sel,
                                                       const float* __restrict__ inv_scale,
                                                       unsigned char* __restrict__ out) {
  const int64_t nchunks = nsup * NT * 256;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const int ki = (int)((c >> 6) & 3);
    const int64_t st = c >> 8;
    const int t = (int)(st % NT);
    const int64_t s = st / NT;
    const int f = t * 32 + (lane & 31);
    const int64_t r = s * 64 + 16 * ki + 8 * (lane >> 5);
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x[j] = 0.0f;
      if (f < d && r + j < n && (sel == nullptr || sel[r + j])) x[j] = load_src(srcs[f], r + j);
    }
    if constexpr (EB == 16) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[j];
      reinterpret_cast<u32x4*>(out)[c] = __builtin_bit_cast(u32x4, v);
    } else {
      const float is = f < d ? inv_scale[f] : 0.0f;
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[0] * is, x[1] * is, 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[2] * is, x[3] * is, lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[4] * is, x[5] * is, 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[6] * is, x[7] * is, hi, true);
      reinterpret_cast<u32x2*>(out)[c] = u32x2{(unsigned)lo, (unsigned)hi};
    }
  }
}

}  // namespace

int64_t wide_tiled_bytes(int eb, int d, int64_t n) {
  const int NT = ((d + 255) / 256) * 8;
  return ((n + 63) / 64) * NT * 4 * 64 * (int64_t)eb;
}

void feature_amax(const PackSrcW* srcs_dev, int d, int64_t n, const uint8_t* sel, float* amax, hipStream_t st) {
  hipLaunchKernelGGL(amax_kernel, dim3(d), dim3(256), 0, st, srcs_dev, n, sel, amax);
  DQ_HIP_CHECK(hipGetLastError());
}

void pack_wide(int eb, const PackSrcW* srcs_dev, int d, int64_t n, int nt, const uint8_t* sel, const float* inv_scale,
               void* out, hipStream_t st) {
  const int64_t nsup = (n + 63) / 64;
  int64_t g = (nsup * nt * 256 + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  unsigned char* o = reinterpret_cast<unsigned char*>(out);
  if (eb == 16) hipLaunchKernelGGL(pack_wide_kernel<16>, dim3(g), dim3(256), 0, st, srcs_dev, d, n, nt, nsup, sel, inv_scale, o);
  else hipLaunchKernelGGL(pack_wide_kernel<8>, dim3(g), dim3(256), 0, st, srcs_dev, d, n, nt, nsup, sel, inv_scale, o);
  DQ_HIP_CHECK(hipGetLastError());
}

int64_t gram_wide_partials(int d, int splitk) {
  const int P = (d + kPanel - 1) / kPanel;
  const int npair = (P + 1) * (P + 2) / 2;
  return (int64_t)npair * splitk * kPanel * kPanel;
}

void gram_wide(int eb, WideArgs a, const int* pairs_dev, const float* scales, double* out, hipStream_t st) {
  a.pairs = pairs_dev;
  const int P = a.npanels;
  const int npair = (P + 1) * (P + 2) / 2;
  const size_t lds = 4 * (size_t)(eb == 16 ? panel_bytes<16>() : panel_bytes<8>());
  if (eb == 16) {
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(gram_wide_kernel<16>, dim3(npair * a.splitk), dim3(kWBlock), lds, st, a);
  } else {
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(gram_wide_kernel<8>, dim3(npair * a.splitk), dim3(kWBlock), lds, st, a);
  }
  DQ_HIP_CHECK(hipGetLastError());
  const int64_t K = 5 + 2 * (int64_t)a.d + (int64_t)a.d * (a.d + 1) / 2;
  int64_t g = (K + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(gram_wide_reduce_kernel, dim3(g), dim3(256), 0, st, a, scales, out);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
