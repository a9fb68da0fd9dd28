// K5-wide exact: LDS-tiled MFMA SYRK for d > 64 at Spark precision (fp64) or exact f32.
//
// The default LinearRegression statistics (gramDtype = fp64) and the fp32 request for any
// 64 < numFeatures <= 4096 (the WLS branch of LinearRegression.fit, reference
// DataQuality4MachineLearningApp.java:126), weighted and DQ-filtered, without a library GEMM:
//
//  * the augmented matrix Z = [X | 1 | y] (p = d + 2 features; the two virtual features are
//    generated in the load path) is cut into 128-feature panels; one block computes the 128 x 128
//    tile of Zᵀ·diag(w)·Z for one upper panel pair (I <= J) over one row range (split-K), so the
//    whole augmented Gram -- count-free sums Σw, Σwy, Σwy², Σw·x, Σw·x·y and the packed upper
//    Σw·x·xᵀ -- comes out of ONE pass over X;
//  * weights and the DQ selection are one f64 row factor w_eff = w·sel (null = 1) applied to the
//    A operand at staging time; rows with w_eff == 0 are zeroed in BOTH operands (Spark's
//    WeightedLeastSquares aggregator skips zero-weight rows, so a NaN there must not leak in);
//  * COMPUTE = double: v_mfma_f64_16x16x4_f64 (4 x 4 tiles of 16 x 16 per wave, f64 accumulate);
//    COMPUTE = float: v_mfma_f32_32x32x2_f32, the exact-f32 MFMA (k-ordered fmaf chain, 2 x 2
//    tiles of 32 x 32 per wave), partials widened to f64;
//  * stages of 16 rows are register-staged (16-byte global loads, convert + weight, ds_write) into
//    a double-buffered LDS image [panel][feature][row] whose feature rows are padded (f64: 18
//    doubles = 144 B, f32: 17 floats) so every MFMA fragment read is bank-conflict free; the next
//    stage's global loads are in flight under the current stage's MFMAs (one barrier per stage);
//  * blockIdx -> (split, pair) is XCD-aware (bijective remap): the blocks an XCD runs together
//    work on the same row range, so the panels they share come from that XCD's L2;
//  * f64 split-K partial tiles, then a coalesced reduction straight into the flat WLS layout.
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "common.h"
#include "gram_syrk.h"

namespace dq4ml {

namespace {

constexpr int kPanel = 128;     // features per panel = block tile edge
constexpr int kSR = 16;         // rows per stage
constexpr int kThreads = 256;   // 4 waves, 2 x 2, 64 x 64 outputs each

template <typename C>
struct SyrkT;

template <>
struct SyrkT<double> {  // v_mfma_f64_16x16x4_f64: A[l&15][k=l>>4], C row (l>>4)+4r, col l&15
  static constexpr int kTile = 16, kK = 4, kRS = 18;
  typedef f64x4 acc_t;
  static constexpr int kAcc = 4;
  static __device__ __forceinline__ acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int crow(int lane, int r) { return (lane >> 4) + 4 * r; }
  static __device__ __forceinline__ int ccol(int lane) { return lane & 15; }
};

template <>
struct SyrkT<float> {  // v_mfma_f32_32x32x2_f32: A[l&31][k=l>>5], C = the 32x32 map
  static constexpr int kTile = 32, kK = 2, kRS = 17;
  typedef f32x16 acc_t;
  static constexpr int kAcc = 16;
  static __device__ __forceinline__ acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int crow(int lane, int r) { return mfma32_row(lane, r); }
  static __device__ __forceinline__ int ccol(int lane) { return lane & 31; }
};

// 8 consecutive rows [r0, r0 + 8) of one feature of X (SDT) as COMPUTE values, zero past n
template <typename C, int SDT>
__device__ __forceinline__ void load8(const void* p, int64_t r0, int64_t n, C v[8]) {
  if (r0 + 8 <= n) {
    if constexpr (SDT == DT_F64) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f64x2 q = *gptr<f64x2>(reinterpret_cast<const double*>(p) + r0 + j);
        v[j] = (C)q[0], v[j + 1] = (C)q[1];
      }
    } else if constexpr (SDT == DT_F32) {
      const f32x4 a = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0);
      const f32x4 b = *gptr<f32x4>(reinterpret_cast<const float*>(p) + r0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (C)a[j], v[4 + j] = (C)b[j];
    } else {  // bf16
      const u32x4 q = *gptr<u32x4>(reinterpret_cast<const uint16_t*>(p) + r0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[2 * j] = (C)__uint_as_float(q[j] << 16);
        v[2 * j + 1] = (C)__uint_as_float(q[j] & 0xffff0000u);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t r = r0 + j;
    C x = (C)0;
    if (r < n) {
      if constexpr (SDT == DT_F64) x = (C)gptr<double>(p)[r];
      else if constexpr (SDT == DT_F32) x = (C)gptr<float>(p)[r];
      else x = (C)bf16_bits_to_f32(gptr<uint16_t>(p)[r]);
    }
    v[j] = x;
  }
}

__device__ __forceinline__ void load8_w(const double* w, int64_t r0, int64_t n, double v[8]) {
  if (r0 + 8 <= n) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f64x2 q = *gptr<f64x2>(w + r0 + j);
      v[j] = q[0], v[j + 1] = q[1];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = r0 + j < n ? gptr<double>(w)[r0 + j] : 0.0;
}

// One thread stages 8 rows of one feature of panel A and of panel B (plus their 8 weights)
template <typename C, int SDT>
struct Staged {
  C a[8], b[8];
};

template <typename C, int SDT, bool HAS_W, bool THIN>
__device__ __forceinline__ void stage_load(const SyrkArgs& s, int I, int J, int64_t r0, Staged<C, SDT>& st) {
  const int fi = threadIdx.x >> 1;
  const int64_t row = r0 + (threadIdx.x & 1) * 8;
  auto feat = [&](int f, C v[8]) {
    if (f < s.d) {
      load8<C, SDT>(reinterpret_cast<const unsigned char*>(s.X) + (int64_t)f * s.ld * (SDT == DT_F64 ? 8 : SDT == DT_F32 ? 4 : 2),
                    row, s.n, v);
    } else if (f == s.d) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = row + j < s.n ? (C)1 : (C)0;
    } else if (f == s.d + 1) {
      load8<C, DT_F64>(s.y, row, s.n, v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (C)0;
    }
  };
  feat(I * kPanel + fi, st.a);
  if (!THIN || fi < SyrkT<C>::kTile) feat(J * kPanel + fi, st.b);  // a thin panel: one MFMA tile of features
  if constexpr (HAS_W) {
    double w[8];
    load8_w(s.w, row, s.n, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool live = w[j] != 0.0;
      st.a[j] = live ? (C)((double)st.a[j] * w[j]) : (C)0;
      st.b[j] = live ? st.b[j] : (C)0;
    }
  }
}

template <typename C, int SDT, bool THIN>
__device__ __forceinline__ void stage_store(C* lds, const Staged<C, SDT>& st) {
  typedef SyrkT<C> T;
  const int fi = threadIdx.x >> 1, h = threadIdx.x & 1;
  C* A = lds + fi * T::kRS + h * 8;
  C* B = lds + kPanel * T::kRS + fi * T::kRS + h * 8;
  const bool wb = !THIN || fi < T::kTile;
  if constexpr (sizeof(C) == 8) {  // 144-B feature rows: 16-B aligned runs
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      *reinterpret_cast<f64x2*>(A + j) = f64x2{st.a[j], st.a[j + 1]};
      if (wb) *reinterpret_cast<f64x2*>(B + j) = f64x2{st.b[j], st.b[j + 1]};
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      A[j] = st.a[j];
      if (wb) B[j] = st.b[j];
    }
  }
}

// THIN: panel J holds at most one MFMA tile of live features (the augmentation columns [1, y]
// spilling past the last full data panel, e.g. d = 256 / 1024 / 4096): only the waves of the
// first column half compute, one tile column each -- such pairs cost ~1/8 of a full one instead
// of a full 128 x 128 tile of zeros.
template <typename C, int SDT, bool HAS_W, bool THIN>
__device__ __forceinline__ void syrk_body(const SyrkArgs& s, C* lds, int I, int J, int pair, int split) {
  typedef SyrkT<C> T;
  constexpr int TW = 64 / T::kTile;                   // MFMA tiles per wave edge
  constexpr int TWN = THIN ? 1 : TW;                  // tile columns computed per wave
  constexpr int kBuf = 2 * kPanel * T::kRS;           // elements of one stage (A + B)
  const int64_t nst = (s.n + kSR - 1) / kSR;
  const int64_t st0 = nst * split / s.splitk, st1 = nst * (split + 1) / s.splitk;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;

  typename T::acc_t acc[TW][TW];
#pragma unroll
  for (int x = 0; x < TW; ++x)
#pragma unroll
    for (int y = 0; y < TW; ++y) acc[x][y] = typename T::acc_t{};

  const bool computes = !THIN || wn == 0;
  if (st0 < st1) {
    Staged<C, SDT> reg;
    stage_load<C, SDT, HAS_W, THIN>(s, I, J, st0 * kSR, reg);
    stage_store<C, SDT, THIN>(lds, reg);
    __syncthreads();
    int cur = 0;
    const int fr = lane & (T::kTile - 1), kr = lane / T::kTile;
    for (int64_t st = st0; st < st1; ++st) {
      const bool more = st + 1 < st1;
      if (more) stage_load<C, SDT, HAS_W, THIN>(s, I, J, (st + 1) * kSR, reg);  // in flight under the MFMAs
      const C* A = lds + cur * kBuf + (wm * 64 + fr) * T::kRS + kr;
      const C* B = lds + cur * kBuf + kPanel * T::kRS + (wn * 64 + fr) * T::kRS + kr;
      if (computes) {
#pragma unroll
        for (int k0 = 0; k0 < kSR; k0 += T::kK) {
          C a[TW], b[TWN];
#pragma unroll
          for (int x = 0; x < TW; ++x) a[x] = A[x * T::kTile * T::kRS + k0];
#pragma unroll
          for (int y = 0; y < TWN; ++y) b[y] = B[y * T::kTile * T::kRS + k0];
#pragma unroll
          for (int x = 0; x < TW; ++x)
#pragma unroll
            for (int y = 0; y < TWN; ++y) acc[x][y] = T::mfma(a[x], b[y], acc[x][y]);
        }
      }
      if (more) stage_store<C, SDT, THIN>(lds + (cur ^ 1) * kBuf, reg);
      __syncthreads();
      cur ^= 1;
    }
  }
  // f64 partial tile [128][128] of this (pair, split)
  double* out = s.part + ((int64_t)pair * s.splitk + split) * kPanel * kPanel;
#pragma unroll
  for (int x = 0; x < TW; ++x)
#pragma unroll
    for (int y = 0; y < TW; ++y)
#pragma unroll
      for (int r = 0; r < T::kAcc; ++r) {
        const int row = wm * 64 + x * T::kTile + T::crow(lane, r);
        const int col = wn * 64 + y * T::kTile + T::ccol(lane);
        out[row * kPanel + col] = (double)acc[x][y][r];
      }
}

template <typename C, int SDT, bool HAS_W>
__global__ __launch_bounds__(kThreads, 2) void syrk_kernel(SyrkArgs s) {
  typedef SyrkT<C> T;
  __shared__ __attribute__((aligned(16))) C lds[2 * 2 * kPanel * T::kRS];
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rem = nwg & 7;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
  const int split = L / s.npair, pair = L - split * s.npair;
  const int I = s.pairs[2 * pair], J = s.pairs[2 * pair + 1];
  if (s.d + 2 - J * kPanel <= T::kTile) syrk_body<C, SDT, HAS_W, true>(s, lds, I, J, pair, split);
  else syrk_body<C, SDT, HAS_W, false>(s, lds, I, J, pair, split);
}

// split-K fold + scatter of the augmented Gram into [count, wSum, wwSum, bSum, bbSum, aSum(d),
// abSum(d), aa packed-upper(d)]; count and wwSum are not Gram entries (the caller fills them).
// Storage-order walk: thread = one (pair, row, col) element, the splits of consecutive threads
// are consecutive doubles.
__global__ __launch_bounds__(256) void syrk_reduce_kernel(SyrkArgs s, double* __restrict__ out) {
  const int d = s.d;
  const int64_t slab = (int64_t)kPanel * kPanel;
  const int64_t tot = (int64_t)s.npair * slab;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < tot; g += (int64_t)gridDim.x * blockDim.x) {
    const int pr = (int)(g / slab);
    const int e = (int)(g - (int64_t)pr * slab);
    const int i = s.pairs[2 * pr] * kPanel + (e >> 7), j = s.pairs[2 * pr + 1] * kPanel + (e & (kPanel - 1));
    if (i > j || j >= d + 2) continue;
    const double* base = s.part + (int64_t)pr * s.splitk * slab + e;
    double v = 0.0;
    for (int k = 0; k < s.splitk; ++k) v += base[(int64_t)k * slab];
    if (j < d) out[5 + 2 * (int64_t)d + i + (int64_t)j * (j + 1) / 2] = v;
    else if (i < d) out[(j == d ? 5 : 5 + d) + i] = v;             // Σw·x, Σw·x·y
    else if (i == d) out[j == d ? 1 : 3] = v;                        // Σw, Σw·y
    else out[4] = v;                                                 // Σw·y²
  }
}

template <typename C, int SDT, bool HAS_W>
void launch(const SyrkArgs& s, hipStream_t st) {
  hipLaunchKernelGGL((syrk_kernel<C, SDT, HAS_W>), dim3(s.npair * s.splitk), dim3(kThreads), 0, st, s);
}

template <typename C, int SDT>
void launch_w(const SyrkArgs& s, hipStream_t st) {
  if (s.w) launch<C, SDT, true>(s, st);
  else launch<C, SDT, false>(s, st);
}

template <typename C>
void launch_dt(const SyrkArgs& s, hipStream_t st) {
  switch (s.xdt) {
    case DT_F64: return launch_w<C, DT_F64>(s, st);
    case DT_F32: return launch_w<C, DT_F32>(s, st);
    case DT_BF16: return launch_w<C, DT_BF16>(s, st);
    default: throw std::invalid_argument("gram_syrk: X must be f64, f32 or bf16");
  }
}

}  // namespace

int syrk_panels(int d) { return (d + 2 + kPanel - 1) / kPanel; }

int64_t syrk_partials(int d, int splitk) {
  const int P = syrk_panels(d);
  return (int64_t)P * (P + 1) / 2 * splitk * kPanel * kPanel;
}

int64_t syrk_stages(int64_t n) { return (n + kSR - 1) / kSR; }

void gram_syrk(int compute_f64, SyrkArgs s, double* out, hipStream_t st) {
  const int P = syrk_panels(s.d);
  if (s.npair != P * (P + 1) / 2) throw std::invalid_argument("gram_syrk: npair must cover the upper panel pairs");
  if (s.splitk < 1 || s.splitk > syrk_stages(s.n) || (int64_t)s.npair * s.splitk > (1LL << 31) - 1)
    throw std::invalid_argument("gram_syrk: bad splitk");
  if (s.xdt == DT_F64 ? (s.ld % 2) : s.xdt == DT_F32 ? (s.ld % 4) : (s.ld % 8))
    throw std::invalid_argument("gram_syrk: feature stride must keep 16-byte alignment");
  if (compute_f64) launch_dt<double>(s, st);
  else launch_dt<float>(s, st);
  DQ_HIP_CHECK(hipGetLastError());
  int64_t g = ((int64_t)s.npair * kPanel * kPanel + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(syrk_reduce_kernel, dim3(g), dim3(256), 0, st, s, out);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
