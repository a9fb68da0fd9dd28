// K9 — the squared-loss l-bfgs / OWLQN path of LinearRegression.fit (solver="l-bfgs", or "auto" with
// numFeatures > 4096: DataQuality4MachineLearningApp.java:120-126).  Spark runs
// one LeastSquaresAggregator treeAggregate per cost evaluation:
//
//   diff_r = x_r . (coef / sigma_x) - y_r / sigma_y + offset,   offset = mean_y/sigma_y - (coef/sigma_x) . mean_x
//   loss   = sum_r w_r diff_r^2 / 2,    grad_j = sum_r w_r diff_r x_rj / sigma_j     (then / weightSum)
//
// Here an evaluation is two streaming passes over the HBM-resident shard plus a fold:
//   lsq_margin   x_r . cf for every row (one wave per 16/32-row fragment unit, the feature sum
//                across the 32 feature lanes by shuffles), writes v_r = w_r diff_r (n f64) and a loss
//                partial per block;
//   lsq_columns  sum_r v_r x_rj: workgroups own (row range, 16-tile feature group) and keep f64
//                per-lane sums in registers; the row ranges' partial slabs are folded in a fixed
//                order (no atomics: repeated evaluations are bitwise identical);
// the (d + 1)-f64 result is what the X4 all-reduce sums across ranks.  The same column pass with
// v = w and an x^2 sum gives the feature moments (Spark's MultivariateOnlineSummarizer pass).
//
// Layouts: the MFMA-fragment tiles the assembler writes (tall bf16 d <= 64, wide bf16, wide fp8 with
// per-feature scales) are read 16 B per lane, one contiguous KiB per wave instruction; plain
// feature-major [d][ld] f64 / f32 / bf16 matrices are read 4 rows per lane.
#include <hip/hip_runtime.h>

#include "common.h"
#include "lsq.h"

namespace dq4ml {

namespace {

constexpr int kMarginThreads = 512;
constexpr int kColThreads = 256;
constexpr int kPlainFB = 16;  // features per workgroup, plain layout

__host__ __device__ constexpr int64_t chunk_bytes(int L) { return L == 3 ? 2048 : 4096; }
__host__ __device__ constexpr int units_per_sup(int L) { return L == 3 ? 2 : 4; }

inline int nt_of(int layout, int d) { return layout == 1 ? (d + 31) / 32 : ((d + 255) / 256) * 8; }
inline int tg_of(int mode) { return mode ? 8 : 16; }

// row of element e of the 16-byte fragment of lane half h in unit `sub` of superstep s
template <int L>
__device__ __forceinline__ int64_t frag_row(int64_t s, int sub, int h, int e) {
  if constexpr (L == 1) return s * 64 + 32 * h + 8 * sub + e;  // tall: k-step i = rows 32h + 8i + j
  else if constexpr (L == 2) return s * 64 + 16 * sub + 8 * h + e;  // wide bf16: k-step = 16 rows
  else return s * 64 + 16 * (2 * sub + (e >> 3)) + 8 * h + (e & 7);  // wide fp8: half = 2 k-steps
}

template <int L>
__device__ __forceinline__ void unpack(const u32x4 q, float* x) {
  if constexpr (L == 3) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = (int)q[k];
      x[4 * k + 0] = __builtin_amdgcn_cvt_f32_fp8(v, 0);
      x[4 * k + 1] = __builtin_amdgcn_cvt_f32_fp8(v, 1);
      x[4 * k + 2] = __builtin_amdgcn_cvt_f32_fp8(v, 2);
      x[4 * k + 3] = __builtin_amdgcn_cvt_f32_fp8(v, 3);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = __uint_as_float(q[j] << 16);
      x[2 * j + 1] = __uint_as_float(q[j] & 0xffff0000u);
    }
  }
}

__device__ __forceinline__ double block_sum_f64(double s, double* red /* >= 16 doubles */) {
  s = wave_sum_f64(s);
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];  // fixed order
  return t;
}

__device__ __forceinline__ void row_epilogue(int64_t r, int64_t n, double m, double offset, double inv_ystd,
                                             const double* __restrict__ y, const double* __restrict__ w,
                                             double* __restrict__ v, double& loss) {
  if (r >= n) return;
  const double wr = w[r];
  double vv = 0.0;
  if (wr != 0.0) {
    const double diff = m + offset - y[r] * inv_ystd;
    vv = wr * diff;
    loss += 0.5 * vv * diff;
  }
  v[r] = vv;
}

// ---- margin pass, fragment layouts ---------------------------------------------------------------
// One wave per unit (bf16: superstep s, k-step -> 16 rows; fp8: superstep s, half -> 32 rows).  Lane l:
// feature (tile t, l & 31), rows of half l >> 5.  Per tile each lane loads its 16 B (the wave: one
// contiguous KiB), 8 tiles in flight; f32 products per 8 tiles, f64 across tiles.  The effective
// coefficients sit in LDS (f32, <= 64 KiB) or are read through L1/L2 (CLDS = false, d > 16384).
template <int L, bool CLDS>
__global__ __launch_bounds__(kMarginThreads) void lsq_margin_frag(
    const unsigned char* __restrict__ X, int d, int NT, int64_t n, int64_t nunits, const float* __restrict__ cf,
    const double* __restrict__ offp, double inv_ystd, const double* __restrict__ y, const double* __restrict__ w,
    double* __restrict__ v, double* __restrict__ lpart) {
  extern __shared__ __attribute__((aligned(16))) double lsq_smem[];
  double* red = lsq_smem;                               // 16 doubles
  float* cs = reinterpret_cast<float*>(lsq_smem + 16);  // ntl * 32 floats
  constexpr int E = L == 3 ? 16 : 8;
  constexpr int64_t CH = chunk_bytes(L);
  constexpr int UPS = units_per_sup(L);
  const int ntl = (d + 31) >> 5;
  const double offset = *offp;  // device scalar: the optimizer never syncs to launch a pass
  if constexpr (CLDS) {
    for (int i = threadIdx.x; i < ntl * 32; i += blockDim.x) cs[i] = i < d ? cf[i] : 0.0f;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fl = lane & 31, h = lane >> 5;
  double loss = 0.0;
  for (int64_t u = (int64_t)blockIdx.x * nw + wave; u < nunits; u += (int64_t)gridDim.x * nw) {
    const int64_t s = u / UPS;
    const int sub = (int)(u % UPS);
    const unsigned char* p = X + s * NT * CH + ((sub * 64 + lane) << 4);
    double acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.0;
    int t = 0;
    for (; t + 8 <= ntl; t += 8) {
      u32x4 q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = *gptr<u32x4>(p + (int64_t)(t + k) * CH);
      float a[E];
#pragma unroll
      for (int e = 0; e < E; ++e) a[e] = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int f = (t + k) * 32 + fl;
        const float c = CLDS ? cs[f] : (f < d ? cf[f] : 0.0f);
        float x[E];
        unpack<L>(q[k], x);
#pragma unroll
        for (int e = 0; e < E; ++e) a[e] = fmaf(x[e], c, a[e]);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += (double)a[e];
    }
    for (; t < ntl; ++t) {
      const u32x4 q = *gptr<u32x4>(p + (int64_t)t * CH);
      const int f = t * 32 + fl;
      const float c = CLDS ? cs[f] : (f < d ? cf[f] : 0.0f);
      float x[E];
      unpack<L>(q, x);
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += (double)(x[e] * c);
    }
    // feature sum across the 32 lanes of each half (offsets < 32 stay inside the half)
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) acc[e] += __shfl_xor(acc[e], o, 64);
    }
    double m = acc[0];
#pragma unroll
    for (int e = 1; e < E; ++e) m = fl == e ? acc[e] : m;
    if (fl < E) row_epilogue(frag_row<L>(s, sub, h, fl), n, m, offset, inv_ystd, y, w, v, loss);
  }
  loss = block_sum_f64(loss, red);
  if (threadIdx.x == 0) lpart[blockIdx.x] = loss;
}

// ---- margin pass, plain feature-major [d][ld] ----------------------------------------------------
template <int XDT>
__device__ __forceinline__ void load4(const void* X, int64_t off, double x[4]) {
  if constexpr (XDT == DT_F64) {
    const f64x2 a = *gptr<f64x2>(reinterpret_cast<const double*>(X) + off);
    const f64x2 b = *gptr<f64x2>(reinterpret_cast<const double*>(X) + off + 2);
    x[0] = a[0], x[1] = a[1], x[2] = b[0], x[3] = b[1];
  } else if constexpr (XDT == DT_F32) {
    const f32x4 a = *gptr<f32x4>(reinterpret_cast<const float*>(X) + off);
    x[0] = a[0], x[1] = a[1], x[2] = a[2], x[3] = a[3];
  } else {
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
    const u32x2 a = *gptr<u32x2>(reinterpret_cast<const uint16_t*>(X) + off);
    x[0] = __uint_as_float(a[0] << 16), x[1] = __uint_as_float(a[0] & 0xffff0000u);
    x[2] = __uint_as_float(a[1] << 16), x[3] = __uint_as_float(a[1] & 0xffff0000u);
  }
}

template <int XDT>
__device__ __forceinline__ double load1(const void* X, int64_t off) {
  if constexpr (XDT == DT_F64) return gptr<double>(X)[off];
  else if constexpr (XDT == DT_F32) return (double)gptr<float>(X)[off];
  else return (double)bf16_bits_to_f32(gptr<uint16_t>(X)[off]);
}

template <int XDT>
__global__ __launch_bounds__(256) void lsq_margin_plain(const void* __restrict__ X, int64_t ld, int d, int64_t n,
                                                       const double* __restrict__ c,
                                                       const double* __restrict__ offp, double inv_ystd,
                                                       const double* __restrict__ y, const double* __restrict__ w,
                                                       double* __restrict__ v, double* __restrict__ lpart) {
  __shared__ double red[16];
  const double offset = *offp;
  double loss = 0.0;
  const int64_t nq = (n + 3) >> 2;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r0 = q * 4;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (r0 + 4 <= n) {
      int f = 0;
      for (; f + 4 <= d; f += 4) {
        double x[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) load4<XDT>(X, (int64_t)(f + k) * ld + r0, x[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double cf = c[f + k];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fma(x[k][j], cf, acc[j]);
        }
      }
      for (; f < d; ++f) {
        double x[4];
        load4<XDT>(X, (int64_t)f * ld + r0, x);
        const double cf = c[f];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fma(x[j], cf, acc[j]);
      }
    } else {
      for (int f = 0; f < d; ++f) {
        const double cf = c[f];
        for (int j = 0; j < 4; ++j)
          if (r0 + j < n) acc[j] = fma(load1<XDT>(X, (int64_t)f * ld + r0 + j), cf, acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) row_epilogue(r0 + j, n, acc[j], offset, inv_ystd, y, w, v, loss);
  }
  loss = block_sum_f64(loss, red);
  if (threadIdx.x == 0) lpart[blockIdx.x] = loss;
}

// ---- column pass, fragment layouts ---------------------------------------------------------------
// Workgroup (row range rho, group of TG tiles); each wave walks supersteps s0 + wave, s0 + wave + 4, ...
// Per superstep a lane loads the v of its 32 rows (4 f64x2 runs per unit) once and reuses it across
// the TG tiles; per tile it reads its 16 B of every unit (the chunk's 4 KiB / 2 KiB in 4 / 2 wave
// loads) and adds an f32 superstep sum into its f64 per-tile accumulator.
template <int L, int MODE, int TG>
__global__ __launch_bounds__(kColThreads) void lsq_cols_frag(const unsigned char* __restrict__ X, int d, int NT,
                                                            int64_t n, int64_t nsup, int R,
                                                            const double* __restrict__ v, double* __restrict__ part) {
  constexpr int E = L == 3 ? 16 : 8;
  constexpr int64_t CH = chunk_bytes(L);
  constexpr int UPS = units_per_sup(L);
  constexpr int NV = UPS * E;  // 32 rows per lane per superstep
  constexpr int NS = TG * (1 + MODE);
  __shared__ double red[4][NS][32];
  const int ntl = (d + 31) >> 5;
  const int G = (ntl + TG - 1) / TG;
  const int tg = (int)(blockIdx.x % G), rho = (int)(blockIdx.x / G);
  const int64_t s0 = nsup * rho / R, s1 = nsup * (rho + 1) / R;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fl = lane & 31, h = lane >> 5;
  const int nt = min(TG, ntl - tg * TG);  // live tiles of this group (uniform)
  double g[TG], g2[TG];
#pragma unroll
  for (int k = 0; k < TG; ++k) g[k] = 0.0, g2[k] = 0.0;
  for (int64_t s = s0 + wave; s < s1; s += 4) {
    float vv[NV];
#pragma unroll
    for (int sub = 0; sub < UPS; ++sub) {
#pragma unroll
      for (int e0 = 0; e0 < E; e0 += 8) {
        const int64_t r0 = frag_row<L>(s, sub, h, e0);  // 8 contiguous rows, r0 % 8 == 0
        if (r0 + 8 <= n) {
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f64x2 a = *gptr<f64x2>(v + r0 + j);
            vv[sub * E + e0 + j] = (float)a[0];
            vv[sub * E + e0 + j + 1] = (float)a[1];
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) vv[sub * E + e0 + j] = r0 + j < n ? (float)v[r0 + j] : 0.0f;
        }
      }
    }
    const unsigned char* p = X + (s * NT + tg * TG) * CH + (lane << 4);
#pragma unroll
    for (int k = 0; k < TG; ++k) {
      if (k < nt) {
        u32x4 q[UPS];
#pragma unroll
        for (int sub = 0; sub < UPS; ++sub) q[sub] = *gptr<u32x4>(p + k * CH + sub * 1024);
        float a = 0.0f, a2 = 0.0f;
#pragma unroll
        for (int sub = 0; sub < UPS; ++sub) {
          float x[E];
          unpack<L>(q[sub], x);
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const float t = vv[sub * E + e] * x[e];
            a += t;
            if constexpr (MODE == 1) a2 = fmaf(t, x[e], a2);
          }
        }
        g[k] += (double)a;
        if constexpr (MODE == 1) g2[k] += (double)a2;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < TG; ++k) {
    g[k] += __shfl_xor(g[k], 32, 64);
    if constexpr (MODE == 1) g2[k] += __shfl_xor(g2[k], 32, 64);
  }
  if (lane < 32) {
#pragma unroll
    for (int k = 0; k < TG; ++k) {
      red[wave][k][lane] = g[k];
      if constexpr (MODE == 1) red[wave][TG + k][lane] = g2[k];
    }
  }
  __syncthreads();
  const int ldp = ntl * 32;
  for (int i = threadIdx.x; i < NS * 32; i += blockDim.x) {
    const int slot = i >> 5, f = i & 31;
    const int mi = slot / TG, k = slot % TG;
    if (k < nt) {
      const double val = (red[0][slot][f] + red[1][slot][f]) + (red[2][slot][f] + red[3][slot][f]);
      part[((int64_t)rho * (1 + MODE) + mi) * ldp + (tg * TG + k) * 32 + f] = val;
    }
  }
}

// ---- column pass, plain feature-major [d][ld] -----------------------------------------------------
template <int XDT, int MODE>
__global__ __launch_bounds__(kColThreads) void lsq_cols_plain(const void* __restrict__ X, int64_t ld, int d, int64_t n,
                                                             int R, const double* __restrict__ v,
                                                             double* __restrict__ part) {
  constexpr int FB = kPlainFB;
  constexpr int NS = FB * (1 + MODE);
  __shared__ double red[4][NS];
  const int G = (d + FB - 1) / FB;
  const int fb = (int)(blockIdx.x % G), rho = (int)(blockIdx.x / G);
  const int64_t nq = (n + 3) >> 2;
  const int64_t q0 = nq * rho / R, q1 = nq * (rho + 1) / R;
  const int nf = min(FB, d - fb * FB);
  double g[FB], g2[FB];
#pragma unroll
  for (int k = 0; k < FB; ++k) g[k] = 0.0, g2[k] = 0.0;
  for (int64_t q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const int64_t r0 = q * 4;
    const bool full = r0 + 4 <= n;
    double vv[4];
    if (full) {
      const f64x2 a = *gptr<f64x2>(v + r0);
      const f64x2 b = *gptr<f64x2>(v + r0 + 2);
      vv[0] = a[0], vv[1] = a[1], vv[2] = b[0], vv[3] = b[1];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) vv[j] = r0 + j < n ? v[r0 + j] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < FB; ++k) {
      if (k < nf) {
        const int64_t off = (int64_t)(fb * FB + k) * ld + r0;
        double x[4];
        if (full) {
          load4<XDT>(X, off, x);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) x[j] = r0 + j < n ? load1<XDT>(X, off + j) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // dead / null rows carry v = 0 whatever their stored value (NaN-safe select)
          const double t = vv[j] * x[j];
          g[k] += vv[j] != 0.0 ? t : 0.0;
          if constexpr (MODE == 1) g2[k] += vv[j] != 0.0 ? t * x[j] : 0.0;
        }
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < FB; ++k) {
    g[k] = wave_sum_f64(g[k]);
    if constexpr (MODE == 1) g2[k] = wave_sum_f64(g2[k]);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < FB; ++k) {
      red[wave][k] = g[k];
      if constexpr (MODE == 1) red[wave][FB + k] = g2[k];
    }
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    const int mi = threadIdx.x / FB, k = threadIdx.x % FB;
    if (k < nf) {
      const double val = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
      part[((int64_t)rho * (1 + MODE) + mi) * d + fb * FB + k] = val;
    }
  }
}

// ---- fold: out[off + mi*d + j] = sum_rho part[rho][mi][j]; out[0] = sum(lpart) (fixed order) -------
__global__ __launch_bounds__(256) void lsq_fold(const double* __restrict__ part, int R, int nm, int d, int ldp,
                                               const double* __restrict__ lpart, int nl, double* __restrict__ out,
                                               int off) {
  __shared__ double red[16];
  const int64_t width = (int64_t)nm * d;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < width; i += (int64_t)gridDim.x * blockDim.x) {
    const int mi = (int)(i / d), j = (int)(i % d);
    double s = 0.0;
    for (int r = 0; r < R; ++r) s += part[((int64_t)r * nm + mi) * ldp + j];
    out[off + i] = s;
  }
  if (lpart != nullptr && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nl; i += blockDim.x) s += lpart[i];
    s = block_sum_f64(s, red);
    if (threadIdx.x == 0) out[0] = s;
  }
}

struct Split {
  int R;       // row ranges
  int G;       // feature groups
  int ldp;     // partial row stride
};

Split col_split(const LsqX& x, int mode) {
  Split sp{};
  if (x.layout == 0) {
    sp.G = (x.d + kPlainFB - 1) / kPlainFB;
    const int64_t nq = (x.n + 3) / 4;
    int64_t R = (2048 + sp.G - 1) / sp.G;
    const int64_t cap = nq / 256 > 1 ? nq / 256 : 1;
    sp.R = (int)(R < cap ? R : cap);
    sp.ldp = x.d;
  } else {
    const int ntl = (x.d + 31) / 32;
    const int tg = tg_of(mode);
    sp.G = (ntl + tg - 1) / tg;
    const int64_t nsup = (x.n + 63) / 64;
    int64_t R = (4096 + sp.G - 1) / sp.G;
    const int64_t cap = nsup > 1 ? nsup : 1;
    sp.R = (int)(R < cap ? R : cap);
    sp.ldp = ntl * 32;
  }
  if (sp.R < 1) sp.R = 1;
  return sp;
}

void check(const LsqX& x) {
  if (x.d < 1 || x.n < 0 || x.layout < 0 || x.layout > 3)
    throw std::invalid_argument("lsq: bad feature-matrix description");
  if (x.layout == 0 && (x.xdt != DT_F64 && x.xdt != DT_F32 && x.xdt != DT_BF16))
    throw std::invalid_argument("lsq: plain layout needs f64 / f32 / bf16 features");
  if (x.layout == 0 && x.d > 1 && x.ld % 4 != 0) throw std::invalid_argument("lsq: plain layout needs ld % 4 == 0");
}

int margin_lds_bytes(const LsqX& x) { return 16 * 8 + ((x.d + 31) / 32) * 32 * 4; }

}  // namespace

int lsq_margin_blocks(const LsqX& x) {
  if (x.layout == 0) {
    const int64_t nq = (x.n + 3) / 4;
    int64_t g = (nq + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
  }
  const int64_t nunits = ((x.n + 63) / 64) * (x.layout == 3 ? 2 : 4);
  const int lds = margin_lds_bytes(x);
  const int per_cu = lds <= 32768 ? 4 : (lds <= 65536 + 128 ? 2 : 1);
  int64_t g = (nunits + 7) / 8;
  const int64_t cap = 256LL * per_cu;
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : g);
}

int64_t lsq_part_doubles(const LsqX& x, int mode) {
  const Split sp = col_split(x, mode);
  return (int64_t)sp.R * (1 + mode) * sp.ldp;
}

void lsq_margin(const LsqX& x, const void* cf, const double* offset, double inv_ystd, const double* y, const double* w,
                double* v, double* lpart, hipStream_t st) {
  check(x);
  const int g = lsq_margin_blocks(x);
  if (x.n == 0) {
    DQ_HIP_CHECK(hipMemsetAsync(lpart, 0, sizeof(double) * g, st));
    return;
  }
  if (x.layout == 0) {
    auto c = reinterpret_cast<const double*>(cf);
    if (x.xdt == DT_F64)
      hipLaunchKernelGGL(lsq_margin_plain<DT_F64>, dim3(g), dim3(256), 0, st, x.X, x.ld, x.d, x.n, c, offset, inv_ystd, y, w, v, lpart);
    else if (x.xdt == DT_F32)
      hipLaunchKernelGGL(lsq_margin_plain<DT_F32>, dim3(g), dim3(256), 0, st, x.X, x.ld, x.d, x.n, c, offset, inv_ystd, y, w, v, lpart);
    else
      hipLaunchKernelGGL(lsq_margin_plain<DT_BF16>, dim3(g), dim3(256), 0, st, x.X, x.ld, x.d, x.n, c, offset, inv_ystd, y, w, v, lpart);
    DQ_HIP_CHECK(hipGetLastError());
    return;
  }
  auto Xb = reinterpret_cast<const unsigned char*>(x.X);
  auto c = reinterpret_cast<const float*>(cf);
  const int NT = nt_of(x.layout, x.d);
  const int64_t nunits = ((x.n + 63) / 64) * (x.layout == 3 ? 2 : 4);
  const int lds = margin_lds_bytes(x);
  const bool clds = lds <= 131072;
  const unsigned smem = clds ? lds : 16 * 8;
#define DQ_LSQ_M(LL, CC)                                                                                       \
  hipLaunchKernelGGL((lsq_margin_frag<LL, CC>), dim3(g), dim3(kMarginThreads), smem, st, Xb, x.d, NT, x.n, nunits, c, \
                     offset, inv_ystd, y, w, v, lpart)
  if (x.layout == 1) { if (clds) DQ_LSQ_M(1, true); else DQ_LSQ_M(1, false); }
  else if (x.layout == 2) { if (clds) DQ_LSQ_M(2, true); else DQ_LSQ_M(2, false); }
  else { if (clds) DQ_LSQ_M(3, true); else DQ_LSQ_M(3, false); }
#undef DQ_LSQ_M
  DQ_HIP_CHECK(hipGetLastError());
}

void lsq_columns(const LsqX& x, int mode, const double* v, const double* lpart, int nl, double* part, double* out,
                 hipStream_t st) {
  check(x);
  if (mode != 0 && mode != 1) throw std::invalid_argument("lsq_columns: mode 0 or 1");
  const Split sp = col_split(x, mode);
  const int nm = 1 + mode;
  if (x.n == 0) {
    DQ_HIP_CHECK(hipMemsetAsync(part, 0, sizeof(double) * (size_t)sp.R * nm * sp.ldp, st));
  } else if (x.layout == 0) {
    const int g = sp.G * sp.R;
#define DQ_LSQ_CP(XD, MM) \
  hipLaunchKernelGGL((lsq_cols_plain<XD, MM>), dim3(g), dim3(kColThreads), 0, st, x.X, x.ld, x.d, x.n, sp.R, v, part)
    if (x.xdt == DT_F64) { if (mode) DQ_LSQ_CP(DT_F64, 1); else DQ_LSQ_CP(DT_F64, 0); }
    else if (x.xdt == DT_F32) { if (mode) DQ_LSQ_CP(DT_F32, 1); else DQ_LSQ_CP(DT_F32, 0); }
    else { if (mode) DQ_LSQ_CP(DT_BF16, 1); else DQ_LSQ_CP(DT_BF16, 0); }
#undef DQ_LSQ_CP
  } else {
    auto Xb = reinterpret_cast<const unsigned char*>(x.X);
    const int NT = nt_of(x.layout, x.d);
    const int64_t nsup = (x.n + 63) / 64;
    const int g = sp.G * sp.R;
#define DQ_LSQ_CF(LL, MM, TT) \
  hipLaunchKernelGGL((lsq_cols_frag<LL, MM, TT>), dim3(g), dim3(kColThreads), 0, st, Xb, x.d, NT, x.n, nsup, sp.R, v, part)
    if (x.layout == 1) { if (mode) DQ_LSQ_CF(1, 1, 8); else DQ_LSQ_CF(1, 0, 16); }
    else if (x.layout == 2) { if (mode) DQ_LSQ_CF(2, 1, 8); else DQ_LSQ_CF(2, 0, 16); }
    else { if (mode) DQ_LSQ_CF(3, 1, 8); else DQ_LSQ_CF(3, 0, 16); }
#undef DQ_LSQ_CF
  }
  DQ_HIP_CHECK(hipGetLastError());
  const int64_t width = (int64_t)nm * x.d;
  int64_t fg = (width + 255) / 256;
  if (fg > 1024) fg = 1024;
  if (fg < 1) fg = 1;
  hipLaunchKernelGGL(lsq_fold, dim3(fg), dim3(256), 0, st, part, sp.R, nm, x.d, sp.ldp, mode == 0 ? lpart : nullptr,
                     nl, out, mode == 0 ? 1 : 0);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
