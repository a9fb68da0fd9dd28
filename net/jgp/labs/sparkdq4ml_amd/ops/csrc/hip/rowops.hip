// Row-wise kernels: K3 stream compaction of a selection vector, K4 column pack (VectorAssembler),
// K7 predict and K8 fused predict + regression metrics.
//
//  * compact: Spark materializes filtered rows through ``take``/collect (show(n) = take(n+1),
//    SURVEY.md S05).  Two passes: per-block live counts (wave ballot + popcount), one-block
//    exclusive scan, then each block writes its indices at its offset — order preserving.
//  * pack: VectorAssembler.transform (DataQuality4MachineLearningApp.java:110-113) — each input
//    column becomes one contiguous row of the feature-major [d, ld] output, cast to the output
//    dtype; dead rows (selection false) can be written as zeros so the Gram kernel needs no mask.
//  * predict / metrics: LinearRegressionModel.transform (:129) and the RegressionMetrics summary
//    (:138-139) in ONE pass: ŷ = x·coef + b is never materialized for the metrics, and the 8
//    moments are reduced per block in f64 (shifted by the label mean for a stable SStot).
#include <hip/hip_runtime.h>

#include "common.h"
#include "rowops.h"

namespace dq4ml {

namespace {

__device__ __forceinline__ double ld_f64(const void* p, int dt, int64_t i) {
  switch (dt) {
    case DT_F64: return reinterpret_cast<const double*>(p)[i];
    case DT_F32: return (double)reinterpret_cast<const float*>(p)[i];
    case DT_BF16: return (double)bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(p)[i]);
    case DT_I32: return (double)reinterpret_cast<const int32_t*>(p)[i];
    case DT_I64: return (double)reinterpret_cast<const int64_t*>(p)[i];
    case DT_U8: return (double)reinterpret_cast<const uint8_t*>(p)[i];
    default: return 0.0;
  }
}

__device__ __forceinline__ void st_from_f64(void* p, int dt, int64_t i, double v) {
  switch (dt) {
    case DT_F64: reinterpret_cast<double*>(p)[i] = v; break;
    case DT_F32: reinterpret_cast<float*>(p)[i] = (float)v; break;
    case DT_BF16: reinterpret_cast<__bf16*>(p)[i] = (__bf16)(float)v; break;
    case DT_I32: reinterpret_cast<int32_t*>(p)[i] = (int32_t)v; break;
    case DT_I64: reinterpret_cast<int64_t*>(p)[i] = (int64_t)v; break;
    default: break;
  }
}

constexpr int kCompactChunk = 4096;  // rows per block (256 threads x 16)

__global__ __launch_bounds__(256) void compact_count_kernel(const uint8_t* __restrict__ sel, int64_t n,
                                                           int64_t* __restrict__ counts) {
  __shared__ int64_t wsum[4];
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  int64_t c = 0;
  for (int k = 0; k < kCompactChunk / 256; ++k) {
    const int64_t r = base + k * 256 + threadIdx.x;
    const bool live = r < n && sel[r] != 0;
    const uint64_t b = __ballot(live);
    c += __popcll(b);
  }
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// exclusive scan in place + total at counts[nb]; single block
__global__ __launch_bounds__(1024) void compact_scan_kernel(int64_t* __restrict__ counts, int64_t nb) {
  __shared__ int64_t part[1024];
  const int64_t per = (nb + 1023) / 1024;
  const int64_t b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
  int64_t s = 0;
  for (int64_t b = b0; b < b1; ++b) s += counts[b];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int i = 0; i < 1024; ++i) {
      const int64_t v = part[i];
      part[i] = run;
      run += v;
    }
    counts[nb] = run;
  }
  __syncthreads();
  int64_t run = part[threadIdx.x];
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t v = counts[b];
    counts[b] = run;
    run += v;
  }
}

__global__ __launch_bounds__(256) void compact_write_kernel(const uint8_t* __restrict__ sel, int64_t n,
                                                           const int64_t* __restrict__ offsets, int64_t limit,
                                                           int64_t* __restrict__ out) {
  __shared__ int64_t woff[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  int64_t off = offsets[blockIdx.x];
  if (off >= limit) return;  // uniform per block
  for (int k = 0; k < kCompactChunk / 256; ++k) {
    const int64_t r = base + k * 256 + threadIdx.x;
    const bool live = r < n && sel[r] != 0;
    const uint64_t b = __ballot(live);
    if (lane == 0) woff[wave] = __popcll(b);
    __syncthreads();
    int64_t before = 0;
    for (int w = 0; w < wave; ++w) before += woff[w];
    const int64_t total = woff[0] + woff[1] + woff[2] + woff[3];
    const int64_t pos = off + before + __popcll(b & ((1ull << lane) - 1ull));
    if (live && pos < limit) out[pos] = r;
    off += total;
    __syncthreads();
  }
}

// ---- pack --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(const PackSrc* __restrict__ srcs, int d, int64_t n,
                                                  void* __restrict__ out, int odt, int64_t ld,
                                                  const uint8_t* __restrict__ sel) {
  const int f = blockIdx.y;
  if (f >= d) return;
  const PackSrc s = srcs[f];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < ld; r += (int64_t)gridDim.x * blockDim.x) {
    double v = 0.0;
    if (r < n && (sel == nullptr || sel[r] != 0)) v = ld_f64(s.ptr, s.dt, r);
    st_from_f64(out, odt, (int64_t)f * ld + r, v);
  }
}

// ---- predict / metrics -----------------------------------------------------------------------
// element offset of (feature f, row r) in the MFMA-fragment-ordered bf16 layout (gram.h)
__device__ __forceinline__ int64_t tiled_offset(int f, int64_t r, int NT) {
  const int64_t s = r >> 6;
  const int h = (int)((r >> 5) & 1), i = (int)((r >> 3) & 3), j = (int)(r & 7);
  const int t = f >> 5, lane = 32 * h + (f & 31);
  return ((((s * NT + t) * 4 + i) * 64 + lane) << 3) + j;
}

// wide layouts (gram_wide.hip): k-step ki = 16 contiguous rows, 8 B (fp8) / 16 B (bf16) per lane
__device__ __forceinline__ int64_t wide_offset(int f, int64_t r, int NT) {
  const int64_t s = r >> 6;
  const int ki = (int)((r >> 4) & 3), h = (int)((r >> 3) & 1), j = (int)(r & 7);
  const int t = f >> 5, lane = 32 * h + (f & 31);
  return ((((s * NT + t) * 4 + ki) * 64 + lane) << 3) + j;  // element index
}

// fp8 wide image: per (superstep, tile) a [2 halves][64 lanes][16 B] chunk; a lane's 32 bytes are
// its k-steps 0..3 (8 rows each), halves = k-steps {0,1} / {2,3} (gram_wide.hip)
__device__ __forceinline__ int64_t wide_offset_fp8(int f, int64_t r, int NT) {
  const int64_t s = r >> 6;
  const int ki = (int)((r >> 4) & 3), h = (int)((r >> 3) & 1), j = (int)(r & 7);
  const int t = f >> 5, lane = 32 * h + (f & 31);
  return (s * NT + t) * 2048 + (((ki >> 1) * 64 + lane) << 4) + ((ki & 1) << 3) + j;  // byte index
}

__device__ __forceinline__ float fp8_to_f32(uint8_t v) {
  return __builtin_amdgcn_cvt_f32_fp8((int)v, 0);
}

__device__ __forceinline__ double predict_row(const void* X, int xdt, int64_t ld, int d, const double* coef,
                                              double b, int64_t r, int tiled) {
  double acc = b;
  if (tiled == 2 || tiled == 3) {  // wide bf16 / wide fp8 (coef pre-multiplied by the fp8 scales)
    const int NT = ((d + 255) >> 8) * 8;
    for (int f = 0; f < d; ++f) {
      const float x = tiled == 2 ? bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(X)[wide_offset(f, r, NT)])
                                 : fp8_to_f32(reinterpret_cast<const uint8_t*>(X)[wide_offset_fp8(f, r, NT)]);
      acc += coef[f] * (double)x;
    }
    return acc;
  }
  if (tiled) {
    const int NT = (d + 31) >> 5;
    const uint16_t* xb = reinterpret_cast<const uint16_t*>(X);
    for (int f = 0; f < d; ++f) acc += coef[f] * (double)bf16_bits_to_f32(xb[tiled_offset(f, r, NT)]);
    return acc;
  }
  for (int f = 0; f < d; ++f) acc += coef[f] * ld_f64(X, xdt, (int64_t)f * ld + r);
  return acc;
}

// columns (PackSrc per feature) -> tiled bf16, dead rows (sel == 0) written as zeros.
// One block-iteration = one (superstep s, tile t) chunk (64 rows x 32 features, 4 KiB out):
// thread (f, q) loads rows [8q, 8q+8) of feature f with 16-B vector loads (8 threads per feature
// -> every wave reads 8 contiguous 256-B column runs) and that run is exactly one lane's
// fragment of k-step q & 3 for lane half q >> 2 -> one 16-B store, no transpose.
__global__ __launch_bounds__(256) void pack_tiled_kernel(const PackSrc* __restrict__ srcs, int d, int64_t n,
                                                        const uint8_t* __restrict__ sel, int NT, int64_t nsup,
                                                        uint16_t* __restrict__ out, const float* __restrict__ shift) {
  const int fl = threadIdx.x >> 3, q = threadIdx.x & 7;
  const int i = q & 3, h = q >> 2;
  const int64_t nchunks = nsup * NT;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int t = (int)(c % NT);
    const int64_t s = c / NT;
    const int f = t * 32 + fl;
    const int64_t r0 = s * 64 + 8 * q;
    float x[8];
    if (f < d) {
      const PackSrc src = srcs[f];
      load8_f32(src.ptr, src.dt, r0, n, x);
      if (shift) sub_shift8(x, shift[f], r0, n);
      mask8(sel, r0, n, x);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = 0.0f;
    }
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[j];
    // chunk c = [4 k-steps][64 lanes][8 bf16]; tall layout: lane 32h + f holds rows 32h + 8i + j
    reinterpret_cast<u32x4*>(out)[c * 256 + i * 64 + h * 32 + fl] = __builtin_bit_cast(u32x4, v);
  }
}

__global__ __launch_bounds__(256) void predict_kernel(const void* __restrict__ X, int xdt, int64_t ld, int d,
                                                     int64_t n, const double* __restrict__ coef, double b,
                                                     double* __restrict__ out, int tiled) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
    out[r] = predict_row(X, xdt, ld, d, coef, b, r, tiled);
}

__global__ __launch_bounds__(256) void metrics_kernel(const void* __restrict__ X, int xdt, int64_t ld, int d,
                                                     int64_t n, const void* __restrict__ y, int ydt,
                                                     const uint8_t* __restrict__ sel,
                                                     const double* __restrict__ coef, double b, double shift,
                                                     double* __restrict__ partials, int tiled) {
  double m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (sel != nullptr && sel[r] == 0) continue;
    const double p = predict_row(X, xdt, ld, d, coef, b, r, tiled);
    const double yy = ld_f64(y, ydt, r);
    const double ys = yy - shift, ps = p - shift, res = yy - p;
    m[0] += 1.0;
    m[1] += ys;
    m[2] += ys * ys;
    m[3] += res;
    m[4] += res * res;
    m[5] += fabs(res);
    m[6] += ps;
    m[7] += ps * ps;
  }
  __shared__ double red[4][8];
#pragma unroll
  for (int k = 0; k < 8; ++k) m[k] = wave_sum_f64(m[k]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x >> 6][k] = m[k];
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    partials[(int64_t)blockIdx.x * 8 + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
  }
}

// ---- predict / metrics over the MFMA-fragment layouts (tiled codes 1 tall bf16, 2 wide bf16,
// 3 wide fp8): block-iteration = one superstep (64 rows).  Thread (f, q) walks the tiles reading
// its 16-B (8-B fp8) fragment = rows [8q, 8q+8) of feature t*32 + f in every layout and
// accumulates coef * x (f64) for those 8 rows.  The 8 feature-threads of a wave fold with
// shuffles, the 4 waves through a double-buffered 2 KiB LDS slab (one barrier per superstep),
// and the next superstep's fragments are loaded before that barrier.
template <int TILED>
__device__ __forceinline__ void frag8(const unsigned char* X, int64_t ch, int q, int fl, float x[8]) {
  if constexpr (TILED == 3) {
    const int ki = q >> 1, lane = 32 * (q & 1) + fl;
    const uint64_t v = *gptr<uint64_t>(X + ch * 2048 + (((ki >> 1) * 64 + lane) << 4) + ((ki & 1) << 3));
    const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    x[0] = __builtin_amdgcn_cvt_f32_fp8(lo, 0);
    x[1] = __builtin_amdgcn_cvt_f32_fp8(lo, 1);
    x[2] = __builtin_amdgcn_cvt_f32_fp8(lo, 2);
    x[3] = __builtin_amdgcn_cvt_f32_fp8(lo, 3);
    x[4] = __builtin_amdgcn_cvt_f32_fp8(hi, 0);
    x[5] = __builtin_amdgcn_cvt_f32_fp8(hi, 1);
    x[6] = __builtin_amdgcn_cvt_f32_fp8(hi, 2);
    x[7] = __builtin_amdgcn_cvt_f32_fp8(hi, 3);
    return;
  }
  const int64_t unit = TILED == 1 ? ch * 256 + (q & 3) * 64 + (q >> 2) * 32 + fl
                                  : ch * 256 + (q >> 1) * 64 + 32 * (q & 1) + fl;
  const u32x4 v = gptr<u32x4>(X)[unit];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[2 * j] = __uint_as_float(v[j] << 16);
    x[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
  }
}

template <int MODE, int YDT, int TILED>  // MODE 0: predictions -> out, 1: the 8 metric sums -> partials
__global__ __launch_bounds__(256) void tiled_rows_kernel(const unsigned char* __restrict__ X, int tiled, int d,
                                                        int64_t n, const double* __restrict__ coef, double b,
                                                        const void* __restrict__ y, int ydt,
                                                        const uint8_t* __restrict__ sel, double shift,
                                                        double* __restrict__ out) {
  __shared__ double part[2][4][64];
  __shared__ double wpart[4][8][65];  // per wave: [feature-thread][row] (+1 pad)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fl = tid >> 3, q = tid & 7;
  const int NT = TILED == 1 ? (d + 31) >> 5 : ((d + 255) >> 8) * 8;
  // tall layouts (<= 2 tiles): the thread's coefficients live in registers
  double c2[2] = {fl < d ? coef[fl] : 0.0, 32 + fl < d ? coef[32 + fl] : 0.0};
  const int ntiles = (d + 31) >> 5;
  const int64_t nsup = (n + 63) >> 6;
  double m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int buf = 0;
  for (int64_t s = blockIdx.x; s < nsup; s += gridDim.x) {
    // the row scalars are requested together with the fragments: one memory round trip per superstep
    double yy = 0.0;
    bool live = false;
    const int64_t rr = s * 64 + tid;
    if (MODE == 1 && tid < 64 && rr < n) {
      live = sel == nullptr || gptr<uint8_t>(sel)[rr] != 0;
      yy = YDT == DT_F64 ? gptr<double>(y)[rr] : YDT == DT_F32 ? (double)gptr<float>(y)[rr] : ld_f64(y, ydt, rr);
    }
    double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (TILED == 1) {  // tall: <= 2 tiles, both fragments requested before use
      float x0[8], x1[8];
      frag8<1>(X, s * NT, q, fl, x0);
      if (ntiles > 1) frag8<1>(X, s * NT + 1, q, fl, x1);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = c2[0] * (double)x0[j];
      if (ntiles > 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += c2[1] * (double)x1[j];
      }
    } else {
      for (int t = 0; t < ntiles; ++t) {
        const int f = t * 32 + fl;
        float x[8];
        frag8<TILED>(X, s * NT + t, q, fl, x);
        const double c = f < d ? coef[f] : 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += c * (double)x[j];
      }
    }
    // fold the wave's 8 feature-threads through a per-wave LDS transpose (no cross-wave sync)
    const int fw = lane >> 3;  // feature-thread within the wave
#pragma unroll
    for (int j = 0; j < 8; ++j) wpart[wave][fw][q * 8 + j] = acc[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double rowp = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) rowp += wpart[wave][k][lane];
    part[buf][wave][lane] = rowp;
    __syncthreads();
    if (tid < 64) {
      const int64_t r = s * 64 + tid;
      const double p = b + part[buf][0][tid] + part[buf][1][tid] + part[buf][2][tid] + part[buf][3][tid];
      if (r < n) {
        if (MODE == 0) {
          out[r] = p;
        } else if (live) {
          const double ys = yy - shift, ps = p - shift, res = yy - p;
          m[0] += 1.0;
          m[1] += ys;
          m[2] += ys * ys;
          m[3] += res;
          m[4] += res * res;
          m[5] += fabs(res);
          m[6] += ps;
          m[7] += ps * ps;
        }
      }
    }
    buf ^= 1;  // the other slab is free: its readers passed this superstep's barrier
  }
  if (MODE == 1) {  // only wave 0 accumulated metrics
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = wave_sum_f64(m[k]);
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) out[(int64_t)blockIdx.x * 8 + k] = m[k];
    }
  }
}

__global__ __launch_bounds__(256) void sum_slabs_kernel(const double* __restrict__ partials, int nslab, int width,
                                                       double* __restrict__ out) {
  // fixed-order (deterministic) block reduction of nslab x width slabs: strided per-thread sums,
  // wave shuffles, then 4 wave totals
  __shared__ double wsum[4];
  for (int k = 0; k < width; ++k) {
    double s = 0.0;
    for (int b = threadIdx.x; b < nslab; b += blockDim.x) s += partials[(int64_t)b * width + k];
    s = wave_sum_f64(s);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[k] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __syncthreads();
  }
}

}  // namespace

int64_t compact_blocks(int64_t n) { return (n + kCompactChunk - 1) / kCompactChunk; }

void compact_count_scan(const uint8_t* sel, int64_t n, int64_t* counts, hipStream_t st) {
  const int64_t nb = compact_blocks(n);
  if (nb == 0) {
    DQ_HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int64_t), st));
    return;
  }
  hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(256), 0, st, sel, n, counts);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nb);
  DQ_HIP_CHECK(hipGetLastError());
}

void compact_write(const uint8_t* sel, int64_t n, const int64_t* offsets, int64_t limit, int64_t* out,
                   hipStream_t st) {
  const int64_t nb = compact_blocks(n);
  if (nb == 0 || limit <= 0) return;
  hipLaunchKernelGGL(compact_write_kernel, dim3(nb), dim3(256), 0, st, sel, n, offsets, limit, out);
  DQ_HIP_CHECK(hipGetLastError());
}

void pack_columns(const PackSrc* srcs_dev, int d, int64_t n, void* out, int odt, int64_t ld, const uint8_t* sel,
                  hipStream_t st) {
  if (d <= 0 || ld <= 0) return;
  int64_t gx = (ld + 255) / 256;
  if (gx > 2048) gx = 2048;
  hipLaunchKernelGGL(pack_kernel, dim3(gx, d), dim3(256), 0, st, srcs_dev, d, n, out, odt, ld, sel);
  DQ_HIP_CHECK(hipGetLastError());
}

void pack_tiled(const PackSrc* srcs_dev, int d, int64_t n, const uint8_t* sel, void* out, hipStream_t st,
                const float* shift) {
  const int NT = (d + 31) / 32;
  const int64_t nsup = (n + 63) / 64;
  int64_t g = nsup * NT;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(pack_tiled_kernel, dim3(g), dim3(256), 0, st, srcs_dev, d, n, sel, NT, nsup,
                     reinterpret_cast<uint16_t*>(out), shift);
  DQ_HIP_CHECK(hipGetLastError());
}

void predict(const void* X, int xdt, int64_t ld, int d, int64_t n, const double* coef, double b, double* out,
             hipStream_t st, int tiled) {
  if (n <= 0) return;
  if (tiled) {
    int64_t g = (n + 63) / 64;
    if (g > 8192) g = 8192;
    auto xb = reinterpret_cast<const unsigned char*>(X);
    if (tiled == 1) hipLaunchKernelGGL((tiled_rows_kernel<0, DT_F64, 1>), dim3(g), dim3(256), 0, st, xb, tiled, d, n, coef, b, nullptr, 0, nullptr, 0.0, out);
    else if (tiled == 2) hipLaunchKernelGGL((tiled_rows_kernel<0, DT_F64, 2>), dim3(g), dim3(256), 0, st, xb, tiled, d, n, coef, b, nullptr, 0, nullptr, 0.0, out);
    else hipLaunchKernelGGL((tiled_rows_kernel<0, DT_F64, 3>), dim3(g), dim3(256), 0, st, xb, tiled, d, n, coef, b, nullptr, 0, nullptr, 0.0, out);
    DQ_HIP_CHECK(hipGetLastError());
    return;
  }
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(predict_kernel, dim3(g), dim3(256), 0, st, X, xdt, ld, d, n, coef, b, out, tiled);
  DQ_HIP_CHECK(hipGetLastError());
}

int metrics_blocks(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;  // enough resident blocks to keep fragment loads in flight
  if (g < 1) g = 1;
  return (int)g;
}

void regression_metrics(const void* X, int xdt, int64_t ld, int d, int64_t n, const void* y, int ydt,
                        const uint8_t* sel, const double* coef, double b, double shift, double* partials,
                        double* out, hipStream_t st, int tiled) {
  const int g = metrics_blocks(n);
  if (tiled)
  {
    auto xb = reinterpret_cast<const unsigned char*>(X);
#define DQ_TR(YT, TC)                                                                                      \
  hipLaunchKernelGGL((tiled_rows_kernel<1, YT, TC>), dim3(g), dim3(256), 0, st, xb, tiled, d, n, coef, b, y, ydt, \
                     sel, shift, partials)
#define DQ_TRY(TC)                      \
  if (ydt == DT_F64) DQ_TR(DT_F64, TC); \
  else if (ydt == DT_F32) DQ_TR(DT_F32, TC); \
  else DQ_TR(-1, TC);
    if (tiled == 1) { DQ_TRY(1) } else if (tiled == 2) { DQ_TRY(2) } else { DQ_TRY(3) }
#undef DQ_TRY
#undef DQ_TR
  }  else
    hipLaunchKernelGGL(metrics_kernel, dim3(g), dim3(256), 0, st, X, xdt, ld, d, n, y, ydt, sel, coef, b, shift,
                       partials, tiled);
  hipLaunchKernelGGL(sum_slabs_kernel, dim3(1), dim3(256), 0, st, partials, g, 8, out);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml

// ---- K9: huber loss / gradient pass (LinearRegression loss="huber", Spark HuberAggregator) ------
namespace dq4ml {
namespace {

__device__ __forceinline__ double load_x(const void* X, int xdt, int64_t ld, int d, int f, int64_t r, int tiled) {
  if (tiled == 1) return (double)bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(X)[tiled_offset(f, r, (d + 31) >> 5)]);
  if (tiled == 2)
    return (double)bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(X)[wide_offset(f, r, ((d + 255) >> 8) * 8)]);
  if (tiled == 3)
    return (double)fp8_to_f32(reinterpret_cast<const uint8_t*>(X)[wide_offset_fp8(f, r, ((d + 255) >> 8) * 8)]);
  return ld_f64(X, xdt, (int64_t)f * ld + r);
}

// One row's Huber terms (Spark HuberAggregator): loss, the gradient multiplier m_r of x_r (the
// coefficient of x_j / σ_j), the intercept and σ contributions.
__device__ __forceinline__ double huber_row(double lin, double wt, double sigma, double eps, double acc[4]) {
  double m;
  if (fabs(lin) <= sigma * eps) {
    const double q = lin / sigma;
    acc[0] += 0.5 * wt * (sigma + lin * lin / sigma);
    m = -wt * q;
    acc[2] += -wt * q;
    acc[3] += 0.5 * wt * (1.0 - q * q);
  } else {
    const double sgn = lin >= 0 ? -1.0 : 1.0;
    acc[0] += 0.5 * wt * (sigma + 2.0 * eps * fabs(lin) - sigma * eps * eps);
    m = wt * sgn * eps;
    acc[2] += wt * sgn * eps;
    acc[3] += 0.5 * wt * (1.0 - eps * eps);
  }
  acc[1] += wt;
  return m;
}

// The Huber pass over rows.  D > 0 (d <= D): fused -- after a row's margin each thread adds
// m_r x_r (the row's features again, from cache) into D per-thread sums: one block partial of
// 4 + d values (loss, W, g_b, g_sigma, Σ m x), the features read from HBM once.  D = 0: the margin pass only
// (4 partials + the multipliers in `mult`), Xᵀm by xt_part_kernel.
//
// Device-steered form (huber_qn.hip): `act` non-null -> ceff = the trial [c_eff (d) | intercept |
// sigma] in HBM, and the pass is skipped once the optimizer is done (act != kHuberEval).
template <int D>
__global__ __launch_bounds__(256) void huber_rows_kernel(const void* __restrict__ X, int xdt, int64_t ld, int d,
                                                        int64_t n, int tiled, const void* __restrict__ y, int ydt,
                                                        const void* __restrict__ w, int wdt,
                                                        const uint8_t* __restrict__ sel,
                                                        const double* __restrict__ ceff /* c_j/σ_j */,
                                                        double icpt, double sigma, double eps,
                                                        double* __restrict__ mult, double* __restrict__ partials,
                                                        const int* __restrict__ act) {
  if (act != nullptr) {
    if (*act != kHuberEval) return;
    icpt = ceff[d];
    sigma = ceff[d + 1];
  }
  constexpr int W = D > 0 ? D : 1;
  double acc[4] = {0, 0, 0, 0};
  double ax[W];
#pragma unroll
  for (int j = 0; j < W; ++j) ax[j] = 0.0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    double m = 0.0;
    const bool live = sel == nullptr || sel[r] != 0;
    const double wt = live ? (w ? ld_f64(w, wdt, r) : 1.0) : 0.0;
    if (wt != 0.0) {
      if constexpr (D > 0) {
        const double margin = predict_row(X, xdt, ld, d, ceff, icpt, r, tiled);
        m = huber_row(ld_f64(y, ydt, r) - margin, wt, sigma, eps, acc);
#pragma unroll
        for (int f = 0; f < D; ++f)  // (the row's features again: cache hits)
          if (f < d) ax[f] += m * load_x(X, xdt, ld, d, f, r, tiled);
      } else {
        const double margin = predict_row(X, xdt, ld, d, ceff, icpt, r, tiled);
        m = huber_row(ld_f64(y, ydt, r) - margin, wt, sigma, eps, acc);
      }
    }
    if constexpr (D == 0) mult[r] = m;
  }
  constexpr int K = 4 + (D > 0 ? D : 0);
  __shared__ double red[4][K];
  const int width = D > 0 ? 4 + d : 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = wave_sum_f64(acc[k]);
#pragma unroll
  for (int j = 0; j < (D > 0 ? D : 0); ++j)
    if (j < d) ax[j] = wave_sum_f64(ax[j]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[threadIdx.x >> 6][k] = acc[k];
#pragma unroll
    for (int j = 0; j < (D > 0 ? D : 0); ++j)
      if (j < d) red[threadIdx.x >> 6][4 + j] = ax[j];
  }
  __syncthreads();
  if (threadIdx.x < width)
    partials[(int64_t)blockIdx.x * width + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// The fused pass over dense feature-major columns of T (f32 / f64), d <= D: a row's d features
// are loaded together into registers (no per-element dtype switch between the loads, so they are
// all in flight at once), used for the margin and again for Σ m x.  Same partial layout and the
// same per-row arithmetic as huber_rows_kernel<D>.  The feature loads are non-temporal (each
// evaluation streams X once and X exceeds the MALL): 3.66 -> 3.51-3.55 ms per 1e7 x 16 fit on
// one box, 4.00 -> 3.66 (mean of three noisy pairs) on another (profiles/r6_huber_device.md).
template <typename T, int D>
__global__ __launch_bounds__(256) void huber_rows_dense_kernel(const T* __restrict__ X, int64_t ld, int d, int64_t n,
                                                              const void* __restrict__ y, int ydt,
                                                              const void* __restrict__ w, int wdt,
                                                              const uint8_t* __restrict__ sel,
                                                              const double* __restrict__ ceff, double icpt,
                                                              double sigma, double eps,
                                                              double* __restrict__ partials,
                                                              const int* __restrict__ act) {
  if (act != nullptr) {
    if (*act != kHuberEval) return;
    icpt = ceff[d];
    sigma = ceff[d + 1];
  }
  double acc[4] = {0, 0, 0, 0};
  double ax[D];
  double cf[D];
#pragma unroll
  for (int j = 0; j < D; ++j) ax[j] = 0.0, cf[j] = j < d ? ceff[j] : 0.0;
  // software-pipelined: the next row's features are in flight while this row computes (two rows'
  // loads per thread outstanding; the last trip re-loads its own row)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  T xn[D];
#pragma unroll
  for (int f = 0; f < D; ++f) xn[f] = (f < d && r < n) ? __builtin_nontemporal_load(X + (int64_t)f * ld + r) : T(0);
  for (; r < n; r += stride) {
    T xs[D];
#pragma unroll
    for (int f = 0; f < D; ++f) xs[f] = xn[f];
    const int64_t rn = r + stride < n ? r + stride : r;
#pragma unroll
    for (int f = 0; f < D; ++f) xn[f] = f < d ? __builtin_nontemporal_load(X + (int64_t)f * ld + rn) : T(0);
    const bool live = sel == nullptr || sel[r] != 0;
    const double wt = live ? (w ? ld_f64(w, wdt, r) : 1.0) : 0.0;
    if (wt == 0.0) continue;
    double margin = icpt;
#pragma unroll
    for (int f = 0; f < D; ++f)
      if (f < d) margin += cf[f] * (double)xs[f];
    const double m = huber_row(ld_f64(y, ydt, r) - margin, wt, sigma, eps, acc);
#pragma unroll
    for (int f = 0; f < D; ++f)
      if (f < d) ax[f] += m * (double)xs[f];
  }
  __shared__ double red[4][4 + D];
  const int width = 4 + d;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = wave_sum_f64(acc[k]);
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < d) ax[j] = wave_sum_f64(ax[j]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) red[threadIdx.x >> 6][k] = acc[k];
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j < d) red[threadIdx.x >> 6][4 + j] = ax[j];
  }
  __syncthreads();
  if (threadIdx.x < width)
    partials[(int64_t)blockIdx.x * width + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// Xᵀm for d > kHuberFuseD: block (c, j) sums feature j over row chunk c (fixed order), xt_fold_kernel
// adds the chunks of each feature in order
__global__ __launch_bounds__(256) void xt_part_kernel(const void* __restrict__ X, int xdt, int64_t ld, int d, int64_t n,
                                                     int tiled, const double* __restrict__ v, int64_t chunk,
                                                     double* __restrict__ part, const int* __restrict__ act) {
  if (act != nullptr && *act != kHuberEval) return;
  const int c = blockIdx.x, j = blockIdx.y;
  const int64_t r0 = (int64_t)c * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  double s = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x)
    if (v[r] != 0.0) s += load_x(X, xdt, ld, d, j, r, tiled) * v[r];
  __shared__ double red[4];
  s = wave_sum_f64(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)j * gridDim.x + c] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void xt_fold_kernel(const double* __restrict__ part, int d, int chunks,
                                                     double* __restrict__ out, const int* __restrict__ act) {
  if (act != nullptr && *act != kHuberEval) return;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += part[(int64_t)j * chunks + c];
  out[j] = s;
}

// the storage epilogue of the device-steered pass: fp8 storage q = x / scale; shifted storage x =
// x' + s: Σ m x = Σ m x' + s Σ m (out[2] = Σ m)
__global__ __launch_bounds__(256) void huber_epilogue_kernel(double* __restrict__ out, int d,
                                                            const double* __restrict__ scale,
                                                            const double* __restrict__ shift,
                                                            const int* __restrict__ act) {
#pragma clang fp contract(off)  // two roundings each, as the host-steered fold's torch expressions
  if (*act != kHuberEval) return;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d) return;
  double t = out[4 + j];
  if (scale != nullptr) t *= scale[j];
  if (shift != nullptr) t += shift[j] * out[2];
  out[4 + j] = t;
}

// sum_slabs_kernel with one block per column (the same fixed-order sum of each column)
__global__ __launch_bounds__(256) void sum_cols_kernel(const double* __restrict__ partials, int nslab, int width,
                                                      double* __restrict__ out, const int* __restrict__ act) {
  if (act != nullptr && *act != kHuberEval) return;
  const int k = blockIdx.x;
  __shared__ double wsum[4];
  double s = 0.0;
  for (int b = threadIdx.x; b < nslab; b += blockDim.x) s += partials[(int64_t)b * width + k];
  s = wave_sum_f64(s);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[k] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

constexpr int kHuberFuseD = 16;

int64_t xt_chunks(int64_t n, int d) {
  int64_t c = (n + 65535) / 65536;
  const int64_t cap = d >= 2048 ? 1 : 2048 / d;
  if (c > cap) c = cap;
  return c < 1 ? 1 : c;
}

void launch_huber(const void* X, int xdt, int64_t ld, int d, int64_t n, int tiled, const void* y, int ydt,
                  const void* w, int wdt, const uint8_t* sel, const double* ceff, double icpt, double sigma,
                  double eps, double* mult, double* partials, double* out, const int* act, hipStream_t st) {
  const int g = metrics_blocks(n);
  if (d <= kHuberFuseD && tiled == 0 && (xdt == DT_F32 || xdt == DT_F64)) {
    if (xdt == DT_F32)
      hipLaunchKernelGGL((huber_rows_dense_kernel<float, kHuberFuseD>), dim3(g), dim3(256), 0, st,
                         reinterpret_cast<const float*>(X), ld, d, n, y, ydt, w, wdt, sel, ceff, icpt, sigma, eps,
                         partials, act);
    else
      hipLaunchKernelGGL((huber_rows_dense_kernel<double, kHuberFuseD>), dim3(g), dim3(256), 0, st,
                         reinterpret_cast<const double*>(X), ld, d, n, y, ydt, w, wdt, sel, ceff, icpt, sigma, eps,
                         partials, act);
    hipLaunchKernelGGL(sum_cols_kernel, dim3(4 + d), dim3(256), 0, st, partials, g, 4 + d, out, act);
  } else if (d <= kHuberFuseD) {
    hipLaunchKernelGGL(huber_rows_kernel<kHuberFuseD>, dim3(g), dim3(256), 0, st, X, xdt, ld, d, n, tiled, y, ydt, w, wdt, sel, ceff, icpt, sigma,
                       eps, mult, partials, act);
    hipLaunchKernelGGL(sum_cols_kernel, dim3(4 + d), dim3(256), 0, st, partials, g, 4 + d, out, act);
  } else {
    hipLaunchKernelGGL(huber_rows_kernel<0>, dim3(g), dim3(256), 0, st, X, xdt, ld, d, n, tiled, y, ydt, w, wdt, sel,
                       ceff, icpt, sigma, eps, mult, partials, act);
    hipLaunchKernelGGL(sum_slabs_kernel, dim3(1), dim3(256), 0, st, partials, g, 4, out);
    const int64_t c = xt_chunks(n, d), chunk = (n + c - 1) / c;
    double* part = partials + (int64_t)g * 4;
    hipLaunchKernelGGL(xt_part_kernel, dim3((unsigned)c, (unsigned)d), dim3(256), 0, st, X, xdt, ld, d, n, tiled,
                       mult, chunk, part, act);
    hipLaunchKernelGGL(xt_fold_kernel, dim3((d + 255) / 256), dim3(256), 0, st, part, d, (int)c, out + 4, act);
  }
}

}  // namespace

int64_t huber_partials(int64_t n, int d) {
  const int64_t g = metrics_blocks(n);
  return d <= kHuberFuseD ? g * (4 + d) : g * 4 + (int64_t)d * xt_chunks(n, d);
}

void huber_pass(const void* X, int xdt, int64_t ld, int d, int64_t n, int tiled, const void* y, int ydt,
                const void* w, int wdt, const uint8_t* sel, const double* ceff, double icpt, double sigma, double eps,
                double* mult, double* partials, double* out /* [4 + d] */, hipStream_t st) {
  launch_huber(X, xdt, ld, d, n, tiled, y, ydt, w, wdt, sel, ceff, icpt, sigma, eps, mult, partials, out, nullptr, st);
  DQ_HIP_CHECK(hipGetLastError());
}

void huber_pass_dev(const void* X, int xdt, int64_t ld, int d, int64_t n, int tiled, const void* y, int ydt,
                    const void* w, int wdt, const uint8_t* sel, const double* trial, const int* act, double eps,
                    const double* scale, const double* shift, double* mult, double* partials, double* out,
                    hipStream_t st) {
  if (act == nullptr || trial == nullptr) throw std::invalid_argument("huber_pass_dev: trial and act are required");
  launch_huber(X, xdt, ld, d, n, tiled, y, ydt, w, wdt, sel, trial, 0.0, 1.0, eps, mult, partials, out, act, st);
  if (scale != nullptr || shift != nullptr)
    hipLaunchKernelGGL(huber_epilogue_kernel, dim3((d + 255) / 256), dim3(256), 0, st, out, d, scale, shift, act);
  DQ_HIP_CHECK(hipGetLastError());
}

// Stand-in for a collective kernel of the fit tail (diagnostics / tests: models/regression.py
// DQ4ML_TAIL_STANDIN): `blocks` workgroups that each hold a CU slot for `usec` microseconds
// (s_memrealtime runs at 100 MHz), the shape of an RCCL all-reduce's channel blocks.  The wait is
// bounded (<= 1 ms) so the grid always drains.
namespace {
__global__ __launch_bounds__(256) void standin_kernel(int64_t ticks) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(2);
  }
  __syncthreads();
}
}  // namespace

void standin(int blocks, int usec, hipStream_t st) {
  if (blocks < 1 || blocks > 4096 || usec < 0 || usec > 1000) throw std::invalid_argument("standin: bad shape");
  hipLaunchKernelGGL(standin_kernel, dim3(blocks), dim3(256), 0, st, (int64_t)usec * 100);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
