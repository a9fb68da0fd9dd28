// K5 — WLS sufficient statistics ("Gram") of a feature-major matrix on MFMA.
//
// Replaces Spark's per-row ``WeightedLeastSquares.Aggregator.add`` (BLAS.spr of every row into a
// packed Gram) triggered by LinearRegression.fit at
// DataQuality4MachineLearningApp.java:126.  One streaming pass over
//     X  [d, ld]  feature-major (bf16 / f32 / f64),  y [n],  optional w [n] and selection sel [n]
// produces   count, Σw, Σw², Σwy, Σwy², Σw·x (d), Σw·x·y (d), Σ w·x·xᵀ (upper)   in f64.
//
// Tall-skinny design (d <= 64, memory bound: 1e8 x 32 bf16 = 6.4 GB per pass):
//  * "superstep" = 64 consecutive rows.  Lane l of a wave owns feature f = l & 31 (bf16/f32
//    modes) and the row half h = l >> 5, and loads ITS 32 rows of ITS feature as contiguous
//    16-byte vectors — in feature-major storage that is exactly the A/B fragment of
//    v_mfma_f32_32x32x16_bf16 (A[i=l&31][k=8h+j]) with the K index permuted (allowed: Σ_k is
//    order-free as long as A and B use the same permutation, and they are the same registers).
//    No LDS transpose, no shuffles: 4 loads + 4 MFMAs per 32-feature tile per superstep.
//  * Upper tile pairs only (d <= 32: 1 pair, d <= 64: 3 pairs).
//  * Column sums and Xᵀy ride on a second MFMA with B = [w_hi, w_lo, wy_hi, wy_lo, 0...]: the
//    per-row scalars are computed lane = row (coalesced), split hi/lo into bf16 (≈16-bit
//    mantissa for the label) and handed to the fragment layout through a 512-byte LDS stripe.
//  * f64 mode (Spark-parity path) uses v_mfma_f64_16x16x4_f64 with 16-feature tiles and exact
//    f64 side sums on the VALU.
//  * Per-wave f32 (bf16 mode) / f64 accumulators -> deterministic in-block wave reduction in
//    LDS -> one f64 partial slab per block -> ``gram_reduce`` sums slabs in a fixed order (no
//    atomics: bit-reproducible run to run).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "gram.h"

namespace dq4ml {

namespace {

constexpr int kBlock = 256;  // f64 kernel: 4 waves
constexpr int kWavesPerBlock = kBlock / kWave;
// bf16 kernel: 8 waves per block -- two co-resident per CU at <= 128 VGPRs for d <= 32 (HALF
// below), one per CU at <= 256 VGPRs for d <= 64; the round-4 16-wave block filled a CU alone
// HALF (d <= 32 unmasked; since round 5 -- the 16-wave block lost): 8-wave blocks, two resident per CU, so one block's ramp and reduction overlap the other's
// stream and the next pass's blocks start beside this pass's last ones.  Same box, two reps
// (profiles/r5_shard_drain.md): 1.25e7-row shard 0.1297 / 0.1292 vs 0.1347 / 0.1365 ms per fit,
// 1e8 headline 0.987 / 0.989 vs 0.994 / 0.992 ms.
template <int NT, int XMODE, bool HALF = false>
struct BF16Geom {
  static constexpr int kBlock = (NT == 1 && XMODE == 0 && !HALF) ? 1024 : 512;
  static constexpr int kWaves = kBlock / kWave;
  static constexpr int kMinBlocks = HALF ? 2 : 1;
};
static int bf16_block(int, int) { return 512; }  // (HALF at d <= 32, the 8-wave block elsewhere)

__device__ __forceinline__ double load_as_f64(const void* p, int dt, int64_t i) {
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

// per-row scalars of row r (lane = row): liveness, weight, label
struct RowVals {
  bool live;
  double w, y, wy;
};

__device__ __forceinline__ RowVals row_vals(const GramArgs& a, int64_t r) {
  RowVals v{false, 0.0, 0.0, 0.0};
  if (r < a.n) {
    bool live = a.sel ? (a.sel[r] != 0) : true;
    if (live) {
      double w = a.w ? load_as_f64(a.w, a.wdt, r) : 1.0;
      double y = load_as_f64(a.y, a.ydt, r);
      v.live = true;
      v.w = w;
      v.y = y;
      v.wy = w * y;
    }
  }
  return v;
}

struct RowAcc {
  double cnt = 0, ws = 0, wws = 0, bs = 0, bbs = 0;
  __device__ __forceinline__ void add(const RowVals& v) {
    if (v.live) {
      cnt += 1.0;
      ws += v.w;
      wws += v.w * v.w;
      bs += v.wy;
      bbs += v.wy * v.y;
    }
  }
};

// ---- 32 rows of one feature as 4 bf16x8 fragments --------------------------------------------
template <typename T>
__device__ __forceinline__ void load_rows32_bf16(const T* p, int64_t rows_left, bf16x8 (&fr)[4]);

template <>
__device__ __forceinline__ void load_rows32_bf16<uint16_t>(const uint16_t* p, int64_t rows_left, bf16x8 (&fr)[4]) {
  if (rows_left >= 32) {
    const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      u32x4 u = __builtin_nontemporal_load(q + i);
      fr[i] = __builtin_bit_cast(bf16x8, u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 8 * i + j;
        uint16_t b = e < rows_left ? p[e] : uint16_t(0);
        fr[i][j] = __builtin_bit_cast(__bf16, b);
      }
    }
  }
}

template <>
__device__ __forceinline__ void load_rows32_bf16<float>(const float* p, int64_t rows_left, bf16x8 (&fr)[4]) {
  if (rows_left >= 32) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 a = __builtin_nontemporal_load(q + 2 * i);
      f32x4 b = __builtin_nontemporal_load(q + 2 * i + 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fr[i][j] = (__bf16)a[j];
        fr[i][4 + j] = (__bf16)b[j];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 8 * i + j;
        fr[i][j] = (__bf16)(e < rows_left ? p[e] : 0.0f);
      }
  }
}

template <>
__device__ __forceinline__ void load_rows32_bf16<double>(const double* p, int64_t rows_left, bf16x8 (&fr)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = 8 * i + j;
      fr[i][j] = (__bf16)(float)(e < rows_left ? p[e] : 0.0);
    }
}

// zero the elements of dead rows (binary mask): bits = liveness of the lane's 32 rows
__device__ __forceinline__ void mask_frags(bf16x8 (&fr)[4], uint32_t bits) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!((bits >> (8 * i + j)) & 1u)) fr[i][j] = (__bf16)0.0f;
}

__device__ __forceinline__ void weight_frags(bf16x8 (&fr)[4], const float* wl /* lane's 32 row weights in LDS */) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) fr[i][j] = (__bf16)((float)fr[i][j] * wl[8 * i + j]);
}

// slab element o (storage order: head, then T x T tiles of the row-major upper pairs I <= J < NT)
// -> its packed-upper destination; lower halves of the diagonal tiles and padding features drop
__device__ __forceinline__ void fold_store(int o, double t, int d, int T, int NT, double* __restrict__ out) {
  const int head = 5 + 2 * d;
  if (o < head) {
    out[o] = t;
    return;
  }
  const int e = o - head, pr = e / (T * T), w = e - pr * T * T, r = w / T, cc = w - (w / T) * T;
  int I = 0, rem = pr;
  while (rem >= NT - I) {
    rem -= NT - I;
    ++I;
  }
  const int J = I + rem;
  const int64_t i = (int64_t)I * T + r, j = (int64_t)J * T + cc;
  if (i <= j && j < d) out[head + i + j * (j + 1) / 2] = t;
}

// Slab stores: the slabs are folded by gram_fold_kernel after the kernel boundary (an in-kernel
// fold by the last block of each XCD group was measured slower at the 8-GPU shard: 155 us vs
// 142-148 us per fit, profiles/r3_fixed_cost.md; removed in round 4).  Relaxed agent-scope
// stores write through to memory (nothing is left dirty in this XCD's L2 for the fold kernel's
// boundary to flush) -- the form the round-3 headline was measured with.
__device__ __forceinline__ void slab_put(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// =============================================================================================
// bf16 MFMA kernel
// =============================================================================================
template <typename TX, int NT, int XMODE, bool TILED, bool HALF = false>
__global__ __launch_bounds__((BF16Geom<NT, XMODE, HALF>::kBlock), (BF16Geom<NT, XMODE, HALF>::kMinBlocks)) void
gram_tall_bf16_kernel(GramArgs a) {
  typedef BF16Geom<NT, XMODE, HALF> Geo;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  // LDS: per wave 4 cols x 64 rows bf16 (W fragments) + 64 f32 row weights; reused for the
  // block reduction afterwards.
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int f = lane & 31, h = lane >> 5;
  __bf16* wl = reinterpret_cast<__bf16*>(smem) + wave * (4 * 64);
  float* wrow = reinterpret_cast<float*>(smem + Geo::kWaves * 4 * 64 * 2) + wave * 64;

  f32x16 acc[NPAIR];
  f32x16 accw[NT];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = f32x16{};
#pragma unroll
  for (int t = 0; t < NT; ++t) accw[t] = f32x16{};
  RowAcc ra;

  const TX* X = reinterpret_cast<const TX*>(a.X);
  const TX* fp[NT];
  bool fvalid[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int feat = t * 32 + f;
    fvalid[t] = feat < a.d;
    fp[t] = X + (int64_t)(fvalid[t] ? feat : 0) * a.ld + 32 * h;
  }

  const int64_t gw = (int64_t)blockIdx.x * Geo::kWaves + wave;
  const int64_t total_waves = (int64_t)gridDim.x * Geo::kWaves;
  int64_t s0 = gw * a.spw;
  int64_t s1 = s0 + a.spw;
  if (s1 > a.nsuper) s1 = a.nsuper;
  const bool do_tail = (gw == total_waves - 1) && (a.n > a.nsuper * 64);

  // One superstep of compute on already-loaded feature fragments.
  auto compute = [&](int64_t r0, bf16x8 (&fr)[NT][4]) {
    // 1) per-row scalars, lane = row
    RowVals rv = row_vals(a, r0 + lane);
    ra.add(rv);
    {
      const float w_hi = (float)(__bf16)(float)rv.w;
      const __bf16 wy_hi = (__bf16)(float)rv.wy;
      wl[0 * 64 + lane] = (__bf16)(float)rv.w;
      wl[1 * 64 + lane] = (__bf16)(float)(rv.w - (double)w_hi);
      wl[2 * 64 + lane] = wy_hi;
      wl[3 * 64 + lane] = (__bf16)(float)(rv.wy - (double)(float)wy_hi);
      if (XMODE == 2) wrow[lane] = (float)rv.w;
    }
    const uint64_t live_bits = __ballot(rv.live);
    __builtin_amdgcn_wave_barrier();
    // 2) W fragments (lanes f < 4 read their column; everyone else multiplies zeros)
    bf16x8 wf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) wf[i] = bf16x8{};
    if (f < 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) wf[i] = *reinterpret_cast<const bf16x8*>(wl + f * 64 + 32 * h + 8 * i);
    }
    // 3) masking / weighting of one operand of XᵀX
    bf16x8 frw[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) frw[t][i] = fr[t][i];
    if (XMODE == 1) {
      const uint32_t bits = (uint32_t)(live_bits >> (32 * h));
#pragma unroll
      for (int t = 0; t < NT; ++t) mask_frags(frw[t], bits);
    } else if (XMODE == 2) {
#pragma unroll
      for (int t = 0; t < NT; ++t) weight_frags(frw[t], wrow + 32 * h);
    }
    // 4) MFMAs
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[I][i], frw[J][i], acc[p], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) accw[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[t][i], wf[i], accw[t], 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
  };
  auto load = [&](int64_t r0, int64_t rows_left, bf16x8 (&fr)[NT][4]) {
    if constexpr (TILED) {
      // MFMA-fragment-ordered storage: superstep s, tile t, k-step i = 1 KiB contiguous
      const u32x4* q = reinterpret_cast<const u32x4*>(a.X) + ((r0 >> 6) * NT) * 4 * 64 + lane;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) fr[t][i] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(q + (t * 4 + i) * 64));
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (fvalid[t]) {
        load_rows32_bf16<TX>(fp[t] + r0, rows_left, fr[t]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) fr[t][i] = bf16x8{};
      }
    }
  };

  // full supersteps: register double buffer (loads of s+1 in flight while s computes)
  if (a.interleave) {
    if (gw < a.nsuper) {
      bf16x8 cur[NT][4], nxt[NT][4];
      load(gw * 64, 64, cur);
      for (int64_t s = gw; s < a.nsuper; s += total_waves) {
        if (s + total_waves < a.nsuper) load((s + total_waves) * 64, 64, nxt);
        compute(s * 64, cur);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) cur[t][i] = nxt[t][i];
      }
    }
  } else if (s0 < s1) {
    bf16x8 cur[NT][4], nxt[NT][4];
    load(s0 * 64, 64, cur);
    for (int64_t s = s0; s < s1; ++s) {
      if (s + 1 < s1) load((s + 1) * 64, 64, nxt);
      compute(s * 64, cur);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) cur[t][i] = nxt[t][i];
    }
  }
  // ragged tail (rows not filling a 64-row superstep): last wave only, guarded loads
  if (do_tail) {
    bf16x8 tl[NT][4];
    const int64_t r0 = a.nsuper * 64;
    load(r0, a.n - (r0 + 32 * h), tl);  // tiled storage is zero padded to a whole superstep
    compute(r0, tl);
  }

  // ---- block reduction: fixed-shape tree over the waves (deterministic), 4 rounds ------------
  constexpr int W = Geo::kWaves;
  constexpr int NV = (NPAIR + NT) * 16;  // f32 accumulator values per lane
  const int d = a.d;
  double sc[5] = {ra.cnt, ra.ws, ra.wws, ra.bs, ra.bbs};
#pragma unroll
  for (int k = 0; k < 5; ++k) sc[k] = wave_sum_f64(sc[k]);
  __syncthreads();  // W stripes are dead from here on: reuse the LDS
  float* tr = reinterpret_cast<float*>(smem);
  double* scl = reinterpret_cast<double*>(smem + (size_t)(W / 2) * NV * 64 * sizeof(float));
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 5; ++k) scl[wave * 5 + k] = sc[k];
  }
#pragma unroll
  for (int step = W / 2; step >= 1; step >>= 1) {
    if (wave >= step && wave < 2 * step) {
      float* dst = tr + (size_t)(wave - step) * NV * 64 + lane;
      int v = 0;
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(v++) * 64] = acc[p][r];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(v++) * 64] = accw[t][r];
    }
    __syncthreads();
    if (wave < step) {
      const float* src = tr + (size_t)wave * NV * 64 + lane;
      int v = 0;
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][r] += src[(v++) * 64];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accw[t][r] += src[(v++) * 64];
    }
    __syncthreads();
  }
  if (wave == 0) {
    double* out = a.partials + (int64_t)blockIdx.x * a.P;
    if (lane < 5) {
      double t = 0.0;
      for (int w = 0; w < W; ++w) t += scl[w * 5 + lane];
      slab_put(out + lane, t);
    }
    const int col = mfma32_col(lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      // accw[t]: rows = features t*32 + row, cols 0..3 = [w_hi, w_lo, wy_hi, wy_lo]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = accw[t][r];
        const float vn = __shfl_down(v, 1, 64);  // col+1 (same row)
        const int feat = t * 32 + mfma32_row(lane, r);
        if (feat < d) {
          if (col == 0) slab_put(out + 5 + feat, (double)v + (double)vn);
          if (col == 2) slab_put(out + 5 + d + feat, (double)v + (double)vn);
        }
      }
    }
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++p) {
        double* tile = out + 5 + 2 * d + p * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) slab_put(tile + mfma32_row(lane, r) * 32 + col, (double)acc[p][r]);
      }
  }
}

// =============================================================================================
// Fused assemble + Gram over SOURCE COLUMNS (d <= 64): the VectorAssembler output is never
// materialized.  Block-cooperative superstep: 256 threads vector-load 64 rows x 32*NT features
// with 16-B loads (thread (f, q) = rows [8q, 8q+8) of feature f: coalesced 256-B column runs),
// convert to bf16 (dead rows of the selection -> 0) and store them in MFMA-fragment order in LDS
// (that octet IS one lane's fragment of k-step q & 3, half q >> 2); wave w then runs k-step w's
// MFMAs for every tile pair.  Next superstep's global loads are in flight during the MFMAs;
// double-buffered LDS, one barrier per superstep.  Partials use the bf16 kernel's slab layout.
// =============================================================================================
template <int NT, int SDT, int YDT>  // SDT: common source dtype (-1 mixed); YDT: label dtype (F32/F64)
__global__ __launch_bounds__(256, (NT == 1 ? 3 : 2)) void gram_cols_kernel(GramArgs a, const PackSrcG* __restrict__ srcs) {
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int FR = NT * 4 * 64 * 16;   // fragment bytes per superstep
  constexpr int BUF = FR + 4 * 64 * 2;   // + W stripe [4 cols][64 rows] bf16
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int f = lane & 31, h = lane >> 5;
  const int fl = tid >> 3, q = tid & 7;

  f32x16 acc[NPAIR];
  f32x16 accw[NT];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) acc[p] = f32x16{};
#pragma unroll
  for (int t = 0; t < NT; ++t) accw[t] = f32x16{};
  RowAcc ra;

  PackSrcG src[NT];
  bool fv[NT];
  float sh[NT];  // the thread's feature shifts (GramArgs::xshift; 0 without one)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int feat = t * 32 + fl;
    fv[t] = feat < a.d;
    src[t] = srcs[fv[t] ? feat : 0];  // padding features load column 0 (branch-free) and stage zeros
    sh[t] = (a.xshift && fv[t]) ? a.xshift[feat] : 0.0f;
  }
  const int64_t nsup = (a.n + 63) / 64, nfull = a.n / 64;
  const int64_t s0 = (int64_t)blockIdx.x * a.spw;
  const int64_t s1 = s0 + a.spw < nsup ? s0 + a.spw : nsup;
  const int64_t e1 = s1 < nfull ? s1 : nfull;  // full supersteps of this block: [s0, e1)

  // Everything a superstep needs is PREFETCHED into registers (features, selection bytes, the
  // label of row tid for the 64 row-scalar threads) with branch-free typed loads, so the only
  // vmcnt waits in the loop are the compiler's counted ones at first use — no scalar load in the
  // loop can drain the prefetch.
  struct Pref {
    float x[NT][8];
    uint64_t m;
    double yv;
    uint32_t live;
  };
  auto gload = [&](int64_t s, Pref& p) {
    const int64_t r0 = s * 64 + 8 * q;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr (SDT >= 0) load8_typed<SDT, true>(src[t].ptr, r0, a.n, p.x[t]);
      else load8_f32(src[t].ptr, src[t].dt, r0, a.n, p.x[t]);
    }
    // branch-free: the host always passes a selection (all ones when there is none) and every
    // wave loads the row scalars (only wave 0 uses them) so the compiler can count the loads
    p.m = *gptr<uint64_t>(a.sel + r0);
    const int64_t r = s * 64 + (tid & 63);
    p.yv = YDT == DT_F64 ? gptr<double>(a.y)[r] : (double)gptr<float>(a.y)[r];
    p.live = gptr<uint8_t>(a.sel)[r];
  };
  auto stage_w = [&](unsigned char* base, const RowVals& rv) {
    __bf16* wl = reinterpret_cast<__bf16*>(base + FR);
    const float w_hi = (float)(__bf16)(float)rv.w;
    const __bf16 wy_hi = (__bf16)(float)rv.wy;
    wl[0 * 64 + tid] = (__bf16)(float)rv.w;
    wl[1 * 64 + tid] = (__bf16)(float)(rv.w - (double)w_hi);
    wl[2 * 64 + tid] = wy_hi;
    wl[3 * 64 + tid] = (__bf16)(float)(rv.wy - (double)(float)wy_hi);
  };
  // x - s of the live rows to bf16 (dead rows and padding features exactly 0); sub = false: x
  // is already shifted and masked (the guarded last superstep)
  auto stage_x = [&](unsigned char* base, float (&x)[NT][8], uint64_t m, bool sub = true) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float s_t = sub ? sh[t] : 0.0f;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)(fv[t] && ((m >> (8 * j)) & 0xff) ? x[t][j] - s_t : 0.0f);
      *reinterpret_cast<u32x4*>(base + (((t * 4 + (q & 3)) * 64 + 32 * (q >> 2) + fl) << 4)) = __builtin_bit_cast(u32x4, v);
    }
  };
  auto stage = [&](int buf, Pref& p) {
    unsigned char* base = smem + buf * BUF;
    stage_x(base, p.x, p.m);
    if (tid < 64) {
      RowVals rv{p.live != 0, 0.0, 0.0, 0.0};
      if (rv.live) {
        rv.w = 1.0;
        rv.y = p.yv;
        rv.wy = p.yv;
      }
      ra.add(rv);
      stage_w(base, rv);
    }
  };
  auto compute = [&](int buf) {
    const unsigned char* base = smem + buf * BUF;
    const int i = wave;  // this wave's k-step
    bf16x8 fr[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) fr[t] = *reinterpret_cast<const bf16x8*>(base + (((t * 4 + i) * 64 + lane) << 4));
    bf16x8 wf = bf16x8{};
    if (f < 4) wf = *reinterpret_cast<const bf16x8*>(base + FR + (f * 64 + 32 * h + 8 * i) * 2);
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++p) acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[I], fr[J], acc[p], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < NT; ++t) accw[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[t], wf, accw[t], 0, 0, 0);
  };

  Pref pa, pb;
  if (s0 < e1) gload(s0, pa);
  if (s0 + 1 < e1) gload(s0 + 1, pb);
  int64_t s = s0;
  // unrolled by two so the register ring has static names; prefetches past the end re-load the
  // last superstep (unconditional, so the compiler counts vmcnt instead of draining to 0)
  for (; s + 1 < e1; s += 2) {
    stage(0, pa);
    gload(s + 2 < e1 ? s + 2 : e1 - 1, pa);
    __syncthreads();
    compute(0);
    stage(1, pb);
    gload(s + 3 < e1 ? s + 3 : e1 - 1, pb);
    __syncthreads();
    compute(1);
  }
  if (s < e1) {
    stage(0, pa);
    __syncthreads();
    compute(0);
    __syncthreads();
  }
  if (s1 > nfull && s0 <= nfull) {  // ragged last superstep: guarded loads (once in the grid)
    const int64_t st = nfull, r0 = st * 64 + 8 * q;
    float x[NT][8];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (fv[t]) load8_f32(src[t].ptr, src[t].dt, r0, a.n, x[t]);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) x[t][j] = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (r0 + j < a.n) x[t][j] -= sh[t];  // rows past n stay 0
      mask8(a.sel, r0, a.n, x[t]);
    }
    stage_x(smem + BUF, x, ~0ull, false);
    if (tid < 64) {
      const RowVals rv = row_vals(a, st * 64 + tid);
      ra.add(rv);
      stage_w(smem + BUF, rv);
    }
    __syncthreads();
    compute(1);
  }

  // ---- block reduction over the 4 waves (two tree rounds) + partial slab -----------------------
  constexpr int NV = (NPAIR + NT) * 16;
  double sc[5] = {ra.cnt, ra.ws, ra.wws, ra.bs, ra.bbs};
#pragma unroll
  for (int k = 0; k < 5; ++k) sc[k] = wave_sum_f64(sc[k]);
  __syncthreads();
  float* tr = reinterpret_cast<float*>(smem);
  double* scl = reinterpret_cast<double*>(smem + (size_t)2 * NV * 64 * sizeof(float));
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 5; ++k) scl[wave * 5 + k] = sc[k];
  }
#pragma unroll
  for (int step = 2; step >= 1; step >>= 1) {
    if (wave >= step && wave < 2 * step) {
      float* dst = tr + (size_t)(wave - step) * NV * 64 + lane;
      int v = 0;
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(v++) * 64] = acc[p][r];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(v++) * 64] = accw[t][r];
    }
    __syncthreads();
    if (wave < step) {
      const float* srcp = tr + (size_t)wave * NV * 64 + lane;
      int v = 0;
#pragma unroll
      for (int p = 0; p < NPAIR; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][r] += srcp[(v++) * 64];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accw[t][r] += srcp[(v++) * 64];
    }
    __syncthreads();
  }
  if (wave == 0) {
    const int d = a.d;
    double* out = a.partials + (int64_t)blockIdx.x * a.P;
    if (lane < 5) slab_put(out + lane, scl[lane] + scl[5 + lane] + scl[10 + lane] + scl[15 + lane]);
    const int col = mfma32_col(lane);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = accw[t][r];
        const float vn = __shfl_down(v, 1, 64);
        const int feat = t * 32 + mfma32_row(lane, r);
        if (feat < d) {
          if (col == 0) slab_put(out + 5 + feat, (double)v + (double)vn);
          if (col == 2) slab_put(out + 5 + d + feat, (double)v + (double)vn);
        }
      }
    }
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++p) {
        double* tile = out + 5 + 2 * d + p * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) slab_put(tile + mfma32_row(lane, r) * 32 + col, (double)acc[p][r]);
      }
  }
}

constexpr int kStageLd = 66;  // f64 staging row stride (doubles): 2-double pad spreads the banks

// Cooperative load of features [f0, f0 + 16) x rows [r0, r0 + 64) of a feature-major matrix into a
// per-wave LDS tile xs[f][row] (f64), zeros for features >= d.  Chunk c = i * 64 + lane.
template <typename TX>
__device__ __forceinline__ void stage_tile(const TX* __restrict__ X, int64_t ld, int d, int f0, int64_t r0, int lane,
                                           double* xs) {
  constexpr int kPer = 16 / sizeof(TX);     // elements per 16-byte chunk
  constexpr int kChunksPerRow = 64 / kPer;  // chunks per feature row segment
  constexpr int kIters = 16 * kChunksPerRow / 64;
  typedef __attribute__((ext_vector_type(kPer))) TX vec;
  vec v[kIters];
#pragma unroll
  for (int i = 0; i < kIters; ++i) {  // all loads in flight first
    const int c = i * 64 + lane;
    const int fl = c / kChunksPerRow, k = c % kChunksPerRow;
    const int feat = f0 + fl;
    const TX* src = X + (int64_t)(feat < d ? feat : 0) * ld + r0 + k * kPer;
    v[i] = feat < d ? __builtin_nontemporal_load(reinterpret_cast<const vec*>(src)) : vec{};
  }
#pragma unroll
  for (int i = 0; i < kIters; ++i) {
    const int c = i * 64 + lane;
    const int fl = c / kChunksPerRow, k = c % kChunksPerRow;
    double* dst = xs + fl * kStageLd + k * kPer;
#pragma unroll
    for (int j = 0; j < kPer; j += 2) *reinterpret_cast<f64x2*>(dst + j) = f64x2{(double)v[i][j], (double)v[i][j + 1]};
  }
}

// =============================================================================================
// f64 MFMA kernel (v_mfma_f64_16x16x4_f64): Spark-parity precision
// =============================================================================================
template <typename TX, int NT>
__global__ __launch_bounds__(kBlock) void gram_tall_f64_kernel(GramArgs a) {
  constexpr int NPAIR = NT * (NT + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int f = lane & 15, q = lane >> 4;
  double* lw = reinterpret_cast<double*>(smem) + wave * 128;  // [w(64), wy(64)]
  // per-wave staging of one 16-feature x 64-row tile, rows padded to kStageLd doubles
  double* xs = reinterpret_cast<double*>(smem) + kWavesPerBlock * 128 + wave * (16 * kStageLd);

  // kChains independent accumulators per tile pair: 16 back-to-back dependent f64 MFMAs per
  // superstep otherwise serialize on the MFMA latency
  constexpr int kChains = NT >= 2 ? 2 : 4;  // fewer for many pairs: VGPRs -> occupancy
  f64x4 acc[NPAIR][kChains];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p)
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[p][c] = f64x4{};
  double cs[NT], ab[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) cs[t] = ab[t] = 0.0;
  RowAcc ra;

  const TX* X = reinterpret_cast<const TX*>(a.X);
  const TX* fp[NT];
  bool fvalid[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int feat = t * 16 + f;
    fvalid[t] = feat < a.d;
    fp[t] = X + (int64_t)(fvalid[t] ? feat : 0) * a.ld + 16 * q;
  }
  const bool weighted = (a.sel != nullptr) || (a.w != nullptr);

  const int64_t gw = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const int64_t total_waves = (int64_t)gridDim.x * kWavesPerBlock;
  int64_t s0 = gw * a.spw;
  int64_t s1 = s0 + a.spw;
  if (s1 > a.nsuper) s1 = a.nsuper;
  const bool do_tail = (gw == total_waves - 1) && (a.n > a.nsuper * 64);
  const int64_t s_end = do_tail ? a.nsuper + 1 : s1;
  if (do_tail && s0 > a.nsuper) s0 = a.nsuper;

  for (int64_t s = s0; s < s_end; ++s) {
    const int64_t r0 = s * 64;
    RowVals rv = row_vals(a, r0 + lane);
    ra.add(rv);
    lw[lane] = rv.live ? rv.w : 0.0;
    lw[64 + lane] = rv.live ? rv.wy : 0.0;
    __builtin_amdgcn_wave_barrier();
    const int64_t rows_left = a.n - (r0 + 16 * q);
    double wv[16], wyv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      wv[e] = lw[16 * q + e];
      wyv[e] = lw[64 + 16 * q + e];
    }
    double x[NT][16];
    if (s < a.nsuper) {
      // full superstep: the wave loads each tile cooperatively — lane-contiguous 16-byte chunks,
      // 512 B (f64) / 256 B (f32) runs per feature — and stages it in LDS, then every lane reads
      // its 16 rows of its feature back (8 x ds_read_b128).  The per-lane strided scalar loads of
      // the first version touched 64 cache lines per instruction (~3 TB/s at d = 16..32).
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        stage_tile<TX>(X, a.ld, a.d, t * 16, r0, lane, xs);
        __builtin_amdgcn_wave_barrier();
        const f64x2* src = reinterpret_cast<const f64x2*>(xs + f * kStageLd + 16 * q);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const f64x2 v = src[i];
          x[t][2 * i] = v[0];
          x[t][2 * i + 1] = v[1];
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          double v = 0.0;
          if (fvalid[t] && e < rows_left) v = (double)fp[t][r0 + e];
          x[t][e] = v;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        cs[t] += x[t][e] * wv[e];
        ab[t] += x[t][e] * wyv[e];
      }
    int p = 0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J, ++p)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const double b = weighted ? x[J][e] * wv[e] : x[J][e];
          acc[p][e % kChains] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[I][e], b, acc[p][e % kChains], 0, 0, 0);
        }
    __builtin_amdgcn_wave_barrier();
  }

  const int d = a.d;
  const int P = a.P;
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
  for (int i = threadIdx.x; i < P; i += kBlock) red[i] = 0.0;
  double sc[5] = {ra.cnt, ra.ws, ra.wws, ra.bs, ra.bbs};
#pragma unroll
  for (int k = 0; k < 5; ++k) sc[k] = wave_sum_f64(sc[k]);
  // combine the 4 row-groups q of each feature
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    cs[t] += __shfl_xor(cs[t], 16, 64);
    cs[t] += __shfl_xor(cs[t], 32, 64);
    ab[t] += __shfl_xor(ab[t], 16, 64);
    ab[t] += __shfl_xor(ab[t], 32, 64);
  }
  __syncthreads();
  for (int wvi = 0; wvi < kWavesPerBlock; ++wvi) {
    if (wave == wvi) {
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) red[k] += sc[k];
      }
      if (q == 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int feat = t * 16 + f;
          if (feat < d) {
            red[5 + feat] += cs[t];
            red[5 + d + feat] += ab[t];
          }
        }
      }
      int p = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = I; J < NT; ++J, ++p) {
          double* tile = red + 5 + 2 * d + p * 256;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double v = 0.0;
#pragma unroll
            for (int c = 0; c < kChains; ++c) v += acc[p][c][r];
            tile[mfma16d_row(lane, r) * 16 + mfma16d_col(lane)] += v;
          }
        }
    }
    __syncthreads();
  }
  double* out = a.partials + (int64_t)blockIdx.x * P;
  for (int i = threadIdx.x; i < P; i += kBlock) out[i] = red[i];
}

// =============================================================================================
// f64 "skinny" kernel, d <= 8 (the lab's own shape: d = 1): lane = row, every statistic a running
// f64 register sum on the VALU.  The MFMA kernel maps 16 features to lanes, so at d = 1 15/16 of
// its lanes idle and each load instruction fetches 4 x 8 B (0.9 TB/s measured); here every lane
// streams its own rows' x / y / w / sel with branch-free selects (dead rows contribute exact
// zeros, their garbage never enters a product), 4 rows in flight per thread.  Slab layout = the
// f64 MFMA kernel's (16 x 16 tile), so the slab fold is shared.
// =============================================================================================
// 4 consecutive elements [r0, r0 + 4) of a typed column as f64, ONE vector load (the caller
// guarantees 16-byte-aligned bases and r0 % 4 == 0; the switch is wave-uniform)
__device__ __forceinline__ void load4_as_f64(const void* p, int dt, int64_t r0, double out[4]) {
  typedef __attribute__((ext_vector_type(4))) int i32x4_t;
  typedef __attribute__((ext_vector_type(2))) long long i64x2_t;
  typedef __attribute__((ext_vector_type(4))) unsigned char u8x4_t;
  typedef __attribute__((ext_vector_type(4))) unsigned short u16x4_t;
  switch (dt) {
    case DT_F64: {
      const f64x2 a = reinterpret_cast<const f64x2*>(p)[r0 / 2], b = reinterpret_cast<const f64x2*>(p)[r0 / 2 + 1];
      out[0] = a[0]; out[1] = a[1]; out[2] = b[0]; out[3] = b[1];
      break;
    }
    case DT_F32: {
      const f32x4 v = reinterpret_cast<const f32x4*>(p)[r0 / 4];
      for (int u = 0; u < 4; ++u) out[u] = (double)v[u];
      break;
    }
    case DT_I32: {
      const i32x4_t v = reinterpret_cast<const i32x4_t*>(p)[r0 / 4];
      for (int u = 0; u < 4; ++u) out[u] = (double)v[u];
      break;
    }
    case DT_I64: {
      const i64x2_t a = reinterpret_cast<const i64x2_t*>(p)[r0 / 2], b = reinterpret_cast<const i64x2_t*>(p)[r0 / 2 + 1];
      out[0] = (double)a[0]; out[1] = (double)a[1]; out[2] = (double)b[0]; out[3] = (double)b[1];
      break;
    }
    case DT_U8: {
      const u8x4_t v = reinterpret_cast<const u8x4_t*>(p)[r0 / 4];
      for (int u = 0; u < 4; ++u) out[u] = (double)v[u];
      break;
    }
    case DT_BF16: {
      const u16x4_t v = reinterpret_cast<const u16x4_t*>(p)[r0 / 4];
      for (int u = 0; u < 4; ++u) out[u] = (double)bf16_bits_to_f32(v[u]);
      break;
    }
    default:
      for (int u = 0; u < 4; ++u) out[u] = 0.0;
  }
}

// VEC (columnar sources only, host-checked 16-byte-aligned pointers): each lane owns 4
// CONSECUTIVE rows and reads each column / the label / weights / selection with one vector load
// (the row-strided form moves 1-8 bytes per lane per load); the partial last quad takes clamped
// scalar loads.
template <typename TX, int D, bool COLS = false, bool VEC = false>
__global__ __launch_bounds__(kBlock) void gram_skinny_f64_kernel(GramArgs a) {
  constexpr int NA = D * (D + 1) / 2;
  constexpr int NV = 5 + 2 * D + NA;
  constexpr int UNR = 4;
  __shared__ double red[kWavesPerBlock][NV];
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  const TX* X = reinterpret_cast<const TX*>(a.X);
  const int64_t n = a.n;
  const int64_t step = (int64_t)gridDim.x * kBlock * UNR;
  const int64_t first = VEC ? ((int64_t)blockIdx.x * kBlock + threadIdx.x) * UNR
                            : (int64_t)blockIdx.x * kBlock * UNR + threadIdx.x;
  for (int64_t r0 = first; r0 < n; r0 += step) {
    double x[UNR][D], yv[UNR], wv[UNR];
    bool live[UNR];
    if (VEC && r0 + UNR <= n) {
      double t[UNR];
      load4_as_f64(a.y, a.ydt, r0, yv);
      if (a.w) {
        load4_as_f64(a.w, a.wdt, r0, wv);
      } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) wv[u] = 1.0;
      }
      if (a.sel) {
        load4_as_f64(a.sel, DT_U8, r0, t);
#pragma unroll
        for (int u = 0; u < UNR; ++u) live[u] = t[u] != 0.0;
      } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) live[u] = true;
      }
#pragma unroll
      for (int f = 0; f < D; ++f) {
        load4_as_f64(a.colp[f], a.coldt[f], r0, t);
#pragma unroll
        for (int u = 0; u < UNR; ++u) x[u][f] = t[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {  // loads of all UNR rows first (clamped, unconditional)
        const int64_t r = VEC ? r0 + u : r0 + (int64_t)u * kBlock;
        const int64_t rc = r < n ? r : n - 1;
        live[u] = r < n && (a.sel == nullptr || a.sel[rc] != 0);
        yv[u] = load_as_f64(a.y, a.ydt, rc);
        wv[u] = a.w ? load_as_f64(a.w, a.wdt, rc) : 1.0;
#pragma unroll
        for (int f = 0; f < D; ++f) {
          if constexpr (COLS) {
            x[u][f] = load_as_f64(a.colp[f], a.coldt[f], rc);  // wave-uniform dtype switch
          } else {
            x[u][f] = (double)X[(int64_t)f * a.ld + rc];
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const double w = live[u] ? wv[u] : 0.0;
      const double y = live[u] ? yv[u] : 0.0;
      const double wy = w * y;
      v[0] += live[u] ? 1.0 : 0.0;
      v[1] += w;
      v[2] += w * w;
      v[3] += wy;
      v[4] += wy * y;
      int q = 0;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const double xi = live[u] ? x[u][i] : 0.0;
        v[5 + i] += w * xi;
        v[5 + D + i] += wy * xi;
        const double wxi = w * xi;
#pragma unroll
        for (int j = i; j < D; ++j, ++q) v[5 + 2 * D + q] += wxi * (live[u] ? x[u][j] : 0.0);
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double t = wave_sum_f64(v[k]);
    if (lane == 0) red[wave][k] = t;
  }
  __syncthreads();
  double* out = a.partials + (int64_t)blockIdx.x * a.P;
  for (int k = threadIdx.x; k < NV; k += kBlock) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) t += red[w][k];
    int64_t dst;
    if (k < 5 + 2 * D) {
      dst = k;  // scalars, Σw x (D), Σw x y (D): d == D
    } else {
      int q = k - 5 - 2 * D, i = 0;
      while (q >= D - i) {
        q -= D - i;
        ++i;
      }
      dst = 5 + 2 * D + i * 16 + (i + q);  // (i, j = i + q) of the 16 x 16 f64 tile
    }
    out[dst] = t;
  }
}

// =============================================================================================
// slab reduction -> packed-upper flat layout
// =============================================================================================

// Storage-order fold: thread = one slab element (consecutive threads read consecutive doubles of
// every slab: 512-B coalesced runs), 16 slab groups per block with independent loads, fixed-order
// LDS combine (deterministic), then the element's packed-upper destination (lower halves of the
// diagonal tiles and padding features are dropped).  The output-order first version gathered
// each packed entry from 256-B-strided tile rows.
__global__ __launch_bounds__(1024) void gram_fold_kernel(const double* __restrict__ partials, int nslab, int P, int d,
                                                        int T, int NT, double* __restrict__ out) {
  __shared__ double part[16][65];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + c;
  double s = 0.0;
  if (o < P) {
    const double* p = partials + o;
    int b = g;
    for (; b + 48 < nslab; b += 64) {
      const double v0 = p[(int64_t)b * P], v1 = p[(int64_t)(b + 16) * P];
      const double v2 = p[(int64_t)(b + 32) * P], v3 = p[(int64_t)(b + 48) * P];
      s += (v0 + v1) + (v2 + v3);
    }
    for (; b < nslab; b += 16) s += p[(int64_t)b * P];
  }
  part[g][c] = s;
  __syncthreads();
  if (g == 0 && o < P) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][c];
    fold_store(o, t, d, T, NT, out);
  }
}

// one block per statistic column: thread t sums rows t, t + 256, ... in order, then a fixed LDS
// tree over the 256 partial sums (deterministic run to run)
__global__ __launch_bounds__(256) void window_fold_kernel(const double* __restrict__ part, int64_t rows, int gw,
                                                          double* __restrict__ flat) {
  __shared__ double red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double s = 0.0;
  for (int64_t r = t; r < rows; r += 256) s += part[r * gw + c];
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) {
    if (c == 0) {
      flat[0] = red[0];
      flat[1] = red[0];
      flat[2] = red[0];
    } else {
      flat[c + 2] = red[0];
    }
  }
}

// feature-major [d, ld] (any dtype) -> MFMA-fragment-ordered bf16 tiles (see gram.h)
template <typename TS>
__global__ __launch_bounds__(256) void tile_bf16_kernel(const TS* __restrict__ X, int64_t ld, int d, int64_t n,
                                                       int NT, int64_t nsup, uint16_t* __restrict__ out,
                                                       const float* __restrict__ shift) {
  // one thread = one 16-byte chunk (8 rows of one feature)
  const int64_t nchunks = nsup * NT * 4 * 64;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const int i = (int)((c >> 6) & 3);
    const int64_t st = c >> 8;  // superstep * NT + t
    const int t = (int)(st % NT);
    const int64_t s = st / NT;
    const int f = t * 32 + (lane & 31);
    const int64_t r = s * 64 + 32 * (lane >> 5) + 8 * i;
    const float sh = (shift && f < d) ? shift[f] : 0.0f;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = 0.0f;
      if (f < d && r + j < n) {
        if constexpr (sizeof(TS) == 8) x = (float)((double)X[(int64_t)f * ld + r + j] - (double)sh);
        else x = (float)X[(int64_t)f * ld + r + j] - sh;
      }
      v[j] = (__bf16)x;
    }
    reinterpret_cast<u32x4*>(out)[c] = __builtin_bit_cast(u32x4, v);
  }
}

template <>
__global__ __launch_bounds__(256) void tile_bf16_kernel<uint16_t>(const uint16_t* __restrict__ X, int64_t ld, int d,
                                                                 int64_t n, int NT, int64_t nsup,
                                                                 uint16_t* __restrict__ out,
                                                                 const float* __restrict__ shift) {
  const int64_t nchunks = nsup * NT * 4 * 64;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const int i = (int)((c >> 6) & 3);
    const int64_t st = c >> 8;
    const int t = (int)(st % NT);
    const int64_t s = st / NT;
    const int f = t * 32 + (lane & 31);
    const int64_t r = s * 64 + 32 * (lane >> 5) + 8 * i;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (f < d) {
      if (r + 8 <= n && ((ld & 7) == 0)) {
        v = *reinterpret_cast<const u32x4*>(X + (int64_t)f * ld + r);
      } else {
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = (r + j < n) ? X[(int64_t)f * ld + r + j] : (uint16_t)0;
        v = __builtin_bit_cast(u32x4, e);
      }
      if (shift) {  // bf16 source and a bf16-representable shift: x - s is usually exact
        const float sh = shift[f];
        bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (r + j < n) ? (__bf16)((float)b[j] - sh) : (__bf16)0.0f;
        v = __builtin_bit_cast(u32x4, b);
      }
    }
    reinterpret_cast<u32x4*>(out)[c] = v;
  }
}

// Un-shift of the packed statistics (gram.h: stats_unshift).  Pass 1 rewrites the Σxxᵀ entries
// (reading the shifted column sums and Σw, which it does not write), pass 2 the column sums.
__global__ __launch_bounds__(256) void unshift_aa_kernel(double* __restrict__ flat, const float* __restrict__ shift,
                                                        int d) {
  const double W = flat[1];
  const double* as = flat + 5;
  double* aa = flat + 5 + 2 * (int64_t)d;
  const int64_t tot = (int64_t)d * (d + 1) / 2;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    // packed upper, column-major: e = i + j (j + 1) / 2, i <= j
    int64_t j = (int64_t)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
    while (j * (j + 1) / 2 > e) --j;
    while ((j + 1) * (j + 2) / 2 <= e) ++j;
    const int64_t i = e - j * (j + 1) / 2;
    const double si = (double)shift[i], sj = (double)shift[j];
    aa[e] += si * as[j] + sj * as[i] + si * sj * W;
  }
}

__global__ __launch_bounds__(256) void unshift_head_kernel(double* __restrict__ flat, const float* __restrict__ shift,
                                                          int d) {
  const double W = flat[1], B = flat[3];
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < d; j += gridDim.x * blockDim.x) {
    const double s = (double)shift[j];
    flat[5 + d + j] += s * B;
    flat[5 + j] += s * W;
  }
}

}  // namespace

void stats_unshift(double* flat, const float* shift, int d, hipStream_t st) {
  if (d < 1) return;
  const int64_t tot = (int64_t)d * (d + 1) / 2;
  int64_t g = (tot + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(unshift_aa_kernel, dim3(g), dim3(256), 0, st, flat, shift, d);
  hipLaunchKernelGGL(unshift_head_kernel, dim3((d + 255) / 256), dim3(256), 0, st, flat, shift, d);
  DQ_HIP_CHECK(hipGetLastError());
}

int64_t tiled_elems(int d, int64_t n) {
  const int NT = (d + 31) / 32;
  return ((n + 63) / 64) * NT * 4 * 64 * 8;
}

void tile_bf16(const void* X, int xdt, int64_t ld, int d, int64_t n, void* out, hipStream_t st, const float* shift) {
  const int NT = (d + 31) / 32;
  const int64_t nsup = (n + 63) / 64;
  const int64_t nchunks = nsup * NT * 256;
  int64_t g = (nchunks + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  uint16_t* o = reinterpret_cast<uint16_t*>(out);
  switch (xdt) {
    case DT_BF16: hipLaunchKernelGGL(tile_bf16_kernel<uint16_t>, dim3(g), dim3(256), 0, st, (const uint16_t*)X, ld, d, n, NT, nsup, o, shift); break;
    case DT_F32: hipLaunchKernelGGL(tile_bf16_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)X, ld, d, n, NT, nsup, o, shift); break;
    case DT_F64: hipLaunchKernelGGL(tile_bf16_kernel<double>, dim3(g), dim3(256), 0, st, (const double*)X, ld, d, n, NT, nsup, o, shift); break;
    case DT_I32: hipLaunchKernelGGL(tile_bf16_kernel<int32_t>, dim3(g), dim3(256), 0, st, (const int32_t*)X, ld, d, n, NT, nsup, o, shift); break;
    default: throw std::invalid_argument("tile_bf16: unsupported dtype");
  }
  DQ_HIP_CHECK(hipGetLastError());
}

int64_t gram_partial_stride(int mode, int d) {
  if (mode == GRAM_F64) {
    const int NT = (d + 15) / 16;
    return 5 + 2 * (int64_t)d + (int64_t)NT * (NT + 1) / 2 * 256;
  }
  const int NT = (d + 31) / 32;
  return 5 + 2 * (int64_t)d + (int64_t)NT * (NT + 1) / 2 * 1024;
}

int gram_default_blocks(int64_t n) {
  const int64_t nsuper = (n + 63) / 64;
  // aim: >= 16 waves per CU on 256 CUs, but >= 8 supersteps per wave
  int64_t blocks = (nsuper + 8 * kWavesPerBlock - 1) / (8 * kWavesPerBlock);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

template <typename K>
static int occupancy_blocks(K kern, size_t lds, int block) {
  int per = 0, dev = 0, cus = 0;
  DQ_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, block, lds));
  DQ_HIP_CHECK(hipGetDevice(&dev));
  DQ_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (per < 1) per = 1;
  return per * cus;
}

static size_t bf16_lds(int d, int xmode) {
  const int W = bf16_block(d, xmode) / kWave;
  const int NT = (d + 31) / 32;
  const size_t stripes = (size_t)W * (4 * 64 * 2 + 64 * 4);
  const size_t tree = (size_t)(W / 2) * ((NT * (NT + 1) / 2 + NT) * 16) * 64 * sizeof(float) + (size_t)W * 5 * 8;
  return tree > stripes ? tree : stripes;
}

static size_t f64_lds(int d) {
  size_t lds = kWavesPerBlock * (128 + 16 * kStageLd) * sizeof(double);
  const size_t red = (size_t)gram_partial_stride(GRAM_F64, d) * sizeof(double);
  return red > lds ? red : lds;
}

// Dispatch table: call F with the kernel instantiation for (mode, xdt, d, xmode).
template <typename F>
static void with_kernel(int mode, int xdt, int d, int xmode, bool tiled, F&& f) {
  if (mode == GRAM_BF16) {
    const int NT = (d + 31) / 32;
#define DQ_BF16_CASE(TX, NTV, TL)                                                 \
    if (xmode == 0 && NTV == 1) return f(gram_tall_bf16_kernel<TX, 1, 0, TL, true>); \
    if (xmode == 0) return f(gram_tall_bf16_kernel<TX, NTV, 0, TL>);              \
    if (xmode == 1) return f(gram_tall_bf16_kernel<TX, NTV, 1, TL>);              \
    return f(gram_tall_bf16_kernel<TX, NTV, 2, TL>);
    if (xdt == DT_BF16 && tiled) { if (NT == 1) { DQ_BF16_CASE(uint16_t, 1, true) } else { DQ_BF16_CASE(uint16_t, 2, true) } }
    if (tiled) throw std::invalid_argument("gram_tall: tiled storage must be bf16");
    if (xdt == DT_BF16) { if (NT == 1) { DQ_BF16_CASE(uint16_t, 1, false) } else { DQ_BF16_CASE(uint16_t, 2, false) } }
    if (xdt == DT_F32) { if (NT == 1) { DQ_BF16_CASE(float, 1, false) } else { DQ_BF16_CASE(float, 2, false) } }
    if (xdt == DT_F64) { if (NT == 1) { DQ_BF16_CASE(double, 1, false) } else { DQ_BF16_CASE(double, 2, false) } }
#undef DQ_BF16_CASE
    throw std::invalid_argument("gram_tall(bf16): unsupported feature dtype");
  }
  if (mode == GRAM_F64) {
    const int NT = (d + 15) / 16;
#define DQ_F64_CASE(TX)                                        \
    switch (NT) {                                              \
      case 1: return f(gram_tall_f64_kernel<TX, 1>);           \
      case 2: return f(gram_tall_f64_kernel<TX, 2>);           \
      case 3: return f(gram_tall_f64_kernel<TX, 3>);           \
      default: return f(gram_tall_f64_kernel<TX, 4>);          \
    }
    if (xdt == DT_F64) { DQ_F64_CASE(double) }
    if (xdt == DT_F32) { DQ_F64_CASE(float) }
#undef DQ_F64_CASE
    throw std::invalid_argument("gram_tall(f64): unsupported feature dtype");
  }
  throw std::invalid_argument("gram_tall: unsupported mode");
}

constexpr int kSkinnyMaxD = 8;

template <typename F>
static void with_skinny(int xdt, int d, F&& f) {
#define DQ_SKINNY(TX)                                          \
  switch (d) {                                                 \
    case 1: return f(gram_skinny_f64_kernel<TX, 1>);           \
    case 2: return f(gram_skinny_f64_kernel<TX, 2>);           \
    case 3: return f(gram_skinny_f64_kernel<TX, 3>);           \
    case 4: return f(gram_skinny_f64_kernel<TX, 4>);           \
    case 5: return f(gram_skinny_f64_kernel<TX, 5>);           \
    case 6: return f(gram_skinny_f64_kernel<TX, 6>);           \
    case 7: return f(gram_skinny_f64_kernel<TX, 7>);           \
    default: return f(gram_skinny_f64_kernel<TX, 8>);          \
  }
  if (xdt == DT_F64) { DQ_SKINNY(double) }
  if (xdt == DT_F32) { DQ_SKINNY(float) }
#undef DQ_SKINNY
  throw std::invalid_argument("gram_skinny: unsupported feature dtype");
}

template <bool VEC, typename F>
static void with_skinny_cols_t(int d, F&& f) {
  switch (d) {
    case 1: return f(gram_skinny_f64_kernel<double, 1, true, VEC>);
    case 2: return f(gram_skinny_f64_kernel<double, 2, true, VEC>);
    case 3: return f(gram_skinny_f64_kernel<double, 3, true, VEC>);
    case 4: return f(gram_skinny_f64_kernel<double, 4, true, VEC>);
    case 5: return f(gram_skinny_f64_kernel<double, 5, true, VEC>);
    case 6: return f(gram_skinny_f64_kernel<double, 6, true, VEC>);
    case 7: return f(gram_skinny_f64_kernel<double, 7, true, VEC>);
    default: return f(gram_skinny_f64_kernel<double, 8, true, VEC>);
  }
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <typename F>
static void with_skinny_cols(const GramArgs& a, F&& f) {
  bool vec = aligned16(a.y) && aligned16(a.w) && aligned16(a.sel);
  for (int i = 0; i < a.cols; ++i) vec = vec && aligned16(a.colp[i]);
  if (vec)
    with_skinny_cols_t<true>(a.d, f);
  else
    with_skinny_cols_t<false>(a.d, f);
}

static bool use_skinny(int mode, int d, int xdt, int tiled) {
  return mode == GRAM_F64 && !tiled && d <= kSkinnyMaxD && (xdt == DT_F64 || xdt == DT_F32);
}

// DQ4ML_GRAM_STREAM=0 keeps the round-1 register-staged f64 kernel (A/B measurements only)
static bool use_stream() {
  static const bool on = [] {
    const char* e = getenv("DQ4ML_GRAM_STREAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

int gram_plan_blocks(int mode, int d, int64_t n, int xdt, int xmode) {
  if (mode == GRAM_F32 || mode == GRAM_F32S || (use_stream() && ((mode == GRAM_F64 && !use_skinny(mode, d, xdt, 0) &&
                                              (xdt == DT_F64 || xdt == DT_F32)) ||
                                             (mode == GRAM_BF16 && xdt == DT_F32))))
    return gram_stream_blocks(mode, d, n, xdt);
  if (use_skinny(mode, d, xdt, 0)) {
    int full = 1;
    with_skinny(xdt, d, [&](auto kern) { full = occupancy_blocks(kern, 0, kBlock); });
    // >= 8 iterations of 4 rows per thread, at most one resident wave of blocks
    int64_t want = (n + (int64_t)kBlock * 4 * 8 - 1) / ((int64_t)kBlock * 4 * 8);
    if (want < 1) want = 1;
    return (int)(want < full ? want : full);
  }
  const size_t lds = mode == GRAM_BF16 ? bf16_lds(d, xmode) : f64_lds(d);
  int full = 1;
  const int block = mode == GRAM_BF16 ? bf16_block(d, xmode) : kBlock;
  with_kernel(mode, xdt, d, xmode, false, [&](auto kern) { full = occupancy_blocks(kern, lds, block); });
  // at least ~4 supersteps per wave, at most one full residency wave of blocks
  const int64_t nsuper = (n + 63) / 64;
  const int wpb = block / kWave;
  int64_t want = (nsuper + 4 * wpb - 1) / (4 * wpb);
  if (want < 1) want = 1;
  return (int)(want < full ? want : full);
}

void gram_window_fold(const double* part, int64_t rows, int gw, double* flat, hipStream_t st) {
  if (gw < 1 || rows < 0) throw std::invalid_argument("gram_window_fold: bad shape");
  hipLaunchKernelGGL(window_fold_kernel, dim3(gw), dim3(256), 0, st, part, rows, gw, flat);
  DQ_HIP_CHECK(hipGetLastError());
}

void gram_reduce(int mode, const double* partials, int blocks, int d, double* out, hipStream_t st) {
  const int T = mode == GRAM_F64 ? 16 : 32;
  const int NT = (d + T - 1) / T;
  const int P = (int)gram_partial_stride(mode, d);
  // output-order gather (first version): 4.4 / 7.9 us at d = 32 / 64; storage order: 3.8 / 3.9 us
  hipLaunchKernelGGL(gram_fold_kernel, dim3((P + 63) / 64), dim3(1024), 0, st, partials, blocks, P, d, T, NT, out);
  DQ_HIP_CHECK(hipGetLastError());
}

int gram_interleave() {
  // always on: same-box A/B against contiguous ranges (5 alternations) 1e8 rows 1.011-1.015 vs
  // 1.020-1.026 ms, 1.25e7 rows 0.1426-0.1441 vs 0.1471-0.1476 ms per fit (tall bf16 kernel)
  return 1;
}

void gram_tall(int mode, GramArgs a, int xmode, int blocks, double* out, hipStream_t st, bool reduce) {
  if (a.d < 1 || a.d > 64) throw std::invalid_argument("gram_tall: d must be in [1, 64]");
  if (blocks < 1) throw std::invalid_argument("gram_tall: blocks must be >= 1");
  a.nsuper = a.n / 64;
  const int block = mode == GRAM_BF16 ? bf16_block(a.d, xmode) : kBlock;
  const int64_t total_waves = (int64_t)blocks * (block / kWave);
  a.spw = (a.nsuper + total_waves - 1) / total_waves;
  if (a.spw < 1) a.spw = 1;
  a.interleave = gram_interleave();
  a.P = (int)gram_partial_stride(mode, a.d);
  const size_t lds = mode == GRAM_BF16 ? bf16_lds(a.d, xmode) : f64_lds(a.d);
  if (a.tiled && mode != GRAM_BF16) throw std::invalid_argument("gram_tall: tiled storage needs bf16 mode");
  if (a.xshift) {
    // only the f32 stream kernels subtract a shift (tiled storage is shifted when it is tiled)
    if (!((mode == GRAM_F32 || mode == GRAM_BF16 || mode == GRAM_F32S) && a.xdt == DT_F32 && !a.tiled && a.cols == 0 &&
          gram_stream_ok(mode, a)))
      throw std::invalid_argument("gram_tall: a feature shift needs 16-byte aligned f32 features (stream kernel)");
    gram_stream(mode, a, 1, blocks, out, st, reduce);  // XM = 1: dead / padding rows weigh 0, not -s
    return;
  }
  if (a.cols > 0) {
    if (mode != GRAM_F64 || a.cols != a.d || a.d > kSkinnyMaxD || a.tiled)
      throw std::invalid_argument("gram_tall: columnar sources need f64 mode and d <= 8");
    with_skinny_cols(a, [&](auto kern) { hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), 0, st, a); });
  } else if (use_skinny(mode, a.d, a.xdt, a.tiled)) {
    with_skinny(a.xdt, a.d, [&](auto kern) { hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), 0, st, a); });
  } else if ((mode == GRAM_F32 || mode == GRAM_F32S ||
              (use_stream() && (mode == GRAM_F64 || (mode == GRAM_BF16 && a.xdt == DT_F32)))) &&
             gram_stream_ok(mode, a)) {
    gram_stream(mode, a, xmode, blocks, out, st, reduce);
    return;
  } else if (mode == GRAM_F32 || mode == GRAM_F32S) {
    throw std::invalid_argument("gram_tall(f32): needs 16-byte aligned f32 features and f32/f64 labels");
  } else {
    with_kernel(mode, a.xdt, a.d, xmode, a.tiled != 0,
                [&](auto kern) { hipLaunchKernelGGL(kern, dim3(blocks), dim3(block), lds, st, a); });
  }
  DQ_HIP_CHECK(hipGetLastError());
  if (reduce) gram_reduce(mode, a.partials, blocks, a.d, out, st);
}

static size_t cols_lds(int NT) {
  const size_t bufs = 2 * ((size_t)NT * 4 * 64 * 16 + 4 * 64 * 2);
  const size_t tree = (size_t)2 * ((NT * (NT + 1) / 2 + NT) * 16) * 64 * sizeof(float) + 4 * 5 * sizeof(double);
  return bufs > tree ? bufs : tree;
}

template <typename F>
static void with_cols_kernel(int NT, int sdt, int ydt, F&& f) {
#define DQ_COLS(NTV, YT)                                                 \
  switch (sdt) {                                                         \
    case DT_F32: return f(gram_cols_kernel<NTV, DT_F32, YT>);            \
    case DT_F64: return f(gram_cols_kernel<NTV, DT_F64, YT>);            \
    case DT_BF16: return f(gram_cols_kernel<NTV, DT_BF16, YT>);          \
    default: return f(gram_cols_kernel<NTV, -1, YT>);                    \
  }
  if (ydt == DT_F64) {
    if (NT == 1) { DQ_COLS(1, DT_F64) } else { DQ_COLS(2, DT_F64) }
  }
  if (NT == 1) { DQ_COLS(1, DT_F32) } else { DQ_COLS(2, DT_F32) }
#undef DQ_COLS
}

int gram_cols_blocks(int d, int64_t n) {
  const int NT = (d + 31) / 32;
  int full = 1;
  with_cols_kernel(NT, DT_F32, DT_F64, [&](auto k) { full = occupancy_blocks(k, cols_lds(NT), 256); });
  const int64_t nsup = (n + 63) / 64;
  int64_t want = (nsup + 3) / 4;  // >= 4 supersteps per block
  if (want < 1) want = 1;
  return (int)(want < full ? want : full);
}

void gram_cols(GramArgs a, const PackSrcG* srcs_dev, int sdt, int blocks, double* out, hipStream_t st) {
  if (a.sel == nullptr) throw std::invalid_argument("gram_cols: pass an all-ones selection when there is none");
  if (a.d < 1 || a.d > 64) throw std::invalid_argument("gram_cols: d must be in [1, 64]");
  if (a.w != nullptr) throw std::invalid_argument("gram_cols: instance weights need the materialized path");
  if (blocks < 1) throw std::invalid_argument("gram_cols: blocks must be >= 1");
  const int64_t nsup = (a.n + 63) / 64;
  a.spw = (nsup + blocks - 1) / blocks;
  if (a.spw < 1) a.spw = 1;
  a.nsuper = nsup;
  a.P = (int)gram_partial_stride(GRAM_BF16, a.d);
  const int NT = (a.d + 31) / 32;
  const size_t lds = cols_lds(NT);
  if (a.ydt != DT_F64 && a.ydt != DT_F32) throw std::invalid_argument("gram_cols: label must be f32 or f64");
  with_cols_kernel(NT, sdt, a.ydt,
                   [&](auto k) { hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, st, a, srcs_dev); });
  DQ_HIP_CHECK(hipGetLastError());
  gram_reduce(GRAM_BF16, a.partials, blocks, a.d, out, st);
}

}  // namespace dq4ml
