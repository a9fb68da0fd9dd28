// K5 — LDS-DMA streamed tall Gram kernels (d <= 64) for the f64 statistics (Spark-parity
// precision, the LinearRegression default) and the exact-f32 statistics.
//
// Same statistics and slab layouts as gram.hip (count, Σw, Σw², Σwy, Σwy², Σw·x, Σw·x·y,
// Σ w·x·xᵀ) for the fit at DataQuality4MachineLearningApp.java:126 (Spark's
// WeightedLeastSquares aggregator).  What is different is the load path:
//
//  * every wave streams its own contiguous range of row "stages" through a private two-deep LDS
//    ring filled by global_load_lds_dwordx4 (LDS-DMA): stage s+1's features, labels, weights
//    and selection bytes are in flight while stage s runs its MFMAs.  No VGPR staging, no block
//    barriers in the loop, and no ordinary global load inside the loop (hipcc drains every glds
//    with vmcnt(0) at the first use of one) — the row scalars travel by DMA as well;
//  * each DMA wave-instruction reads 1 KiB as 16-B chunks whose SOURCE addresses are permuted so
//    that the lane-linear LDS image is XOR-swizzled per feature: the later ds_read_b128 of a
//    lane's rows is bank-conflict free (tests/test_gram_stream_swizzle.py checks every variant
//    against the gfx950 ds_read_b128 lane groups);
//  * f64: v_mfma_f64_16x16x4_f64, 16-feature tiles, upper tile pairs, f64 side sums on the VALU.
//    The round-1 kernel (wave-cooperative register staging, load -> wait -> MFMA per superstep)
//    took 6.88 ms for 1e8 x 32 f64 (3.7 TB/s): its loads and MFMAs did not overlap;
//  * exact-f32: v_mfma_f32_32x32x2_f32 (f32 products and sums, bitwise an fmaf chain), one
//    32-feature tile per 32 features, f32 accumulators flushed into f64 registers every
//    kFlush stages (1024 rows) so the error stays that of a 1024-term f32 sum.
//
// Stage = RS rows (64; 32 for f64 storage at d > 32 to keep four waves per CU).  Per-wave LDS:
// 2 x (NT tiles of TF features x RS rows + 1.25 KiB row scalars) + the (w, wy) stripe.
#ifndef __HIPCC_RTC__  // (ops/streamfuse.py compiles the device part below with hipRTC too)
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "gram.h"
#endif

namespace dq4ml {

namespace {

constexpr int kSW = 4;  // waves per block
constexpr int kSB = kSW * kWave;
constexpr int kRawBytes = 1280;  // [y | w]: 1 KiB (lanes 0-31 | 32-63 x 16 B); sel: 64 x 4 B
constexpr int kFlush = 16;       // exact-f32 kernel: stages per f32 accumulation chunk

// cache policy of the stream's DMA loads: every byte is read once per pass (the rows stream
// through, nothing is re-read from L2 / MALL), so non-temporal (aux 2 = nt) by default
#ifndef DQ4ML_GLDS_AUX
#define DQ4ML_GLDS_AUX 2
#endif
__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g),
                                   (__attribute__((address_space(3))) void*)(l), 16, 0, DQ4ML_GLDS_AUX);
}
__device__ __forceinline__ void glds4(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g),
                                   (__attribute__((address_space(3))) void*)(l), 4, 0, DQ4ML_GLDS_AUX);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct RowVals {
  bool live;
  double w, y, wy;
};
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

template <typename TX, int TF, int NT, int RS, int RING>
struct SGeom {
  static constexpr int kFeatBytes = RS * (int)sizeof(TX);  // one feature's rows in a stage
  static constexpr int kCPF = kFeatBytes / 16;             // 16-B chunks per feature
  static constexpr int kEPC = 16 / (int)sizeof(TX);        // elements per chunk
  static constexpr int kTileBytes = TF * kFeatBytes;
  static constexpr int kPieces = kTileBytes / 1024;        // 1-KiB DMA pieces per tile
  static constexpr int kStageX = NT * kTileBytes;
  static constexpr int kStage = kStageX + kRawBytes;
  static constexpr int kStripe = RS * 16;
  static constexpr int kWaveBytes = RING * kStage + kStripe;
  static constexpr int kGlds = NT * kPieces + 2;           // DMA wave-instructions per stage
  static_assert(kTileBytes % 1024 == 0, "a tile must be whole 1-KiB pieces");
};

// XOR swizzle of a feature's chunk slots (an involution: slot = chunk ^ g, chunk = slot ^ g).
// f64 kernel, lane (f = l & 15, q = l >> 4) reads chunks [q*CPL, q*CPL + CPL): the ds_read_b128
// lane groups {0-3,12-15,20-27} / {4-11,16-19,28-31} mix q = 0 and 1, so features 4-11 flip the
// bit that separates them.
template <int CPL>
__device__ __forceinline__ int swz16(int f) { return f ^ ((f >= 4 && f <= 11) ? CPL : 0); }
// f32-storage kernel, lane (f = l & 31, h = l >> 5): every 16-lane group is one h, 16 distinct f&15.
// 64-row stages (CPL = 4, 256-B feature rows): slot = chunk ^ (f & 15); 32-row stages (CPL = 2,
// 128-B feature rows, two features per 256-B bank row): slot = chunk ^ ((f >> 1) & 7), so the 16
// lanes of a read group hit 16 distinct (f & 1, slot) 16-B bank slots.
template <int CPL>
__device__ __forceinline__ int swz32(int f) {
  if constexpr (CPL == 4) return f & 15;
  else return (f >> 1) & 7;
}

template <int TF, int CPL>
__device__ __forceinline__ int swz(int f) {
  if constexpr (TF == 16) return swz16<CPL>(f);
  else return swz32<CPL>(f);
}

// Per-lane DMA source of every (tile, piece): the lane's feature (clamped into [0, d): padding
// features re-read the last one and are zeroed on read) and its swizzled chunk.  Matrix storage:
// X + feat * ld; column storage (a.srcs): the feature's own column.  Computed once per wave, so
// a stage's issue is one 64-bit add per piece.
template <typename TX, int TF, int NT, int RS, int RING>
struct SrcBases {
  const TX* p[NT][SGeom<TX, TF, NT, RS, RING>::kPieces];
#ifdef DQ4ML_ROW_PRED
  // the row-scalar area's two DMA instructions: per-lane source base and bytes per row (the DQ
  // predicate's input columns, laid out by ops/streamfuse.py)
  const unsigned char* rb1;
  const unsigned char* rb2;
  int64_t rs1, rs2;
#endif
  __device__ __forceinline__ void init(const GramArgs& a, int lane) {
    typedef SGeom<TX, TF, NT, RS, RING> G;
#ifdef DQ4ML_ROW_PRED
    rb1 = reinterpret_cast<const unsigned char*>(a.rawtab[lane * 4 + 0]);
    rs1 = a.rawtab[lane * 4 + 1];
    rb2 = reinterpret_cast<const unsigned char*>(a.rawtab[lane * 4 + 2]);
    rs2 = a.rawtab[lane * 4 + 3];
#endif
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int k = 0; k < G::kPieces; ++k) {
        const int slot = k * 64 + lane;
        const int fl = slot / G::kCPF, pos = slot % G::kCPF;
        int feat = t * TF + fl;
        if (feat >= a.d) feat = a.d - 1;
        const int c = pos ^ swz<TF, G::kCPF / 4>(fl);
        const TX* base = a.srcs ? reinterpret_cast<const TX*>(a.srcs[2 * feat])
                                : reinterpret_cast<const TX*>(a.X) + (int64_t)feat * a.ld;
        p[t][k] = base + c * G::kEPC;
      }
  }
};

// Issue stage r0's DMA into stage buffer st: NT*kPieces feature pieces, [y | w], sel.  The number
// of wave-instructions is fixed (kGlds) so the counted vmcnt waits stay exact: absent w / sel
// and out-of-range features re-read valid bytes that nothing consumes.
template <typename TX, int TF, int NT, int RS, int RING>
__device__ __forceinline__ void issue_stage(const GramArgs& a, const SrcBases<TX, TF, NT, RS, RING>& sb,
                                            int64_t r0, unsigned char* st, int lane) {
  typedef SGeom<TX, TF, NT, RS, RING> G;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int k = 0; k < G::kPieces; ++k) glds16(sb.p[t][k] + r0, st + t * G::kTileBytes + k * 1024);
#ifdef DQ4ML_ROW_PRED
  glds16(sb.rb1 + r0 * sb.rs1, st + G::kStageX);
  glds4(sb.rb2 + r0 * sb.rs2, st + G::kStageX + 1024);
  return;
#endif
  const int ysz = a.ydt == DT_F64 ? 8 : 4;
  const unsigned char* yb = reinterpret_cast<const unsigned char*>(a.y) + r0 * ysz;
  const void* src;
  if (lane < 32) {
    src = yb + ((lane * 16 < RS * ysz) ? lane * 16 : 0);
  } else {
    const int wl = lane - 32;
    if (a.w) {
      const int wsz = a.wdt == DT_F64 ? 8 : 4;
      src = reinterpret_cast<const unsigned char*>(a.w) + r0 * wsz + ((wl * 16 < RS * wsz) ? wl * 16 : 0);
    } else {
      src = yb;
    }
  }
  glds16(src, st + G::kStageX);
  const unsigned char* selb = a.sel ? reinterpret_cast<const unsigned char*>(a.sel) + r0 : yb;
  glds4(selb + ((lane * 4 < RS) ? lane * 4 : 0), st + G::kStageX + 1024);
}

// Tail stage (rows [r0, n), fewer than RS): the same LDS image written with guarded plain loads
// and ds stores; rows >= n are zero and dead.
template <typename TX, int TF, int NT, int RS, int RING>
__device__ __forceinline__ void fill_stage_guarded(const GramArgs& a, const SrcBases<TX, TF, NT, RS, RING>& sb,
                                                   int64_t r0, unsigned char* st, int lane) {
  typedef SGeom<TX, TF, NT, RS, RING> G;
  typedef __attribute__((ext_vector_type(G::kEPC))) TX vec;
  // element j of piece (t, k) for this lane is row r0 + c * EPC + j of its feature; the chunk
  // offset c * EPC is folded into the base, so the row of element j is r0 + off + j where
  // off = (p - feature base) — recomputed from the slot as in SrcBases::init
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int k = 0; k < G::kPieces; ++k) {
      const int slot = k * 64 + lane;
      const int fl = slot / G::kCPF, pos = slot % G::kCPF;
      const int c = pos ^ swz<TF, G::kCPF / 4>(fl);
      vec v;
#pragma unroll
      for (int j = 0; j < G::kEPC; ++j) {
        const int64_t r = r0 + c * G::kEPC + j;
        v[j] = r < a.n ? sb.p[t][k][r0 + j] : TX(0);
      }
      *reinterpret_cast<vec*>(st + t * G::kTileBytes + k * 1024 + lane * 16) = v;
    }
  unsigned char* raw = st + G::kStageX;
#ifdef DQ4ML_ROW_PRED
  dq_fill_raw(a, raw, lane, r0);  // the predicate's columns, rows >= n zero
  return;
#endif
  if (lane < RS) {
    const int64_t r = r0 + lane;
    const bool in = r < a.n;
    if (a.ydt == DT_F64) reinterpret_cast<double*>(raw)[lane] = in ? reinterpret_cast<const double*>(a.y)[r] : 0.0;
    else reinterpret_cast<float*>(raw)[lane] = in ? reinterpret_cast<const float*>(a.y)[r] : 0.0f;
    if (a.w) {
      if (a.wdt == DT_F64) reinterpret_cast<double*>(raw + 512)[lane] = in ? reinterpret_cast<const double*>(a.w)[r] : 0.0;
      else reinterpret_cast<float*>(raw + 512)[lane] = in ? reinterpret_cast<const float*>(a.w)[r] : 0.0f;
    }
    raw[1024 + lane] = (in && a.sel) ? a.sel[r] : (unsigned char)(in && !a.sel ? 1 : 0);
  }
}

// Row scalars of a stage (lane = row < RS): liveness, weight, label -> RowAcc, and the
// per-row effective (w, w*y) for the feature phase.  sel_any: the raw sel bytes are meaningful
// (a selection exists, or this is a guarded tail stage whose bytes mark the rows < n).
__device__ __forceinline__ void stage_rows(const GramArgs& a, const unsigned char* raw, int lane, int rows_valid,
                                           bool sel_any, RowAcc& ra, double& w_eff, double& wy_eff) {
#ifdef DQ4ML_ROW_PRED
  {  // the DQ chain on the row's staged columns gives liveness and the label (unit weights)
    double yv = 0.0;
    const bool keep = dq_row_pred(raw, lane, yv);
    const bool lv = lane < rows_valid && keep;
    RowVals rv{lv, lv ? 1.0 : 0.0, lv ? yv : 0.0, lv ? yv : 0.0};
    ra.add(rv);
    w_eff = rv.w;
    wy_eff = rv.wy;
    (void)sel_any;
    return;
  }
#endif
  bool live = lane < rows_valid;
  if (sel_any) live = live && raw[1024 + lane] != 0;
  const double y = a.ydt == DT_F64 ? reinterpret_cast<const double*>(raw)[lane]
                                   : (double)reinterpret_cast<const float*>(raw)[lane];
  double w = 1.0;
  if (a.w)
    w = a.wdt == DT_F64 ? reinterpret_cast<const double*>(raw + 512)[lane]
                        : (double)reinterpret_cast<const float*>(raw + 512)[lane];
  RowVals rv{live, live ? w : 0.0, live ? y : 0.0, live ? w * y : 0.0};
  ra.add(rv);
  w_eff = rv.w;
  wy_eff = rv.wy;
}

// per-lane RowAcc -> 5 wave sums
__device__ __forceinline__ void wave_scalars(const RowAcc& ra, double sc[5]) {
  sc[0] = ra.cnt, sc[1] = ra.ws, sc[2] = ra.wws, sc[3] = ra.bs, sc[4] = ra.bbs;
#pragma unroll
  for (int k = 0; k < 5; ++k) sc[k] = wave_sum_f64(sc[k]);
}

// The wave's stage loop: RING-deep DMA ring (RING - 1 stages in flight while one computes),
// counted vmcnt waits, then the guarded tail stage on the last wave.
template <typename G, typename SB, typename ISSUE, typename PROC, typename TAIL>
__device__ __forceinline__ void stage_loop(const GramArgs& a, int RS, int RING, int64_t gw, int64_t total_waves,
                                           unsigned char* wb, ISSUE&& issue, PROC&& process, TAIL&& tail) {
  const int64_t nstage = a.n / RS;
  // the wave's stages: base + i * step, i < cnt (interleaved: every wave sweeps the whole range
  // in step with the others; else one contiguous range of spw stages)
  const int64_t base = a.interleave ? gw : gw * a.spw;
  const int64_t step = a.interleave ? total_waves : 1;
  int64_t cnt;
  if (a.interleave) {
    cnt = gw < nstage ? (nstage - 1 - gw) / total_waves + 1 : 0;
  } else {
    const int64_t e = base + a.spw < nstage ? base + a.spw : nstage;
    cnt = e > base ? e - base : 0;
  }
  for (int i = 0; i < RING - 1; ++i)
    if (i < cnt) issue(base + i * step, wb + i * G::kStage);
  int b = 0;
  for (int64_t s = 0; s < cnt; ++s) {
    const int64_t nx = s + RING - 1;
    if (nx < cnt) issue(base + nx * step, wb + ((b + RING - 1) % RING) * G::kStage);
    const int64_t ahead = (cnt - 1 - s) < (RING - 1) ? (cnt - 1 - s) : (RING - 1);
    if (ahead >= 2) wait_vm<2 * G::kGlds>();
    else if (ahead == 1) wait_vm<G::kGlds>();
    else wait_vm<0>();
    process(wb + b * G::kStage, RS, a.sel != nullptr);
    b = b + 1 == RING ? 0 : b + 1;
  }
  if (gw == total_waves - 1 && a.n > nstage * RS) {
    tail(nstage * RS, wb);
    __builtin_amdgcn_wave_barrier();
    process(wb, (int)(a.n - nstage * RS), true);
  }
}

// =============================================================================================
// f64 statistics: v_mfma_f64_16x16x4_f64
// =============================================================================================
template <typename TX, int NT, int RS, int RING, int XM>
__global__ __launch_bounds__(kSB) void gram_stream_f64_kernel(GramArgs a) {
  typedef SGeom<TX, 16, NT, RS, RING> G;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int E = RS / 4;         // rows per lane per stage
  constexpr int CPL = G::kCPF / 4;  // chunks per lane per feature
  constexpr int kChains = NPAIR >= 3 ? 1 : (NPAIR == 1 ? 4 : 2);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = lane & 15, q = lane >> 4;
  unsigned char* wb = smem + wave * G::kWaveBytes;
  double* stripe = reinterpret_cast<double*>(wb + RING * G::kStage);  // [w (RS) | wy (RS)]
  SrcBases<TX, 16, NT, RS, RING> sb;
  sb.init(a, lane);

  f64x4 acc[NPAIR][kChains];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p)
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[p][c] = f64x4{};
  double cs[NT], ab[NT];
  bool fvalid[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) cs[t] = ab[t] = 0.0, fvalid[t] = t * 16 + f < a.d;
  RowAcc ra;

  auto process = [&](const unsigned char* st, int rows_valid, bool sel_any) {
    double w_eff, wy_eff;
    stage_rows(a, st + G::kStageX, lane, rows_valid, sel_any, ra, w_eff, wy_eff);
    if (lane < RS) stripe[lane] = w_eff, stripe[RS + lane] = wy_eff;
    __builtin_amdgcn_wave_barrier();
    double x[NT][E];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const unsigned char* fb = st + t * G::kTileBytes + f * G::kFeatBytes;
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int p = (q * CPL + i) ^ swz16<CPL>(f);
        if constexpr (sizeof(TX) == 8) {
          const f64x2 v = *reinterpret_cast<const f64x2*>(fb + p * 16);
          x[t][2 * i] = fvalid[t] ? v[0] : 0.0;
          x[t][2 * i + 1] = fvalid[t] ? v[1] : 0.0;
        } else {
          const f32x4 v = *reinterpret_cast<const f32x4*>(fb + p * 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[t][4 * i + j] = fvalid[t] ? (double)v[j] : 0.0;
        }
      }
    }
    double wv[E], wyv[E];
#pragma unroll
    for (int e = 0; e < E; e += 2) {
      const f64x2 u = *reinterpret_cast<const f64x2*>(stripe + q * E + e);
      const f64x2 v = *reinterpret_cast<const f64x2*>(stripe + RS + q * E + e);
      wv[e] = u[0], wv[e + 1] = u[1], wyv[e] = v[0], wyv[e + 1] = v[1];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        cs[t] += x[t][e] * wv[e];
        ab[t] += x[t][e] * wyv[e];
      }
      int p = 0;
#pragma unroll
      for (int I = 0; I < NT; ++I)
#pragma unroll
        for (int J = I; J < NT; ++J, ++p) {
          const double b = XM ? x[J][e] * wv[e] : x[J][e];
          acc[p][e % kChains] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[I][e], b, acc[p][e % kChains], 0, 0, 0);
        }
    }
    wait_lgkm0();  // every read of this buffer has landed before the next DMA may target it
  };

  stage_loop<G, decltype(sb)>(
      a, RS, RING, (int64_t)blockIdx.x * kSW + wave, (int64_t)gridDim.x * kSW, wb,
      [&](int64_t s, unsigned char* st) { issue_stage<TX, 16, NT, RS, RING>(a, sb, s * RS, st, lane); }, process,
      [&](int64_t r0, unsigned char* st) { fill_stage_guarded<TX, 16, NT, RS, RING>(a, sb, r0, st, lane); });

  // ---- block reduction into one f64 slab (serial over the waves: deterministic) --------------
  const int d = a.d, P = a.P;
  double sc[5];
  wave_scalars(ra, sc);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    cs[t] += __shfl_xor(cs[t], 16, 64);
    cs[t] += __shfl_xor(cs[t], 32, 64);
    ab[t] += __shfl_xor(ab[t], 16, 64);
    ab[t] += __shfl_xor(ab[t], 32, 64);
  }
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
  for (int i = threadIdx.x; i < P; i += kSB) red[i] = 0.0;
  __syncthreads();
  for (int wvi = 0; wvi < kSW; ++wvi) {
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
  for (int i = threadIdx.x; i < P; i += kSB) out[i] = red[i];
}

// =============================================================================================
// f32 storage, 32-feature tiles: exact-f32 statistics (CMP 0: v_mfma_f32_32x32x2_f32) or bf16
// statistics (CMP 1: tiles converted to bf16 on the LDS read, v_mfma_f32_32x32x16_bf16 — the
// "32 float features" storage of the headline config).  Side sums Σw·x, Σw·x·y on the f32 VALU
// from the unrounded features in both.
// =============================================================================================
template <int NT, int RING, int CMP, int XM, int RS = 64>
__device__ __forceinline__ void gram_stream_f32_body(const GramArgs& a) {
  static_assert(RS == 64 || RS == 32, "f32 stream kernel: 64- or 32-row stages");
  typedef SGeom<float, 32, NT, RS, RING> G;
  constexpr int HC = G::kCPF / 2;  // chunks per half stage: lane h reads rows [h * RS / 2, (h + 1) * RS / 2)
  constexpr int NPAIR = NT * (NT + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = lane & 31, h = lane >> 5;
  unsigned char* wb = smem + wave * G::kWaveBytes;
  float* stripe = reinterpret_cast<float*>(wb + RING * G::kStage);  // [w (64) | wy (64)]
  SrcBases<float, 32, NT, RS, RING> sb;
  sb.init(a, lane);

  f32x16 acc[NPAIR];
  double acc64[NPAIR][16];
#pragma unroll
  for (int p = 0; p < NPAIR; ++p) {
    acc[p] = f32x16{};
#pragma unroll
    for (int r = 0; r < 16; ++r) acc64[p][r] = 0.0;
  }
  double cs[NT], ab[NT];
  bool fvalid[NT];
  float sh[NT];  // GramArgs::xshift of the lane's features (the host launches XM = 1 with a shift)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    cs[t] = ab[t] = 0.0, fvalid[t] = t * 32 + f < a.d;
    sh[t] = (a.xshift && fvalid[t]) ? a.xshift[t * 32 + f] : 0.0f;
  }
  RowAcc ra;
  int chunk = 0;

  auto flush = [&]() {
#pragma unroll
    for (int p = 0; p < NPAIR; ++p) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc64[p][r] += (double)acc[p][r];
      acc[p] = f32x16{};
    }
  };

  auto process = [&](const unsigned char* st, int rows_valid, bool sel_any) {
    double w_eff, wy_eff;
    stage_rows(a, st + G::kStageX, lane, rows_valid, sel_any, ra, w_eff, wy_eff);
    stripe[lane] = (float)w_eff;
    stripe[64 + lane] = (float)wy_eff;
    __builtin_amdgcn_wave_barrier();
    float c32[NT], a32[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) c32[t] = a32[t] = 0.0f;
    constexpr int RPS = CMP == 0 ? 4 : 8;  // rows per step: one f32x4 chunk / one bf16x8 fragment
#pragma unroll
    for (int i = 0; i < (RS / 2) / RPS; ++i) {
      float x[NT][RPS], w8[RPS], wy8[RPS];
#pragma unroll
      for (int u = 0; u < RPS / 4; ++u) {
        const int c = HC * h + (RPS / 4) * i + u;
        const int p = c ^ swz32<G::kCPF / 4>(f);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(st + t * G::kTileBytes + f * G::kFeatBytes + p * 16);
#pragma unroll
          for (int j = 0; j < 4; ++j) x[t][4 * u + j] = fvalid[t] ? v[j] - sh[t] : 0.0f;
        }
        const f32x4 w4 = *reinterpret_cast<const f32x4*>(stripe + (RS / 2) * h + RPS * i + 4 * u);
        const f32x4 wy4 = *reinterpret_cast<const f32x4*>(stripe + 64 + (RS / 2) * h + RPS * i + 4 * u);
#pragma unroll
        for (int j = 0; j < 4; ++j) w8[4 * u + j] = w4[j], wy8[4 * u + j] = wy4[j];
      }
      if constexpr (CMP == 2) {  // even / odd rows in the two halves of packed FMAs
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          f32x2 c2 = {c32[t], 0.0f}, a2 = {a32[t], 0.0f};
#pragma unroll
          for (int j = 0; j < RPS; j += 2) {
            const f32x2 xv = {x[t][j], x[t][j + 1]};
            c2 = __builtin_elementwise_fma(xv, f32x2{w8[j], w8[j + 1]}, c2);
            a2 = __builtin_elementwise_fma(xv, f32x2{wy8[j], wy8[j + 1]}, a2);
          }
          c32[t] = c2.x + c2.y;
          a32[t] = a2.x + a2.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < RPS; ++j)
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            c32[t] = __builtin_fmaf(x[t][j], w8[j], c32[t]);
            a32[t] = __builtin_fmaf(x[t][j], wy8[j], a32[t]);
          }
      }
      if constexpr (CMP == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int pp = 0;
#pragma unroll
          for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = I; J < NT; ++J, ++pp) {
              const float b = XM ? x[J][j] * w8[j] : x[J][j];
              acc[pp] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[I][j], b, acc[pp], 0, 0, 0);
            }
        }
      } else if constexpr (CMP == 1) {
        bf16x8 fa[NT], fb[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            fa[t][j] = (__bf16)x[t][j];
            fb[t][j] = XM ? (__bf16)(x[t][j] * w8[j]) : fa[t][j];
          }
        int pp = 0;
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
          for (int J = I; J < NT; ++J, ++pp) acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[I], fb[J], acc[pp], 0, 0, 0);
      } else {
        // CMP 2 (GRAM_F32S): x = hi + mid + lo exactly, by truncation: hi = the top 16 bits of
        // x (sign, exponent, 7 mantissa bits), mid = the top 16 bits of r = x - hi (<= 16
        // significant bits, exact), lo = r - mid (<= 8 significant bits: its top 16 bits ARE it).
        // x·z ~ hi·hi' + hi·mid' + mid·hi' + mid·mid' + hi·lo' + lo·hi' (the dropped terms are
        // below 2^-24 relative), every bf16 product exact in the f32 accumulator — exact-f32-class
        // error on six bf16 MFMAs per pair and k-step.  VALU: two masks and one packed subtract
        // per residual and element pair, one byte permute per packed bf16 pair (no conversions)
        bf16x8 ah[NT], am[NT], al[NT], bh[NT], bm[NT], bl[NT];
        auto split = [&](const float (&v)[8], bf16x8& h8, bf16x8& m8, bf16x8& l8) {
          u32x4 hw, mw, lw;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x2 xv = {v[2 * q], v[2 * q + 1]};
            const u32x2 xu = __builtin_bit_cast(u32x2, xv);
            const f32x2 r = xv - __builtin_bit_cast(f32x2, xu & 0xFFFF0000u);
            const u32x2 ru = __builtin_bit_cast(u32x2, r);
            const u32x2 lu = __builtin_bit_cast(u32x2, r - __builtin_bit_cast(f32x2, ru & 0xFFFF0000u));
            hw[q] = __builtin_amdgcn_perm(xu.y, xu.x, 0x07060302u);
            mw[q] = __builtin_amdgcn_perm(ru.y, ru.x, 0x07060302u);
            lw[q] = __builtin_amdgcn_perm(lu.y, lu.x, 0x07060302u);
          }
          h8 = __builtin_bit_cast(bf16x8, hw);
          m8 = __builtin_bit_cast(bf16x8, mw);
          l8 = __builtin_bit_cast(bf16x8, lw);
        };
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          split(x[t], ah[t], am[t], al[t]);
          if constexpr (XM) {
            float xb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) xb[j] = x[t][j] * w8[j];
            split(xb, bh[t], bm[t], bl[t]);
          } else {
            bh[t] = ah[t], bm[t] = am[t], bl[t] = al[t];
          }
        }
        int pp = 0;
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
          for (int J = I; J < NT; ++J, ++pp) {
            // smallest terms first into the running f32 sum
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[I], bh[J], acc[pp], 0, 0, 0);
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[I], bl[J], acc[pp], 0, 0, 0);
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[I], bm[J], acc[pp], 0, 0, 0);
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[I], bh[J], acc[pp], 0, 0, 0);
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[I], bm[J], acc[pp], 0, 0, 0);
            acc[pp] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[I], bh[J], acc[pp], 0, 0, 0);
          }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) cs[t] += (double)c32[t], ab[t] += (double)a32[t];
    wait_lgkm0();
    if (++chunk == kFlush * 64 / RS) {  // f32 accumulation chunks of 1024 rows
      flush();
      chunk = 0;
    }
  };

  stage_loop<G, decltype(sb)>(
      a, RS, RING, (int64_t)blockIdx.x * kSW + wave, (int64_t)gridDim.x * kSW, wb,
      [&](int64_t s, unsigned char* st) { issue_stage<float, 32, NT, RS, RING>(a, sb, s * RS, st, lane); }, process,
      [&](int64_t r0, unsigned char* st) { fill_stage_guarded<float, 32, NT, RS, RING>(a, sb, r0, st, lane); });
  flush();

  const int d = a.d, P = a.P;
  double sc[5];
  wave_scalars(ra, sc);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    cs[t] += __shfl_xor(cs[t], 32, 64);
    ab[t] += __shfl_xor(ab[t], 32, 64);
  }
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
  for (int i = threadIdx.x; i < P; i += kSB) red[i] = 0.0;
  __syncthreads();
  const int col = mfma32_col(lane);
  for (int wvi = 0; wvi < kSW; ++wvi) {
    if (wave == wvi) {
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) red[k] += sc[k];
      }
      if (h == 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int feat = t * 32 + f;
          if (feat < d) {
            red[5 + feat] += cs[t];
            red[5 + d + feat] += ab[t];
          }
        }
      }
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        double* tile = red + 5 + 2 * d + p * 1024;
#pragma unroll
        for (int r = 0; r < 16; ++r) tile[mfma32_row(lane, r) * 32 + col] += acc64[p][r];
      }
    }
    __syncthreads();
  }
  double* out = a.partials + (int64_t)blockIdx.x * P;
  for (int i = threadIdx.x; i < P; i += kSB) out[i] = red[i];
}

template <int NT, int RING, int CMP, int XM, int RS = 64>
__global__ __launch_bounds__(kSB) void gram_stream_f32_kernel(GramArgs a) {
  gram_stream_f32_body<NT, RING, CMP, XM, RS>(a);
}

// ---- dispatch --------------------------------------------------------------------------------
#ifndef __HIPCC_RTC__
constexpr int kLdsMax = 160 * 1024;

// DQ4ML_GRAM_STREAM_RING=2|3 (A/B): ring depth where a 3-deep ring still fits four waves per CU
static int ring_pref() {
  static const int r = [] {
    const char* e = getenv("DQ4ML_GRAM_STREAM_RING");
    return e ? atoi(e) : 3;
  }();
  return r;
}

// measured (1e8 x 32, 1x MI355X): bf16 on f32 columns 2.24 (ring 3) vs 2.29 ms (ring 2); exact
// f32 3.15 vs 3.00 ms — its MFMA share wants the second block per CU that ring 3 costs
template <typename G3, typename F, typename K2, typename K3>
static void pick_ring(F&& f, K2 k2, int wb2, K3 k3, bool mfma_heavy = false) {
  const int want = getenv("DQ4ML_GRAM_STREAM_RING") ? ring_pref() : (mfma_heavy ? 2 : 3);
  if (want >= 3 && kSW * G3::kWaveBytes <= kLdsMax) return f(k3, G3::kWaveBytes);
  return f(k2, wb2);
}

// f32 storage, 64 features (NT = 2): 64-row stages.  32-row stages (a deeper DMA ring, four waves
// per CU) were measured and lost: config 4 (1.25e8 x 64, one box, one run) 6.18 ms at 64 rows /
// ring 2, 6.45 at 32 / ring 3, 6.53 at 32 / ring 4 -- the per-stage fixed work (row scalars,
// waits) doubles and the extra bytes in flight buy nothing.
static int f32_rs(int) { return 64; }

template <int NT, int CMP, int XM, typename F>
static void f32_rs32(F&& f) {
  const char* e = getenv("DQ4ML_GRAM_STREAM_RING");
  const int want = e ? atoi(e) : (CMP == 0 ? 2 : 4);
  if (want >= 4 && kSW * SGeom<float, 32, NT, 32, 4>::kWaveBytes <= kLdsMax)
    return f(gram_stream_f32_kernel<NT, 4, CMP, XM, 32>, SGeom<float, 32, NT, 32, 4>::kWaveBytes);
  if (want == 3) return f(gram_stream_f32_kernel<NT, 3, CMP, XM, 32>, SGeom<float, 32, NT, 32, 3>::kWaveBytes);
  return f(gram_stream_f32_kernel<NT, 2, CMP, XM, 32>, SGeom<float, 32, NT, 32, 2>::kWaveBytes);
}

template <typename F>
static void with_stream_kernel(int mode, int xdt, int d, int xm, F&& f) {
  // split-bf16 f32 statistics: 64-row stages, ring 2 (two blocks per CU: one wave's split VALU
  // overlaps the other's MFMAs; 1e8 x 32 same box 2.55 vs 2.81 ms at ring 3)
  if (mode == GRAM_F32S) {
    if (xdt != DT_F32) throw std::invalid_argument("gram_stream(f32s): needs f32 features");
#define DQ_SF32S(NTV, XMV)                                                                             \
  return pick_ring<SGeom<float, 32, NTV, 64, 3>>(f, gram_stream_f32_kernel<NTV, 2, 2, XMV>,            \
                                                 SGeom<float, 32, NTV, 64, 2>::kWaveBytes,              \
                                                 gram_stream_f32_kernel<NTV, 3, 2, XMV>, true);
    if ((d + 31) / 32 == 1) { if (xm) { DQ_SF32S(1, 1) } else { DQ_SF32S(1, 0) } }
    if (xm) { DQ_SF32S(2, 1) } else { DQ_SF32S(2, 0) }
#undef DQ_SF32S
  }
  if (mode == GRAM_F32 || mode == GRAM_BF16) {
    if (xdt != DT_F32) throw std::invalid_argument("gram_stream(f32/bf16): needs f32 features");
    const int NT = (d + 31) / 32;
    if (f32_rs(d) == 32) {
      if (NT == 1) {
        if (mode == GRAM_F32) return xm ? f32_rs32<1, 0, 1>(f) : f32_rs32<1, 0, 0>(f);
        return xm ? f32_rs32<1, 1, 1>(f) : f32_rs32<1, 1, 0>(f);
      }
      if (mode == GRAM_F32) return xm ? f32_rs32<2, 0, 1>(f) : f32_rs32<2, 0, 0>(f);
      return xm ? f32_rs32<2, 1, 1>(f) : f32_rs32<2, 1, 0>(f);
    }
#define DQ_SF32(NTV, CMPV, XMV)                                                                        \
  return pick_ring<SGeom<float, 32, NTV, 64, 3>>(f, gram_stream_f32_kernel<NTV, 2, CMPV, XMV>,         \
                                                 SGeom<float, 32, NTV, 64, 2>::kWaveBytes,              \
                                                 gram_stream_f32_kernel<NTV, 3, CMPV, XMV>, CMPV == 0);
    if (mode == GRAM_F32) {
      if (NT == 1) { if (xm) { DQ_SF32(1, 0, 1) } else { DQ_SF32(1, 0, 0) } }
      if (xm) { DQ_SF32(2, 0, 1) } else { DQ_SF32(2, 0, 0) }
    }
    if (NT == 1) { if (xm) { DQ_SF32(1, 1, 1) } else { DQ_SF32(1, 1, 0) } }
    if (xm) { DQ_SF32(2, 1, 1) } else { DQ_SF32(2, 1, 0) }
#undef DQ_SF32
  }
  if (mode != GRAM_F64) throw std::invalid_argument("gram_stream: f64 / f32 / bf16 modes only");
  const int NT = (d + 15) / 16;
#define DQ_SF64(TX, NTV, RSV)                                                                          \
  if (xm) return pick_ring<SGeom<TX, 16, NTV, RSV, 3>>(f, gram_stream_f64_kernel<TX, NTV, RSV, 2, 1>,  \
                                                       SGeom<TX, 16, NTV, RSV, 2>::kWaveBytes,          \
                                                       gram_stream_f64_kernel<TX, NTV, RSV, 3, 1>);     \
  return pick_ring<SGeom<TX, 16, NTV, RSV, 3>>(f, gram_stream_f64_kernel<TX, NTV, RSV, 2, 0>,           \
                                               SGeom<TX, 16, NTV, RSV, 2>::kWaveBytes,                  \
                                               gram_stream_f64_kernel<TX, NTV, RSV, 3, 0>);
  if (xdt == DT_F64) {
    switch (NT) {
      case 1: DQ_SF64(double, 1, 64)
      case 2: DQ_SF64(double, 2, 64)
      case 3: DQ_SF64(double, 3, 32)
      default: DQ_SF64(double, 4, 32)
    }
  }
  if (xdt == DT_F32) {
    switch (NT) {
      case 1: DQ_SF64(float, 1, 64)
      case 2: DQ_SF64(float, 2, 64)
      case 3: DQ_SF64(float, 3, 64)
      default: DQ_SF64(float, 4, 64)
    }
  }
#undef DQ_SF64
  throw std::invalid_argument("gram_stream(f64): f64 / f32 features only");
}

static int stream_rs(int mode, int xdt, int d) {
  if (mode == GRAM_F32S) return 64;
  if (mode == GRAM_F32 || mode == GRAM_BF16) return f32_rs(d);
  return (mode == GRAM_F64 && xdt == DT_F64 && d > 32) ? 32 : 64;
}

static size_t stream_lds(int wave_bytes, int mode, int d) {
  const size_t ring = (size_t)kSW * wave_bytes;
  const size_t red = (size_t)gram_partial_stride(mode, d) * sizeof(double);
  return ring > red ? ring : red;
}

static bool al(const void* p, uintptr_t m) { return (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; }

}  // namespace

bool gram_stream_ok(int mode, const GramArgs& a) {
  if (a.tiled || a.cols > 0 || a.d < 1 || a.d > 64 || a.n < 1) return false;
  if ((mode == GRAM_F32 || mode == GRAM_BF16 || mode == GRAM_F32S) && a.xdt != DT_F32) return false;
  if (mode != GRAM_F32 && mode != GRAM_F64 && mode != GRAM_BF16 && mode != GRAM_F32S) return false;
  if (a.xdt != DT_F32 && a.xdt != DT_F64) return false;
  const int xs = a.xdt == DT_F64 ? 8 : 4;
  if (a.srcs == nullptr && (!al(a.X, 16) || (a.d > 1 && ((a.ld * xs) & 15) != 0))) return false;
  if ((a.ydt != DT_F32 && a.ydt != DT_F64) || !al(a.y, 16)) return false;
  if (a.w && ((a.wdt != DT_F32 && a.wdt != DT_F64) || !al(a.w, 16))) return false;
  if (a.sel && !al(a.sel, 4)) return false;
  return true;
}

int gram_stream_blocks(int mode, int d, int64_t n, int xdt) {
  int full = 1;
  with_stream_kernel(mode, xdt, d, 0, [&](auto kern, int wave_bytes) {
    int per = 0, dev = 0, cus = 0;
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)stream_lds(wave_bytes, mode, d)));
    DQ_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kSB, stream_lds(wave_bytes, mode, d)));
    DQ_HIP_CHECK(hipGetDevice(&dev));
    DQ_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    full = (per < 1 ? 1 : per) * cus;
  });
  const int64_t nstage = n / stream_rs(mode, xdt, d);
  int64_t want = (nstage + 4 * kSW - 1) / (4 * kSW);  // >= 4 stages per wave
  if (want < 1) want = 1;
  return (int)(want < full ? want : full);
}

void gram_stream(int mode, GramArgs a, int xmode, int blocks, double* out, hipStream_t st, bool reduce) {
  if (!gram_stream_ok(mode, a)) throw std::invalid_argument("gram_stream: unsupported operands (dtype/alignment)");
  if (blocks < 1) throw std::invalid_argument("gram_stream: blocks must be >= 1");
  const int rs = stream_rs(mode, a.xdt, a.d);
  const int64_t nstage = a.n / rs;
  const int64_t total_waves = (int64_t)blocks * kSW;
  a.spw = (nstage + total_waves - 1) / total_waves;
  if (a.spw < 1) a.spw = 1;
  a.nsuper = nstage;
  // contiguous stage ranges per wave: interleaved stages measured neutral for f64 / f32, +1 % for
  // bf16 on f32 storage and +2.6 % for config 4's 64 separate column streams (each wave's 256-B
  // column pieces lose their DRAM page locality); the interleaved A/B knob was removed in round 4
  a.interleave = 0;
  a.P = (int)gram_partial_stride(mode, a.d);
  if (a.xshift && mode == GRAM_F64) throw std::invalid_argument("gram_stream: f64 statistics take no feature shift");
  // a shift makes the stored zeros of dead / padding rows -s: those rows must weigh 0 (XM = 1)
  const int xm = (xmode != 0 || a.xshift) ? 1 : 0;
  with_stream_kernel(mode, a.xdt, a.d, xm, [&](auto kern, int wave_bytes) {
    const size_t lds = stream_lds(wave_bytes, mode, a.d);
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kSB), lds, st, a);
  });
  DQ_HIP_CHECK(hipGetLastError());
  if (reduce) gram_reduce(mode, a.partials, blocks, a.d, out, st);
}

void gram_stream_rtc(void* fn, int mode, GramArgs a, int blocks, size_t lds, double* out, hipStream_t st) {
  if (mode != GRAM_F32 && mode != GRAM_BF16 && mode != GRAM_F32S)
    throw std::invalid_argument("gram_stream_rtc: f32 / bf16 / split-f32 modes");
  if (a.xdt != DT_F32 || a.srcs == nullptr || a.rawtab == nullptr || a.d < 1 || a.d > 64 || a.n < 1)
    throw std::invalid_argument("gram_stream_rtc: f32 source columns and a row-scalar table");
  if (blocks < 1 || lds > (size_t)kLdsMax) throw std::invalid_argument("gram_stream_rtc: blocks / lds");
  const int64_t nstage = a.n / 64;
  const int64_t total_waves = (int64_t)blocks * kSW;
  a.spw = (nstage + total_waves - 1) / total_waves;
  if (a.spw < 1) a.spw = 1;
  a.nsuper = nstage;
  a.interleave = 0;
  a.P = (int)gram_partial_stride(mode, a.d);
  void* args[] = {&a};
  DQ_HIP_CHECK(hipModuleLaunchKernel(reinterpret_cast<hipFunction_t>(fn), blocks, 1, 1, kSB, 1, 1, (unsigned)lds, st,
                                     args, nullptr));
  gram_reduce(mode, a.partials, blocks, a.d, out, st);
}

}  // namespace dq4ml
#else
}  // namespace
}  // namespace dq4ml
#endif
