// K5 Gram / WLS-statistics kernels (see gram.hip).
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <cstdint>
#endif

namespace dq4ml {

// GRAM_F32S: f32 statistics from split-bf16 products (each f32 = hi + mid + lo bf16, the six
// leading cross products on the bf16 MFMA; f32 accumulation) — exact-f32-class error at the bf16
// MFMA rate (gram_stream.hip)
enum GramMode : int { GRAM_F64 = 0, GRAM_F32 = 1, GRAM_BF16 = 2, GRAM_FP8 = 3, GRAM_F32S = 4 };

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
  int tiled;           // X is MFMA-fragment-ordered bf16 (tile_bf16 layout)
  // columnar skinny f64 mode (cols = d <= 8, X unused): feature f is the source column colp[f]
  // of DType coldt[f] — a VectorAssembler output read straight from its inputs, never packed
  const void* colp[8];
  int coldt[8];
  int cols;
  // stream kernels over source columns (gram_stream_cols): [2 * d] int64 device table of
  // (column pointer, dtype) pairs — feature f is column srcs[2 f] (all of X's dtype xdt)
  const int64_t* srcs;
  // bf16 + stream kernels: 1 = wave w takes supersteps (stages) w, w + W, w + 2W, ... (W = total waves) instead of
  // one contiguous range (default; DQ4ML_GRAM_INTERLEAVE=0 restores the contiguous ranges; both orders are fixed, so run-to-run
  // deterministic).  Every wave sweeps the whole row range in step with the others: measured ~1 % faster
  // at 1e8 rows and ~2.5 % at the 1.25e7-row 8-GPU shard (the waves' drain is more even)
  int interleave;
  // stream kernels compiled with a DQ row predicate (ops/streamfuse.py, hipRTC): per-lane DMA
  // sources of the stage's row-scalar area — [64 lanes][(base, bytes per row) x 2 instructions]
  // int64 pairs, then the region pointers the guarded tail stage copies from
  const int64_t* rawtab;
  // per-feature f32 shift s (null: none): kernels that round the features (bf16 / exact-f32 /
  // split-f32 MFMA) accumulate the statistics of x - s, so a column with |mean| >> std keeps its
  // digits through the cast and the f32 accumulators; stats_unshift restores those of x in f64
  // (SURVEY.md §7e.2).  Dead and padding rows stay exactly zero.
  const float* xshift;
};

#ifndef __HIPCC_RTC__
// MFMA-fragment-ordered bf16 feature storage ("tiled"): for superstep s (64 rows), 32-feature
// tile t, k-step i: 64 lanes x 16 B contiguous, lane l = 32h + f holding rows s*64+32h+8i..+8 of
// feature 32t+f.  One wave load instruction = 1 KiB contiguous; zero padded to whole supersteps.
int64_t tiled_elems(int d, int64_t n);

// GramArgs::interleave for the tall bf16 kernel (1 unless DQ4ML_GRAM_INTERLEAVE=0); the stream
// kernels always keep contiguous ranges (their interleaved A/B lost and was removed)
int gram_interleave();
// shift: per-feature f32 shift subtracted before the bf16 cast (null: none; rows >= n stay zero)
void tile_bf16(const void* X, int xdt, int64_t ld, int d, int64_t n, void* out, hipStream_t st,
               const float* shift = nullptr);

int64_t gram_partial_stride(int mode, int d);
int gram_default_blocks(int64_t n);
// grid that exactly fills the chip for the kernel instantiation (occupancy-sized, persistent-style)
int gram_plan_blocks(int mode, int d, int64_t n, int xdt, int xmode);
// xmode: 0 = X already zero on dead rows (or no sel/w), 1 = binary mask from sel, 2 = general weights
// reduce = false: only the per-block partial slabs; gram_reduce (same mode/blocks/d) folds them
// later, possibly on another stream
void gram_tall(int mode, GramArgs a, int xmode, int blocks, double* out, hipStream_t st, bool reduce = true);
void gram_reduce(int mode, const double* partials, int blocks, int d, double* out, hipStream_t st);
// flat statistics of x' = x - s (GramArgs::xshift) -> those of x, in place, in f64:
//   Σw·x = Σw·x' + s·Σw,  Σw·x·y = Σw·x'·y + s·Σw·y,
//   Σw·xᵢ·xⱼ = Σw·x'ᵢ·x'ⱼ + sᵢ·Σw·x'ⱼ + sⱼ·Σw·x'ᵢ + sᵢ·sⱼ·Σw
// (exact algebra for any fixed s: DQ selections and weights are already in the sums)
void stats_unshift(double* flat, const float* shift, int d, hipStream_t st);

// The fused CSV scans' per-window statistics part[rows][gw] (gw = 3 + 2d + d(d+1)/2: live count,
// Σy, Σy², Σx, Σxy, packed-upper Σxx) -> the flat gram_stats layout [n, n, n, Σy, Σy², ...]
// (unit weights), every column summed in one fixed order: one launch instead of a column-sum
// kernel plus a concatenation (ops/scanfuse.py, ops/scancut.py)
void gram_window_fold(const double* part, int64_t rows, int gw, double* flat, hipStream_t st);

// LDS-DMA streamed tall kernels (gram_stream.hip): GRAM_F64 on f64/f32 features, GRAM_F32
// (exact-f32 MFMA) on f32 features.  gram_stream_ok: operand dtypes/alignment the DMA path needs.
bool gram_stream_ok(int mode, const GramArgs& a);
int gram_stream_blocks(int mode, int d, int64_t n, int xdt);
void gram_stream(int mode, GramArgs a, int xmode, int blocks, double* out, hipStream_t st, bool reduce = true);
// GRAM_BF16 on f32 storage rides the same stream kernel (bf16 MFMA on converted LDS tiles); with
// a.srcs set the features are d separate f32 columns (fused VectorAssembler + Gram)

// fused VectorAssembler + bf16 Gram over d <= 64 source columns (a.X unused; a.sel masks rows)
struct PackSrcG {
  const void* ptr;
  int dt;
  int pad;
};
int gram_cols_blocks(int d, int64_t n);
// sdt: the common source dtype (DT_F32 / DT_F64 / DT_BF16, 16-byte aligned columns) or -1 (mixed)
void gram_cols(GramArgs a, const PackSrcG* srcs_dev, int sdt, int blocks, double* out, hipStream_t st);

// a stream kernel compiled by hipRTC with a DQ row predicate (ops/streamfuse.py): the same
// argument setup as gram_stream (mode GRAM_F32 / GRAM_BF16, binary row mask), launched through
// the module function ``fn`` with ``lds`` bytes of dynamic LDS
void gram_stream_rtc(void* fn, int mode, GramArgs a, int blocks, size_t lds, double* out, hipStream_t st);
#endif

}  // namespace dq4ml
