// K1 + K2: device CSV scan with fused type inference (SURVEY.md S03 contract, numeric columns).
//
// Spark reads ``data/dataset-abstract.csv`` with ``inferSchema=true`` (DataQuality4MachineLearningApp
// .java:53-55): one full pass to infer the per-column type lattice, then univocity parses every
// line again on every action.  Here the file bytes go to HBM once and three kernels produce typed
// columns in one parse:
//   1. line terminators (\n, \r, \r\n — Hadoop LineRecordReader semantics; the lab's files are
//      CR-only with no trailing terminator): per-block wave-ballot counts -> one-block scan ->
//      ordered line-end offsets;
//   2. one thread per line: split on the separator, parse every field to its exact f64 value
//      (Clinger's fast path: mantissa < 2^53 and |exp10| <= 22, i.e. correctly rounded like
//      java.lang.Double.parseDouble; integers up to 2^53), classify it into the lattice null < int
//      < long < decimal < double < boolean < string, OR the class bits into a per-column mask and
//      count null fields / empty lines (wave ballots, LDS, one global atomic per block and
//      column) — K2 fused into K1, no second pass;
//   3. ONE host read of the stats merges the masks into the column types (X3 all-reduce across
//      ranks when sharded); double columns are the parsed planes as-is, int / long / boolean ones
//      one conversion, validity masks only materialized for columns that hold nulls.  Fields
//      outside the fast path (quotes, >19 digits, huge exponents, strings) raise a flag and the
//      whole scan is re-done by the host scanner.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.h"
#include "csv_scan.h"

namespace dq4ml {

namespace {

// Line-boundary passes: a thread owns 64 contiguous bytes = four 16-byte granules (vector loads),
// a block 256 threads = 16 KiB.  Granules are taken in ABSOLUTE 16-byte alignment (a chunk of a
// larger buffer starts anywhere): the first / last granule may cover bytes outside [0, n), which
// are masked — a 16-byte granule never crosses a page, so those loads cannot fault.  The
// byte-per-thread first version (4 KiB blocks, two loads per byte for the CRLF rule) ran at
// ~1 TB/s.
constexpr int kBytesPerThread = 64;
constexpr int kChunk = 256 * kBytesPerThread;  // bytes per block

using dq4ml_csv::byte_eq4;

// terminator bitmask of the thread's 64-byte window; window byte k <-> buffer index base + k.
// Terminators: \r, and \n not preceded by \r (CR LF is one terminator, at the CR).  With facts:
// the window's separator count and its terminator kinds (CR, lone LF, CR followed by LF -- a
// CR LF pair across two windows counts in the second) for the cutter's scan facts.
struct WinFacts {
  int sep, cr, lf, crlf;
};

template <bool FACTS = false>
__device__ __forceinline__ uint64_t term_mask(const uint8_t* __restrict__ b, int64_t n, int64_t base,
                                              uint32_t sep4 = 0, WinFacts* wf = nullptr) {
  const uint8_t* ab = b - (reinterpret_cast<uintptr_t>(b) & 15);  // granule-aligned view
  const int64_t off = b - ab;                                    // 0..15
  const int64_t g0 = base + off;                                  // aligned position of window byte 0
  uint64_t cr = 0, lf = 0, sp = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t ga = g0 + 16 * j;  // aligned, multiple of 16
    if (ga - off >= n || ga - off + 16 <= 0) continue;
    const u32x4 v = *reinterpret_cast<const u32x4*>(ab + ga);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      cr |= (uint64_t)byte_eq4(v[w], 0x0D0D0D0Du) << (16 * j + 4 * w);
      lf |= (uint64_t)byte_eq4(v[w], 0x0A0A0A0Au) << (16 * j + 4 * w);
      if (FACTS) sp |= (uint64_t)byte_eq4(v[w], sep4) << (16 * j + 4 * w);
    }
  }
  // bytes outside [0, n) of the edge windows
  const int64_t lo = base < 0 ? -base : 0, hi = n - base;
  if (lo > 0 || hi < 64) {
    const uint64_t keep_lo = lo >= 64 ? 0ull : (~0ull << lo);
    const uint64_t keep_hi = hi <= 0 ? 0ull : (hi >= 64 ? ~0ull : ((1ull << hi) - 1));
    cr &= keep_lo & keep_hi;
    lf &= keep_lo & keep_hi;
    if (FACTS) sp &= keep_lo & keep_hi;
  }
  const uint64_t prev_cr = (base >= 1 && base - 1 < n && b[base - 1] == '\r') ? 1ull : 0ull;
  const uint64_t lone_lf = lf & ~((cr << 1) | prev_cr);
  if (FACTS) {
    wf->sep = __popcll(sp);
    wf->cr = __popcll(cr);
    wf->lf = __popcll(lone_lf);
    wf->crlf = __popcll(cr & (lf >> 1)) + (int)(prev_cr & lf & 1ull);
  }
  return cr | lone_lf;
}

__global__ __launch_bounds__(256) void csv_count_kernel(const uint8_t* __restrict__ b, int64_t n,
                                                       int64_t* __restrict__ counts) {
  __shared__ int ws[4];
  const int64_t base = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kBytesPerThread -
                       (int64_t)(reinterpret_cast<uintptr_t>(b) & 15);
  int c = __popcll(term_mask(b, n, base));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = (int64_t)ws[0] + ws[1] + ws[2] + ws[3];
}

// Exclusive scan of the per-block counts in place, total at counts[nb].  One block walks the
// array in 4096-entry tiles: each thread owns 4 consecutive entries, a wave shfl_up scan and the
// 16 wave totals in LDS give the tile prefix, a running carry joins the tiles.  (The first version
// had each thread sum a contiguous 1/1024 of the array serially: 150 us for a 0.9 GB input.)
__global__ __launch_bounds__(1024) void csv_scan_counts_kernel(int64_t* __restrict__ counts, int64_t nb) {
  __shared__ int wsum[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t carry = 0;
  for (int64_t t0 = 0; t0 < nb; t0 += 4096) {
    const int64_t i0 = t0 + 4 * (int64_t)threadIdx.x;
    int v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = i0 + k < nb ? (int)counts[i0 + k] : 0;  // <= kChunk each
    const int s = v[0] + v[1] + v[2] + v[3];
    int inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int64_t before = carry + (inc - s), tot = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const int x = wsum[w];
      before += w < wave ? x : 0;
      tot += x;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < nb) counts[i0 + k] = before;
      before += v[k];
    }
    carry += tot;
    __syncthreads();  // wsum is rewritten by the next tile
  }
  if (threadIdx.x == 0) counts[nb] = carry;
}

constexpr int kEndsStage = 8192;  // line ends per block staged in LDS (block-relative int32)

// Each thread finds its window's line ends; a block with at most kEndsStage of them collects them
// in LDS (in order) and writes them out as one coalesced run — per-thread direct stores put 64
// lanes on 64 different cache lines per instruction.
//
// facts (or null): per block [separators, CR ends, lone-LF ends, CR LF ends] (int32 x 4), the
// scan facts the host used to derive with whole-chunk torch passes (ops/csvscan.py _scan_chunk)
template <typename IT>
__global__ __launch_bounds__(256) void csv_ends_kernel(const uint8_t* __restrict__ b, int64_t n,
                                                      const int64_t* __restrict__ offsets, IT* __restrict__ ends,
                                                      uint32_t sep4, int32_t* __restrict__ facts) {
  __shared__ int wtot[4];
  __shared__ int wfact[4][4];
  __shared__ int sends[kEndsStage];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t bbase = (int64_t)blockIdx.x * kChunk - (int64_t)(reinterpret_cast<uintptr_t>(b) & 15);
  const int64_t base = bbase + (int64_t)threadIdx.x * kBytesPerThread;
  uint64_t m;
  if (facts != nullptr) {
    WinFacts wf;
    m = term_mask<true>(b, n, base, sep4, &wf);
    int f[4] = {wf.sep, wf.cr, wf.lf, wf.crlf};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) f[k] += __shfl_xor(f[k], o, 64);
      if (lane == 0) wfact[wave][k] = f[k];
    }
  } else {
    m = term_mask(b, n, base);
  }
  const int c = __popcll(m);
  // exclusive prefix of the per-thread counts: wave scan (shfl_up) + wave totals in LDS
  int inc = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  if (facts != nullptr && threadIdx.x < 4)
    facts[(int64_t)blockIdx.x * 4 + threadIdx.x] =
        wfact[0][threadIdx.x] + wfact[1][threadIdx.x] + wfact[2][threadIdx.x] + wfact[3][threadIdx.x];
  int before = inc - c;
  for (int w = 0; w < wave; ++w) before += wtot[w];
  const int64_t o0 = offsets[blockIdx.x];
  const int cnt = (int)(offsets[blockIdx.x + 1] - o0);  // offsets[nb] is the total
  if (cnt <= kEndsStage) {
    int o = before;
    const int rel = threadIdx.x * kBytesPerThread;
    while (m) {
      sends[o++] = rel + __builtin_ctzll(m);
      m &= m - 1;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) ends[o0 + i] = (IT)(bbase + sends[i]);
  } else {
    int64_t o = o0 + before;
    while (m) {
      ends[o++] = (IT)(base + __builtin_ctzll(m));
      m &= m - 1;
    }
  }
}

constexpr int kMaxCols = 256;
// staged bytes per 256-line group: 8 KiB (short lines, <= ~24 B: 8 waves per SIMD — the byte
// loops are latency-bound) or 32 KiB (wider rows; 4 waves per SIMD).  Chosen per launch from the
// chunk's mean line length; a group that does not fit parses from global memory.
constexpr int kParseLdsSmall = 8192;
constexpr int kParseLdsLarge = 32768;

using dq4ml_csv::CsvOpts;

// Parse line li.  Bytes are read as B[i - bias] (global: B = b, bias = 0; LDS-staged: B = the
// block's stage, bias = the buffer index of its first byte).
// Called by EVERY lane of the wave (``active`` false past the last line) so the per-field type
// bits can be OR-reduced across the wave with shuffles: one LDS atomic per wave and field instead
// of 64 same-address atomics (which serialized the first version of this kernel).
// Empty lines and comment lines are skipped (keep = 0).  A malformed record (see
// csv_parse_dev.h; in strict mode also a field that does not convert to the user schema's type)
// keeps its row with every field null, as Spark's PERMISSIVE mode.
template <typename PB, typename IT>
__device__ __forceinline__ bool parse_line(PB B, int64_t bias, int64_t n, const IT* __restrict__ ends,
                                           int64_t li, bool active, int64_t nlines, int ncols, const CsvOpts& o,
                                           const int64_t* __restrict__ dcols, uint8_t* __restrict__ valid,
                                           uint8_t* __restrict__ keep, uint32_t* smask, int* snull, int* sempty,
                                           int* smiss, int* shard, unsigned long long* smaxl,
                                           unsigned long long* sminl) {
  const bool lane0 = (threadIdx.x & 63) == 0;
  int64_t start = 0, end = 0;
  bool line = false;
  int64_t span = 0;  // terminator to terminator (the first line: its end + 1), for the line-length facts
  if (active) {
    int64_t pe = -1;
    if (li > 0) {
      pe = ends[li - 1];
      start = pe + 1 + ((B[pe - bias] == '\r' && pe + 1 < n && B[pe + 1 - bias] == '\n') ? 1 : 0);
    }
    end = ends[li];  // exclusive (position of the terminator or n)
    span = end - pe;
    line = end > start && !(o.comment && B[start - bias] == o.comment);
    keep[li] = line;
  }
  {
    int64_t mx = active ? span : 0, mn = active ? span : ((int64_t)1 << 62);
#pragma unroll
    for (int oo = 1; oo < 64; oo <<= 1) {
      mx = max(mx, (int64_t)__shfl_xor((long long)mx, oo, 64));
      mn = min(mn, (int64_t)__shfl_xor((long long)mn, oo, 64));
    }
    if (lane0) {
      atomicMax(smaxl, (unsigned long long)mx);
      atomicMin(sminl, (unsigned long long)mn);
    }
  }
  const uint64_t empty = __ballot(active && !line);
  if (lane0 && empty) atomicAdd(sempty, (int)__popcll(empty));
  long long pos = start;
  bool slow = false, malformed = false, miss = false, hard = false;
  const bool plain = o.null_len == 0 && !o.trim_lead && !o.trim_trail;
  for (int c = 0; c < ncols; ++c) {
    double dv = 0.0;
    long long lv = 0;
    bool big = false;
    int ty = CT_NULL;
    const int kind = (int)dcols[ncols + c];
    if (kind == 4) {
      // a string column: its field's span (no conversion); the host builds the text when the
      // column is materialized (ops/csvscan.py DeviceStrings)
      long long fs = 0, fe = 0;
      bool raw = false;
      if (pos <= end && line) {
        const bool is_null = dq4ml_csv::csv_field_span(B, (long long)bias, pos, (long long)end, o, fs, fe, raw);
        ty = is_null ? CT_NULL : CT_STRING;
        slow |= fe - fs >= (1ll << 24) || fs >= (1ll << 38);
        miss = hard = true;
      }
      if (active) {
        reinterpret_cast<int64_t*>(reinterpret_cast<void*>(dcols[c]))[li] =
            (fs << 25) | ((long long)raw << 24) | ((fe - fs) & 0xFFFFFF);
        valid[(int64_t)c * nlines + li] = ty == CT_STRING;
      }
      uint32_t bit = line ? (1u << ty) : 0u;
#pragma unroll
      for (int oo = 1; oo < 64; oo <<= 1) bit |= (uint32_t)__shfl_xor((int)bit, oo, 64);
      const uint64_t nulls = __ballot(line && ty != CT_STRING);
      if (lane0) {
        if (bit) atomicOr(&smask[c], bit);
        if (nulls) atomicAdd(&snull[c], (int)__popcll(nulls));
      }
      continue;
    }
    // fslow: this field's value (or class) needs the host -- flagged per column (class-mask bit
    // 8): it only matters when the column does not come out a string
    bool fslow = false;
    if (pos <= end && line) {
      const long long pb = (long long)bias, pe = (long long)end;
      if (!(plain && dq4ml_csv::csv_field_fast(B, pb, pos, pe, o.sep, dv, lv, ty))) {
        miss = true;  // a field outside the fast path (a later fused scan then keeps the general parser)
        if (!(plain && dq4ml_csv::csv_field_fast_quoted(B, pb, pos, pe, o.sep, o.quote, dv, lv, ty))) {
          ty = dq4ml_csv::csv_field_general(B, pb, pos, pe, o, dv, lv, fslow, big, malformed);
          hard = true;  // not even a quoted fast-path number (the cutter's QUOTED build)
        }
      }
    }
    fslow |= big && kind != 2;  // an f64 plane would round it; an int64 store of lv is exact
    bool ok = ty != CT_NULL && ty != CT_STRING;
    if (o.strict && ty != CT_NULL && !dq4ml_csv::csv_conforms(ty, kind)) {
      malformed = true;  // a value the user schema's type does not accept
      ok = false;
    }
    if (active) {
      // one plane per column: f64 by default — ints / longs / booleans as their (exact:
      // |v| <= 2^53, else ``slow``) double value, converted once the column type is known — or,
      // when the type is known (an earlier scan of the same bytes, or the user schema), stored
      // as that type directly (kind = dcols[ncols + c]; a hint mismatch shows in the masks)
      void* dst = reinterpret_cast<void*>(dcols[c]);
      switch (kind) {
        case 1: reinterpret_cast<int32_t*>(dst)[li] = ok ? (int32_t)dv : 0; break;
        case 2:
        case 5: reinterpret_cast<int64_t*>(dst)[li] = ok ? (int64_t)lv : 0; break;  // long / timestamp (us)
        case 3: reinterpret_cast<uint8_t*>(dst)[li] = ok && dv != 0.0; break;
        default: reinterpret_cast<double*>(dst)[li] = dv;
      }
      valid[(int64_t)c * nlines + li] = ok;
    }
    uint32_t bit = line ? ((1u << ty) | (fslow ? 0x100u : 0u)) : 0u;
#pragma unroll
    for (int oo = 1; oo < 64; oo <<= 1) bit |= (uint32_t)__shfl_xor((int)bit, oo, 64);
    const uint64_t nulls = __ballot(line && !ok);
    if (lane0) {
      if (bit) atomicOr(&smask[c], bit);
      if (nulls) atomicAdd(&snull[c], (int)__popcll(nulls));
    }
  }
  const uint64_t misses = __ballot(active && line && miss);
  if (lane0 && misses) atomicAdd(smiss, (int)__popcll(misses));
  const uint64_t hards = __ballot(active && line && hard);
  if (lane0 && hards) atomicAdd(shard, (int)__popcll(hards));
  // a malformed record: every field null (valid = 0) — the null counts above already cover the
  // fields that failed; the rest are counted here
  const uint64_t bad = __ballot(active && line && malformed);
  if (bad) {
    if (active && line && malformed) {
      for (int c = 0; c < ncols; ++c) {
        if (valid[(int64_t)c * nlines + li]) {
          valid[(int64_t)c * nlines + li] = 0;
          atomicAdd(&snull[c], 1);
        }
      }
    }
  }
  return slow;
}

// One thread per line, 256-line groups per block.  A group whose bytes fit kParseLds is first
// staged into LDS by the whole block with 16-byte granule loads (coalesced; absolute alignment
// as in the line-boundary passes), then every thread parses its line from LDS — the first
// version walked each line with dependent byte loads from global memory (~180 GB/s).  Longer
// groups (very wide rows) parse straight from global memory.
template <int LDS, int WPE, typename IT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void csv_parse_kernel(
    const uint8_t* __restrict__ b, int64_t n, const IT* __restrict__ ends, int64_t nlines, int ncols, CsvOpts o,
    const int64_t* __restrict__ dcols, uint8_t* __restrict__ valid, uint8_t* __restrict__ keep,
    unsigned long long* __restrict__ stats) {
  __shared__ uint32_t smask[kMaxCols];
  __shared__ int snull[kMaxCols];
  __shared__ int sempty, sflag, smiss, shard;
  __shared__ unsigned long long smaxl, sminl;
  __shared__ __attribute__((aligned(16))) uint8_t stage[LDS];
  for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
    smask[c] = 0;
    snull[c] = 0;
  }
  if (threadIdx.x == 0) {
    sflag = 0;
    sempty = 0;
    smiss = 0;
    shard = 0;
    smaxl = 0;
    sminl = 1ull << 62;
  }
  const uint8_t* ab = b - (reinterpret_cast<uintptr_t>(b) & 15);
  const int64_t off = b - ab;
  bool slow = false;
  const int64_t ngroups = (nlines + 255) / 256;
  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t l0 = grp * 256;
    const int64_t l1 = min(nlines, l0 + 256);
    const int64_t li = l0 + threadIdx.x;
    // bytes the group touches: [previous terminator, last line's end)
    const int64_t lo = l0 > 0 ? ends[l0 - 1] : 0;
    const int64_t hi = ends[l1 - 1];
    const int64_t glo = (lo + off) & ~(int64_t)15;  // aligned-view granule bounds
    const int64_t ghi = (hi + 1 + off + 15) & ~(int64_t)15;
    __syncthreads();  // previous group's readers are done with the stage
    if (ghi - glo <= LDS) {
      for (int64_t g = glo + 16 * threadIdx.x; g < ghi; g += 16 * blockDim.x) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (g - off < n) v = *reinterpret_cast<const u32x4*>(ab + g);  // granule overlaps [0, n)
        *reinterpret_cast<u32x4*>(stage + (g - glo)) = v;
      }
      __syncthreads();
      slow |= parse_line(stage, glo - off, n, ends, li, li < l1, nlines, ncols, o, dcols, valid, keep, smask,
                         snull, &sempty, &smiss, &shard, &smaxl, &sminl);
    } else {
      slow |= parse_line(b, 0, n, ends, li, li < l1, nlines, ncols, o, dcols, valid, keep, smask, snull, &sempty,
                         &smiss, &shard, &smaxl, &sminl);
    }
  }
  if (slow) sflag = 1;
  __syncthreads();
  // stats: [0] slow flag, [1] empty lines, [2, 2+ncols) null fields, [2+ncols, 2+2*ncols) class masks
  // (bit 8: a field whose value or class needs the host),
  // [2+2*ncols] lines with a field outside the numeric fast path, [3+2*ncols] those with a field that
  // is not even a quoted fast-path number
  for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
    if (snull[c]) atomicAdd(&stats[2 + c], (unsigned long long)snull[c]);
    if (smask[c]) atomicOr(&stats[2 + ncols + c], (unsigned long long)smask[c]);
  }
  if (threadIdx.x == 0) {
    if (sempty) atomicAdd(&stats[1], (unsigned long long)sempty);
    if (sflag) atomicOr(&stats[0], 1ull);
    if (smiss) atomicAdd(&stats[2 + 2 * ncols], (unsigned long long)smiss);
    if (shard) atomicAdd(&stats[3 + 2 * ncols], (unsigned long long)shard);
    atomicMax(&stats[4 + 2 * ncols], smaxl);  // longest line (terminator to terminator)
    atomicMin(&stats[6 + 2 * ncols], sminl);  // shortest (the caller initializes it high)
  }
}

// A raw (quoted / escaped) field's text compared with the literal as it is produced: the host
// tokenizer's state machine for one field (ops/csrc/host/csv.cpp split_record with no separator,
// so a NUL outside quotes ends the field), emitting bytes straight into the comparison.
__device__ __forceinline__ uint8_t raw_field_eq(const uint8_t* __restrict__ p, int64_t n,
                                                const uint8_t* __restrict__ lit, int L, int quote, int escape) {
  bool in_q = false, was_q = false;
  int k = 0;  // bytes of the field's text produced (and matched) so far
  for (int64_t i = 0; i < n; ++i) {
    int c = p[i], e = -1;  // e: the byte this step appends to the text, if any
    if (in_q) {
      if (c == escape && escape != quote && i + 1 < n && (p[i + 1] == quote || p[i + 1] == escape)) {
        e = p[++i];
      } else if (c == quote) {
        if (i + 1 < n && p[i + 1] == quote) {
          e = quote;
          ++i;
        } else {
          in_q = false;
        }
      } else {
        e = c;
      }
    } else if (c == 0) {
      break;  // the separator of a one-field record
    } else if (c == quote && k == 0 && !was_q) {
      in_q = was_q = true;
    } else if (c == escape && escape != quote && i + 1 < n && p[i + 1] == quote) {
      e = p[++i];
    } else {
      e = c;
    }
    if (e >= 0) {
      if (k >= L || lit[k] != (uint8_t)e) return 0;
      ++k;
    }
  }
  return k == L ? 1 : 0;
}

// A device string column (kind-4 spans into buf) compared with a constant: 1 equal, 0 not equal.
// Plain fields compare their bytes; raw (quoted / escaped) ones their unescaped text, produced on
// the fly -- no field's text is ever built on the host.
__global__ __launch_bounds__(256) void csv_span_eq_kernel(const uint8_t* __restrict__ buf, int64_t nbuf,
                                                          const int64_t* __restrict__ spans, int64_t n,
                                                          const uint8_t* __restrict__ lit, int L, int quote,
                                                          int escape, uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = spans[i];
    const int64_t fs = v >> 25, len = v & 0xFFFFFF;
    uint8_t r;
    if (fs < 0 || fs + len > nbuf) {
      r = 0;
    } else if ((v >> 24) & 1) {
      r = raw_field_eq(buf + fs, len, lit, L, quote, escape);
    } else if (len != L) {
      r = 0;
    } else {
      r = 1;
      for (int k = 0; k < L && r; ++k) r = buf[fs + k] == lit[k];
    }
    out[i] = r;
  }
}

}  // namespace

void csv_span_eq(const uint8_t* buf, int64_t nbuf, const int64_t* spans, int64_t n, const uint8_t* lit, int L,
                 int quote, int escape, uint8_t* out, hipStream_t st) {
  if (n <= 0) return;
  int64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(csv_span_eq_kernel, dim3(g), dim3(256), 0, st, buf, nbuf, spans, n, lit, L, quote, escape, out);
  DQ_HIP_CHECK(hipGetLastError());
}

// + 1: the window grid starts at the granule boundary below the buffer start
int64_t csv_count_blocks(int64_t n) { return (n + kChunk - 1) / kChunk + 1; }

bool csv_ends_i32(int64_t n) { return n < ((int64_t)1 << 31) - 1; }

void csv_line_ends(const uint8_t* buf, int64_t n, int64_t* counts, void* ends, hipStream_t st, int sep,
                   int32_t* facts) {
  const int64_t nb = csv_count_blocks(n);
  const uint32_t sep4 = (uint32_t)(sep & 0xFF) * 0x01010101u;
  if (facts != nullptr && (sep < 0 || sep > 255)) throw std::invalid_argument("csv_line_ends: facts need a separator byte");
  if (ends == nullptr) {  // pass 1: per-block counts -> exclusive offsets, total at counts[nb]
    hipLaunchKernelGGL(csv_count_kernel, dim3(nb), dim3(256), 0, st, buf, n, counts);
    hipLaunchKernelGGL(csv_scan_counts_kernel, dim3(1), dim3(1024), 0, st, counts, nb);
  } else if (csv_ends_i32(n)) {  // pass 2 (ends sized from counts[nb]); int32 offsets below 2 GiB
    hipLaunchKernelGGL((csv_ends_kernel<int32_t>), dim3(nb), dim3(256), 0, st, buf, n, counts,
                       static_cast<int32_t*>(ends), sep4, facts);
  } else {
    hipLaunchKernelGGL((csv_ends_kernel<int64_t>), dim3(nb), dim3(256), 0, st, buf, n, counts,
                       static_cast<int64_t*>(ends), sep4, facts);
  }
  DQ_HIP_CHECK(hipGetLastError());
}

// The parse stats' initial values plus the ends pass's per-block facts folded in: one block,
// launched between the ends pass and the parse (whose atomics then accumulate on top) -- it
// replaces a zero fill, a min-slot fill, a column sum of the facts and two copies (five launches).
// Layout (csv_scan.h): [parse counters 0 .. 4 + 2 ncols], 5 + 2 ncols separators, 6 + 2 ncols the
// shortest line (a min from above), 7 + 2 ncols .. 9 + 2 ncols CR / lone-LF / CR LF ends.
__global__ __launch_bounds__(256) void csv_stats_init_kernel(const int32_t* __restrict__ facts, int64_t nb,
                                                            int64_t* __restrict__ stats, int ncols) {
  __shared__ long long part[4][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long f[4] = {0, 0, 0, 0};
  for (int64_t i = threadIdx.x; i < nb; i += 256) {
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] += facts[4 * i + k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) f[k] += __shfl_xor(f[k], o, 64);
    if (lane == 0) part[wave][k] = f[k];
  }
  __syncthreads();
  const int nstat = 10 + 2 * ncols;
  for (int i = threadIdx.x; i < nstat; i += 256) {
    int64_t v = 0;
    if (i == 5 + 2 * ncols) v = part[0][0] + part[1][0] + part[2][0] + part[3][0];
    else if (i == 6 + 2 * ncols) v = (int64_t)1 << 30;
    else if (i >= 7 + 2 * ncols) {
      const int k = i - (6 + 2 * ncols);
      v = part[0][k] + part[1][k] + part[2][k] + part[3][k];
    }
    stats[i] = v;
  }
}

void csv_stats_init(const int32_t* facts, int64_t nb, int64_t* stats, int ncols, hipStream_t st) {
  hipLaunchKernelGGL(csv_stats_init_kernel, dim3(1), dim3(256), 0, st, facts, nb, stats, ncols);
  DQ_HIP_CHECK(hipGetLastError());
}

template <typename IT>
static void launch_parse(bool small, int64_t g, hipStream_t st, const uint8_t* buf, int64_t n, const IT* ends,
                         int64_t nlines, int ncols, const CsvOpts& o, const int64_t* dcols, uint8_t* valid,
                         uint8_t* keep, unsigned long long* stats) {
  if (small)
    hipLaunchKernelGGL((csv_parse_kernel<kParseLdsSmall, 8, IT>), dim3(g), dim3(256), 0, st, buf, n, ends, nlines,
                       ncols, o, dcols, valid, keep, stats);
  else
    hipLaunchKernelGGL((csv_parse_kernel<kParseLdsLarge, 4, IT>), dim3(g), dim3(256), 0, st, buf, n, ends, nlines,
                       ncols, o, dcols, valid, keep, stats);
}

void csv_parse(const uint8_t* buf, int64_t n, const void* ends, int64_t nlines, int ncols, const CsvOpts& o,
               const int64_t* dcols, uint8_t* valid, uint8_t* keep, int64_t* stats, hipStream_t st) {
  if (ncols > kMaxCols) throw std::invalid_argument("csv_parse: too many columns for the device scanner");
  if (nlines <= 0) return;
  int64_t g = (nlines + 255) / 256;
  if (g > 16384) g = 16384;
  // variant: DQ4ML_CSV_PARSE_LDS (8192 | 32768) forces one; default by mean line length
  static const int forced = [] {
    const char* e = getenv("DQ4ML_CSV_PARSE_LDS");
    return e ? atoi(e) : 0;
  }();
  const bool small = forced ? forced == kParseLdsSmall : (n / nlines) * 256 * 5 / 4 <= kParseLdsSmall;
  auto* stats64 = reinterpret_cast<unsigned long long*>(stats);
  if (csv_ends_i32(n))
    launch_parse(small, g, st, buf, n, static_cast<const int32_t*>(ends), nlines, ncols, o, dcols, valid, keep,
                 stats64);
  else
    launch_parse(small, g, st, buf, n, static_cast<const int64_t*>(ends), nlines, ncols, o, dcols, valid, keep,
                 stats64);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
