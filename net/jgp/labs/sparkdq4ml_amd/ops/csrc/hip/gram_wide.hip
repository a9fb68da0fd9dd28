// K5-wide: LDS-tiled MFMA SYRK for d > 64 (BASELINE config 5: 1e7 rows x 4096 features, fp8).
//
// G = Xᵀ X over rows, upper 256x256 panel pairs only, split-K over row ranges.  MI355X design:
//  * storage is the MFMA-fragment-ordered tiling (ops/layout.py): per superstep s (64 rows) and
//    32-feature tile t one 2 KiB chunk holding exactly the operand fragments of the 64 lanes —
//    bf16: [4 k-steps][64 lanes][16 B] (v_mfma_f32_32x32x16_bf16, K = 16 per k-step); fp8 e4m3:
//    [2 halves][64 lanes][16 B] (a lane's 32 B = all 64 rows: ONE block-scaled
//    v_mfma_scale_f32_32x32x64_f8f6f4 with unit E8M0 scales = 2x the bf16 MFMA rate);
//  * a "stage" is 32 rows (bf16) / 64 rows (fp8) = 16 KiB per 256-feature panel; stages stream
//    HBM/L2 -> LDS with global_load_lds (16 B per lane, lane-linear, so every later ds_read_b128 is
//    conflict-free with no swizzle) through a 4-deep ring (128 KiB LDS, 1 block per CU) with COUNTED
//    vmcnt: three stages stay in flight across the one barrier per stage;
//  * 8 waves (2 x 4) per 256x256 block, 128 x 64 per wave = 4 x 2 accumulators (2 waves/SIMD: one
//    wave's LDS reads hide under the other's MFMAs; the 4-wave 128 x 128 tiling halved the LDS
//    reads per MFMA but ran 86 vs 75 ms at 1 wave/SIMD, profiles/r3_wide_gang.md);
//  * the label and the intercept column ride along as an "augmentation" panel [1, y_hi, y_lo]
//    (a 32-feature tile of its own; the other 7 tiles stream from a zero page so every wave issues
//    the same number of loads), so count, Σy, Σy², Σx, Σxy fall out of the same SYRK — the
//    augmented [X | 1 | y] Gram of SURVEY.md K5 without re-streaming X; augmentation blocks skip
//    the all-zero MFMAs;
//  * blockIdx -> (split, pair) is XCD-aware (bijective): the blocks one XCD runs together are
//    consecutive pairs of the same row range, so the panels they share hit that XCD's L2;
//  * per-column fp8 scales are applied in the f64 slab reduction (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <stdexcept>

#include "common.h"
#include "gram_wide.h"

namespace dq4ml {

namespace {

constexpr int kPanel = 256;           // features per panel
constexpr int kTilesPerPanel = 8;     // 32-feature tiles
constexpr int kChunk = 2048;          // bytes of one (tile, stage) image
constexpr int kPanelStage = kTilesPerPanel * kChunk;  // 16 KiB
constexpr int kStageBytes = 2 * kPanelStage;          // A + B images
constexpr int kMaxRing = 5;                           // LDS stages (5 x 32 KiB = all 160 KiB)
constexpr int kWaves = 8;                             // waves per block (2 per SIMD)

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(8))) int i32x8;

template <int EB>
struct WideTraits;

template <>
struct WideTraits<16> {  // bf16: a stage = 32 rows = 2 k-steps of v_mfma_f32_32x32x16_bf16
  static constexpr int kStagesPerSup = 2;
  static constexpr int kSteps = 2;
  typedef bf16x8 frag;
  static __device__ __forceinline__ frag read(const unsigned char* tile, int kk, int lane) {
    return *reinterpret_cast<const frag*>(tile + kk * 1024 + lane * 16);
  }
  static __device__ __forceinline__ f32x16 mfma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  // byte offset of the (stage st, tile T) image = sdelta(st, NT) + T * kTileStride
  static constexpr int kTileStride = 4096;
  static __device__ __forceinline__ int64_t sdelta(int64_t st, int NT) {
    return (st >> 1) * (int64_t)NT * 4096 + (st & 1) * 2048;
  }
};

template <>
struct WideTraits<8> {  // fp8 e4m3 (OCP): a stage = 64 rows = 1 block-scaled K=64 MFMA
  static constexpr int kStagesPerSup = 1;
  static constexpr int kSteps = 1;
  typedef i32x8 frag;
  static __device__ __forceinline__ frag read(const unsigned char* tile, int, int lane) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(tile + lane * 16);
    const u32x4 hi = *reinterpret_cast<const u32x4*>(tile + 1024 + lane * 16);
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  }
  static __device__ __forceinline__ f32x16 mfma(frag a, frag b, f32x16 c) {
    // FMT 0/0 = e4m3 x e4m3, E8M0 scale 127 = 1.0 for both operands
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  }
  static constexpr int kTileStride = kChunk;
  static __device__ __forceinline__ int64_t sdelta(int64_t st, int NT) { return st * (int64_t)NT * kChunk; }
};

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g),
                                   (__attribute__((address_space(3))) void*)(l), 16, 0, 0);
}

__device__ __forceinline__ int pair_index(int I, int J, int P) {
  // pairs listed row-major over I <= J in [0, P] (P = augmentation panel)
  return I * (P + 1) - I * (I - 1) / 2 + (J - I);
}

template <bool TABLE>
__device__ __forceinline__ int64_t tile_of(const WideArgs& a, int pair, int slot) {
  if constexpr (TABLE) return (int64_t)a.tile_base[pair] + slot;
  else return (int64_t)pair * a.splitk + slot;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename F>
struct StageFrags {
  F a[2][4];  // [k-step][A tile]
  F b[2][2];  // [k-step][B tile]
};

// One (pair, split) block's K loop + epilogue.  MODE 0: off-diagonal panel pair; 3: diagonal pair
// (one panel, loaded once); 1: (I, augmentation);
// 2: (augmentation, augmentation).  Gang schedule (8 waves): a diagonal unit also carries the
// augmentation products of its panel — it loads panel I plus the augmentation tile, and the two
// waves whose 128 x 64 tiles lie entirely below the diagonal (wm = 1, wn < 2) compute (I, aug)
// instead (MODE 5; panel I = 0 adds (aug, aug)); the other six are MODE 4 (waves 0-1, which also load
// the augmentation tile) and MODE 6.  Separate instantiations keep the accumulators in AGPRs with no
// control-flow merge inside the loop (a merge there costs a full AGPR<->VGPR copy per stage).
//
// Schedule per stage i (fragments of stage i already in registers `cur`):
//   MFMAs on A tiles 0-1 | wait stage i+1 (counted vmcnt) + s_barrier | ds_read stage i+1 -> `nxt`,
//   glds stage i+4 into the buffer stage i vacated | MFMAs on A tiles 2-3 | lgkmcnt(0)
// so the LDS reads and the barrier skew hide under half a stage of MFMAs, and three stages of
// global_load_lds stay in flight across every barrier.
template <int EB, int MODE, int RING, bool TABLE = false>
__device__ __forceinline__ void syrk_block(const WideArgs& a, unsigned char* smem, int I, int J, int s_lo, int s_hi,
                                           int slot) {
  typedef WideTraits<EB> Tr;
  typedef typename Tr::frag F;
  // 2 x 4 waves of 128 x 64 (2 waves/SIMD)
  constexpr int kWBlock = 64 * kWaves;
  constexpr int WN = 2;  // 32-col tiles per wave
  constexpr int kLoadsPerPanel = kPanelStage / (kWBlock * 16);
  // loads per thread per stage: an augmentation side needs only piece 0 (tile 0 = [1, y_hi, y_lo]
  // for threads < 128, the zero page into tile 1 for the rest — waves whose tiles are all zero
  // read tile 1); a diagonal pair (MODE 3) loads its one panel once
  //
  // gang diagonal unit (MODE 4 / 5 / 6): the B region holds only the augmentation tile, read by
  // the MODE-5 waves; its 2 KiB are loaded by waves 0-1 alone (MODE 4).  The other waves (MODE
  // 5 / 6) issue no B piece -- theirs would be the zero page: 14 KiB of L2 -> LDS traffic per
  // stage for nothing.  vmcnt is per wave, so each mode's counted waits use its own loads.
  constexpr int LA = MODE == 2 ? 1 : kLoadsPerPanel;
  constexpr int LB = (MODE == 3 || MODE == 5 || MODE == 6) ? 0 : (MODE >= 1 ? 1 : kLoadsPerPanel);
  constexpr bool kDiagPanel = MODE == 3 || MODE == 4 || MODE == 6;  // B operand = the A panel
  constexpr bool kFullWave = MODE == 0 || kDiagPanel;
  constexpr int kLoadsPerStage = LA + LB;
  typedef StageFrags<F> SF;
  // The wave index is a scalar (readfirstlane): every LDS-DMA destination (M0) is SALU
  // arithmetic.
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t nst = a.nsup * Tr::kStagesPerSup;
  const int64_t st0 = nst * s_lo / a.splitk, st1 = nst * s_hi / a.splitk;  // rows of splits [s_lo, s_hi)
  const int64_t cnt = st1 - st0;

  // Each thread moves kLoadsPerPanel 16-byte pieces of every panel-stage image: piece r is byte o
  // = (r * 512 + tid) * 16 of the 16 KiB image, at a 32-bit panel-relative offset that never
  // changes; the stage adds a wave-uniform base (X + panel + Tr::sdelta, or the zero page for the
  // padding stages past cnt, or the augmentation tile), so a load is one uniform base + one
  // lane offset (no 64-bit per-lane address math and no per-lane select in the K loop).
  uint32_t offT[kLoadsPerPanel];  // panel-relative offset of piece r in the tiled image
  uint32_t offO[kLoadsPerPanel];  // o itself (augmentation tile / zero page, 2 KiB stride images)
#pragma unroll
  for (int r = 0; r < kLoadsPerPanel; ++r) {
    const uint32_t o = (uint32_t)(r * kWBlock + tid) * 16u;
    offO[r] = o;
    offT[r] = (o >> 11) * (uint32_t)Tr::kTileStride + (o & (kChunk - 1));
  }
  // (I, J come from a table every lane loads: readfirstlane keeps the panel bases scalar)
  const int Iu = __builtin_amdgcn_readfirstlane(I), Ju = __builtin_amdgcn_readfirstlane(J);
  const unsigned char* pA = a.X + (int64_t)Iu * kTilesPerPanel * Tr::kTileStride;
  const unsigned char* pB = a.X + (int64_t)Ju * kTilesPerPanel * Tr::kTileStride;
  const int cnt32 = (int)cnt;  // (a 32-bit scalar compare per stage: s_cmp, not a 64-bit v_cmp)
  // stages at or beyond cnt stream the zero page: the K loop then runs an even number of stages
  // with no branch at all (a branch there lets the compiler sink MFMAs past the barrier) and
  // every wait is the same counted vmcnt — the extra stage multiplies zeros
  auto issue = [&](int64_t st, int buf) {
    unsigned char* base = smem + buf * kStageBytes;
    const bool live = (int)st < cnt32;
    const int64_t dx = Tr::sdelta(st0 + st, a.NT), dg = Tr::sdelta(st0 + st, 1);
    const unsigned char* zx = a.zeros;
#pragma unroll
    for (int r = 0; r < LA; ++r) {
      unsigned char* dst = base + (r * kWBlock + wave * 64) * 16;
      if constexpr (MODE == 2) {  // (aug, aug): piece 0 of the first 128 threads is real
        const bool real = offO[r] < (uint32_t)kChunk;
        glds16((live && real ? a.Xaug + dg : zx) + offO[r], dst);
      } else {
        glds16((live ? pA + dx : zx) + offT[r], dst);
      }
    }
#pragma unroll
    for (int r = 0; r < LB; ++r) {
      unsigned char* dst = base + kPanelStage + (r * kWBlock + wave * 64) * 16;
      if constexpr (MODE == 0) {
        glds16((live ? pB + dx : zx) + offT[r], dst);
      } else if constexpr (MODE == 4) {  // waves 0-1 of a gang diagonal unit: all real aug rows
        glds16((live ? a.Xaug + dg : zx) + offO[r], dst);
      } else {  // MODE 1: the first 128 threads real, the rest the zero page
        const bool real = offO[r] < (uint32_t)kChunk;
        glds16((live && real ? a.Xaug + dg : zx) + offO[r], dst);
      }
    }
  };
  auto read = [&](SF& f, int buf) {
    const unsigned char* A = smem + buf * kStageBytes;
    const unsigned char* B = kDiagPanel ? A : A + kPanelStage;
    const int ta = MODE == 2 ? (wm == 0 ? 0 : 1) : (MODE == 5 ? wn * 4 : wm * 4);  // first A tile
    const int tb = (MODE == 1 || MODE == 2) ? (wn == 0 ? 0 : 1) : (MODE == 5 ? 0 : wn * WN);  // first B tile
#pragma unroll
    for (int kk = 0; kk < Tr::kSteps; ++kk) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
        if (MODE != 2 || x == 0) f.a[kk][x] = Tr::read(A + (ta + x) * kChunk, kk, lane);
#pragma unroll
      for (int y = 0; y < WN; ++y)
        if (kFullWave || y == 0) f.b[kk][y] = Tr::read(B + (tb + y) * kChunk, kk, lane);
    }
  };

  f32x16 acc[4][WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x16{};
  // (augmentation modes: waves whose B (or A) tiles come from the zero page multiply zeros —
  // cheaper than a data-dependent branch around the accumulators)
  auto mfmas = [&](const SF& f, int x0) {
#pragma unroll
    for (int kk = 0; kk < Tr::kSteps; ++kk)
#pragma unroll
      for (int x = x0; x < x0 + 2; ++x) {
        if (MODE == 2 && x != 0) continue;
#pragma unroll
        for (int y = 0; y < WN; ++y) {
          if (!kFullWave && y != 0) continue;
          acc[x][y] = Tr::mfma(f.a[kk][x], f.b[kk][y], acc[x][y]);
        }
      }
    if (MODE == 5 && x0 == 0)  // (aug, aug) into the wave's free accumulator (kept for I == 0)
#pragma unroll
      for (int kk = 0; kk < Tr::kSteps; ++kk) acc[0][1] = Tr::mfma(f.b[kk][0], f.b[kk][0], acc[0][1]);
  };
  // one stage: MFMAs(A tiles 0-1 of cur) | vmcnt: stage i+1 landed | s_barrier | MFMAs(A tiles
  // 2-3 of cur) interleaved with ds_read stage i+1 -> nxt and glds stage i+RING into the buffer
  // stage i vacated (the issue slots ride in the MFMA shadow) | lgkmcnt(0)
  int rb = 0;  // ring buffer of stage i
  auto step = [&](SF& cur, SF& nxt, int64_t i) {
    const int nb = rb + 1 == RING ? 0 : rb + 1;
    mfmas(cur, 0);
    __builtin_amdgcn_sched_barrier(0);
    wait_vm<(RING - 2) * kLoadsPerStage>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    mfmas(cur, 2);
    read(nxt, nb);
    issue(i + RING, rb);
    if (kFullWave) {
#pragma unroll
      for (int g = 0; g < 2 * WN; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, (4 + WN) * Tr::kSteps * (EB == 8 ? 2 : 1) / (2 * WN), 0);  // DS reads
        __builtin_amdgcn_sched_group_barrier(0x020, (kLoadsPerStage + 2 * WN - 1) / (2 * WN), 0);  // glds
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);                  // VALU address math
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    rb = nb;
  };

  if (cnt > 0) {
#pragma unroll
    for (int p = 0; p < RING; ++p) issue(p, p);
    wait_vm<(RING - 1) * kLoadsPerStage>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    SF f0, f1;
    read(f0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    for (int64_t i = 0; i < cnt; i += 2) {
      step(f0, f1, i);
      step(f1, f0, i + 1);
    }
    wait_vm<0>();  // drain the zero-page prefetches before the block can exit
  }
  if constexpr (MODE == 5) {  // (I, aug): 256 rows x the augmentation tile's 32 columns
    float* out = a.part + tile_of<TABLE>(a, pair_index(I, a.npanels, a.npanels), slot) * kPanel * kPanel;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        out[(wn * 128 + x * 32 + mfma32_row(lane, r)) * kPanel + mfma32_col(lane)] = acc[x][0][r];
    if (I == 0 && wn == 0) {
      float* o2 = a.part + tile_of<TABLE>(a, pair_index(a.npanels, a.npanels, a.npanels), slot) * kPanel * kPanel;
#pragma unroll
      for (int r = 0; r < 16; ++r) o2[mfma32_row(lane, r) * kPanel + mfma32_col(lane)] = acc[0][1][r];
    }
    return;
  }
  // f32 partial tile [256][256] of this (pair, slot)
  float* out = a.part + tile_of<TABLE>(a, pair_index(I, J, a.npanels), slot) * kPanel * kPanel;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < WN; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 128 + x * 32 + mfma32_row(lane, r);
        const int col = wn * 32 * WN + y * 32 + mfma32_col(lane);
        out[row * kPanel + col] = acc[x][y][r];
      }
}

template <int EB, int RING>
__global__ __launch_bounds__(64 * kWaves, 1) void gram_wide_kernel(WideArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // XCD-aware bijective remap: dispatch puts block b on XCD b % 8; give each XCD a contiguous
  // run of logical ids (split-major, pairs consecutive) so co-resident blocks share panels in L2
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rem = nwg & 7;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
  const int npair = (a.npanels + 1) * (a.npanels + 2) / 2;
  const int split = L / npair, pair = L - split * npair;
  const int I = a.pairs[2 * pair], J = a.pairs[2 * pair + 1];
  if (I == J && J != a.npanels) syrk_block<EB, 3, RING>(a, smem, I, J, split, split + 1, split);
  else if (J != a.npanels) syrk_block<EB, 0, RING>(a, smem, I, J, split, split + 1, split);
  else if (I != a.npanels) syrk_block<EB, 1, RING>(a, smem, I, J, split, split + 1, split);
  else syrk_block<EB, 2, RING>(a, smem, I, J, split, split + 1, split);
}

// Persistent, XCD-grouped schedule.  The grid is one block per CU; block b belongs to group
// g = b % 8 (blocks dispatched round-robin over the 8 XCDs: a group shares one XCD's L2 -- for
// speed only, any placement is correct).  Group g owns the row ranges (splits) g*h .. g*h+h-1 and
// pulls (split, pair) work units from its own queue head in list order: the ~32 blocks of a group
// always run a sliding window of consecutive units of the SAME row range whose panels overlap
// (Z-order pair list), so each panel-stage is fetched from HBM about once per window and then
// served from that XCD's L2 to every block of the window.  With the static one-pair-per-block
// grid, co-resident blocks of an XCD mix row ranges and finish at different times (diagonal and
// augmentation pairs are cheaper), which left the L2 hit rate at 54 % and the fabric reading each
// input byte ~8x.  The dynamic queue also absorbs the unequal unit costs.
template <int EB, int RING>
__global__ __launch_bounds__(64 * kWaves, 1) void gram_wide_queue_kernel(WideArgs a, int* __restrict__ heads, int h) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* slot = reinterpret_cast<int*>(smem + RING * kStageBytes);  // same LDS array as the ring
  const int g = blockIdx.x & 7;
  const int npair = (a.npanels + 1) * (a.npanels + 2) / 2;
  const int units = npair * h;
  for (;;) {
    if (threadIdx.x == 0) slot[0] = atomicAdd(&heads[g], 1);
    __syncthreads();
    const int u = slot[0];
    __syncthreads();  // every wave has read the slot (and finished the previous unit's LDS reads)
    if (u >= units) break;
    const int k = u / npair, pos = u - k * npair;
    const int split = g * h + k;
    const int I = a.pairs[2 * pos], J = a.pairs[2 * pos + 1];
    if (I == J && J != a.npanels) syrk_block<EB, 3, RING>(a, smem, I, J, split, split + 1, split);
    else if (J != a.npanels) syrk_block<EB, 0, RING>(a, smem, I, J, split, split + 1, split);
    else if (I != a.npanels) syrk_block<EB, 1, RING>(a, smem, I, J, split, split + 1, split);
    else syrk_block<EB, 2, RING>(a, smem, I, J, split, split + 1, split);
  }
}


// Gang schedule (one block per CU, 8 waves): group g = b % 8 (one XCD under round-robin dispatch)
// owns the row ranges [g*S, g*S+S) and its G blocks walk the unit list (range-major, then the
// P(P+1)/2 panel pairs I <= J < P in Z-order; a diagonal unit carries its augmentation products)
// statically: block l takes units l, l + G, l + 2G, ...  Every unit costs about the same (a
// diagonal unit's busiest SIMD runs as many MFMAs as an off-diagonal one's), so the G blocks of a
// group stay in step: round k runs units [kG, kG + G) of ONE row range (two at a range boundary),
// every panel-stage is fetched from HBM / MALL once per round and served from the XCD's L2 to the
// other blocks of the round.  The queue schedule's blocks drift apart (unequal unit costs,
// dynamic dequeue), so there each block re-fetched its panels (L2 hit 61 %, ~6.6x the unique
// bytes from the fabric).  S is chosen on the host so that npu * S is a multiple of G.
// unit u of a gang group -> (row range s, pair index pos): the S * P(P-1)/2 off-diagonal units
// first (range-major, Z-order pairs), then the S * P diagonal ones.  A diagonal unit streams one
// panel instead of two: the K loop is data-bound, so it ran in 3.1 ms against 4.6 ms (per-unit
// stamps, profiles/r5_wide_limiter.md); mixed into a round it let its block run ahead into the
// next round, and the blocks of an XCD drifted ~0.5 ms apart -- out of reach of each other's
// panel-stages in L2.  Segregated, every round holds units of one cost.  The pair table lists the
// off-diagonal pairs, then the diagonal ones.
// round barrier of a gang group (bar: 8 groups x 32 ints, zeroed per launch, or null): the block
// arrives after its unit k - 1 and waits until all G blocks of its group have -- the round's
// blocks then start their units together and share each panel-stage through the XCD's L2.  For
// speed only, never for correctness:
//  * only FULL rounds synchronize (round k runs G units iff k*G + G <= units): the blocks of a
//    partial last round would wait for arrivals that never come;
//  * the wait is bounded (kGangSpin polls), and a group whose wait ever times out -- its blocks
//    are not all co-resident: another kernel holds CU slots, a CU-masked stream, a placement that
//    is not round-robin -- turns its barrier off for the rest of the launch (bar[g*32 + 1]), so a
//    non-co-resident grid loses one bounded wait per group, not one per round.
constexpr int kGangSpin = 1 << 13;

__device__ __forceinline__ void gang_round_sync(int* bar, int g, int k, int G, int units) {
  if (bar == nullptr || k == 0 || k * G + G > units) return;
  if (threadIdx.x == 0) {
    int* c = bar + g * 32;
    __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_load(c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      const int target = k * G;
      int it = 0;
      for (; it < kGangSpin && __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++it)
        __builtin_amdgcn_s_sleep(4);
      if (it == kGangSpin) __hip_atomic_store(c + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

// unit u of the classic gang list (no long units): the S * P(P-1)/2 off-diagonal units range-major,
// then the S * P diagonal ones; `pos` indexes a.pairs (off-diagonal pairs in Z-order, then the
// diagonal ones)
__device__ __forceinline__ void gang_unit(int u, int S, int P, int& s, int& pos) {
  const int noff = P * (P - 1) / 2;
  if (u < S * noff) {
    s = u / noff;
    pos = u - s * noff;
  } else {
    const int v = u - S * noff;
    s = v / P;
    pos = noff + (v - s * P);
  }
}

// TABLE: units from the int4 table (long units over all S ranges for some pairs, per-pair tile
// prefix); else the classic list decoded from u (one range per unit, uniform tile layout)
template <int EB, int RING, bool TABLE>
__global__ __launch_bounds__(64 * kWaves, 1) void gram_wide_gang_kernel(WideArgs a, int S, int units,
                                                                       const int4* __restrict__ table,
                                                                       int* __restrict__ bar) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int g = blockIdx.x & 7, l = blockIdx.x >> 3, G = gridDim.x >> 3;
  const int wave = threadIdx.x >> 6;
  // the waves whose tiles lie entirely below a diagonal unit's diagonal
  const bool aug_wave = (wave >> 2) == 1 && (wave & 3) < 2;
  int k = 0;
  for (int u = l; u < units; u += G, ++k) {
    int I, J, lo, ns, slot;
    if constexpr (TABLE) {
      // unit u of every group: panels (I, J), row ranges [s0, s0 + ns) of the group's S, and the
      // unit's slot kk among the K units its pair has per group (slot g K + kk of the pair's tiles)
      const int4 e = table[u];
      I = e.x, J = e.y;
      const int s0 = e.z & 0xffff, kk = e.w & 0xffff, K = e.w >> 16;
      ns = e.z >> 16;
      lo = g * S + s0, slot = g * K + kk;
    } else {
      int s, pos;
      gang_unit(u, S, a.npanels, s, pos);
      I = a.pairs[2 * pos], J = a.pairs[2 * pos + 1];
      lo = g * S + s, ns = 1, slot = lo;
    }
    gang_round_sync(bar, g, k, G, units);
    if (I != J) syrk_block<EB, 0, RING, TABLE>(a, smem, I, J, lo, lo + ns, slot);
    else if (aug_wave) syrk_block<EB, 5, RING, TABLE>(a, smem, I, J, lo, lo + ns, slot);
    else if (wave < 2) syrk_block<EB, 4, RING, TABLE>(a, smem, I, J, lo, lo + ns, slot);  // + the aug tile's loads
    else syrk_block<EB, 6, RING, TABLE>(a, smem, I, J, lo, lo + ns, slot);
    __syncthreads();  // every wave is done reading the ring before the next unit's first glds
  }
}

// f64 reduction of the split-K slabs, fp8 scales applied, straight into the flat WLS layout:
// [count, wSum, wwSum, bSum, bbSum, aSum(d), abSum(d), aa packed-upper(d)]


// Walks the partial tiles in STORAGE order (thread = one (pair, row, col) element; the split-K
// slabs of consecutive threads are consecutive floats, so every read is coalesced) and scatters
// the f64 sums into the flat WLS layout.  Augmentation columns [1, y_hi, y_lo] fold into
// aSum / abSum / the five scalars.
//
// Banded form (data-parallel fits, X1): only the pairs of panel COLUMNS [J0, J1) — a contiguous
// range of the packed-upper layout (J = npanels: the head [count .. abSum]) — and, with out32, the
// values go to an f32 wire buffer (same flat indexing) that the bucketed RCCL all-reduce of that
// band ships while the next band folds.
__device__ __forceinline__ void wide_store(double* __restrict__ out, float* __restrict__ out32, int64_t idx, double v) {
  if (out32) out32[idx] = (float)v;
  else out[idx] = v;
}

__global__ __launch_bounds__(256) void gram_wide_reduce_kernel(WideArgs a, const float* __restrict__ scales,
                                                              double* __restrict__ out, float* __restrict__ out32,
                                                              int J0, int J1) {
  // one thread = 4 consecutive columns of one partial-tile row: float4 loads, 4 independent f64
  // chains per slab walk (the same k order per element as a scalar fold: bitwise the same sums).
  // Quads with nothing to fold skip their loads: the strictly-lower quads of a diagonal tile
  // (only i <= j is stored), and every augmentation quad but the first (columns 0-2 carry
  // [1, y_hi, y_lo]).
  const int d = a.d, P = a.npanels;
  int64_t npb = 0;  // pairs of the band's panel columns: column J holds pairs I = 0..J
  for (int J = J0; J < J1; ++J) npb += J + 1;
  const int64_t slab = (int64_t)kPanel * kPanel;
  const int64_t tot = npb * (slab / 4);
  const double s1 = a.aug_scale[0], syh = a.aug_scale[1], syl = a.aug_scale[2];  // device f64[3]
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < tot; g += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(g / (slab / 4));
    const int e = (int)(g - (int64_t)q * (slab / 4)) * 4, r = e >> 8, c0 = e & (kPanel - 1);
    int J = J0, I = q;  // band-local pair index (column-major) -> (I, J)
    while (I >= J + 1) { I -= J + 1; ++J; }
    const int pr = I * (P + 1) - I * (I - 1) / 2 + (J - I);  // row-major storage index of (I, J)
    const int64_t t0 = a.tile_base ? (int64_t)a.tile_base[pr] : (int64_t)pr * a.splitk;
    const int nsl = a.tile_base ? a.tile_base[pr + 1] - a.tile_base[pr] : a.splitk;  // this pair's slots
    const float* base = a.part + t0 * slab + e;
    const int i = I * kPanel + r;
    if (J < P) {  // Gram block
      if (i >= d || (I == J && r > c0 + 3)) continue;
      double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
      for (int k = 0; k < nsl; ++k) {
        const float4 x = *reinterpret_cast<const float4*>(base + (int64_t)k * slab);
        v0 += (double)x.x;
        v1 += (double)x.y;
        v2 += (double)x.z;
        v3 += (double)x.w;
      }
      const double v[4] = {v0, v1, v2, v3};
      const double si = scales ? (double)scales[i] : 1.0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = J * kPanel + c0 + t;
        if (j < d && i <= j) {
          const double sc = scales ? si * (double)scales[j] : 1.0;
          wide_store(out, out32, 5 + 2 * (int64_t)d + i + (int64_t)j * (j + 1) / 2, v[t] * sc);
        }
      }
      continue;
    }
    if (c0 != 0) continue;  // augmentation column: only columns 0-2 hold data
    if (I < P) {  // (X panel, augmentation): column 0 -> aSum, columns 1 + 2 -> abSum
      if (i >= d) continue;
      double v0 = 0.0, v1 = 0.0, v2 = 0.0;  // one float4 per slab (the same k order per element)
#pragma unroll 4
      for (int k = 0; k < nsl; ++k) {
        const float4 x = *reinterpret_cast<const float4*>(base + (int64_t)k * slab);
        v0 += (double)x.x;
        v1 += (double)x.y;
        v2 += (double)x.z;
      }
      const double si = scales ? (double)scales[i] : 1.0;
      wide_store(out, out32, 5 + i, v0 * si * s1);
      wide_store(out, out32, 5 + d + i, (v1 * syh + v2 * syl) * si);
    } else if (r == 0) {  // (augmentation, augmentation): the five scalars from rows 0-2
      double g00 = 0.0, g01 = 0.0, g02 = 0.0, g11 = 0.0, g12 = 0.0, g22 = 0.0;
#pragma unroll 2
      for (int k = 0; k < nsl; ++k) {
        const float* t = base + (int64_t)k * slab;
        const float4 x0 = *reinterpret_cast<const float4*>(t);
        const float4 x1 = *reinterpret_cast<const float4*>(t + kPanel);
        const float4 x2 = *reinterpret_cast<const float4*>(t + 2 * kPanel);
        g00 += (double)x0.x;
        g01 += (double)x0.y;
        g02 += (double)x0.z;
        g11 += (double)x1.y;
        g12 += (double)x1.z;
        g22 += (double)x2.z;
      }
      const double w = g00 * s1 * s1;
      wide_store(out, out32, 0, w);  // count, wSum, wwSum (unit weights; dead rows are zero)
      wide_store(out, out32, 1, w);
      wide_store(out, out32, 2, w);
      wide_store(out, out32, 3, g01 * s1 * syh + g02 * s1 * syl);                            // Σy
      wide_store(out, out32, 4, g11 * syh * syh + 2.0 * (g12 * syh * syl) + g22 * syl * syl);  // Σy²
    }
  }
}

// ---- packing into the wide tiled layouts ----------------------------------------------------
// per-feature amax (for fp8 scales): one block per feature
__global__ __launch_bounds__(256) void amax_kernel(const PackSrcW* __restrict__ srcs, int64_t n,
                                                  const uint8_t* __restrict__ sel, float* __restrict__ amax,
                                                  const float* __restrict__ shift) {
  const PackSrcW s = srcs[blockIdx.x];
  const float sh = shift ? shift[blockIdx.x] : 0.0f;  // amax of the shifted column x - s
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
    m = fmaxf(m, fabsf(v - sh));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// columns -> wide fragment-ordered tiles (EB = 16: bf16, EB = 8: fp8 with 1/scale pre-multiplied).
// One block-iteration = one (superstep s, tile t) chunk: thread (f, q) vector-loads rows
// [8q, 8q+8) of feature f (8 threads per feature: coalesced 256-B column runs); in the wide
// layout that run is lane 32(q & 1) + f's fragment of k-step q >> 1 -> one 16-B (bf16) or 8-B
// (fp8) store.
template <int EB>
__global__ __launch_bounds__(256) void pack_wide_kernel(const PackSrcW* __restrict__ srcs, int d, int64_t n, int NT,
                                                       int64_t nsup, const uint8_t* __restrict__ sel,
                                                       const float* __restrict__ inv_scale,
                                                       unsigned char* __restrict__ out,
                                                       const float* __restrict__ shift) {
  const int fl = threadIdx.x >> 3, q = threadIdx.x & 7;
  const int ki = q >> 1, lane = 32 * (q & 1) + fl;
  const int64_t nchunks = nsup * NT;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int t = (int)(c % NT);
    const int64_t s = c / NT;
    const int f = t * 32 + fl;
    const int64_t r0 = s * 64 + 8 * q;
    float x[8];
    if (f < d) {
      const PackSrcW src = srcs[f];
      load8_f32(src.ptr, src.dt, r0, n, x);
      if (shift) sub_shift8(x, shift[f], r0, n);
      mask8(sel, r0, n, x);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = 0.0f;
    }
    if constexpr (EB == 16) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[j];
      reinterpret_cast<u32x4*>(out)[c * 256 + ki * 64 + lane] = __builtin_bit_cast(u32x4, v);
    } else {  // saturate to the e4m3 range (the conversion maps overflow to NaN)
      const float is = f < d ? inv_scale[f] : 0.0f;
      float qv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[j] = fminf(fmaxf(x[j] * is, -448.0f), 448.0f);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(qv[0], qv[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(qv[2], qv[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(qv[4], qv[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(qv[6], qv[7], hi, true);
      // chunk (s, t) = [2 halves][64 lanes][16 B]; k-step ki -> half ki >> 1, byte 8 * (ki & 1)
      const int64_t o = c * 2048 + (((ki >> 1) * 64 + lane) << 4) + ((ki & 1) << 3);
      *reinterpret_cast<u32x2*>(out + o) = u32x2{(unsigned)lo, (unsigned)hi};
    }
  }
}

// ---- the label's augmentation panel [1, y_hi, y_lo] of the wide SYRK, on the device --------
// (the label split of models/regression -> ops/device.py _label_split, fused: three launches and
// no host read instead of ~40 elementwise / reduction ops between the fit's SYRKs)
//  1. wide_label_stats_kernel: per-block f64 partials [Σ live y, Σ live, max live y, min live y]
//     over a fixed grid (fixed summation order: deterministic);
//  2. wide_label_scales_kernel (one thread): fp8 -- the live mean t (the label is centred before
//     its split: two e4m3 digits of y - t carry ~8 bits relative to the label's spread), s_h =
//     max|y - t| / 448, s_l = s_h / 28 (the e4m3 rounding error of a value in [-448, 448] is at
//     most half an ulp of the top binade, 16, so (y - t) - y_hi stays within 16 s_h = 448 s_l);
//     bf16 -- t = 0 and unit scales.  aux = [1, s_h, s_l | t, 1/s_h, 1/s_l];
//  3. wide_label_pack_kernel: the 1-tile fragment panel (columns 0-2 live, y_hi, y_lo; 3-31 zero).
constexpr int kLabelBlocks = 256;

__global__ __launch_bounds__(256) void wide_label_stats_kernel(const void* __restrict__ y, int ydt, int64_t n,
                                                               const uint8_t* __restrict__ sel,
                                                               double* __restrict__ part) {
  __shared__ double red[4][4];
  double sy = 0.0, sw = 0.0, mx = -INFINITY, mn = INFINITY;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    if (sel != nullptr && !sel[r]) continue;
    const double v = ydt == 0 ? reinterpret_cast<const double*>(y)[r] : (double)reinterpret_cast<const float*>(y)[r];
    sy += v;
    sw += 1.0;
    mx = fmax(mx, v);
    mn = fmin(mn, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sy += __shfl_xor(sy, o);
    sw += __shfl_xor(sw, o);
    mx = fmax(mx, __shfl_xor(mx, o));
    mn = fmin(mn, __shfl_xor(mn, o));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w][0] = sy, red[w][1] = sw, red[w][2] = mx, red[w][3] = mn;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      red[0][0] += red[i][0];
      red[0][1] += red[i][1];
      red[0][2] = fmax(red[0][2], red[i][2]);
      red[0][3] = fmin(red[0][3], red[i][3]);
    }
    for (int i = 0; i < 4; ++i) part[blockIdx.x * 4 + i] = red[0][i];
  }
}

__global__ __launch_bounds__(64) void wide_label_scales_kernel(const double* __restrict__ part, int nb, int eb,
                                                                double* __restrict__ aux) {
  // one wave: lane l folds blocks l, l + 64, ... then a fixed butterfly (deterministic)
  double sy = 0.0, sw = 0.0, mx = -INFINITY, mn = INFINITY;
  for (int b = threadIdx.x; b < nb; b += 64) {
    sy += part[4 * b];
    sw += part[4 * b + 1];
    mx = fmax(mx, part[4 * b + 2]);
    mn = fmin(mn, part[4 * b + 3]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sy += __shfl_xor(sy, o);
    sw += __shfl_xor(sw, o);
    mx = fmax(mx, __shfl_xor(mx, o));
    mn = fmin(mn, __shfl_xor(mn, o));
  }
  if (threadIdx.x != 0) return;
  double t = 0.0, sh = 1.0, sl = 1.0;
  if (eb == 8) {
    t = sy / fmax(sw, 1.0);
    const double amax = sw > 0.0 ? fmax(mx - t, t - mn) : 0.0;
    sh = amax > 0.0 ? amax / 448.0 : 1.0;
    sl = sh / 28.0;
  }
  aux[0] = 1.0;
  aux[1] = sh;
  aux[2] = sl;
  aux[3] = t;
  aux[4] = 1.0 / sh;
  aux[5] = 1.0 / sl;
}

template <int EB>
__global__ __launch_bounds__(256) void wide_label_pack_kernel(const void* __restrict__ y, int ydt, int64_t n,
                                                              int64_t nsup, const uint8_t* __restrict__ sel,
                                                              const double* __restrict__ aux,
                                                              unsigned char* __restrict__ out) {
  const int fl = threadIdx.x >> 3, q = threadIdx.x & 7;
  const int ki = q >> 1, lane = 32 * (q & 1) + fl;
  const double t = aux[3], sh = aux[1], ish = aux[4], isl = aux[5];
  for (int64_t s = blockIdx.x; s < nsup; s += gridDim.x) {  // one 64-row superstep per iteration
    const int64_t r0 = s * 64 + 8 * q;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t r = r0 + j;
      const bool live = r < n && (sel == nullptr || sel[r]);
      float v = 0.0f;
      if (live && fl < 3) {
        if (fl == 0) {
          v = 1.0f;
        } else {
          const double yv = (ydt == 0 ? reinterpret_cast<const double*>(y)[r]
                                      : (double)reinterpret_cast<const float*>(y)[r]) - t;
          if constexpr (EB == 16) {
            const double hi = (double)(float)(__bf16)(float)yv;
            v = fl == 1 ? (float)hi : (float)(yv - hi);
          } else {
            const float qh = fminf(fmaxf((float)(yv * ish), -448.0f), 448.0f);
            if (fl == 1) {
              v = qh;
            } else {
              const float dh = __builtin_amdgcn_cvt_f32_fp8(__builtin_amdgcn_cvt_pk_fp8_f32(qh, 0.0f, 0, false), 0);
              v = fminf(fmaxf((float)((yv - (double)dh * sh) * isl), -448.0f), 448.0f);
            }
          }
        }
      }
      x[j] = v;
    }
    if constexpr (EB == 16) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[j];
      reinterpret_cast<u32x4*>(out)[s * 256 + ki * 64 + lane] = __builtin_bit_cast(u32x4, v);
    } else {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[0], x[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(x[2], x[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[4], x[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(x[6], x[7], hi, true);
      const int64_t o = s * 2048 + (((ki >> 1) * 64 + lane) << 4) + ((ki & 1) << 3);
      *reinterpret_cast<u32x2*>(out + o) = u32x2{(unsigned)lo, (unsigned)hi};
    }
  }
}

// Zero the dead rows of a wide fragment-ordered matrix (a DQ selection applied AFTER the pack):
// one pass over the storage, 16 B per thread, no dequantize / re-pack.  In both layouts a 16-B
// unit holds 8-row runs of ONE feature: bf16 = rows s*64 + 16ki + 8h + [0, 8) (unit = (s, t, ki,
// lane)), fp8 = two runs 16 rows apart, k-steps 2kh and 2kh + 1 (unit = (s, t, kh, lane));
// lane = 32h + feature % 32.
template <int EB>
__global__ __launch_bounds__(256) void wide_mask_rows_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                            int64_t units, int NT, int64_t n,
                                                            const uint8_t* __restrict__ sel) {
  constexpr int kUnitsPerChunk = EB == 8 ? 128 : 256;
  auto run_mask = [&](int64_t r0) -> uint64_t {  // 0x01 per live row byte, rows past n dead
    if (r0 + 8 <= n) return *gptr<uint64_t>(sel + r0);
    uint64_t m = 0;
    for (int j = 0; j < 8; ++j)
      if (r0 + j < n && sel[r0 + j]) m |= 1ull << (8 * j);
    return m;
  };
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = u / kUnitsPerChunk;
    const int q = (int)(u - c * kUnitsPerChunk);
    const int64_t s = c / NT;
    const int lane = q & 63, h = lane >> 5;
    u32x4 v = in[u];
    if constexpr (EB == 8) {
      const int kh = q >> 6;
      const int64_t base = s * 64 + 32 * kh + 8 * h;
      const uint64_t m0 = run_mask(base) * 0xffull, m1 = run_mask(base + 16) * 0xffull;  // bytes 0x01 -> 0xff
      v[0] &= (unsigned)m0, v[1] &= (unsigned)(m0 >> 32), v[2] &= (unsigned)m1, v[3] &= (unsigned)(m1 >> 32);
    } else {
      const int ki = q >> 6;
      const uint64_t m = run_mask(s * 64 + 16 * ki + 8 * h);
#pragma unroll
      for (int w = 0; w < 4; ++w) {  // dword w = rows 2w, 2w+1
        const unsigned lo = (unsigned)((m >> (16 * w)) & 1) * 0xffffu;
        const unsigned hi = (unsigned)((m >> (16 * w + 8)) & 1) * 0xffff0000u;
        v[w] &= lo | hi;
      }
    }
    out[u] = v;
  }
}

}  // namespace


void wide_mask_rows(int eb, const void* in, void* out, int d, int64_t n, const uint8_t* sel, hipStream_t st) {
  const int NT = ((d + 255) / 256) * 8;
  const int64_t units = wide_tiled_bytes(eb, d, n) / 16;
  int64_t g = (units + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  if (eb == 8)
    hipLaunchKernelGGL(wide_mask_rows_kernel<8>, dim3(g), dim3(256), 0, st, reinterpret_cast<const u32x4*>(in),
                       reinterpret_cast<u32x4*>(out), units, NT, n, sel);
  else
    hipLaunchKernelGGL(wide_mask_rows_kernel<16>, dim3(g), dim3(256), 0, st, reinterpret_cast<const u32x4*>(in),
                       reinterpret_cast<u32x4*>(out), units, NT, n, sel);
  DQ_HIP_CHECK(hipGetLastError());
}

int64_t wide_tiled_bytes(int eb, int d, int64_t n) {
  const int NT = ((d + 255) / 256) * 8;
  return ((n + 63) / 64) * NT * 4 * 64 * (int64_t)eb;
}

void feature_amax(const PackSrcW* srcs_dev, int d, int64_t n, const uint8_t* sel, float* amax, hipStream_t st,
                  const float* shift) {
  hipLaunchKernelGGL(amax_kernel, dim3(d), dim3(256), 0, st, srcs_dev, n, sel, amax, shift);
  DQ_HIP_CHECK(hipGetLastError());
}

void pack_wide(int eb, const PackSrcW* srcs_dev, int d, int64_t n, int nt, const uint8_t* sel, const float* inv_scale,
               void* out, hipStream_t st, const float* shift) {
  const int64_t nsup = (n + 63) / 64;
  int64_t g = nsup * nt;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  unsigned char* o = reinterpret_cast<unsigned char*>(out);
  if (eb == 16) hipLaunchKernelGGL(pack_wide_kernel<16>, dim3(g), dim3(256), 0, st, srcs_dev, d, n, nt, nsup, sel, inv_scale, o, shift);
  else hipLaunchKernelGGL(pack_wide_kernel<8>, dim3(g), dim3(256), 0, st, srcs_dev, d, n, nt, nsup, sel, inv_scale, o, shift);
  DQ_HIP_CHECK(hipGetLastError());
}

// statistics of a label shifted by t = aux[3] (y' = y - t) -> those of y, in place (f64), after the
// head fold: Σy² += 2tΣy' + t²W, Σy += tW, Σx·y += tΣx (one thread per feature; thread 0 the
// scalars, reading Σy' before anyone writes it)
__global__ __launch_bounds__(256) void wide_unshift_label_kernel(double* __restrict__ out, int d,
                                                                 const double* __restrict__ aux) {
  const double t = aux[3];
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < d) out[5 + d + j] += t * out[5 + j];
  if (j == 0) {
    const double W = out[1], b = out[3];
    out[4] += (2.0 * t) * b + (t * t) * W;
    out[3] = b + t * W;
  }
}

void wide_unshift_label(double* out, int d, const double* aux, hipStream_t st) {
  hipLaunchKernelGGL(wide_unshift_label_kernel, dim3((d + 255) / 256 > 0 ? (d + 255) / 256 : 1), dim3(256), 0, st,
                     out, d, aux);
  DQ_HIP_CHECK(hipGetLastError());
}

int wide_label_part_doubles() { return 4 * kLabelBlocks; }

void wide_label_aug(int eb, const void* y, int ydt, int64_t n, const uint8_t* sel, double* part, double* aux,
                    void* out, hipStream_t st) {
  if (eb != 8 && eb != 16) throw std::invalid_argument("wide_label_aug: eb must be 8 or 16");
  if (ydt != 0 && ydt != 1) throw std::invalid_argument("wide_label_aug: label must be f64 or f32");
  const int64_t nsup = (n + 63) / 64;
  hipLaunchKernelGGL(wide_label_stats_kernel, dim3(kLabelBlocks), dim3(256), 0, st, y, ydt, n, sel, part);
  hipLaunchKernelGGL(wide_label_scales_kernel, dim3(1), dim3(64), 0, st, part, kLabelBlocks, eb, aux);
  int64_t g = nsup < 1 ? 1 : (nsup > 2048 ? 2048 : nsup);  // (grid-stride: ~10 supersteps per block)
  unsigned char* o = reinterpret_cast<unsigned char*>(out);
  if (eb == 16) hipLaunchKernelGGL(wide_label_pack_kernel<16>, dim3(g), dim3(256), 0, st, y, ydt, n, nsup, sel, aux, o);
  else hipLaunchKernelGGL(wide_label_pack_kernel<8>, dim3(g), dim3(256), 0, st, y, ydt, n, nsup, sel, aux, o);
  DQ_HIP_CHECK(hipGetLastError());
}

int64_t gram_wide_partials(int d, int splitk) {
  const int P = (d + kPanel - 1) / kPanel;
  const int npair = (P + 1) * (P + 2) / 2;
  return (int64_t)npair * splitk * kPanel * kPanel;
}

template <int EB, int RING>
static void launch_wide(const WideArgs& a, int nblocks, hipStream_t st) {
  const size_t lds = (size_t)RING * kStageBytes;
  DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_kernel<EB, RING>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((gram_wide_kernel<EB, RING>), dim3(nblocks), dim3(64 * kWaves), lds, st, a);
  DQ_HIP_CHECK(hipGetLastError());
}

template <int EB, int RING>
static void launch_wide_queue(const WideArgs& a, int grid, int* heads, int h, hipStream_t st) {
  const size_t lds = (size_t)RING * kStageBytes + 16;
  DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_queue_kernel<EB, RING>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((gram_wide_queue_kernel<EB, RING>), dim3(grid), dim3(64 * kWaves), lds, st, a, heads, h);
  DQ_HIP_CHECK(hipGetLastError());
}

static void launch_fold(const WideArgs& a, const float* scales, double* out, float* out32, int J0, int J1,
                        hipStream_t st) {
  int64_t npb = 0;
  for (int J = J0; J < J1; ++J) npb += J + 1;
  int64_t g = (npb * kPanel * kPanel / 4 + 255) / 256;  // one thread per 4 columns
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(gram_wide_reduce_kernel, dim3(g), dim3(256), 0, st, a, scales, out, out32, J0, J1);
  DQ_HIP_CHECK(hipGetLastError());
}

void gram_wide_fold(WideArgs a, const float* scales, double* out, float* out32, int J0, int J1, hipStream_t st) {
  if (J0 < 0 || J1 > a.npanels + 1 || J0 >= J1) throw std::invalid_argument("gram_wide_fold: bad panel-column band");
  if ((out == nullptr) == (out32 == nullptr)) throw std::invalid_argument("gram_wide_fold: exactly one output");
  launch_fold(a, scales, out, out32, J0, J1, st);
}

void gram_wide_queue(int eb, WideArgs a, const int* pairs_dev, const float* scales, double* out, int* heads, int h,
                     int grid, hipStream_t st, bool fold) {
  a.pairs = pairs_dev;
  if (a.splitk != 8 * h) throw std::invalid_argument("gram_wide_queue: splitk must be 8 * h");
  if (grid < 8 || grid % 8) throw std::invalid_argument("gram_wide_queue: grid must be a positive multiple of 8");
  DQ_HIP_CHECK(hipMemsetAsync(heads, 0, 8 * sizeof(int), st));
  if (eb == 16) launch_wide_queue<16, 4>(a, grid, heads, h, st);
  else launch_wide_queue<8, 4>(a, grid, heads, h, st);
  if (fold) launch_fold(a, scales, out, nullptr, 0, a.npanels + 1, st);
}

template <int EB>
static void launch_wide_gang(const WideArgs& a, int grid, int S, int units, const int4* table, hipStream_t st,
                             int* bar) {
  const size_t lds = (size_t)5 * kStageBytes;
  if (bar != nullptr) DQ_HIP_CHECK(hipMemsetAsync(bar, 0, 8 * 32 * sizeof(int), st));
  if (table != nullptr) {
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_gang_kernel<EB, 5, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((gram_wide_gang_kernel<EB, 5, true>), dim3(grid), dim3(64 * kWaves), lds, st, a, S, units,
                       table, bar);
  } else {
    DQ_HIP_CHECK(hipFuncSetAttribute((const void*)gram_wide_gang_kernel<EB, 5, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((gram_wide_gang_kernel<EB, 5, false>), dim3(grid), dim3(64 * kWaves), lds, st, a, S, units,
                       table, bar);
  }
  DQ_HIP_CHECK(hipGetLastError());
}

void gram_wide_gang(int eb, WideArgs a, const int* table, int units, const float* scales, double* out, int S, int grid,
                    hipStream_t st, bool fold, int* bar) {
  if (S < 1 || a.splitk != 8 * S) throw std::invalid_argument("gram_wide_gang: splitk must be 8 * S");
  if (grid < 8 || grid % 8) throw std::invalid_argument("gram_wide_gang: grid must be a positive multiple of 8");
  if ((int64_t)a.splitk > a.nsup) throw std::invalid_argument("gram_wide_gang: more row ranges than supersteps");
  if (units < 1) throw std::invalid_argument("gram_wide_gang: no units");
  // the table form needs its tile prefix; the classic form decodes units from a.pairs (off-diagonal
  // pairs, then diagonal ones) over the uniform splitk tile layout
  if (table != nullptr && a.tile_base == nullptr) throw std::invalid_argument("gram_wide_gang: table needs tile_base");
  if (table == nullptr && (a.pairs == nullptr || a.tile_base != nullptr || units != S * a.npanels * (a.npanels + 1) / 2))
    throw std::invalid_argument("gram_wide_gang: the classic unit list needs the pair list and the uniform layout");
  const int4* t = reinterpret_cast<const int4*>(table);
  if (eb == 16) launch_wide_gang<16>(a, grid, S, units, t, st, bar);
  else launch_wide_gang<8>(a, grid, S, units, t, st, bar);
  if (fold) launch_fold(a, scales, out, nullptr, 0, a.npanels + 1, st);
}

void gram_wide(int eb, WideArgs a, const int* pairs_dev, const float* scales, double* out, hipStream_t st, int ring,
               bool fold) {
  a.pairs = pairs_dev;
  const int P = a.npanels;
  const int npair = (P + 1) * (P + 2) / 2;
  const int nb = npair * a.splitk;
  if (ring != 4 && ring != 5) throw std::invalid_argument("gram_wide: ring must be 4 or 5");
  if (eb == 16) ring == 5 ? launch_wide<16, 5>(a, nb, st) : launch_wide<16, 4>(a, nb, st);
  else ring == 5 ? launch_wide<8, 5>(a, nb, st) : launch_wide<8, 4>(a, nb, st);
  if (fold) launch_fold(a, scales, out, nullptr, 0, P + 1, st);
}

}  // namespace dq4ml
