// K5-wide: LDS-tiled MFMA SYRK for d > 64 (see gram_wide.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

struct PackSrcW {
  const void* ptr;
  int dt;
  int pad;
};

struct WideArgs {
  const unsigned char* X;     // wide tiled storage, NT = npanels * 8 tiles
  const unsigned char* Xaug;  // 1-tile tiled storage of [1, y_hi, y_lo] (same element type)
  const unsigned char* zeros; // >= 16 KiB zero page (streams the empty tiles of the augmentation panel)
  int NT;
  int npanels;                // ceil(d / 256)
  int d;
  int64_t nsup;               // supersteps (64 rows)
  int splitk;
  const int* pairs;           // [npair][2] panel pairs I <= J over [0, npanels] (npanels = augmentation)
  float* part;                // [npair * splitk][256][256] f32 partial tiles
  const double* aug_scale;    // device f64[3]: scales of [1, y_hi, y_lo] (made on the device with the
                              // label split, so no launch reads them on the host)
  const int* tile_base;       // (or null: splitk slots per pair) [npair + 1] prefix table of the
                              // partial tiles per pair (the gang schedule's merged units)
};

constexpr int kWideZeroBytes = 32768;  // >= the largest panel-relative piece offset (bf16 tiles: 30 KiB)

int64_t wide_tiled_bytes(int eb, int d, int64_t n);
int64_t gram_wide_partials(int d, int splitk);
// shift (null: none): per-feature f32 shift s; the amax is that of x - s and the pack stores
// (x - s) [* inv_scale] (the Gram statistics are un-shifted in f64 afterwards: gram.h stats_unshift)
void feature_amax(const PackSrcW* srcs_dev, int d, int64_t n, const uint8_t* sel, float* amax, hipStream_t st,
                  const float* shift = nullptr);
// the label's augmentation panel [1, y_hi, y_lo] (1 tile, eb's layout) of rows with sel != 0
// (null: all), split on the device: aux (f64[6]) = [1, s_h, s_l | t, 1/s_h, 1/s_l] -- aux[0:3] is
// the fold's aug_scale, aux[3] the label shift t (fp8: the live mean; bf16: 0); part:
// wide_label_part_doubles() f64 of scratch.  y: f64 (ydt 0) or f32 (ydt 1).
// head statistics of the label shifted by aux[3] -> those of the label, in place (after the head fold)
void wide_unshift_label(double* out, int d, const double* aux, hipStream_t st);
int wide_label_part_doubles();
void wide_label_aug(int eb, const void* y, int ydt, int64_t n, const uint8_t* sel, double* part, double* aux,
                    void* out, hipStream_t st);
// eb = 16 (bf16) or 8 (fp8 e4m3, values multiplied by inv_scale[f] before conversion)
void pack_wide(int eb, const PackSrcW* srcs_dev, int d, int64_t n, int nt, const uint8_t* sel, const float* inv_scale,
               void* out, hipStream_t st, const float* shift = nullptr);
// zero the rows with sel[r] == 0 (and rows >= n) of a wide tiled matrix: in -> out (may alias)
void wide_mask_rows(int eb, const void* in, void* out, int d, int64_t n, const uint8_t* sel, hipStream_t st);
// out: flat WLS layout [count, wSum, wwSum, bSum, bbSum, aSum(d), abSum(d), aa packed-upper(d)]
// fold = false: partial tiles only (the caller folds them band by band with gram_wide_fold)
void gram_wide(int eb, WideArgs a, const int* pairs_dev, const float* scales, double* out, hipStream_t st,
               int ring = 4, bool fold = true);
// persistent XCD-grouped schedule: grid blocks (one per CU, a multiple of 8), group b % 8 owns
// splits [g*h, g*h+h) (a.splitk == 8*h) and dequeues (split, pair) units from heads[g] (8 ints,
// zeroed here on the stream)
void gram_wide_queue(int eb, WideArgs a, const int* pairs_dev, const float* scales, double* out, int* heads, int h,
                     int grid, hipStream_t st, bool fold = true);
// gang schedule: grid blocks (one per CU, a multiple of 8) of 8 waves; group b % 8 owns splits
// [g*S, g*S+S) (a.splitk == 8*S) and its blocks walk `units` entries of `table` (int4 per unit:
// I, J, s0 | ns << 16, kk | K << 16 -- panels, row ranges [s0, s0 + ns) of the group, the unit's
// slot kk of the K its pair has per group) statically, block l taking l, l + G, ...; partial
// tiles at a.tile_base[pair] + g K + kk; bar (or null): 256 ints of scratch for the per-round
// group barrier (zeroed here on the stream; full rounds only, bounded, self-disabling:
// gram_wide.hip gang_round_sync)
void gram_wide_gang(int eb, WideArgs a, const int* table, int units, const float* scales, double* out, int S, int grid,
                    hipStream_t st, bool fold = true, int* bar = nullptr);
// fold the pairs of panel columns [J0, J1) (J = npanels: the augmentation column -> the head of
// the flat layout) into out (f64) or out32 (f32 wire buffer, same flat indexing)
void gram_wide_fold(WideArgs a, const float* scales, double* out, float* out32, int J0, int J1, hipStream_t st);

}  // namespace dq4ml
