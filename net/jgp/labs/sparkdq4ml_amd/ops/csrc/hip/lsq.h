// K9: per-evaluation data passes of the squared-loss l-bfgs / OWLQN path (lsq.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

// Feature-matrix layouts (the ``tiled`` codes of rowops): 0 plain feature-major [d][ld] of xdt
// (f64 / f32 / bf16), 1 tall bf16 tiles (TiledBF16), 2 wide bf16 tiles, 3 wide fp8 tiles (TiledWide).
struct LsqX {
  const void* X;
  int layout;
  int xdt;      // layout 0 only
  int64_t ld;   // layout 0 only
  int d;
  int64_t n;
};

// workspace sizes (doubles) of one evaluation / one moments pass
int64_t lsq_part_doubles(const LsqX& x, int mode);
int lsq_margin_blocks(const LsqX& x);

// Margin pass: v[r] = w[r] * (x_r . cf + *offset - y[r] * inv_ystd), loss partial sum of 1/2 w diff^2 per
// block (lpart[lsq_margin_blocks]).  cf: effective coefficients (f32 for the tile layouts, f64 plain).
void lsq_margin(const LsqX& x, const void* cf, const double* offset, double inv_ystd, const double* y, const double* w,
                double* v, double* lpart, hipStream_t st);

// Column pass: mode 0 -> out[1 + j] = sum_r v[r] x[r][j] and out[0] = sum(lpart) (the evaluation);
// mode 1 -> out[j] = sum_r v[r] x[r][j], out[d + j] = sum_r v[r] x[r][j]^2 (feature moments, v = w).
// part: lsq_part_doubles(x, mode) doubles of workspace.  Fixed-order reductions (deterministic).
void lsq_columns(const LsqX& x, int mode, const double* v, const double* lpart, int nl, double* part, double* out,
                 hipStream_t st);

// The whole squared-loss l-bfgs / OWLQN fit as one cooperative launch (lsq_qn.hip): wide tile
// layouts (2 bf16, 3 fp8), d <= kLsqQnMaxD, one rank.  head: the summarizer pass [count, W, W2,
// Σwy, Σwy², Σwx (d), Σwx² (d)]; out: [coef(d), intercept, status, reason, H, iterations, evaluations,
// head(5), history(hist_cap)] (status 0 ok, 1 empty data, 2 constant label, 8 history overflow:
// the host path owns those).  work: lsq_qn_work(d, blocks, n) doubles.
constexpr int kLsqQnMaxD = 16384;
int lsq_qn_blocks(int layout, int d);
int64_t lsq_qn_work(int d, int blocks, int64_t n);
void lsq_qn(const LsqX& x, const double* y, const double* w, const double* scale, const double* shift,
            const double* head, bool fit_icpt, bool std_f, double reg, double enet, int max_iter, double tol,
            int hist_cap, double* work, int blocks, double* out, hipStream_t st);

// Data-parallel form of lsq_qn (X4, lsq_qn.hip): the same fit as separate launches around an
// all-reduce.  phase 0 starts the fit (head = the ALL-REDUCED summarizer head), phase 1 enqueues
// one evaluation's pass over this rank's rows and leaves [Σ v x_j (d), loss, Σ v] at
// work + lsq_qn_dp_red_offset (the caller all-reduces those d + 2 doubles), phase 2 the control
// step; the state's action (int, 3 = done) is the first word at work + lsq_qn_dp_ctl_offset.
// Every kernel returns at once after the fit is done.  work: lsq_qn_dp_work doubles.
int64_t lsq_qn_dp_work(int d, int blocks, int64_t n);
int64_t lsq_qn_dp_red_offset(int d, int blocks, int64_t n);
int64_t lsq_qn_dp_ctl_offset(int d, int blocks, int64_t n);
void lsq_qn_dp(int phase, const LsqX& x, const double* y, const double* w, const double* scale, const double* shift,
               const double* head, bool fit_icpt, bool std_f, double reg, double enet, int max_iter, double tol,
               int hist_cap, double* work, int blocks, double* out, hipStream_t st);

}  // namespace dq4ml
