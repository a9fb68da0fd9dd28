// Row-wise kernels (see rowops.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "huber_qn.h"

namespace dq4ml {

struct PackSrc {
  const void* ptr;
  int dt;
  int pad;
};

int64_t compact_blocks(int64_t n);
// counts must hold compact_blocks(n) + 1 int64: exclusive offsets + total at [nb]
void compact_count_scan(const uint8_t* sel, int64_t n, int64_t* counts, hipStream_t st);
void compact_write(const uint8_t* sel, int64_t n, const int64_t* offsets, int64_t limit, int64_t* out,
                   hipStream_t st);

void pack_columns(const PackSrc* srcs_dev, int d, int64_t n, void* out, int odt, int64_t ld, const uint8_t* sel,
                  hipStream_t st);

// shift: per-feature f32 shift subtracted before the bf16 cast (null: none)
void pack_tiled(const PackSrc* srcs_dev, int d, int64_t n, const uint8_t* sel, void* out, hipStream_t st,
                const float* shift = nullptr);
void predict(const void* X, int xdt, int64_t ld, int d, int64_t n, const double* coef, double b, double* out,
             hipStream_t st, int tiled);
int metrics_blocks(int64_t n);
void regression_metrics(const void* X, int xdt, int64_t ld, int d, int64_t n, const void* y, int ydt,
                        const uint8_t* sel, const double* coef, double b, double shift, double* partials,
                        double* out, hipStream_t st, int tiled);

// K9 huber: out = [lossSum, weightSum, g_intercept, g_sigma, Σ_r m_r x_jr (d)]; `partials` holds
// huber_partials(n, d) doubles, `mult` n (used for d > 16 only)
int64_t huber_partials(int64_t n, int d);
void huber_pass(const void* X, int xdt, int64_t ld, int d, int64_t n, int tiled, const void* y, int ydt,
                const void* w, int wdt, const uint8_t* sel, const double* ceff, double icpt, double sigma, double eps,
                double* mult, double* partials, double* out, hipStream_t st);

// the same pass steered by the device l-bfgs-b (huber_qn.hip): trial = [c_eff * scale (d) | intercept
// (shift folded in) | sigma], skipped when *act != kHuberEval; out[4 + j] gets the fp8 scale and the
// storage shift applied (either may be null)
void huber_pass_dev(const void* X, int xdt, int64_t ld, int d, int64_t n, int tiled, const void* y, int ydt,
                    const void* w, int wdt, const uint8_t* sel, const double* trial, const int* act, double eps,
                    const double* scale, const double* shift, double* mult, double* partials, double* out,
                    hipStream_t st);

// a bounded stand-in for a collective's channel blocks (diagnostics): blocks x 256 threads, usec each
void standin(int blocks, int usec, hipStream_t st);

}  // namespace dq4ml
