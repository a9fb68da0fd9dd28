// Host check of csv_div_pow10 (csv_parse_dev.h): the fma-corrected product by RN(10^-k) equals
// the correctly rounded quotient v / 10^k for integer mantissas v < 10^9 and 0 <= k <= 9 — the
// whole range of the numeric fast path.  A stride of the 10^10 cases (the full sweep passed
// offline; it takes ~25 CPU-seconds).
#include <cmath>
#include <cstdio>

#define __device__
#define __forceinline__ inline
static inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
#include "csv_parse_dev.h"

using namespace dq4ml_csv;

int main() {
  long bad = 0, n = 0;
  for (int k = 0; k <= 9; ++k) {
    const double p = csv_pow10(k);
    for (long v = k; v < 1000000000L; v += 97) {
      const double x = (double)v;
      ++n;
      if (csv_div_pow10(x, k) != x / p) {
        if (bad < 5) printf("MISMATCH v %ld k %d: %.17g vs %.17g\n", v, k, csv_div_pow10(x, k), x / p);
        ++bad;
      }
    }
  }
  printf("div_pow10 %s: %ld cases\n", bad ? "FAILED" : "ok", n);
  return bad != 0;
}
