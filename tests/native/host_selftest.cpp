// Native self-test of the host runtime library (solvers, WLS driver, CSV scanner), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py (SURVEY.md §5b:
// sanitizers run on host code; GPU ASan is not available on this pool).  Exit code 0 = pass.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "csv.h"
#include "solvers.h"
#include "wls.h"

using namespace dq4ml;

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

static bool close(double a, double b, double tol) { return std::fabs(a - b) <= tol * (1.0 + std::fabs(b)); }

static void test_cholesky() {
  // A = [[4,2,0],[2,5,1],[0,1,3]] packed upper column-major
  std::vector<double> ap = {4, 2, 5, 0, 1, 3};
  std::vector<double> b = {2, 1, 4};
  auto x = cholesky_solve(3, ap, b);
  std::vector<double> y(3);
  dspmv(3, ap.data(), x.data(), y.data());
  for (int i = 0; i < 3; ++i) CHECK(close(y[i], b[i], 1e-12));
  auto inv = cholesky_inverse(3, ap);
  // A * inv(:,0) == e0
  std::vector<double> col = {inv[pk(0, 0)], inv[pk(0, 1)], inv[pk(0, 2)]};
  dspmv(3, ap.data(), col.data(), y.data());
  CHECK(close(y[0], 1.0, 1e-12) && std::fabs(y[1]) < 1e-12 && std::fabs(y[2]) < 1e-12);
  bool threw = false;
  try {
    std::vector<double> sing = {1, 1, 1};  // [[1,1],[1,1]]
    cholesky_solve(2, sing, {1, 1});
  } catch (const SingularMatrixError&) {
    threw = true;
  }
  CHECK(threw);
}

static std::vector<double> flat_stats(const std::vector<std::vector<double>>& X, const std::vector<double>& y) {
  const int d = (int)X.size();
  const size_t n = y.size();
  std::vector<double> f(5 + 2 * d + d * (d + 1) / 2, 0.0);
  for (size_t r = 0; r < n; ++r) {
    f[0] += 1;
    f[1] += 1;
    f[2] += 1;
    f[3] += y[r];
    f[4] += y[r] * y[r];
    for (int j = 0; j < d; ++j) {
      f[5 + j] += X[j][r];
      f[5 + d + j] += X[j][r] * y[r];
      for (int i = 0; i <= j; ++i) f[5 + 2 * d + pk(i, j)] += X[i][r] * X[j][r];
    }
  }
  return f;
}

static void test_wls() {
  // exact linear data: y = 2 x0 - 3 x1 + 0.5
  std::vector<std::vector<double>> X(2, std::vector<double>(50));
  std::vector<double> y(50);
  for (int r = 0; r < 50; ++r) {
    X[0][r] = std::sin(0.3 * r) + 0.1 * r;
    X[1][r] = std::cos(0.7 * r);
    y[r] = 2 * X[0][r] - 3 * X[1][r] + 0.5;
  }
  auto f = flat_stats(X, y);
  WlsResult c = wls_fit(f.data(), 2, true, 0.0, 0.0, true, true, 0, 100, 1e-9, true);
  CHECK(c.status == WLS_OK && c.solver == "cholesky");
  CHECK(close(c.coefficients[0], 2.0, 1e-9) && close(c.coefficients[1], -3.0, 1e-9) && close(c.intercept, 0.5, 1e-9));
  WlsResult q = wls_fit(f.data(), 2, true, 0.01, 1.0, true, true, 0, 100, 1e-10, false);  // OWLQN (L1)
  CHECK(q.solver == "owlqn" && q.objective_history.size() >= 2);
  CHECK(std::fabs(q.coefficients[0] - 2.0) < 0.1 && std::fabs(q.coefficients[1] + 3.0) < 0.1);
  for (size_t i = 1; i < q.objective_history.size(); ++i)
    CHECK(q.objective_history[i] <= q.objective_history[i - 1] + 1e-12);
  std::vector<double> constant = f;
  constant[4] = constant[3] * constant[3] / constant[1];  // zero label variance
  WlsResult k = wls_fit(constant.data(), 2, true, 0.0, 0.0, true, true, 0, 10, 1e-6, false);
  CHECK(k.status == WLS_CONST_LABEL || k.status == WLS_ZERO_LABEL);
  std::vector<double> empty(f.size(), 0.0);
  CHECK(wls_fit(empty.data(), 2, true, 0, 0, true, true, 0, 10, 1e-6, false).status == WLS_EMPTY);
}

static void test_csv(const char* root) {
  const char* txt = "3,25.5\r4,\r5,30\r16,95.25";
  CsvOptions o;
  o.infer_schema = true;
  CsvTable t = csv_scan(txt, std::strlen(txt), o, {}, {});
  CHECK(t.nrows == 4 && t.cols.size() == 2);
  CHECK(t.cols[0].type == T_INT && t.cols[1].type == T_DOUBLE);
  CHECK(t.cols[1].valid[1] == 0 && close(t.cols[1].dvals[3], 95.25, 0));
  CHECK(csv_merge_types(T_INT, T_DOUBLE) == T_DOUBLE && csv_merge_types(T_BOOL, T_INT) == T_STRING);
  CHECK(csv_infer_field("12", 2) == T_INT && csv_infer_field("1.5", 3) == T_DOUBLE);
  CsvTable e = csv_scan("", 0, o, {}, {});
  CHECK(e.nrows == 0);
  // the reference datasets (CR-only terminators, no trailing terminator)
  for (const char* name : {"dataset-small.csv", "dataset-abstract.csv", "dataset-full.csv"}) {
    std::ifstream in(std::string(root) + "/data/" + name, std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string s = ss.str();
    CsvTable d = csv_scan(s.data(), s.size(), o, {}, {});
    CHECK(d.cols.size() == 2 && d.cols[0].type == T_INT && d.cols[1].type == T_DOUBLE);
    CHECK(d.nrows == (std::strcmp(name, "dataset-small.csv") == 0 ? 27 : std::strcmp(name, "dataset-abstract.csv") == 0 ? 40 : 1040));
  }
  // quotes, escapes, header, forced types, garbage
  const char* q = "a,b\n\"x,1\",2\n\"y\\\"z\",3\nbad,row,extra\n";
  CsvOptions oh;
  oh.header = true;
  oh.infer_schema = true;
  CsvTable h = csv_scan(q, std::strlen(q), oh, {}, {});
  CHECK(h.nrows == 3 && h.cols[0].name == "a" && h.cols[0].svals[0] == "x,1");
  CsvTable forced = csv_scan(q, std::strlen(q), oh, {T_DOUBLE, T_INT}, {"u", "v"});
  CHECK(forced.cols[1].type == T_INT);
}

int main(int argc, char** argv) {
  const char* root = argc > 1 ? argv[1] : ".";
  test_cholesky();
  test_wls();
  test_csv(root);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("host selftest ok\n");
  return 0;
}
