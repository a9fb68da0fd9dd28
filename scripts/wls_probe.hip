// Phase timing of the device WLS solve (wls_small.hip built with DQ4ML_WLS_PROBE).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<ops/csrc/hip> scripts/wls_probe.hip -o /tmp/wls_probe
#define DQ4ML_WLS_PROBE 1
#include "wls_small.hip"

#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  const int nf = argc > 1 ? atoi(argv[1]) : 32;
  const int n = 4096;
  std::mt19937_64 g(1);
  std::normal_distribution<double> N;
  std::vector<double> X((size_t)n * nf), y(n);
  for (auto& v : X) v = N(g);
  for (int i = 0; i < n; ++i) {
    double s = 0.5;
    for (int j = 0; j < nf; ++j) s += (j - nf / 2) * 0.1 * X[(size_t)i * nf + j];
    y[i] = s + 0.01 * N(g);
  }
  const size_t P = 5 + 2 * nf + (size_t)nf * (nf + 1) / 2;
  std::vector<double> flat(P, 0.0);
  for (int i = 0; i < n; ++i) {
    const double* x = &X[(size_t)i * nf];
    flat[0] += 1; flat[1] += 1; flat[2] += 1; flat[3] += y[i]; flat[4] += y[i] * y[i];
    for (int j = 0; j < nf; ++j) {
      flat[5 + j] += x[j];
      flat[5 + nf + j] += x[j] * y[i];
      for (int k = 0; k <= j; ++k) flat[5 + 2 * nf + k + (size_t)j * (j + 1) / 2] += x[k] * x[j];
    }
  }
  double *dflat, *dout;
  long long* dprobe;
  hipMalloc(&dflat, P * 8);
  hipMalloc(&dout, (nf + 16) * 8);
  hipMalloc(&dprobe, 16 * 8);
  hipMemcpy(dflat, flat.data(), P * 8, hipMemcpyHostToDevice);
  hipMemcpyToSymbol(HIP_SYMBOL(dq4ml::g_wls_probe), &dprobe, sizeof(dprobe));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double acc[8] = {0};
  const int reps = 50;
  float ms_tot = 0;
  for (int r = 0; r < reps + 5; ++r) {
    hipEventRecord(e0, 0);
    dq4ml::wls_small(dflat, nf, 1, 0.0, 0.0, 1, 1, dout, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long pr[5];
    hipMemcpy(pr, dprobe, sizeof(pr), hipMemcpyDeviceToHost);
    if (r >= 5) {
      ms_tot += ms;
      for (int i = 1; i < 5; ++i) acc[i] += (double)(pr[i] - pr[i - 1]);
    }
  }
  std::vector<double> out(nf + 7);
  hipMemcpy(out.data(), dout, (nf + 7) * 8, hipMemcpyDeviceToHost);
  printf("nf=%d status=%g coef[0]=%.6f coef[last]=%.6f intercept=%.6f\n", nf, out[nf + 1], out[0], out[nf - 1], out[nf]);
  printf("event ms/launch %.2f us\n", ms_tot / reps * 1e3);
  const char* names[5] = {"", "load+std", "assemble", "eliminate", "backsub"};
  for (int i = 1; i < 5; ++i) printf("  %-10s %10.0f memtime ticks\n", names[i], acc[i] / reps);
  return 0;
}
