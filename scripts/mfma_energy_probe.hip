// Config-5 shape / tiling energy probe: the SYRK K-loop's LDS-fed MFMA work in
// three forms -- 32x32x64 on 128 x 64 wave tiles (the kernel's, 8 waves per CU), 16x16x128 on the
// same tiles, and 32x32x64 on 128 x 128 wave tiles (4 waves per CU: a third fewer LDS reads) --
// each run for ~2 s while a host thread samples the board's hwmon power and sclk, so every form
// gets ms, PF/s, W, pJ per MAC and MHz on the same box.
//
// (Round 4's question, kept:) does the block-scaled fp8 MFMA hold a higher clock as 16x16x128 than as
// 32x32x64 (MI355X_MICROARCH.md 'DVFS give-back' item 7 measured 1.12-1.15x for bf16 16x16x32 vs
// 32x32x16 on random data)?  Two loops of EQUAL work per iteration, fed from LDS like the SYRK's
// 128 x 64 wave tile (gram_wide.hip): per 128 rows of K, 12 fragments of 32 B per lane (24
// ds_read_b128) and 128 x 64 x 128 MACs -- 16 x v_mfma_scale_f32_32x32x64_f8f6f4 or
// 32 x v_mfma_scale_f32_16x16x128_f8f6f4.  8 waves (2 per SIMD) per CU, random finite e4m3 bytes
// in LDS, the LDS offsets walk so nothing is hoisted.  Prints PF/s per variant, interleaved rounds.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/mfma_shape_probe scripts/mfma_shape_probe.hip
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include <glob.h>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

constexpr int kLds = 64 * 1024;

__device__ __forceinline__ i32x8 frag(const unsigned char* lds, int off, int lane) {
  const u32x4 lo = *reinterpret_cast<const u32x4*>(lds + off + lane * 16);
  const u32x4 hi = *reinterpret_cast<const u32x4*>(lds + off + 1024 + lane * 16);
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

template <int SHAPE>  // 32: 32x32x64, 16: 16x16x128
__global__ __launch_bounds__(SHAPE == 128 ? 256 : 512, 1) void shape_loop(float* out, int iters, unsigned seed) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  for (int i = threadIdx.x; i < kLds / 4; i += blockDim.x) {
    unsigned v = (seed + i) * 2654435761u;
    v ^= v >> 13;
    v *= 0x5bd1e995u;
    reinterpret_cast<unsigned*>(lds)[i] = v & 0x77777777u;  // finite e4m3 bytes, random signs
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if constexpr (SHAPE == 32) {
    f32x16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[x][0] = acc[x][1] = f32x16{};
    for (int it = 0; it < iters; ++it) {
      const int base = ((it * 7 + wave) & 7) * 4096;
#pragma unroll
      for (int st = 0; st < 2; ++st) {  // two 64-row stages
        i32x8 a[4], b[2];
#pragma unroll
        for (int x = 0; x < 4; ++x) a[x] = frag(lds, (base + st * 2048 + x * 6144) & (kLds - 2048), lane);
#pragma unroll
        for (int y = 0; y < 2; ++y) b[y] = frag(lds, (base + 30720 + st * 2048 + y * 4096) & (kLds - 2048), lane);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[x], b[y], acc[x][y], 0, 0, 0, 127, 0, 127);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc[x][0][r] + acc[x][1][r];
    if (s == 12345.678f) out[threadIdx.x] = s;
  } else if constexpr (SHAPE == 128) {  // 128 x 128 wave tiles, 4 waves per block
    f32x16 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = f32x16{};
    for (int it = 0; it < iters; ++it) {
      const int base = ((it * 7 + wave) & 7) * 4096;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        i32x8 a[4], b[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) a[x] = frag(lds, (base + st * 2048 + x * 6144) & (kLds - 2048), lane);
#pragma unroll
        for (int y = 0; y < 4; ++y) b[y] = frag(lds, (base + 30720 + st * 2048 + y * 4096) & (kLds - 2048), lane);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[x], b[y], acc[x][y], 0, 0, 0, 127, 0, 127);
      }
    }
    float s = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[x][y][r];
    if (s == 12345.678f) out[threadIdx.x] = s;
  } else {
    f32x4 acc[8][4];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{};
    for (int it = 0; it < iters; ++it) {
      const int base = ((it * 7 + wave) & 7) * 4096;
      i32x8 a[8], b[4];  // one 128-row K step: 8 A frags (16 features each), 4 B frags
#pragma unroll
      for (int x = 0; x < 8; ++x) a[x] = frag(lds, (base + x * 3072) & (kLds - 2048), lane);
#pragma unroll
      for (int y = 0; y < 4; ++y) b[y] = frag(lds, (base + 30720 + y * 2048) & (kLds - 2048), lane);
#pragma unroll
      for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[x], b[y], acc[x][y], 0, 0, 0, 127, 0, 127);
    }
    float s = 0.f;
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[x][y][r];
    if (s == 12345.678f) out[threadIdx.x] = s;
  }
}

// ---- board power / clock from hwmon (sampled by a host thread while a kernel runs) -----------
static std::string hwmon_dir() {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) == hipSuccess) {
    for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
    glob_t g;
    std::string pat = std::string("/sys/bus/pci/devices/") + bus + "/hwmon/hwmon*";
    if (glob(pat.c_str(), 0, nullptr, &g) == 0 && g.gl_pathc > 0) {
      std::string d = g.gl_pathv[0];
      globfree(&g);
      return d;
    }
  }
  return "";
}

static double read_num(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return -1.0;
  double v = -1.0;
  if (fscanf(f, "%lf", &v) != 1) v = -1.0;
  fclose(f);
  return v;
}

struct Sampler {
  std::string dir;
  std::atomic<bool> run{false};
  std::vector<double> watts, mhz;
  std::thread th;
  void start() {
    watts.clear(), mhz.clear();
    run = true;
    th = std::thread([this] {
      while (run) {
        double p = read_num(dir + "/power1_average");
        if (p < 0) p = read_num(dir + "/power1_input");
        const double f = read_num(dir + "/freq1_input");
        if (p >= 0) watts.push_back(p * 1e-6);
        if (f >= 0) mhz.push_back(f * 1e-6);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    });
  }
  void stop() {
    run = false;
    th.join();
  }
  static double mean_mid(const std::vector<double>& v) {  // the middle 80 % of the samples
    if (v.empty()) return -1.0;
    const size_t a = v.size() / 10, b = v.size() - v.size() / 10;
    double s = 0.0;
    for (size_t i = a; i < b; ++i) s += v[i];
    return b > a ? s / (double)(b - a) : v[0];
  }
};

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  float* out;
  CHECK(hipMalloc(&out, 4096));
  const int iters = argc > 1 ? atoi(argv[1]) : 3000000;  // ~1.6 s per launch
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  Sampler smp;
  smp.dir = hwmon_dir();
  printf("{\"hwmon\": \"%s\", \"cus\": %d}\n", smp.dir.c_str(), cus);
  // one iteration = 128 x 64 x 128 MACs per 64-thread slice of the block (every form: same MACs per block)
  const double macs = 128.0 * 64 * 128 * 8.0 * cus * iters;
  hipLaunchKernelGGL(shape_loop<32>, dim3(cus), dim3(512), 0, 0, out, 200, 1u);
  hipLaunchKernelGGL(shape_loop<16>, dim3(cus), dim3(512), 0, 0, out, 200, 1u);
  hipLaunchKernelGGL(shape_loop<128>, dim3(cus), dim3(256), 0, 0, out, 200, 1u);
  CHECK(hipDeviceSynchronize());
  for (int rep = 0; rep < reps; ++rep) {
    for (int shape : {32, 16, 128}) {
      std::this_thread::sleep_for(std::chrono::milliseconds(500));  // settle between forms
      smp.start();
      CHECK(hipEventRecord(e0));
      if (shape == 32) hipLaunchKernelGGL(shape_loop<32>, dim3(cus), dim3(512), 0, 0, out, iters, 7u + rep);
      else if (shape == 16) hipLaunchKernelGGL(shape_loop<16>, dim3(cus), dim3(512), 0, 0, out, iters, 7u + rep);
      else hipLaunchKernelGGL(shape_loop<128>, dim3(cus), dim3(256), 0, 0, out, iters, 7u + rep);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      smp.stop();
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double w = Sampler::mean_mid(smp.watts), f = Sampler::mean_mid(smp.mhz);
      const char* name = shape == 32 ? "32x32x64, 128x64 wave tiles, 8 waves"
                         : shape == 16 ? "16x16x128, 128x64 wave tiles, 8 waves"
                                       : "32x32x64, 128x128 wave tiles, 4 waves";
      printf("{\"form\": \"%s\", \"rep\": %d, \"ms\": %.2f, \"pflops\": %.3f, \"board_w\": %.1f, \"pj_per_mac\": %.4f, "
             "\"sclk_mhz\": %.0f, \"samples\": %zu}\n",
             name, rep, ms, 2.0 * macs / (ms * 1e-3) / 1e15, w, w > 0 ? w * (ms * 1e-3) / macs * 1e12 : -1.0, f,
             smp.watts.size());
      fflush(stdout);
    }
  }
  CHECK(hipFree(out));
  return 0;
}
