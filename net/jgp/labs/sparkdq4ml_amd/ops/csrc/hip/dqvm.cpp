// Whole-stage code generation for the DQ path (the HIP analogue of Spark's Janino whole-stage
// codegen that runs the lab's UDF + filter chain, DataQuality4MachineLearningApp.java:68-90).
//
// ops/dqvm.py lowers a chain of Project/Filter plan nodes (DQ rule UDF bodies, casts, the
// ``WHERE price_no_min > 0`` clean-ups, null checks) to ONE straight-line HIP kernel — one row
// per thread, every column read once, selection vector and derived columns written once — and
// this file compiles it for gfx950 with hipRTC and launches it on the caller's stream.
#include "dqvm.h"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace dq4ml {

namespace {

struct Compiled {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};

std::mutex g_mu;
std::unordered_map<std::string, int64_t> g_by_src;
std::vector<Compiled> g_mods;

#define RTC_CHECK(expr)                                                                             \
  do {                                                                                              \
    hiprtcResult _r = (expr);                                                                       \
    if (_r != HIPRTC_SUCCESS) throw std::runtime_error(std::string("hipRTC: ") + hiprtcGetErrorString(_r)); \
  } while (0)

}  // namespace

// The cache lookup and insert hold the lock; the compile itself does not, so a compile on one
// thread (the process's hipRTC warm-up, dqvm.prewarm) never blocks another thread's launches.
int64_t rtc_compile(const std::string& src, const std::string& entry, std::string* log) {
  const std::string key = entry + "\n" + src;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_by_src.find(key);
    if (it != g_by_src.end()) return it->second;
  }
  hiprtcProgram prog;
  RTC_CHECK(hiprtcCreateProgram(&prog, src.c_str(), "dq_fused.hip", 0, nullptr, nullptr));
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string lg(ls, '\0');
  if (ls) hiprtcGetProgramLog(prog, &lg[0]);
  if (log) *log = lg;
  if (rc != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hipRTC compile failed: " + lg + "\n--- source ---\n" + src);
  }
  size_t cs = 0;
  RTC_CHECK(hiprtcGetCodeSize(prog, &cs));
  std::vector<char> code(cs);
  RTC_CHECK(hiprtcGetCode(prog, code.data()));
  hiprtcDestroyProgram(&prog);
  Compiled c;
  DQ_HIP_CHECK(hipModuleLoadData(&c.mod, code.data()));
  DQ_HIP_CHECK(hipModuleGetFunction(&c.fn, c.mod, entry.c_str()));
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_by_src.find(key);
  if (it != g_by_src.end()) {  // another thread compiled the same source meanwhile: keep theirs
    hipModuleUnload(c.mod);
    return it->second;
  }
  g_mods.push_back(c);
  const int64_t h = (int64_t)g_mods.size() - 1;
  g_by_src[key] = h;
  return h;
}

void* rtc_function(int64_t handle) {
  std::lock_guard<std::mutex> g(g_mu);
  if (handle < 0 || handle >= (int64_t)g_mods.size()) throw std::invalid_argument("rtc_function: bad handle");
  return reinterpret_cast<void*>(g_mods[handle].fn);
}

void rtc_launch(int64_t handle, int grid, int block, void* const* ptrs_dev, int64_t n, hipStream_t st) {
  hipFunction_t fn;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (handle < 0 || handle >= (int64_t)g_mods.size()) throw std::invalid_argument("rtc_launch: bad handle");
    fn = g_mods[handle].fn;
  }
  long long nn = (long long)n;
  void* p = (void*)ptrs_dev;
  void* args[] = {&p, &nn};
  DQ_HIP_CHECK(hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, st, args, nullptr));
}

void rtc_launch_args(int64_t handle, int grid, int block, const int64_t* ptrs_host, int nptr, int64_t n,
                     hipStream_t st) {
  if (nptr < 1 || nptr * 8 + 8 > 4096) throw std::invalid_argument("rtc_launch_args: pointer slots do not fit the kernarg segment");
  hipFunction_t fn;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (handle < 0 || handle >= (int64_t)g_mods.size()) throw std::invalid_argument("rtc_launch_args: bad handle");
    fn = g_mods[handle].fn;
  }
  long long nn = (long long)n;
  // the struct argument's bytes are read from ptrs_host when the launch is enqueued
  void* args[] = {const_cast<int64_t*>(ptrs_host), &nn};
  DQ_HIP_CHECK(hipModuleLaunchKernel(fn, grid, 1, 1, block, 1, 1, 0, st, args, nullptr));
}

}  // namespace dq4ml
