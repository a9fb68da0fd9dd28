// pybind11 bindings of the gfx950 kernel module (_dq4ml_hip).  Every entry point takes raw device
// pointers (ints) plus the HIP stream handle of the calling torch stream; buffers are allocated by
// the python side (ops/device.py) from torch's caching allocator, so there is no hipMalloc in any
// launch path (graph-capturable) and kernels run on the same stream as the surrounding torch work.
#include <map>
#include <utility>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "common.h"
#include "csv_scan.h"
#include "dqvm.h"
#include "gram.h"
#include "gram_wide.h"
#include "gram_syrk.h"
#include "wls_small.h"
#include "wls_large.h"
#include "rowops.h"
#include "lsq.h"

namespace py = pybind11;
using namespace dq4ml;

template <typename T>
static T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}

// Reusable event rings for stream ordering on the asynchronous fit's issue path: torch's
// wait_stream / Event create a Python Event object (and a HIP event) per call.  One ring per
// (device, key): key 0 serves stream_wait (the wait is enqueued right after the record and keeps
// the record it saw, whatever later records do); event_record keys its ring by the recording
// stream, so a ring event is only ever re-recorded LATER on that same stream.
static hipEvent_t ring_event(uintptr_t key) {
  constexpr int kRing = 64;
  struct Ring {
    hipEvent_t ev[kRing];
    int next = 0;
  };
  static std::map<std::pair<int, uintptr_t>, Ring*> rings;
  int dev = 0;
  DQ_HIP_CHECK(hipGetDevice(&dev));
  Ring*& r = rings[{dev, key}];
  if (!r) {
    r = new Ring();
    for (auto& e : r->ev) DQ_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipEvent_t e = r->ev[r->next];
  r->next = (r->next + 1) % kRing;
  return e;
}

PYBIND11_MODULE(_dq4ml_hip, m) {
  m.doc() = "dq4ml gfx950 kernels: MFMA Gram, fused DQ VM, compaction, pack, predict/metrics, CSV scan";

  // dst waits for everything enqueued on src so far (stream.wait_stream without a torch Event)
  m.def("stream_wait", [](uintptr_t dst, uintptr_t src) {
    hipEvent_t e = ring_event(0);
    DQ_HIP_CHECK(hipEventRecord(e, as_stream(src)));
    DQ_HIP_CHECK(hipStreamWaitEvent(as_stream(dst), e, 0));
  });
  // a ring event recorded on st: re-recorded only on st, 64 records later, which only moves it
  // later on the same stream -- waiting on it still orders after the original record
  m.def("event_record", [](uintptr_t st) {
    hipEvent_t e = ring_event(st);
    DQ_HIP_CHECK(hipEventRecord(e, as_stream(st)));
    return reinterpret_cast<uintptr_t>(e);
  });
  m.def("stream_wait_event", [](uintptr_t dst, uintptr_t ev) {
    DQ_HIP_CHECK(hipStreamWaitEvent(as_stream(dst), reinterpret_cast<hipEvent_t>(ev), 0));
  });

  m.def("standin", [](int blocks, int usec, uintptr_t st) { standin(blocks, usec, as_stream(st)); });
  // a stream whose kernels only dispatch to the CUs set in mask (32 CUs per word, logical CU order)
  m.def("stream_create_cumask", [](const std::vector<uint32_t>& mask) {
    hipStream_t s = nullptr;
    DQ_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    return reinterpret_cast<uintptr_t>(s);
  });
  // drain and destroy a stream this module created (runtime/streams.py releases its CU-masked
  // streams at interpreter exit, before the HIP runtime's own teardown)
  m.def("stream_destroy", [](uintptr_t st) {
    DQ_HIP_CHECK(hipStreamSynchronize(as_stream(st)));
    DQ_HIP_CHECK(hipStreamDestroy(as_stream(st)));
  });
  m.def("device_info", []() {
    int dev = 0;
    DQ_HIP_CHECK(hipGetDevice(&dev));
    hipDeviceProp_t p;
    DQ_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    py::dict d;
    d["name"] = std::string(p.name);
    d["gcnArchName"] = std::string(p.gcnArchName);
    d["multiProcessorCount"] = p.multiProcessorCount;
    d["totalGlobalMem"] = (uint64_t)p.totalGlobalMem;
    d["sharedMemPerBlock"] = (uint64_t)p.sharedMemPerBlock;
    return d;
  });

  // ---- Gram (K5) ---------------------------------------------------------------------------
  m.def("gram_partial_stride", &gram_partial_stride);
  m.def("gram_default_blocks", &gram_default_blocks);
  m.def("gram_plan_blocks", &gram_plan_blocks);
  m.def("gram_tall",
        [](int mode, uintptr_t X, int64_t ld, int d, int64_t n, int xdt, uintptr_t y, int ydt, uintptr_t w, int wdt,
           uintptr_t sel, int xmode, uintptr_t partials, int blocks, uintptr_t out, uintptr_t stream, int tiled,
           bool reduce, uintptr_t xshift) {
          GramArgs a{};
          a.tiled = tiled;
          a.xshift = P<const float>(xshift);
          a.X = P<const void>(X);
          a.ld = ld;
          a.d = d;
          a.n = n;
          a.xdt = xdt;
          a.y = P<const void>(y);
          a.ydt = ydt;
          a.w = P<const void>(w);
          a.wdt = wdt;
          a.sel = P<const uint8_t>(sel);
          a.partials = P<double>(partials);
          gram_tall(mode, a, xmode, blocks, P<double>(out), as_stream(stream), reduce);
        });
  m.def("gram_stream_cols",
        [](int mode, uintptr_t srcs, int d, int64_t n, int xdt, uintptr_t y, int ydt, uintptr_t w, int wdt,
           uintptr_t sel, uintptr_t partials, int blocks, uintptr_t out, uintptr_t stream, uintptr_t xshift) {
          GramArgs a{};
          a.srcs = P<const int64_t>(srcs);
          a.xshift = P<const float>(xshift);
          a.d = d;
          a.n = n;
          a.xdt = xdt;
          a.y = P<const void>(y);
          a.ydt = ydt;
          a.w = P<const void>(w);
          a.wdt = wdt;
          a.sel = P<const uint8_t>(sel);
          a.partials = P<double>(partials);
          gram_stream(mode, a, (w || sel || xshift) ? 1 : 0, blocks, P<double>(out), as_stream(stream), true);
        });
  m.def("gram_stream_blocks", &gram_stream_blocks);
  m.def("gram_stream_rtc",
        [](int64_t handle, int mode, uintptr_t srcs, int d, int64_t n, uintptr_t rawtab, uintptr_t partials, int blocks,
           int64_t lds, uintptr_t out, uintptr_t stream, uintptr_t xshift) {
          GramArgs a{};
          a.srcs = P<const int64_t>(srcs);
          a.xshift = P<const float>(xshift);
          a.d = d;
          a.n = n;
          a.xdt = DT_F32;
          a.ydt = DT_F64;
          a.rawtab = P<const int64_t>(rawtab);
          a.partials = P<double>(partials);
          gram_stream_rtc(rtc_function(handle), mode, a, blocks, (size_t)lds, P<double>(out), as_stream(stream));
        });
  m.def("gram_skinny_cols",
        [](const std::vector<uintptr_t>& cols, const std::vector<int>& dts, int64_t n, uintptr_t y, int ydt,
           uintptr_t w, int wdt, uintptr_t sel, uintptr_t partials, int blocks, uintptr_t out, uintptr_t stream) {
          const int d = (int)cols.size();
          if (d < 1 || d > 8 || (int)dts.size() != d) throw std::invalid_argument("gram_skinny_cols: 1 <= d <= 8");
          GramArgs a{};
          for (int f = 0; f < d; ++f) {
            a.colp[f] = P<const void>(cols[f]);
            a.coldt[f] = dts[f];
          }
          a.cols = d;
          a.d = d;
          a.n = n;
          a.xdt = DT_F64;
          a.y = P<const void>(y);
          a.ydt = ydt;
          a.w = P<const void>(w);
          a.wdt = wdt;
          a.sel = P<const uint8_t>(sel);
          a.partials = P<double>(partials);
          gram_tall(GRAM_F64, a, w ? 2 : (sel ? 1 : 0), blocks, P<double>(out), as_stream(stream), true);
        });
  m.def("gram_reduce", [](int mode, uintptr_t partials, int blocks, int d, uintptr_t out, uintptr_t stream) {
    gram_reduce(mode, P<const double>(partials), blocks, d, P<double>(out), as_stream(stream));
  });
  m.def("gram_window_fold", [](uintptr_t part, int64_t rows, int gw, uintptr_t flat, uintptr_t stream) {
    gram_window_fold(P<const double>(part), rows, gw, P<double>(flat), as_stream(stream));
  });
  m.def("stats_unshift", [](uintptr_t flat, uintptr_t shift, int d, uintptr_t stream) {
    stats_unshift(P<double>(flat), P<const float>(shift), d, as_stream(stream));
  });
  m.def("gram_cols_blocks", &gram_cols_blocks);
  m.def("gram_cols", [](uintptr_t srcs, int sdt, int d, int64_t n, uintptr_t y, int ydt, uintptr_t sel,
                        uintptr_t partials, int blocks, uintptr_t out, uintptr_t stream, uintptr_t xshift) {
    GramArgs a{};
    a.xshift = P<const float>(xshift);
    a.d = d;
    a.n = n;
    a.xdt = DT_F32;
    a.y = P<const void>(y);
    a.ydt = ydt;
    a.sel = P<const uint8_t>(sel);
    a.partials = P<double>(partials);
    gram_cols(a, P<const PackSrcG>(srcs), sdt, blocks, P<double>(out), as_stream(stream));
  });
  m.def("tiled_elems", &tiled_elems);
  m.def("tile_bf16", [](uintptr_t X, int xdt, int64_t ld, int d, int64_t n, uintptr_t out, uintptr_t stream,
                        uintptr_t shift) {
    tile_bf16(P<const void>(X), xdt, ld, d, n, P<void>(out), as_stream(stream), P<const float>(shift));
  });
  m.def("wls_small", [](uintptr_t flat, int nf, bool fit_intercept, double reg, double enet, bool std_f, bool std_l,
                        uintptr_t out, uintptr_t stream) {
    wls_small(P<const double>(flat), nf, fit_intercept, reg, enet, std_f, std_l, P<double>(out), as_stream(stream));
  });
  m.def("wls_assemble", [](uintptr_t flat, int nf, bool fit_intercept, double reg, double enet, bool std_f,
                           bool std_l, uintptr_t A, uintptr_t b, uintptr_t minv, uintptr_t aStd, uintptr_t aBar,
                           uintptr_t lam, uintptr_t o, uintptr_t stream) {
    wls_assemble(P<const double>(flat), nf, fit_intercept, reg, enet, std_f, std_l, P<double>(A), P<double>(b),
                 P<double>(minv), P<double>(aStd), P<double>(aBar), P<double>(lam), P<double>(o), as_stream(stream));
  });
  m.def("wls_pcg_init", [](uintptr_t b, uintptr_t minv, int k, double rtol, uintptr_t o, uintptr_t r, uintptr_t p,
                           uintptr_t stream) {
    wls_pcg_init(P<const double>(b), P<const double>(minv), k, rtol, P<double>(o), P<double>(r), P<double>(p),
                 as_stream(stream));
  });
  m.def("wls_pcg_chunk", [](uintptr_t A, uintptr_t b, uintptr_t minv, uintptr_t aStd, int k, int nf, int iters,
                            uintptr_t o, uintptr_t r, uintptr_t p, uintptr_t Ap, uintptr_t stream) {
    wls_pcg_chunk(P<const double>(A), P<const double>(b), P<const double>(minv), P<const double>(aStd), k, nf, iters,
                  P<double>(o), P<double>(r), P<double>(p), P<double>(Ap), as_stream(stream));
  });
  m.attr("PCG_STATE_WORDS") = (int)PCG_STATE_WORDS;
  m.attr("PCG_CONV") = (int)PCG_CONV;
  m.attr("PCG_BAD") = (int)PCG_BAD;
  m.attr("PCG_OK") = (int)PCG_OK;
  m.attr("PCG_ITERS") = (int)PCG_ITERS;
  m.attr("PCG_STATUS") = (int)PCG_STATUS;
  m.attr("PCG_HEAD") = (int)PCG_HEAD;
  m.attr("PCG_WSUM") = (int)PCG_WSUM;
  m.attr("PCG_BSTD") = (int)PCG_BSTD;
  m.def("wls_qn_small", [](uintptr_t flat, int nf, bool fit_intercept, double reg, double enet, bool std_f,
                           bool std_l, int max_iter, double tol, int hist_cap, uintptr_t out, uintptr_t stream) {
    wls_qn_small(P<const double>(flat), nf, fit_intercept, reg, enet, std_f, std_l, max_iter, tol, hist_cap,
                 P<double>(out), as_stream(stream));
  });
  m.attr("WLS_QN_MAX_K") = kWlsQnMaxK;
  m.attr("WLS_QN_GRID_MAX_K") = kWlsQnGridMaxK;
  m.def("wls_qn_grid_work", &wls_qn_grid_work);
  m.def("wls_qn_grid_blocks", &wls_qn_grid_blocks);
  m.def("wls_qn_grid", [](uintptr_t flat, int nf, bool fit_intercept, double reg, double enet, bool std_f, bool std_l,
                          int max_iter, double tol, int hist_cap, uintptr_t work, int blocks, uintptr_t out,
                          uintptr_t stream) {
    wls_qn_grid(P<const double>(flat), nf, fit_intercept, reg, enet, std_f, std_l, max_iter, tol, hist_cap,
                P<double>(work), blocks, P<double>(out), as_stream(stream));
  });
  m.attr("WLS_SMALL_MAX_FEATURES") = kWlsSmallMaxFeatures;
  m.def("wide_tiled_bytes", &wide_tiled_bytes);
  m.attr("WIDE_ZERO_BYTES") = kWideZeroBytes;
  m.def("gram_wide_partials", &gram_wide_partials);
  m.def("pack_wide", [](int eb, uintptr_t srcs_dev, int d, int64_t n, int nt, uintptr_t sel, uintptr_t inv_scale,
                        uintptr_t out, uintptr_t stream, uintptr_t shift) {
    pack_wide(eb, P<const PackSrcW>(srcs_dev), d, n, nt, P<const uint8_t>(sel), P<const float>(inv_scale), P<void>(out),
              as_stream(stream), P<const float>(shift));
  });
  m.def("wide_label_part_doubles", &wide_label_part_doubles);
  m.def("wide_unshift_label", [](uintptr_t out, int d, uintptr_t aux, uintptr_t stream) {
    wide_unshift_label(P<double>(out), d, P<const double>(aux), as_stream(stream));
  });
  m.def("wide_label_aug", [](int eb, uintptr_t y, int ydt, int64_t n, uintptr_t sel, uintptr_t part, uintptr_t aux,
                             uintptr_t out, uintptr_t stream) {
    wide_label_aug(eb, P<const void>(y), ydt, n, P<const uint8_t>(sel), P<double>(part), P<double>(aux), P<void>(out),
                   as_stream(stream));
  });
  m.def("wide_mask_rows", [](int eb, uintptr_t in, uintptr_t out, int d, int64_t n, uintptr_t sel, uintptr_t stream) {
    wide_mask_rows(eb, P<const void>(in), P<void>(out), d, n, P<const uint8_t>(sel), as_stream(stream));
  });
  m.def("feature_amax", [](uintptr_t srcs_dev, int d, int64_t n, uintptr_t sel, uintptr_t amax, uintptr_t stream,
                           uintptr_t shift) {
    feature_amax(P<const PackSrcW>(srcs_dev), d, n, P<const uint8_t>(sel), P<float>(amax), as_stream(stream),
                 P<const float>(shift));
  });
  auto wide_args = [](uintptr_t X, uintptr_t Xaug, uintptr_t zeros, int nt, int npanels, int d, int64_t nsup,
                      int splitk, uintptr_t part, uintptr_t aug_scale, uintptr_t tile_base = 0) {
    WideArgs a{};
    a.X = P<const unsigned char>(X);
    a.Xaug = P<const unsigned char>(Xaug);
    a.zeros = P<const unsigned char>(zeros);
    a.NT = nt;
    a.npanels = npanels;
    a.d = d;
    a.nsup = nsup;
    a.splitk = splitk;
    a.part = P<float>(part);
    a.aug_scale = P<const double>(aug_scale);
    a.tile_base = P<const int>(tile_base);
    return a;
  };
  // aug_scale: device f64[3] scales of the augmentation columns [1, y_hi, y_lo] (read by the fold)
  m.def("gram_wide", [wide_args](int eb, uintptr_t X, uintptr_t Xaug, uintptr_t zeros, int nt, int npanels, int d,
                                 int64_t nsup, int splitk, uintptr_t pairs, uintptr_t part, uintptr_t aug_scale,
                                 uintptr_t scales, uintptr_t out, uintptr_t stream, int ring, bool fold) {
    WideArgs a = wide_args(X, Xaug, zeros, nt, npanels, d, nsup, splitk, part, aug_scale);
    gram_wide(eb, a, P<const int>(pairs), P<const float>(scales), P<double>(out), as_stream(stream), ring, fold);
  });
  m.def("gram_wide_queue", [wide_args](int eb, uintptr_t X, uintptr_t Xaug, uintptr_t zeros, int nt, int npanels,
                                       int d, int64_t nsup, int h, uintptr_t pairs, uintptr_t part, uintptr_t aug_scale,
                                       uintptr_t scales, uintptr_t out, uintptr_t heads, int grid, uintptr_t stream,
                                       bool fold) {
    WideArgs a = wide_args(X, Xaug, zeros, nt, npanels, d, nsup, 8 * h, part, aug_scale);
    gram_wide_queue(eb, a, P<const int>(pairs), P<const float>(scales), P<double>(out), P<int>(heads), h, grid,
                    as_stream(stream), fold);
  });
  m.def("gram_wide_gang", [wide_args](int eb, uintptr_t X, uintptr_t Xaug, uintptr_t zeros, int nt, int npanels,
                                      int d, int64_t nsup, int S, uintptr_t table, uintptr_t pairs, int units,
                                      uintptr_t tile_base, uintptr_t part, uintptr_t aug_scale, uintptr_t scales,
                                      uintptr_t out, int grid, uintptr_t stream, bool fold, uintptr_t bar) {
    WideArgs a = wide_args(X, Xaug, zeros, nt, npanels, d, nsup, 8 * S, part, aug_scale, tile_base);
    a.pairs = P<const int>(pairs);
    gram_wide_gang(eb, a, P<const int>(table), units, P<const float>(scales), P<double>(out), S, grid,
                   as_stream(stream), fold, P<int>(bar));
  });
  m.def("gram_wide_fold", [wide_args](int npanels, int d, int splitk, uintptr_t part, uintptr_t aug_scale,
                                      uintptr_t tile_base, uintptr_t scales, uintptr_t out, uintptr_t out32, int J0,
                                      int J1, uintptr_t stream) {
    WideArgs a = wide_args(0, 0, 0, 0, npanels, d, 0, splitk, part, aug_scale, tile_base);
    gram_wide_fold(a, P<const float>(scales), P<double>(out), P<float>(out32), J0, J1, as_stream(stream));
  });

  m.def("syrk_panels", &syrk_panels);
  m.def("syrk_partials", &syrk_partials);
  m.def("syrk_stages", &syrk_stages);
  m.def("gram_syrk", [](int compute_f64, uintptr_t X, int64_t ld, int d, int64_t n, int xdt, uintptr_t y, uintptr_t w,
                        uintptr_t pairs, int npair, int splitk, uintptr_t part, uintptr_t out, uintptr_t stream) {
    SyrkArgs s{};
    s.X = P<const void>(X);
    s.ld = ld;
    s.d = d;
    s.n = n;
    s.xdt = xdt;
    s.y = P<const double>(y);
    s.w = P<const double>(w);
    s.pairs = P<const int>(pairs);
    s.npair = npair;
    s.splitk = splitk;
    s.part = P<double>(part);
    gram_syrk(compute_f64, s, P<double>(out), as_stream(stream));
  });

  // ---- compaction (K3) -----------------------------------------------------------------------
  m.def("compact_blocks", &compact_blocks);
  m.def("compact_count_scan", [](uintptr_t sel, int64_t n, uintptr_t counts, uintptr_t stream) {
    compact_count_scan(P<const uint8_t>(sel), n, P<int64_t>(counts), as_stream(stream));
  });
  m.def("compact_write", [](uintptr_t sel, int64_t n, uintptr_t offsets, int64_t limit, uintptr_t out,
                            uintptr_t stream) {
    compact_write(P<const uint8_t>(sel), n, P<const int64_t>(offsets), limit, P<int64_t>(out), as_stream(stream));
  });

  // ---- pack (K4) -----------------------------------------------------------------------------
  m.def("pack_columns", [](uintptr_t srcs_dev, int d, int64_t n, uintptr_t out, int odt, int64_t ld, uintptr_t sel,
                           uintptr_t stream) {
    pack_columns(P<const PackSrc>(srcs_dev), d, n, P<void>(out), odt, ld, P<const uint8_t>(sel), as_stream(stream));
  });
  m.def("pack_src_bytes", []() { return (int)sizeof(PackSrc); });

  // ---- predict / metrics (K7/K8) ---------------------------------------------------------------
  m.def("pack_tiled", [](uintptr_t srcs_dev, int d, int64_t n, uintptr_t sel, uintptr_t out, uintptr_t stream,
                         uintptr_t shift) {
    pack_tiled(P<const PackSrc>(srcs_dev), d, n, P<const uint8_t>(sel), P<void>(out), as_stream(stream),
               P<const float>(shift));
  });
  m.def("predict", [](uintptr_t X, int xdt, int64_t ld, int d, int64_t n, uintptr_t coef, double b, uintptr_t out,
                      uintptr_t stream, int tiled) {
    predict(P<const void>(X), xdt, ld, d, n, P<const double>(coef), b, P<double>(out), as_stream(stream), tiled);
  });
  m.def("metrics_blocks", &metrics_blocks);
  m.def("huber_pass", [](uintptr_t X, int xdt, int64_t ld, int d, int64_t n, int tiled, uintptr_t y, int ydt, uintptr_t w,
                         int wdt, uintptr_t sel, uintptr_t ceff, double icpt, double sigma, double eps, uintptr_t mult,
                         uintptr_t partials, uintptr_t out, uintptr_t stream) {
    huber_pass(P<const void>(X), xdt, ld, d, n, tiled, P<const void>(y), ydt, P<const void>(w), wdt,
               P<const uint8_t>(sel), P<const double>(ceff), icpt, sigma, eps, P<double>(mult), P<double>(partials),
               P<double>(out), as_stream(stream));
  });
  m.def("huber_pass_dev", [](uintptr_t X, int xdt, int64_t ld, int d, int64_t n, int tiled, uintptr_t y, int ydt,
                             uintptr_t w, int wdt, uintptr_t sel, uintptr_t trial, uintptr_t act, double eps,
                             uintptr_t scale, uintptr_t shift, uintptr_t mult, uintptr_t partials, uintptr_t out,
                             uintptr_t stream) {
    huber_pass_dev(P<const void>(X), xdt, ld, d, n, tiled, P<const void>(y), ydt, P<const void>(w), wdt,
                   P<const uint8_t>(sel), P<const double>(trial), P<const int>(act), eps, P<const double>(scale),
                   P<const double>(shift), P<double>(mult), P<double>(partials), P<double>(out), as_stream(stream));
  });
  m.def("huber_partials", &huber_partials);
  m.def("huber_qn_work", &huber_qn_work);
  m.def("huber_qn_out", &huber_qn_out);
  m.attr("HUBER_EVAL") = kHuberEval;
  m.attr("HUBER_DONE") = kHuberDone;
  m.def("huber_qn_init", [](int d, bool fit_icpt, int max_iter, double tol, int hist_cap, uintptr_t sx, uintptr_t lam,
                            uintptr_t scale, uintptr_t shift, uintptr_t work, uintptr_t trial, uintptr_t out,
                            uintptr_t stream) {
    huber_qn_init(d, fit_icpt, max_iter, tol, hist_cap, P<const double>(sx), P<const double>(lam),
                  P<const double>(scale), P<const double>(shift), P<double>(work), P<double>(trial), P<double>(out),
                  as_stream(stream));
  });
  m.def("huber_qn_ctl", [](int d, bool fit_icpt, int max_iter, double tol, int hist_cap, uintptr_t sx, uintptr_t lam,
                           uintptr_t scale, uintptr_t shift, uintptr_t work, uintptr_t trial, uintptr_t red,
                           uintptr_t out, uintptr_t stream) {
    huber_qn_ctl(d, fit_icpt, max_iter, tol, hist_cap, P<const double>(sx), P<const double>(lam),
                 P<const double>(scale), P<const double>(shift), P<double>(work), P<double>(trial),
                 P<const double>(red), P<double>(out), as_stream(stream));
  });
  // ---- K9: squared-loss l-bfgs evaluation passes ----------------------------------------------
  auto lsqx = [](uintptr_t X, int layout, int xdt, int64_t ld, int d, int64_t n) {
    LsqX x{};
    x.X = P<const void>(X);
    x.layout = layout;
    x.xdt = xdt;
    x.ld = ld;
    x.d = d;
    x.n = n;
    return x;
  };
  m.def("lsq_margin_blocks", [lsqx](uintptr_t X, int layout, int xdt, int64_t ld, int d, int64_t n) {
    return lsq_margin_blocks(lsqx(X, layout, xdt, ld, d, n));
  });
  m.def("lsq_part_doubles", [lsqx](uintptr_t X, int layout, int xdt, int64_t ld, int d, int64_t n, int mode) {
    return lsq_part_doubles(lsqx(X, layout, xdt, ld, d, n), mode);
  });
  m.def("lsq_margin", [lsqx](uintptr_t X, int layout, int xdt, int64_t ld, int d, int64_t n, uintptr_t cf,
                             uintptr_t offset, double inv_ystd, uintptr_t y, uintptr_t w, uintptr_t v, uintptr_t lpart,
                             uintptr_t stream) {
    lsq_margin(lsqx(X, layout, xdt, ld, d, n), P<const void>(cf), P<const double>(offset), inv_ystd, P<const double>(y),
               P<const double>(w), P<double>(v), P<double>(lpart), as_stream(stream));
  });
  m.def("lsq_columns", [lsqx](uintptr_t X, int layout, int xdt, int64_t ld, int d, int64_t n, int mode, uintptr_t v,
                              uintptr_t lpart, int nl, uintptr_t part, uintptr_t out, uintptr_t stream) {
    lsq_columns(lsqx(X, layout, xdt, ld, d, n), mode, P<const double>(v), P<const double>(lpart), nl, P<double>(part),
                P<double>(out), as_stream(stream));
  });
  m.attr("LSQ_QN_MAX_D") = kLsqQnMaxD;
  m.def("lsq_qn_blocks", &lsq_qn_blocks);
  m.def("lsq_qn_work", &lsq_qn_work);
  m.def("lsq_qn", [lsqx](uintptr_t X, int layout, int d, int64_t n, uintptr_t y, uintptr_t w, uintptr_t scale,
                         uintptr_t shift, uintptr_t head, bool fit_icpt, bool std_f, double reg, double enet,
                         int max_iter, double tol, int hist_cap, uintptr_t work, int blocks, uintptr_t out,
                         uintptr_t stream) {
    lsq_qn(lsqx(X, layout, 2, 0, d, n), P<const double>(y), P<const double>(w), P<const double>(scale),
           P<const double>(shift), P<const double>(head), fit_icpt, std_f, reg, enet, max_iter, tol, hist_cap,
           P<double>(work), blocks, P<double>(out), as_stream(stream));
  });
  m.def("lsq_qn_dp_work", &lsq_qn_dp_work);
  m.def("lsq_qn_dp_red_offset", &lsq_qn_dp_red_offset);
  m.def("lsq_qn_dp_ctl_offset", &lsq_qn_dp_ctl_offset);
  m.def("lsq_qn_dp", [lsqx](int phase, uintptr_t X, int layout, int d, int64_t n, uintptr_t y, uintptr_t w,
                            uintptr_t scale, uintptr_t shift, uintptr_t head, bool fit_icpt, bool std_f, double reg,
                            double enet, int max_iter, double tol, int hist_cap, uintptr_t work, int blocks,
                            uintptr_t out, uintptr_t stream) {
    lsq_qn_dp(phase, lsqx(X, layout, 2, 0, d, n), P<const double>(y), P<const double>(w), P<const double>(scale),
              P<const double>(shift), P<const double>(head), fit_icpt, std_f, reg, enet, max_iter, tol, hist_cap,
              P<double>(work), blocks, P<double>(out), as_stream(stream));
  });
  m.def("regression_metrics",
        [](uintptr_t X, int xdt, int64_t ld, int d, int64_t n, uintptr_t y, int ydt, uintptr_t sel, uintptr_t coef,
           double b, double shift, uintptr_t partials, uintptr_t out, uintptr_t stream, int tiled) {
          regression_metrics(P<const void>(X), xdt, ld, d, n, P<const void>(y), ydt, P<const uint8_t>(sel),
                             P<const double>(coef), b, shift, P<double>(partials), P<double>(out), as_stream(stream),
                             tiled);
        });

  // ---- CSV scan (K1/K2) ------------------------------------------------------------------------
  m.def("csv_count_blocks", &csv_count_blocks);
  m.def("csv_span_eq", [](uintptr_t buf, int64_t nbuf, uintptr_t spans, int64_t n, uintptr_t lit, int L, int quote,
                          int escape, uintptr_t out, uintptr_t stream) {
    csv_span_eq(P<const uint8_t>(buf), nbuf, P<const int64_t>(spans), n, P<const uint8_t>(lit), L, quote, escape,
                P<uint8_t>(out), as_stream(stream));
  });
  m.def("csv_line_ends", [](uintptr_t buf, int64_t n, uintptr_t counts, uintptr_t ends, uintptr_t stream, int sep,
                            uintptr_t facts) {
    csv_line_ends(P<const uint8_t>(buf), n, P<int64_t>(counts), P<void>(ends), as_stream(stream), sep,
                  P<int32_t>(facts));
  });
  m.def("memset_async", [](uintptr_t p, int v, int64_t nbytes, uintptr_t stream) {
    // (an action's zeroed scratch without torch's fill dispatch: one runtime call)
    if (nbytes > 0) DQ_HIP_CHECK(hipMemsetAsync(P<void>(p), v, (size_t)nbytes, as_stream(stream)));
  });
  m.def("csv_stats_init", [](uintptr_t facts, int64_t nb, uintptr_t stats, int ncols, uintptr_t stream) {
    csv_stats_init(P<const int32_t>(facts), nb, P<int64_t>(stats), ncols, as_stream(stream));
  });
  m.def("csv_ends_i32", &csv_ends_i32);
  m.def("csv_parse", [](uintptr_t buf, int64_t n, uintptr_t ends, int64_t nlines, int ncols, int sep, uintptr_t dcols,
                        uintptr_t valid, uintptr_t keep, uintptr_t stats, uintptr_t stream, int quote, int escape,
                        int comment, bool trim_lead, bool trim_trail, const std::string& null_value, bool strict) {
    dq4ml_csv::CsvOpts o{};
    if (null_value.size() > sizeof(o.null_val)) throw std::invalid_argument("csv_parse: nullValue longer than 16 bytes");
    o.sep = (uint8_t)sep;
    o.quote = (uint8_t)quote;
    o.escape = (uint8_t)escape;
    o.comment = (uint8_t)comment;
    o.trim_lead = trim_lead;
    o.trim_trail = trim_trail;
    o.null_len = (uint8_t)null_value.size();
    for (size_t i = 0; i < null_value.size(); ++i) o.null_val[i] = (uint8_t)null_value[i];
    o.strict = strict;
    csv_parse(P<const uint8_t>(buf), n, P<const void>(ends), nlines, ncols, o, P<const int64_t>(dcols),
              P<uint8_t>(valid), P<uint8_t>(keep), P<int64_t>(stats), as_stream(stream));
  }, pybind11::arg("buf"), pybind11::arg("n"), pybind11::arg("ends"), pybind11::arg("nlines"), pybind11::arg("ncols"),
     pybind11::arg("sep"), pybind11::arg("dcols"), pybind11::arg("valid"), pybind11::arg("keep"), pybind11::arg("stats"),
     pybind11::arg("stream"), pybind11::arg("quote") = '"', pybind11::arg("escape") = '\\', pybind11::arg("comment") = 0,
     pybind11::arg("trim_lead") = false, pybind11::arg("trim_trail") = false, pybind11::arg("null_value") = "",
     pybind11::arg("strict") = false);

  // ---- fused DQ chains: hipRTC whole-stage codegen ----------------------------------------------
  m.def("rtc_compile", [](const std::string& src, const std::string& entry) {
    std::string log;
    int64_t h;
    {
      py::gil_scoped_release nogil;  // (seconds for a cold hipRTC: other Python threads keep running)
      h = rtc_compile(src, entry, &log);
    }
    return py::make_tuple(h, log);
  });
  m.def("rtc_launch_args", [](int64_t handle, int grid, int block, py::buffer ptrs, int64_t n, uintptr_t stream) {
    py::buffer_info bi = ptrs.request();  // a contiguous int64 array of the pointer slots
    if (bi.itemsize != 8 || bi.ndim != 1 || (bi.ndim == 1 && bi.strides[0] != 8))
      throw std::invalid_argument("rtc_launch_args: ptrs must be a contiguous 1-d int64 array");
    rtc_launch_args(handle, grid, block, static_cast<const int64_t*>(bi.ptr), (int)bi.size, n, as_stream(stream));
  });
  m.def("rtc_launch", [](int64_t handle, int grid, int block, uintptr_t ptrs_dev, int64_t n, uintptr_t stream) {
    rtc_launch(handle, grid, block, P<void* const>(ptrs_dev), n, as_stream(stream));
  });
}
