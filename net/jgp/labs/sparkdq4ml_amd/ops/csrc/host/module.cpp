// pybind11 bindings of the host runtime library (_dq4ml_host): normal-equation solvers and the
// CSV scanner.  Device kernels live in the separate gfx950 module (_dq4ml_hip).
#include <cstring>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "csv.h"
#include "solvers.h"
#include "wls.h"

namespace py = pybind11;
using namespace dq4ml;

static std::vector<double> to_vec(const py::array_t<double, py::array::c_style | py::array::forcecast>& a) {
  return std::vector<double>(a.data(), a.data() + a.size());
}

static py::array_t<double> to_np(const std::vector<double>& v) {
  py::array_t<double> a(v.size());
  std::copy(v.begin(), v.end(), a.mutable_data());
  return a;
}

PYBIND11_MODULE(_dq4ml_host, m) {
  m.doc() = "dq4ml host runtime: f64 normal-equation solvers (Breeze-compatible) and CSV scanner";

  py::register_exception<SingularMatrixError>(m, "SingularMatrixError");

  m.def(
      "wls_fit",
      [](py::array_t<double, py::array::c_style | py::array::forcecast> flat, int nf, bool fit_intercept,
         double reg_param, double elastic_net, bool standardize_features, bool standardize_label, int solver_type,
         int max_iter, double tol, bool keep_system) {
        const py::ssize_t need = 5 + 2 * (py::ssize_t)nf + (py::ssize_t)nf * (nf + 1) / 2;
        if (flat.size() != need) throw std::invalid_argument("wls_fit: flat statistics have the wrong length");
        WlsResult r;
        {
          py::gil_scoped_release nogil;
          r = wls_fit(flat.data(), nf, fit_intercept, reg_param, elastic_net, standardize_features,
                      standardize_label, solver_type, max_iter, tol, keep_system);
        }
        py::dict d;
        d["status"] = r.status;
        d["singular_fallback"] = r.singular_fallback;
        d["solver"] = r.solver;
        d["coefficients"] = to_np(r.coefficients);
        d["intercept"] = r.intercept;
        d["objective_history"] = to_np(r.objective_history);
        d["converged_reason"] = r.converged_reason;
        d["ata"] = to_np(r.ata);
        d["a_std"] = to_np(r.a_std);
        d["w_sum"] = r.w_sum;
        return d;
      },
      py::arg("flat"), py::arg("nf"), py::arg("fit_intercept"), py::arg("reg_param"), py::arg("elastic_net"),
      py::arg("standardize_features"), py::arg("standardize_label"), py::arg("solver_type"), py::arg("max_iter"),
      py::arg("tol"), py::arg("keep_system") = true);

  m.def("dspmv", [](int k, py::array_t<double, py::array::c_style | py::array::forcecast> ap,
                    py::array_t<double, py::array::c_style | py::array::forcecast> x) {
    if (ap.size() != (py::ssize_t)k * (k + 1) / 2 || x.size() != k) throw std::invalid_argument("dspmv: bad sizes");
    std::vector<double> y(k);
    dspmv(k, ap.data(), x.data(), y.data());
    return to_np(y);
  });

  m.def("cholesky_solve", [](int k, py::array_t<double, py::array::c_style | py::array::forcecast> ap,
                             py::array_t<double, py::array::c_style | py::array::forcecast> b) {
    if (ap.size() != (py::ssize_t)k * (k + 1) / 2 || b.size() != k) throw std::invalid_argument("cholesky_solve: bad sizes");
    std::vector<double> x;
    {
      py::gil_scoped_release nogil;
      x = cholesky_solve(k, to_vec(ap), to_vec(b));
    }
    return to_np(x);
  });

  m.def("cholesky_inverse", [](int k, py::array_t<double, py::array::c_style | py::array::forcecast> ap) {
    if (ap.size() != (py::ssize_t)k * (k + 1) / 2) throw std::invalid_argument("cholesky_inverse: bad size");
    return to_np(cholesky_inverse(k, to_vec(ap)));
  });

  m.def(
      "quasi_newton",
      [](double bBar, double bbBar, py::array_t<double, py::array::c_style | py::array::forcecast> ab,
         py::array_t<double, py::array::c_style | py::array::forcecast> aa,
         py::array_t<double, py::array::c_style | py::array::forcecast> aBar, bool fit_intercept, int max_iter,
         double tol, py::object l1, int memory) {
        std::vector<double> l1v;
        if (!l1.is_none()) l1v = to_vec(l1.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>());
        const int k = static_cast<int>(ab.size());
        if (aa.size() != (py::ssize_t)k * (k + 1) / 2) throw std::invalid_argument("quasi_newton: aa size");
        QNResult r;
        {
          auto abv = to_vec(ab), aav = to_vec(aa), abar = to_vec(aBar);
          py::gil_scoped_release nogil;
          r = quasi_newton(bBar, bbBar, abv, aav, abar, fit_intercept, max_iter, tol, l1v, memory);
        }
        return py::make_tuple(to_np(r.x), to_np(r.objective_history), r.converged_reason);
      },
      py::arg("bBar"), py::arg("bbBar"), py::arg("ab"), py::arg("aa"), py::arg("aBar"), py::arg("fit_intercept"),
      py::arg("max_iter"), py::arg("tol"), py::arg("l1") = py::none(), py::arg("memory") = 10);

  m.def("csv_infer_field", [](const std::string& s) { return csv_infer_field(s.data(), s.size()); });
  m.def("csv_merge_types", &csv_merge_types);
  m.def("csv_parse_timestamp", [](const std::string& s) -> py::object {
    int64_t us;
    if (!csv_parse_timestamp(s.data(), s.size(), us)) return py::none();
    return py::int_(us);
  });

  // Python strings of a device string column (ops/csvscan.py DeviceStrings), None where not valid:
  // spans are the device scanner's packed (fs << 25) | (raw << 24) | len into data; a raw field
  // (quoted, or holding the escape byte) goes through csv_field_text, the others are their bytes
  // (trimmed when a trim option is set).  Same text and UTF-8 decoding as csv_scan's columns.
  m.def(
      "csv_strings",
      [](py::buffer data, py::array_t<int64_t, py::array::c_style> spans, py::array_t<uint8_t, py::array::c_style> valid,
         std::string quote, std::string escape, bool ilws, bool itws) {
        py::buffer_info bi = data.request();
        const char* base = static_cast<const char*>(bi.ptr);
        const int64_t nb = bi.size * bi.itemsize;
        const int64_t n = spans.size();
        if (valid.size() != n) throw std::invalid_argument("csv_strings: spans / valid length mismatch");
        CsvOptions o;
        o.quote = quote.empty() ? '\0' : quote[0];
        o.escape = escape.empty() ? '\\' : escape[0];
        o.sep = '\0';  // the span holds one field: no separator outside its quotes
        o.ignore_leading_ws = ilws;
        o.ignore_trailing_ws = itws;
        o.null_value = std::string("\xff\xfe", 2);  // never null here: nulls come from valid
        const int64_t* sp = spans.data();
        const uint8_t* vp = valid.data();
        py::list out(n);
        std::string t;
        for (int64_t i = 0; i < n; ++i) {
          if (!vp[i]) {
            Py_INCREF(Py_None);
            PyList_SET_ITEM(out.ptr(), (Py_ssize_t)i, Py_None);
            continue;
          }
          const int64_t fs = sp[i] >> 25, len = sp[i] & 0xFFFFFF;
          if (fs < 0 || fs + len > nb) throw std::out_of_range("csv_strings: span outside the data");
          const char* p = base + fs;
          size_t a = 0, e = (size_t)len;
          if ((sp[i] >> 24) & 1) {
            csv_field_text(p, (size_t)len, o, t);
            p = t.data();
            e = t.size();
          } else {
            if (ilws)
              while (a < e && (p[a] == ' ' || p[a] == '\t')) ++a;
            if (itws)
              while (e > a && (p[e - 1] == ' ' || p[e - 1] == '\t')) --e;
          }
          // ASCII text (the common case): a compact 1-byte string filled by memcpy, no decoder
          const char* q = p + a;
          const size_t m = e - a;
          bool ascii = true;
          for (size_t k = 0; k < m && ascii; ++k) ascii = (unsigned char)q[k] < 0x80;
          PyObject* s;
          if (ascii) {
            s = PyUnicode_New((Py_ssize_t)m, 127);
            if (s) std::memcpy(PyUnicode_DATA(s), q, m);
          } else {
            s = PyUnicode_DecodeUTF8(q, (Py_ssize_t)m, nullptr);
          }
          if (!s) throw py::error_already_set();
          PyList_SET_ITEM(out.ptr(), (Py_ssize_t)i, s);  // steals the reference (PyList_New left the slot NULL)
        }
        return out;
      },
      py::arg("data"), py::arg("spans"), py::arg("valid"), py::arg("quote") = "\"", py::arg("escape") = "\\",
      py::arg("ignore_leading_ws") = false, py::arg("ignore_trailing_ws") = false);

  m.def(
      "csv_scan",
      [](py::bytes data, std::string sep, std::string quote, std::string escape, bool header, bool infer,
         std::string null_value, std::string comment, bool ilws, bool itws, std::vector<int> user_types,
         std::vector<std::string> user_names) {
        std::string buf = data;
        CsvOptions o;
        o.sep = sep.empty() ? ',' : sep[0];
        o.quote = quote.empty() ? '\0' : quote[0];
        o.escape = escape.empty() ? '\\' : escape[0];
        o.header = header;
        o.infer_schema = infer;
        o.null_value = null_value;
        o.comment = comment.empty() ? 0 : comment[0];
        o.ignore_leading_ws = ilws;
        o.ignore_trailing_ws = itws;
        CsvTable t;
        {
          py::gil_scoped_release nogil;
          t = csv_scan(buf.data(), buf.size(), o, user_types, user_names);
        }
        py::list cols;
        for (auto& c : t.cols) {
          py::object vals;
          if (c.type == T_STRING) {
            py::list l;
            for (auto& s : c.svals) l.append(py::str(s));
            vals = l;
          } else if (c.type == T_DOUBLE || c.type == T_DECIMAL) {
            vals = to_np(c.dvals);
          } else {
            py::array_t<int64_t> a(c.ivals.size());
            std::copy(c.ivals.begin(), c.ivals.end(), a.mutable_data());
            vals = a;
          }
          py::array_t<uint8_t> v(c.valid.size());
          std::copy(c.valid.begin(), c.valid.end(), v.mutable_data());
          cols.append(py::make_tuple(c.name, c.type, vals, v));
        }
        return py::make_tuple(t.nrows, cols);
      },
      py::arg("data"), py::arg("sep") = ",", py::arg("quote") = "\"", py::arg("escape") = "\\",
      py::arg("header") = false, py::arg("infer") = false, py::arg("null_value") = "", py::arg("comment") = "",
      py::arg("ignore_leading_ws") = false, py::arg("ignore_trailing_ws") = false,
      py::arg("user_types") = std::vector<int>{}, py::arg("user_names") = std::vector<std::string>{});
}
