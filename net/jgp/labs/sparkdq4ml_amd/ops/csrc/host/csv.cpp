// Host CSV scanner — contract in csv.h.
#include "csv.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>

namespace dq4ml {

namespace {

struct Field {
  std::string text;
  bool is_null;
};

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

bool parse_int64(const char* s, size_t n, int64_t& out) {
  if (n == 0) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
    if (n == 1) return false;
  }
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX;
  for (; i < n; ++i) {
    if (!is_digit(s[i])) return false;
    const uint64_t d = s[i] - '0';
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

bool all_digits_signed(const char* s, size_t n) {
  size_t i = (n && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
  if (i >= n) return false;
  for (; i < n; ++i)
    if (!is_digit(s[i])) return false;
  return true;
}

// java.lang.Double.parseDouble subset: decimal / scientific, NaN, [+-]Infinity, optional d/f suffix
bool parse_double(const char* s, size_t n, double& out) {
  if (n == 0) return false;
  std::string t(s, n);
  if (t == "NaN") { out = std::numeric_limits<double>::quiet_NaN(); return true; }
  if (t == "Infinity" || t == "+Infinity") { out = std::numeric_limits<double>::infinity(); return true; }
  if (t == "-Infinity") { out = -std::numeric_limits<double>::infinity(); return true; }
  char last = t.back();
  if (last == 'd' || last == 'D' || last == 'f' || last == 'F') t.pop_back();
  if (t.empty()) return false;
  // reject hex / inf / nan spellings strtod would take
  bool seen_digit = false;
  for (char c : t) {
    if (is_digit(c)) seen_digit = true;
    else if (!(c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E')) return false;
  }
  if (!seen_digit) return false;
  errno = 0;
  char* end = nullptr;
  out = std::strtod(t.c_str(), &end);
  return end == t.c_str() + t.size();
}

bool parse_bool(const char* s, size_t n, int64_t& out) {
  if (n == 4 && strncasecmp(s, "true", 4) == 0) { out = 1; return true; }
  if (n == 5 && strncasecmp(s, "false", 5) == 0) { out = 0; return true; }
  return false;
}

// split one record into fields (univocity-like: quotes, escapes, separator)
void split_record(const char* p, size_t n, const CsvOptions& o, std::vector<Field>& out) {
  out.clear();
  std::string cur;
  bool in_quotes = false, was_quoted = false;
  for (size_t i = 0; i < n; ++i) {
    char c = p[i];
    if (in_quotes) {
      if (c == o.escape && o.escape != o.quote && i + 1 < n && (p[i + 1] == o.quote || p[i + 1] == o.escape)) {
        cur.push_back(p[++i]);
      } else if (c == o.quote) {
        if (i + 1 < n && p[i + 1] == o.quote) {
          cur.push_back(o.quote);
          ++i;
        } else {
          in_quotes = false;
        }
      } else {
        cur.push_back(c);
      }
    } else if (c == o.sep) {
      out.push_back({cur, false});
      out.back().is_null = !was_quoted && cur == o.null_value;
      cur.clear();
      was_quoted = false;
    } else if (c == o.quote && cur.empty() && !was_quoted) {
      in_quotes = true;
      was_quoted = true;
    } else if (c == o.escape && o.escape != o.quote && i + 1 < n && p[i + 1] == o.quote) {
      cur.push_back(p[++i]);
    } else {
      cur.push_back(c);
    }
  }
  out.push_back({cur, !was_quoted && cur == o.null_value});
  for (auto& f : out) {
    if (f.is_null) continue;
    if (o.ignore_leading_ws) {
      size_t a = 0;
      while (a < f.text.size() && (f.text[a] == ' ' || f.text[a] == '\t')) ++a;
      f.text.erase(0, a);
    }
    if (o.ignore_trailing_ws) {
      while (!f.text.empty() && (f.text.back() == ' ' || f.text.back() == '\t')) f.text.pop_back();
    }
  }
}

// days from 1970-01-01 of the proleptic Gregorian y-m-d (linear in d: day 31 of a 30-day month
// is the 1st of the next, java.util.Date's leniency)
int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

// k digits at s[i..]: their value, i advanced; false when fewer than lo or more than hi digits
bool take_digits(const char* s, size_t n, size_t& i, int lo, int hi, int64_t& v) {
  int k = 0;
  v = 0;
  while (i < n && is_digit(s[i]) && k < hi) {
    v = v * 10 + (s[i] - '0');
    ++i;
    ++k;
  }
  return k >= lo && !(i < n && is_digit(s[i]));
}

}  // namespace

bool csv_parse_timestamp(const char* s, size_t n, int64_t& us) {
  size_t i = 0;
  int64_t y, mo, d;
  if (!take_digits(s, n, i, 4, 4, y) || i >= n || s[i] != '-') return false;
  const size_t m0 = ++i;
  if (!take_digits(s, n, i, 1, 2, mo) || i >= n || s[i] != '-') return false;
  const bool mo2 = i - m0 == 2;
  const size_t d0 = ++i;
  if (!take_digits(s, n, i, 1, 2, d)) return false;
  const bool d2 = i - d0 == 2;
  if (y < 1600 || mo < 1 || mo > 12 || d < 1 || d > 31) return false;
  int64_t secs = 0, ms = 0, off = 0;
  if (i == n) {  // Date.valueOf
  } else if (s[i] == ' ' || s[i] == 'T') {
    const bool iso = s[i] == 'T';
    const int lo = iso ? 2 : 1;
    int64_t h, mi, se;
    ++i;
    if (iso && !(mo2 && d2)) return false;
    if (!take_digits(s, n, i, lo, 2, h) || i >= n || s[i] != ':') return false;
    ++i;
    if (!take_digits(s, n, i, lo, 2, mi) || i >= n || s[i] != ':') return false;
    ++i;
    if (!take_digits(s, n, i, lo, 2, se)) return false;
    if (i < n && s[i] == '.') {  // 1..9 fraction digits, millisecond precision kept
      ++i;
      int k = 0;
      while (i < n && is_digit(s[i]) && k < 9) {
        if (k < 3) ms = ms * 10 + (s[i] - '0');
        ++i;
        ++k;
      }
      if (k == 0 || (i < n && is_digit(s[i]))) return false;
      for (; k < 3; ++k) ms *= 10;
    }
    if (iso) {
      static const int dim[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
      const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
      if (d > dim[mo - 1] + (mo == 2 && leap) || h > 23 || mi > 59 || se > 59) return false;
      if (i < n && s[i] == 'Z') {
        ++i;
      } else if (i < n && (s[i] == '+' || s[i] == '-')) {
        const int64_t sg = s[i] == '-' ? -1 : 1;
        int64_t oh, om;
        ++i;
        if (!take_digits(s, n, i, 2, 2, oh) || i >= n || s[i] != ':') return false;
        ++i;
        if (!take_digits(s, n, i, 2, 2, om) || oh > 23 || om > 59) return false;
        off = sg * (oh * 3600 + om * 60);
      }
    }
    if (i != n) return false;
    secs = h * 3600 + mi * 60 + se - off;
  } else {
    return false;
  }
  us = ((days_from_civil(y, mo, d) * 86400 + secs) * 1000 + ms) * 1000;
  return true;
}

void csv_field_text(const char* p, size_t n, const CsvOptions& o, std::string& out) {
  std::vector<Field> f;
  split_record(p, n, o, f);
  out.swap(f[0].text);
}

int csv_infer_field(const char* s, size_t n) {
  if (n == 0) return T_NULL;
  int64_t iv;
  if (parse_int64(s, n, iv)) return (iv >= INT32_MIN && iv <= INT32_MAX) ? T_INT : T_LONG;
  if (all_digits_signed(s, n)) return T_DECIMAL;  // integer too long for long
  double dv;
  if (parse_double(s, n, dv)) return T_DOUBLE;
  if (csv_parse_timestamp(s, n, iv)) return T_TIMESTAMP;
  if (parse_bool(s, n, iv)) return T_BOOL;
  return T_STRING;
}

int csv_merge_types(int a, int b) {
  if (a == b) return a;
  if (a == T_NULL) return b;
  if (b == T_NULL) return a;
  const bool an = a >= T_INT && a <= T_DOUBLE, bn = b >= T_INT && b <= T_DOUBLE;
  if (an && bn) return a > b ? a : b;  // int < long < decimal < double
  return T_STRING;
}

CsvTable csv_scan(const char* data, size_t len, const CsvOptions& opt, const std::vector<int>& user_types,
                  const std::vector<std::string>& user_names) {
  // 1) records: split on \n, \r, \r\n; skip empty lines and comments
  std::vector<std::pair<size_t, size_t>> recs;
  size_t i = 0;
  while (i < len) {
    size_t s = i;
    while (i < len && data[i] != '\n' && data[i] != '\r') ++i;
    size_t e = i;
    if (i < len) {
      if (data[i] == '\r' && i + 1 < len && data[i + 1] == '\n') i += 2;
      else i += 1;
    }
    if (e == s) continue;
    if (opt.comment && data[s] == opt.comment) continue;
    recs.emplace_back(s, e - s);
  }
  CsvTable t;
  std::vector<Field> fields;
  size_t first = 0;
  std::vector<std::string> names;
  if (!recs.empty()) {
    split_record(data + recs[0].first, recs[0].second, opt, fields);
    for (size_t c = 0; c < fields.size(); ++c) {
      if (opt.header) names.push_back(fields[c].is_null ? ("_c" + std::to_string(c)) : fields[c].text);
      else names.push_back("_c" + std::to_string(c));
    }
    if (opt.header) first = 1;
  }
  if (!user_names.empty()) names = user_names;
  const size_t ncols = user_types.empty() ? names.size() : user_types.size();
  while (names.size() < ncols) names.push_back("_c" + std::to_string(names.size()));

  // 2) tokenize all records once
  const size_t nrec = recs.size() - first;
  std::vector<std::vector<Field>> rows(nrec);
  for (size_t r = 0; r < nrec; ++r) {
    split_record(data + recs[first + r].first, recs[first + r].second, opt, rows[r]);
  }
  // 3) schema
  std::vector<int> types(ncols, T_STRING);
  if (!user_types.empty()) {
    types = user_types;
  } else if (opt.infer_schema) {
    std::fill(types.begin(), types.end(), T_NULL);
    for (auto& row : rows) {
      for (size_t c = 0; c < ncols && c < row.size(); ++c) {
        if (row[c].is_null) continue;
        types[c] = csv_merge_types(types[c], csv_infer_field(row[c].text.data(), row[c].text.size()));
      }
    }
    for (auto& ty : types)
      if (ty == T_NULL) ty = T_STRING;
  }
  // 4) convert
  t.nrows = static_cast<int64_t>(nrec);
  t.cols.resize(ncols);
  for (size_t c = 0; c < ncols; ++c) {
    auto& col = t.cols[c];
    col.name = names[c];
    col.type = types[c];
    col.valid.assign(nrec, 0);
    if (col.type == T_STRING) col.svals.assign(nrec, std::string());
    else if (col.type == T_DOUBLE || col.type == T_DECIMAL) col.dvals.assign(nrec, 0.0);
    else col.ivals.assign(nrec, 0);
  }
  for (size_t r = 0; r < nrec; ++r) {
    const auto& row = rows[r];
    bool malformed = false;
    for (size_t c = 0; c < ncols; ++c) {
      auto& col = t.cols[c];
      if (c >= row.size() || row[c].is_null) continue;
      const std::string& s = row[c].text;
      bool ok = true;
      switch (col.type) {
        case T_INT: {
          int64_t v;
          ok = parse_int64(s.data(), s.size(), v) && v >= INT32_MIN && v <= INT32_MAX;
          if (ok) col.ivals[r] = v;
          break;
        }
        case T_LONG: {
          int64_t v;
          ok = parse_int64(s.data(), s.size(), v);
          if (ok) col.ivals[r] = v;
          break;
        }
        case T_BOOL: {
          int64_t v;
          ok = parse_bool(s.data(), s.size(), v);
          if (ok) col.ivals[r] = v;
          break;
        }
        case T_TIMESTAMP: {
          int64_t v;
          ok = csv_parse_timestamp(s.data(), s.size(), v);
          if (ok) col.ivals[r] = v;
          break;
        }
        case T_DECIMAL:
        case T_DOUBLE: {
          double v;
          ok = parse_double(s.data(), s.size(), v);
          if (ok) col.dvals[r] = v;
          break;
        }
        default:
          col.svals[r] = s;
      }
      if (!ok) {
        malformed = true;
        break;
      }
      col.valid[r] = 1;
    }
    if (malformed) {
      for (auto& col : t.cols) col.valid[r] = 0;
    }
  }
  return t;
}

}  // namespace dq4ml
