// Host check of the device field converters (csv_parse_dev.h): csv_swar_field16, csv_field_r16 and csv_field_r8 must accept
// exactly what the byte-walking fast path csv_field_fast accepts and return the same bits, over
// every field shape the cutter hands it (1..16 bytes: signs, dots, digits, junk).  Compiled with
// g++ (the header is plain C++ once the HIP qualifiers are defined away).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#define __device__
#define __forceinline__ inline
static inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
#include "csv_parse_dev.h"

using namespace dq4ml_csv;

static bool fast(const std::string& f, double& dv, long long& lv, int& ty) {
  std::string s = f + ",";
  int pos = 0;
  const int end = (int)f.size();
  return csv_field_fast((const unsigned char*)s.data(), 0, pos, end, (unsigned char)',', dv, lv, ty);
}

static std::mt19937 junk(7);

// the right-aligned converter: the field at a varying offset in a dword-aligned stage, junk bytes
// before it (they must be masked off) and after it
static bool r16(const std::string& f, double& dv, long long& lv, int& ty) {
  alignas(16) unsigned char buf[64];
  const char pool[] = "0123456789.-+,\r\n x";
  for (auto& c : buf) c = (unsigned char)pool[junk() % (sizeof(pool) - 1)];
  const int off = 16 + (int)(junk() % 16);
  memcpy(buf + off, f.data(), f.size());
  return csv_field_r16(buf, off + (int)f.size(), (int)f.size(), dv, lv, ty);
}

static bool r8(const std::string& f, double& dv, long long& lv, int& ty) {
  alignas(16) unsigned char buf[64];
  const char pool[] = "0123456789.-+,\r\n x";
  for (auto& c : buf) c = (unsigned char)pool[junk() % (sizeof(pool) - 1)];
  const int off = 16 + (int)(junk() % 16);
  memcpy(buf + off, f.data(), f.size());
  return csv_field_r8(buf, off + (int)f.size(), (int)f.size(), dv, lv, ty);
}

// the cutter's sign-stripped 8-byte path (csv_num_r8s + the caller's sign handling)
static bool r8s(const std::string& f, double& dv, long long& lv, int& ty, bool& fits) {
  alignas(16) unsigned char buf[64];
  const char pool[] = "0123456789.-+,\r\n x";
  for (auto& c : buf) c = (unsigned char)pool[junk() % (sizeof(pool) - 1)];
  const int off = 16 + (int)(junk() % 16);
  memcpy(buf + off, f.data(), f.size());
  const int len = (int)f.size();
  const unsigned char c0 = len ? buf[off] : 0;
  const int sg = (c0 == '-' || c0 == '+') ? 1 : 0;
  fits = len - sg <= 8;
  if (!fits) return false;
  unsigned m;
  int fr;
  bool dot;
  const bool ok = csv_num_r8s(buf, off + len, len - sg, m, fr, dot);
  const double v = dot ? csv_div_pow10((double)m, fr) : (double)m;
  dv = ok ? (c0 == '-' ? -v : v) : 0.0;
  lv = ok && !dot ? (c0 == '-' ? -(long long)m : (long long)m) : 0;
  ty = len == 0 ? C_NULL : (dot ? C_DOUBLE : C_INT);
  return len == 0 || ok;
}

// csv_num_r8q (the 32-bit-SWAR form of the same path), same caller
static bool r8q(const std::string& f, double& dv, long long& lv, int& ty, bool& fits) {
  alignas(16) unsigned char buf[64];
  const char pool[] = "0123456789.-+,\r\n x";
  for (auto& c : buf) c = (unsigned char)pool[junk() % (sizeof(pool) - 1)];
  const int off = 16 + (int)(junk() % 16);
  memcpy(buf + off, f.data(), f.size());
  const int len = (int)f.size();
  const unsigned char c0 = len ? buf[off] : 0;
  const int sg = (c0 == '-' || c0 == '+') ? 1 : 0;
  fits = len - sg <= 8;
  if (!fits) return false;
  unsigned m;
  int fr;
  bool dot;
  const bool ok = csv_num_r8q(buf, off + len, len - sg, m, fr, dot);
  const double v = dot ? csv_div_pow10((double)m, fr) : (double)m;
  dv = ok ? (c0 == '-' ? -v : v) : 0.0;
  lv = ok && !dot ? (c0 == '-' ? -(long long)m : (long long)m) : 0;
  ty = len == 0 ? C_NULL : (dot ? C_DOUBLE : C_INT);
  return len == 0 || ok;
}

// csv_swar_field directly, with junk bytes after the field in the same 64-bit word (as the
// per-line scan kernel hands it the field at the start of the line's remaining bytes)
static bool swar8(const std::string& f, double& dv, long long& lv, int& ty) {
  const char pool[] = "0123456789.-+,\r\n x";
  unsigned char b[8];
  for (auto& c : b) c = (unsigned char)pool[junk() % (sizeof(pool) - 1)];
  memcpy(b, f.data(), f.size());
  unsigned long long x;
  memcpy(&x, b, 8);
  return csv_swar_field(x, (int)f.size(), dv, lv, ty);
}

static bool swar(const std::string& f, double& dv, long long& lv, int& ty) {
  unsigned char buf[48] = {0};
  const int off = 5;  // an unaligned start, like a field inside an LDS stage
  memcpy(buf + off, f.data(), f.size());
  unsigned long long lo, hi;
  csv_line16(buf, off, lo, hi);
  return csv_swar_field16(lo, hi, (int)f.size(), dv, lv, ty);
}

int main() {
  std::mt19937_64 rng(12345);
  const char alpha[] = "0123456789.-+e,x ";
  long checked = 0, accepted = 0;
  auto check = [&](const std::string& f) {
    double d1 = 0, d2 = 0;
    long long l1 = 0, l2 = 0;
    int t1 = -1, t2 = -1;
    const bool a = fast(f, d1, l1, t1), b = swar(f, d2, l2, t2);
    ++checked;
    if (a != b || (a && (t1 != t2 || l1 != l2 || memcmp(&d1, &d2, sizeof d1) != 0))) {
      printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | swar16 %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1,
             l1, b, t2, d2, l2);
      return false;
    }
    double d3 = 0;
    long long l3 = 0;
    int t3 = -1;
    const bool c = r16(f, d3, l3, t3);
    if (a != c || (a && (t1 != t3 || l1 != l3 || memcmp(&d1, &d3, sizeof d1) != 0))) {
      printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | r16 %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1, l1,
             c, t3, d3, l3);
      return false;
    }
    {
      double d5 = 0;
      long long l5 = 0;
      int t5 = -1;
      bool fits = false;
      const bool g = r8s(f, d5, l5, t5, fits);
      if (fits && (a != g || (a && (t1 != t5 || l1 != l5 || memcmp(&d1, &d5, sizeof d1) != 0)))) {
        printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | r8s %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1,
               l1, g, t5, d5, l5);
        return false;
      }
    }
    {
      double d7 = 0;
      long long l7 = 0;
      int t7 = -1;
      bool fits = false;
      const bool g = r8q(f, d7, l7, t7, fits);
      if (fits && (a != g || (a && (t1 != t7 || l1 != l7 || memcmp(&d1, &d7, sizeof d1) != 0)))) {
        printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | r8q %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1,
               l1, g, t7, d7, l7);
        return false;
      }
    }
    if (f.size() <= 8) {
      double d6 = 0;
      long long l6 = 0;
      int t6 = -1;
      const bool h = swar8(f, d6, l6, t6);
      if (a != h || (a && (t1 != t6 || l1 != l6 || memcmp(&d1, &d6, sizeof d1) != 0))) {
        printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | swar8 %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1,
               l1, h, t6, d6, l6);
        return false;
      }
    }
    if (f.size() <= 8) {
      double d4 = 0;
      long long l4 = 0;
      int t4 = -1;
      const bool e = r8(f, d4, l4, t4);
      if (a != e || (a && (t1 != t4 || l1 != l4 || memcmp(&d1, &d4, sizeof d1) != 0))) {
        printf("MISMATCH field '%s': fast %d ty %d %.17g %lld | r8 %d ty %d %.17g %lld\n", f.c_str(), a, t1, d1, l1,
               e, t4, d4, l4);
        return false;
      }
    }
    accepted += a;
    return true;
  };
  // numeric shapes: [sign] digits [. digits], 1..16 bytes
  for (int it = 0; it < 3000000; ++it) {
    std::string f;
    const int sg = (int)(rng() % 4);
    if (sg == 1) f += '-';
    if (sg == 2) f += '+';
    const int nd = 1 + (int)(rng() % 12);
    const int dp = (rng() % 3) ? (int)(rng() % (nd + 1)) : -1;
    for (int k = 0; k < nd; ++k) {
      if (k == dp) f += '.';
      f += (char)('0' + rng() % 10);
    }
    if (dp == nd) f += '.';
    if (f.size() > 16) continue;
    if (!check(f)) return 1;
  }
  if (!check("")) return 1;  // the empty field: null
  // arbitrary bytes from a small alphabet (junk, double dots, stray signs)
  for (int it = 0; it < 2000000; ++it) {
    const int len = 1 + (int)(rng() % 16);
    std::string f;
    for (int k = 0; k < len; ++k) f += alpha[rng() % (sizeof(alpha) - 1)];
    if (f.find(',') != std::string::npos) continue;  // the cutter never hands over a separator
    if (!check(f)) return 1;
  }
  // csv_num_r8q_w against csv_num_r8s_w on raw frames: every shift, every field length 0..8,
  // bytes from the field alphabet
  {
    const char pool[] = "0123456789.-+,\r x/";
    for (int it = 0; it < 4000000; ++it) {
      unsigned w[3];
      for (auto& x : w) {
        x = 0;
        for (int k = 0; k < 4; ++k) x |= (unsigned)(unsigned char)pool[rng() % (sizeof(pool) - 1)] << (8 * k);
      }
      const int sft = (int)(rng() % 4), fl = (int)(rng() % 9);
      unsigned m1 = 0, m2 = 0;
      int f1 = 0, f2 = 0;
      bool o1, o2, d1 = false, d2 = false;
      o1 = csv_num_r8s_w(w[0], w[1], w[2], sft, fl, m1, f1, d1);
      o2 = csv_num_r8q_w(w[0], w[1], w[2], sft, fl, m2, f2, d2);
      if (o1 != o2 || (o1 && (m1 != m2 || f1 != f2 || d1 != d2))) {
        printf("MISMATCH frame %08x %08x %08x s %d fl %d: r8s %d %u %d %d | r8q %d %u %d %d\n", w[0], w[1], w[2], sft, fl,
               o1, m1, f1, d1, o2, m2, f2, d2);
        return 1;
      }
    }
  }
  printf("swar16 ok: %ld fields, %ld accepted\n", checked, accepted);
  return 0;
}
