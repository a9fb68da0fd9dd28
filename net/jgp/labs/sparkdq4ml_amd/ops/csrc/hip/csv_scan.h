// K1/K2 device CSV scan (see csv_scan.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csv_parse_dev.h"

namespace dq4ml {

// type lattice codes (same as the host scanner, csrc/host/csv.h)
enum CsvTypeCode : int { CT_NULL = 0, CT_INT = 1, CT_LONG = 2, CT_DECIMAL = 3, CT_DOUBLE = 4, CT_BOOL = 5, CT_STRING = 6,
                         CT_TIMESTAMP = 7 };

int64_t csv_count_blocks(int64_t n);
// Two calls: ends == null -> counts = csv_count_blocks(n)+1 int64 (exclusive per-block offsets,
// total at [nb]); then ends (total entries) -> the ordered line-end offsets, reusing counts.
// ends are int32 when csv_ends_i32(n) (inputs below 2 GiB), else int64
bool csv_ends_i32(int64_t n);
// facts (pass 2 only, or null): csv_count_blocks(n) x 4 int32, per block [separator bytes (sep),
// CR ends, lone-LF ends, CR LF ends]
void csv_line_ends(const uint8_t* buf, int64_t n, int64_t* counts, void* ends, hipStream_t st, int sep = -1,
                   int32_t* facts = nullptr);
// stats (10 + 2 ncols int64) initialised for csv_parse with the ends pass's nb x 4 facts summed in
// (separators at 5 + 2 ncols, the shortest-line slot at 1 << 30, terminator kinds at 7 + 2 ncols ..)
void csv_stats_init(const int32_t* facts, int64_t nb, int64_t* stats, int ncols, hipStream_t st);
// dcols: [2 * ncols] int64 — ncols device pointers to nlines values each, then ncols storage
// kinds (0 f64, 1 int32, 2 int64, 3 bool/uint8, 4 string span: int64 (fs << 25) | (raw << 24) | len
// with fs the field's first byte in buf (csv_field_span), 5 timestamp: int64 microseconds);
// valid: [ncols, nlines]; stats (zeroed):
// [slow flag, empty lines, null fields per column (ncols), class masks per column (ncols; bit 8:
// a field whose value or class needs the host -- harmless when the column is a string),
// lines with a field outside the numeric fast path, lines with a field that is not even a quoted
// fast-path number ("12.5"), the longest line [4 + 2 ncols] and, when the caller made room and set
// it high, the shortest [6 + 2 ncols] (terminator to terminator)]
// o: dialect (csv_parse_dev.h).  o.strict: the kinds are the user schema's types and a field that
// does not convert makes its record malformed (all fields null)
void csv_parse(const uint8_t* buf, int64_t n, const void* ends, int64_t nlines, int ncols, const dq4ml_csv::CsvOpts& o,
               const int64_t* dcols, uint8_t* valid, uint8_t* keep, int64_t* stats, hipStream_t st);
// string column (kind-4 spans into buf[0, nbuf)) == lit[0, L): out 1 / 0; a raw (quoted /
// escaped) field compares its unescaped text (quote / escape bytes, -1: none)
void csv_span_eq(const uint8_t* buf, int64_t nbuf, const int64_t* spans, int64_t n, const uint8_t* lit, int L,
                 int quote, int escape, uint8_t* out, hipStream_t st);

}  // namespace dq4ml
