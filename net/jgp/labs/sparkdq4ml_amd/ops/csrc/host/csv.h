// Host CSV scanner with Spark 2.4 CSV-source semantics:
//   * line terminators \n, \r and \r\n (Hadoop LineRecordReader, non-multiLine mode); the
//     reference datasets use CR only and have no trailing terminator
//   * separator / quote / escape configurable (defaults , " \), empty field -> null
//   * header=false -> columns _c0.._cN-1 with N taken from the first record
//   * inferSchema -> per-field lattice null < int < long < decimal < double < timestamp < boolean
//     < string, per-column tightest common type (a timestamp merges only with timestamps)
//   * timestamps (csv_parse_timestamp): Spark 2.4's fallback parsers -- java.sql.Date.valueOf
//     ("yyyy-[m]m-[d]d"), java.sql.Timestamp.valueOf ("yyyy-[m]m-[d]d [h]h:[m]m:[s]s[.f...]",
//     lenient field ranges) and xsd:dateTime ("yyyy-MM-ddTHH:mm:ss[.f...][Z|+hh:mm]") -- in UTC,
//     millisecond precision (Date.getTime), years 1600..9999 (Gregorian only)
//   * PERMISSIVE: short rows padded with nulls, extra tokens dropped, a field that fails to parse
//     under the final schema nulls the whole row (Spark's malformed-record handling)
// Used for local (CPU) sessions and for small files; the device scanner (csrc/hip/csv_scan.hip)
// implements the same contract for numeric columns on the MI355X.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dq4ml {

// (T_TIMESTAMP sits between double and boolean in the lattice; its code is 7 so that the older
// codes keep their values)
enum CsvType : int { T_NULL = 0, T_INT = 1, T_LONG = 2, T_DECIMAL = 3, T_DOUBLE = 4, T_BOOL = 5, T_STRING = 6,
                     T_TIMESTAMP = 7 };

struct CsvOptions {
  char sep = ',';
  char quote = '"';
  char escape = '\\';
  bool header = false;
  bool infer_schema = false;
  std::string null_value;  // empty string => empty field is null
  char comment = 0;
  bool ignore_leading_ws = false;
  bool ignore_trailing_ws = false;
};

struct CsvColumn {
  std::string name;
  int type = T_STRING;
  std::vector<int64_t> ivals;     // T_INT / T_LONG / T_BOOL
  std::vector<double> dvals;      // T_DOUBLE / T_DECIMAL
  std::vector<std::string> svals; // T_STRING
  std::vector<uint8_t> valid;     // 1 = not null
};

struct CsvTable {
  int64_t nrows = 0;
  std::vector<CsvColumn> cols;
};

// user_types: optional forced schema (empty => infer or all strings)
CsvTable csv_scan(const char* data, size_t len, const CsvOptions& opt, const std::vector<int>& user_types,
                  const std::vector<std::string>& user_names);

// Text of one field whose bytes [p, p + n) the device scanner cut (csrc/hip/csv_parse_dev.h
// csv_field_span): the first field split_record yields from them, trims applied.
void csv_field_text(const char* p, size_t n, const CsvOptions& o, std::string& out);

// Microseconds since the epoch of a timestamp field (see the contract above); false otherwise.
bool csv_parse_timestamp(const char* s, size_t n, int64_t& us);

// Lattice helpers shared with tests.
int csv_infer_field(const char* s, size_t n);
int csv_merge_types(int a, int b);

}  // namespace dq4ml
