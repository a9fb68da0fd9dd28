"""Fused CSV scan + DQ chain: K1 (line boundaries) + K2 (field parse) + K3 (DQ rules, filters,
casts) in ONE hipRTC kernel per action.

Spark re-reads ``dataset-abstract.csv`` on every action and runs the parsed rows through the
rule UDFs and the clean-up filters in one whole-stage-codegen pipeline
(``DataQuality4MachineLearningApp.java:53-55, 68-90``).  The unfused device path here took five
kernels per action: terminator counts, their scan, a materialized ``[nlines]`` line-end array,
the parse (one typed plane per column, validity, keep flags) and the ``dq_fused`` chain kernel
re-reading those planes.  This module generates a kernel that

* takes 16 KiB byte windows per block (the ``csv_count_kernel`` windows, so the exclusive scan of
  the per-window terminator counts gives each block its first global line index — the only
  global intermediate, ``nb`` int64s);
* stages the window plus a head region (bytes of the line that straddles into the window) in
  LDS with 16-byte granule loads, finds the terminators from the staged registers (SWAR), and
  keeps their positions in LDS (uint16, 1024-line rounds) — no line-end array in HBM;
* parses each line (one thread per line, ``csv_parse_dev.h`` field parser) into registers,
  evaluates the DQ chain lowered by ``ops/dqvm.py`` on those registers, and stores only the
  columns the consumer needs plus the selection vector.

It runs only for a relation whose schema, null columns and line count are already known from an
earlier device scan of the SAME cached bytes (``runtime.filecache``; Spark's own schema-inference
job at ``load()`` is that earlier scan), so nothing has to be read back on the host: the action is
asynchronous end to end.  The kernel still verifies every field against those facts and raises a
deferred data error (``runtime/checks.py``) if one ever disagrees."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..runtime import faststream
from ..runtime.checks import defer
from ..utils import tracing
from ..utils import diag

__all__ = ["kernel_source", "ENTRY", "WINDOW", "head_bytes", "STATS"]

ENTRY = "dq_scan_fused"
WINDOW = 16384  # bytes per block: csv_count_kernel's window (256 threads x 64 bytes)
CAP = 1024  # line ends per LDS round
STATS = {"fused_scans": 0, "fused_grams": 0}

_HDR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "hip", "csv_parse_dev.h")
_header_text: Optional[str] = None



class _GramNullable(ValueError):
    """The in-scan Gram epilogue cannot take a chain whose feature / label outputs are nullable;
    only this rejection is cached as "no fused plan" (any other codegen error propagates)."""

def header_text() -> str:
    global _header_text
    if _header_text is None:
        with open(_HDR) as f:
            _header_text = f.read().replace("#pragma once\n", "")
    return _header_text


def head_bytes(mean_line: float) -> int:
    """LDS head region: the part of the line that straddles into the window — 4x the mean line
    length, a power of two in [256, 2048].  A longer straddling line parses from global memory."""
    h = 256
    while h < 4 * mean_line and h < 2048:
        h *= 2
    return h


def ticket_mode() -> str:
    """How a look-back block picks its window (``DQ4ML_SCAN_TICKET``):

    * ``xcd`` (default): one dispatch-order ticket counter per ``blockIdx.x % 8`` class (the
      8 XCDs take workgroups round-robin), on separate cache lines; window = ticket * 8 + class.
    * ``global``: one counter for the grid — strict dispatch order, but every block's ticket
      is an atomic on ONE address, serialised at the memory side: 0.48 of 0.75 ms in a
      1e8-line scan with the per-line work ablated (``scripts/scan_ablation.py``).
    * ``none``: window = ``blockIdx.x`` (relies on in-order dispatch per XCD).

    Either way a predecessor that never publishes ends in the bounded spin (vflag 4, a loud
    fact-check failure), never a hang."""
    m = os.environ.get("DQ4ML_SCAN_TICKET", "xcd")
    if m not in ("xcd", "global", "none"):
        raise ValueError(f"DQ4ML_SCAN_TICKET={m!r}: expected xcd, global or none")
    return m


# status words after the per-window ones: the global ticket, then 8 per-class tickets 128 B apart
TICKET_WORDS = 1 + 8 * 16


def _ticket(lookback: bool, mode: str = "xcd") -> str:
    if not lookback:
        return "  const long long blk = blockIdx.x;"
    if mode == "none":
        return """  DQG unsigned long long* status = (DQG unsigned long long*)offs;
  const long long blk = blockIdx.x;"""
    if mode == "global":
        return """  // window = dispatch-order ticket: every predecessor window's block is already resident, so
  // the look-back below always makes progress
  DQG unsigned long long* status = (DQG unsigned long long*)offs;
  if (tid == 0)
    sblk = (long long)__hip_atomic_fetch_add(status + gridDim.x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const long long blk = sblk;"""
    return """  // window = per-XCD dispatch-order ticket * 8 + class: one counter per blockIdx.x % 8 class
  // (the XCD round-robin), so no single address serialises every block's ticket
  DQG unsigned long long* status = (DQG unsigned long long*)offs;
  if (tid == 0) {
    const unsigned int x = blockIdx.x & 7u;
    sblk = (long long)__hip_atomic_fetch_add(status + gridDim.x + 1 + 16 * x, 1ull, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
  }
  __syncthreads();
  const long long blk = sblk;"""


def _lookback(lookback: bool) -> str:
    if not lookback:
        return "  const long long gl0 = offs[blockIdx.x];"
    return """  if (wave == 0) {
    // decoupled look-back, one wave: publish this window's count (flag 1), then read the 64
    // nearest predecessors at once; their values up to the nearest one carrying its inclusive
    // prefix (flag 2) sum to ours.  Relaxed agent-scope atomics: the status words are
    // self-contained (no other data to order), so no release/acquire cache maintenance.  Bounded
    // spin: a predecessor that never publishes flags the scan (vflag 4) instead of hanging.
    const unsigned long long kVal = (1ull << 62) - 1;
    if (lane == 0)
      __hip_atomic_store(status + blk, (1ull << 62) | (unsigned long long)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long pre = 0;
    long long j0 = blk - 1;
    unsigned int spins = 0;
    bool stuck = false;
    while (j0 >= 0) {
      const long long j = j0 - lane;
      unsigned long long st = 2ull << 62;  // before window 0: an inclusive zero
      if (j >= 0) st = __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned int f = (unsigned int)(st >> 62);
      const unsigned long long inv = __ballot(f == 0), incl = __ballot(f == 2);
      const int k = incl ? (int)__builtin_ctzll(incl) : 64;
      const unsigned long long upto = k >= 63 ? ~0ull : ((2ull << k) - 1);  // lanes 0..k
      if (inv & upto) {
        if (++spins > (1u << 20)) { stuck = true; break; }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      long long v = lane <= k ? (long long)(st & kVal) : 0ll;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      pre += v;
      if (k < 64) break;
      j0 -= 64;
    }
    if (lane == 0) {
      if (stuck) dq_flag(vflag, 4u);
      __hip_atomic_store(status + blk, (2ull << 62) | (unsigned long long)(pre + cnt), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      sgl0 = pre;
    }
  }
  __syncthreads();
  const long long gl0 = sgl0;"""


def _wpe(fast_only: bool = False) -> str:
    """Occupancy hint (``DQ4ML_SCAN_WPE`` waves per SIMD; 0: the compiler's choice).  Default 8:
    the byte walks are latency-bound, and 8 waves with a few spilled VGPRs beat 4 waves without
    (lab CSV pipeline 2.16 / 1.94 / 1.91 ms per step at 4 / 6 / 8 waves, one run)."""
    w = int(os.environ.get("DQ4ML_SCAN_WPE", "8"))
    return f"__attribute__((amdgpu_waves_per_eu({w}))) " if w > 0 else ""


_VALUE = {1: "(int)fzl{c}", 2: "fzl{c}", 0: "fzd{c}", 3: "(fzd{c} != 0.0)", 5: "fzl{c}"}


def _scan_nt() -> bool:
    """Window loads with the non-temporal hint (default; DQ4ML_SCAN_NT=0 turns it off).  Each
    window byte is read once, so the hint keeps the stream out of the caches' way: lab CSV action
    0.913 -> 0.900 ms at 1e8 rows, three alternating pairs, same statistics digest
    (profiles/r6/lab_nt_ab.log)."""
    return os.environ.get("DQ4ML_SCAN_NT", "1") != "0"


def gram_width(d: int) -> int:
    """Statistics per block in Gram mode: live count, Σy, Σy², Σx (d), Σxy (d), packed-upper Σxx."""
    return 3 + 2 * d + d * (d + 1) // 2


def _gram_code(xs, yv) -> str:
    """Per-line accumulation of the Gram statistics (``gram_width`` order) for a live row."""
    d = len(xs)
    lines = ["    if (live) {\n"]
    lines += [f"      const double gx{i} = (double)({v});\n" for i, v in enumerate(xs)]
    lines.append(f"      const double gy = (double)({yv});\n")
    lines.append("      acc[0] += 1.0; acc[1] += gy; acc[2] += gy * gy;\n")
    for i in range(d):
        lines.append(f"      acc[{3 + i}] += gx{i}; acc[{3 + d + i}] += gx{i} * gy;\n")
    q = 3 + 2 * d
    for j in range(d):  # packed upper, column by column: slot j(j+1)/2 + i (the WLS flat layout)
        for i in range(j + 1):
            lines.append(f"      acc[{q}] += gx{i} * gx{j};\n")
            q += 1
    lines.append("    }\n")
    return "".join(lines)


def kernel_source(g, kinds, nullable, used, opts: dict, strict: bool, head: int, slots: dict,
                  lookback: bool = True, fast_only: bool = False, ticket: str = "xcd", gram: int = 0,
                  nolb: bool = False, term_only: Optional[str] = None) -> str:
    """Source of the fused kernel.

    ``g``: the dqvm generator after lowering the chain (its ``lines`` use ``f<c>`` / ``m<c>`` for
    base column ``c``; ``stores`` write row ``li``).  ``kinds``: storage kind per CSV column (0 f64,
    1 int32, 2 int64, 3 bool).  ``nullable``: columns with nulls in the earlier scan (others are
    verified null-free).  ``used``: columns the chain reads.  ``slots``: pointer-slot indices of
    the scan inputs (buf, offs, nalloc, trailing, vflag).

    ``lookback``: single pass — each block takes a ticket (its window, in dispatch order),
    publishes its line count and finds its first line index by decoupled look-back over its
    predecessors' published counts (``offs`` is then the zeroed ``[nb + TICKET_WORDS]`` status
    array, the ticket counters last; ``ticket``: see ``ticket_mode``).  Otherwise ``offs`` holds
    the exclusive scan of ``csv_count_kernel``'s per-window counts (two passes over the bytes).

    ``fast_only``: the earlier scan parsed every field on the numeric fast path (plain dialect):
    only that path is compiled in — the general parser's registers (~60 VGPRs) leave the kernel
    (40 VGPRs instead of 103, full occupancy without spills); a field it cannot take is a fact
    violation (vflag), like a type or null mismatch.

    ``gram`` = d > 0: the chain's outputs are d features and a label (a ``VectorAssembler`` +
    ``LinearRegression`` consumer, ``try_fused_gram``): no row is stored — every live row adds
    to register sums of the f64 normal-equation statistics, and each block writes its
    ``gram_width(d)`` sums (wave shuffles + LDS, fixed order) to ``p[slots['gpart']]`` at its
    window index."""
    from .dqvm import ptr_struct

    ncols = len(kinds)
    ns = len(g.ptrs)
    nv = list(opts.get("null_value", "").encode())
    o = (f"{{(unsigned char){ord(opts.get('sep', ','))}, (unsigned char){int(opts['quote'])}, "
         f"(unsigned char){int(opts['escape'])}, (unsigned char){int(opts['comment'])}, "
         f"(unsigned char){int(bool(opts['trim_lead']))}, (unsigned char){int(bool(opts['trim_trail']))}, "
         f"(unsigned char){len(nv)}, (unsigned char){int(strict)}, "
         f"{{{', '.join(str(x) for x in (nv + [0] * (16 - len(nv))))}}}}}")
    # diagnostic ablation builds (wrong results; scripts/scan_ablation.py), bit flags: 1 no per-line
    # work, 2 no stores, 4 no look-back, 8 no line-end scatter / line loop, 16 no ticket, 32 no LDS
    # staging stores, 64 no SWAR field conversion, 128 no Gram accumulation, 256 no Gram epilogue
    abl = diag.ablation("DQ4ML_SCAN_ABL")  # (refused without DQ4ML_DIAG=1)
    # the window's line-end counts scanned by DPP (six __shfl_up ds_bpermute steps measured 1.2 %
    # slower over the lab action: profiles/r5/lab_dpp_ab.jsonl)
    scan_code = "  int inc = dq_scan_incl(c);"

    def field_code(c: int, swar: bool) -> str:
        if int(kinds[c]) == 4:  # a string column the chain does not read: cut past its field only
            return (f"    bool fzk{c} = false;\n"
                    f"    if (pos <= end && line) {{ decltype(pos) fs{c} = 0, fe{c} = 0; bool rw{c} = false; "
                    f"fzk{c} = !csv_field_span(B, (decltype(pos))bias, pos, (decltype(pos))end, O, fs{c}, fe{c}, rw{c}); }}\n")
        if swar and abl & 64:
            return (f"    double fzd{c} = 0.0; long long fzl{c} = 0; bool fzg{c} = false; int fzy{c} = C_NULL;\n"
                    f"    if (pos <= len && line) {{\n"
                    f"      const unsigned int rest = sepm >> pos;\n"
                    f"      const int q = rest ? pos + (int)__builtin_ctz(rest) : len;\n"
                    f"      fzl{c} = (long long)(csv_bytes8(lo, hi, pos) & 0xFFull) + (q - pos); fzd{c} = (double)fzl{c};\n"
                    f"      fzy{c} = C_INT; pos = q + 1;\n"
                    f"    }}\n"
                    f"    bool fzk{c} = fzy{c} != C_NULL && fzy{c} != C_STRING;\n")
        if swar:  # short line in registers (csv_line16 / csv_swar_field); > 8-byte fields walk the stage
            return (f"    double fzd{c} = 0.0; long long fzl{c} = 0; bool fzg{c} = false; int fzy{c} = C_NULL;\n"
                    f"    if (pos <= len && line) {{\n"
                    f"      const unsigned int rest = sepm >> pos;\n"
                    f"      const int q = rest ? pos + (int)__builtin_ctz(rest) : len;\n"
                    f"      if (q - pos <= 8) {{\n"
                    f"        if (!csv_swar_field(csv_bytes8(lo, hi, pos), q - pos, fzd{c}, fzl{c}, fzy{c})) bad = true;\n"
                    f"      }} else {{\n"
                    f"        int ps = start + pos;\n"
                    f"        if (!csv_field_fast(B, 0, ps, end, O.sep, fzd{c}, fzl{c}, fzy{c})) bad = true;\n"
                    f"      }}\n"
                    f"      pos = q + 1;\n"
                    f"    }}\n"
                    f"    bool fzk{c} = fzy{c} != C_NULL && fzy{c} != C_STRING;\n")
        if fast_only:
            return (f"    double fzd{c} = 0.0; long long fzl{c} = 0; bool fzg{c} = false; int fzy{c} = C_NULL;\n"
                    f"    if (pos <= end && line && !csv_field_fast(B, bias, pos, end, O.sep, fzd{c}, fzl{c}, fzy{c})) bad = true;\n"
                    f"    bool fzk{c} = fzy{c} != C_NULL && fzy{c} != C_STRING;\n")
        return (f"    double fzd{c} = 0.0; long long fzl{c} = 0; bool fzg{c} = false; int fzy{c} = C_NULL;\n"
                f"    if (pos <= end && line) fzy{c} = csv_field(B, bias, pos, end, O, fzd{c}, fzl{c}, slow, fzg{c}, malformed);\n"
                f"    bool fzk{c} = fzy{c} != C_NULL && fzy{c} != C_STRING;\n")

    def parse_code(swar: bool) -> str:
        parse = []
        for c in range(ncols):
            k = int(kinds[c])
            parse.append(field_code(c, swar))
            if k == 4:
                continue
            if strict:
                parse.append(f"    if (fzy{c} != C_NULL && !csv_conforms(fzy{c}, {k})) {{ malformed = true; fzk{c} = false; }}\n")
            else:
                parse.append(f"    bad |= line && fzy{c} != C_NULL && !csv_conforms(fzy{c}, {k});\n")
            if k != 2:
                parse.append(f"    slow |= fzg{c};\n")
        parse.append("    if (malformed) {" + " ".join(f"fzk{c} = false;" for c in range(ncols)) + " }\n")
        for c in range(ncols):
            if not nullable[c]:
                parse.append(f"    bad |= line && !fzk{c};\n")
        for c in sorted(used):
            ct = used[c]
            if int(kinds[c]) == 4:
                from . import dqvm

                raise dqvm.Unfusable("string column")  # the eager scan builds it (DeviceStringColumn)
            val = _VALUE[int(kinds[c])].format(c=c)
            parse.append(f"    const {ct} fzf{c} = fzk{c} ? ({ct})({val}) : ({ct})0;\n")
            if nullable[c]:
                parse.append(f"    const bool fzm{c} = fzk{c};\n")
        return "".join(parse)

    # SWAR rows: fast-only files whose separator cannot be part of a number
    sep_c = opts.get("sep", ",")
    swar = fast_only and sep_c not in "0123456789.+-" and os.environ.get("DQ4ML_SCAN_SWAR", "1") != "0"
    body = ("\n".join("    " + ln.strip() for ln in g.lines).replace("P[", "p[")
            .replace("atomicOr((int*)p[", "dq_flag((unsigned int*)p["))
    stores = "".join(f"    ((DQG {t}*)p[{s}])[li] = ({t})({v});\n" for t, v, s in g.stores)
    if gram:
        vals = {}
        for t, v, s in g.stores:
            tag = g.recipe[s]
            if tag[0] == "outvalid":
                raise _GramNullable("gram mode: nullable outputs")
            if tag[0] == "out":
                vals[tag[1]] = v
        stores = _gram_code([vals[i] for i in range(gram)], vals[gram]) if not abl & 128 else ""
    elif abl & 2:
        stores = "".join(f"    if (li == -7) ((DQG {t}*)p[{s}])[0] = ({t})({v});\n" for t, v, s in g.stores)
    comment = int(opts["comment"])
    H, W = int(head), WINDOW
    # terminator masks: both bytes in general; only the file's one terminator byte when its facts
    # say every line ends the same single way (CR only, as the reference data, or LF only) -- the
    # other byte then occurs nowhere in the cached bytes (the kernel is VALU-issue-bound)
    cr_scan = ("" if term_only == "lf" else
               "      cr |= (unsigned long long)byte_eq4(v[w], 0x0D0D0D0Du) << (16 * j + 4 * w);\n")
    lf_scan = ("" if term_only == "cr" else
               "      lf |= (unsigned long long)byte_eq4(v[w], 0x0A0A0A0Au) << (16 * j + 4 * w);\n")
    swar_row = "" if not swar else f"""
// a line of at most 16 bytes in the LDS stage: held in two 64-bit registers, fields cut by the
// separator bitmask, numeric fields converted SWAR (csv_parse_dev.h) — no per-byte loop
__device__ __forceinline__ void dq_row_swar(const unsigned char* B, int start, int end, long long li,
                                            void* const* p, unsigned int* vflag, double* acc) {{
    const CsvOpts O = {o};
    const int len = end - start;
    const bool line = len > 0 && !({comment} && B[start] == {comment});
    unsigned long long lo, hi;
    csv_line16(B, start, lo, hi);
    const unsigned int sepm = csv_eq16(lo, hi, O.sep) & ((1u << len) - 1u);
    int pos = 0;
    bool slow = false, malformed = false, bad = false;
{parse_code(True)}    bad |= slow;
    if (bad) dq_flag(vflag, 1u);
    bool live = line;
{body}
{stores}}}
"""
    # 10^k / RN(10^-k) for the SWAR converter's decimals: an LDS table (one ds_read2_b64) or VALU
    # selects and products (DQ4ML_SCAN_P10=valu); the kernel is VALU-issue-bound
    p10_lds = swar and os.environ.get("DQ4ML_SCAN_P10", "lds") == "lds"
    p10_decl = ("__shared__ double dq_p10[16];\n#define CSV_P10_TAB dq_p10\n" if p10_lds else "")
    p10_init = ("  if (threadIdx.x < 16) dq_p10[threadIdx.x] = threadIdx.x < 8 ? dq4ml_csv::csv_pow10(threadIdx.x)\n"
                "                                                       : dq4ml_csv::csv_inv_pow10(threadIdx.x - 8);\n"
                if p10_lds else "")
    return ("#define CSV_UDOT4(a, b, c) __builtin_amdgcn_udot4((a), (b), (c), false)\n"
            "#define CSV_MUL24(a, b) __umul24((a), (b))\n" + p10_decl + header_text() + f"""
using namespace dq4ml_csv;
typedef unsigned int csv_u32x4 __attribute__((ext_vector_type(4)));
// every global access names the global address space: generic (flat) accesses count in both
// the VM and the LDS wait counters, so each LDS read after a flat store would wait for that store
#define DQG __attribute__((address_space(1)))

__device__ __forceinline__ void dq_flag(unsigned int* f, unsigned int v) {{
  __hip_atomic_fetch_or((DQG unsigned int*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}}
// inclusive wave scan by DPP: row_shr 1, 2, 4, 8 inside each 16-lane row (zero fill), then
// row_bcast 15 / 31 across rows; lane 63 ends with the wave total
__device__ __forceinline__ int dq_scan_incl(int v) {{
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return v;
}}
// the f64 wave sum by the same DPP steps on the two halves (fixed order); the total in lane 63
template <int CTRL, int RM>
__device__ __forceinline__ double dq_dpp_f64(double x) {{
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, RM, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, RM, 0xF, false);
  return __hiloint2double(hi, lo);
}}
__device__ __forceinline__ double dq_sum63(double x) {{
  x += dq_dpp_f64<0x111, 0xF>(x);
  x += dq_dpp_f64<0x112, 0xF>(x);
  x += dq_dpp_f64<0x114, 0xF>(x);
  x += dq_dpp_f64<0x118, 0xF>(x);
  x += dq_dpp_f64<0x142, 0xA>(x);
  x += dq_dpp_f64<0x143, 0xC>(x);
  return x;
}}

// one line: parse every field into registers, run the DQ chain, store the needed outputs at li
template <typename PB, typename IT>
__device__ __forceinline__ void dq_row(PB B, IT bias, IT start, IT end, long long li,
                                       void* const* p, unsigned int* vflag, double* acc) {{
    const CsvOpts O = {o};
    const bool line = end > start && !({comment} && B[start - bias] == {comment});
    IT pos = start;
    bool slow = false, malformed = false, bad = false;
{parse_code(False)}    bad |= slow;
    if (bad) dq_flag(vflag, 1u);
    bool live = line;
{body}
{stores}}}
{swar_row}
{ptr_struct(ns)}extern "C" __global__ __launch_bounds__(256) {_wpe(fast_only)}void {ENTRY}(const DqPtrs P, long long n) {{
  void* p[{ns}];
#pragma unroll
  for (int i = 0; i < {ns}; ++i) p[i] = P.v[i];
  const DQG unsigned char* __restrict__ b = (const DQG unsigned char*)p[{slots['buf']}];
  const DQG long long* __restrict__ offs = (const DQG long long*)p[{slots['offs']}];
  const long long nalloc = (long long)p[{slots['nalloc']}];
  const bool trailing = (long long)p[{slots['trailing']}] != 0;
  unsigned int* vflag = (unsigned int*)p[{slots['vflag']}];
  __shared__ __attribute__((aligned(16))) unsigned char stage[{H} + {W} + 16];
  __shared__ unsigned short lend[{CAP} + 1];
  __shared__ int wtot[4];
  __shared__ long long sstart0, sblk, sgl0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
{p10_init}{"  const long long blk = blockIdx.x;  // Gram mode: no global line numbering needed" if nolb else _ticket(lookback, ticket if not abl & 16 else "none")}
  const long long a = (long long)(reinterpret_cast<unsigned long long>(b) & 15ull);
  const DQG unsigned char* ab = b - a;                     // 16-byte aligned view
  const long long wbase = blk * {W} - a;                    // buffer index of window byte 0
  const long long sbase = wbase - {H};                     // buffer index of stage[0]
  const long long tb = wbase + 64 * tid;                    // this thread's 64 window bytes
  if (wbase > n) return;  // past the end (block-uniform; the virtual terminator at n is in an earlier window)
  unsigned long long cr = 0ull, lf = 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {{
    const long long gi = tb + 16 * j;
    csv_u32x4 v = {{0u, 0u, 0u, 0u}};
    if (gi < n && gi + 16 > 0) v = {"__builtin_nontemporal_load(" if _scan_nt() else "*("}reinterpret_cast<const DQG csv_u32x4*>(ab + gi + a));
    {"if (v[0] == 0x7F7F7F7Fu && v[1] == 3u) " if abl & 32 else ""}*reinterpret_cast<csv_u32x4*>(stage + {H} + 64 * tid + 16 * j) = v;
#pragma unroll
    for (int w = 0; w < 4; ++w) {{
{cr_scan}{lf_scan}
    }}
  }}
  for (int gq = tid; gq < {H // 16} + 1; gq += 256) {{  // head granules + one tail granule
    const long long gi = gq < {H // 16} ? sbase + 16 * gq : wbase + {W};
    csv_u32x4 v = {{0u, 0u, 0u, 0u}};
    if (gi < n && gi + 16 > 0) v = *reinterpret_cast<const DQG csv_u32x4*>(ab + gi + a);
    *reinterpret_cast<csv_u32x4*>(stage + (gq < {H // 16} ? 16 * gq : {H} + {W})) = v;
  }}
  {{
    const long long lo = tb < 0 ? -tb : 0, hi = n - tb;
    if (lo > 0 || hi < 64) {{
      const unsigned long long keep_lo = lo >= 64 ? 0ull : (~0ull << lo);
      const unsigned long long keep_hi = hi <= 0 ? 0ull : (hi >= 64 ? ~0ull : ((1ull << hi) - 1));
      cr &= keep_lo & keep_hi;
      lf &= keep_lo & keep_hi;
    }}
  }}
  __syncthreads();
  const unsigned long long prev_cr = (tb >= 1 && tb - 1 < n && stage[{H} + 64 * tid - 1] == '\\r') ? 1ull : 0ull;
  unsigned long long m = cr | (lf & ~((cr << 1) | prev_cr));
  // terminators that are the CR of a CR LF: the next line starts one byte later (bit 15 of the
  // LDS line-end word), so no line reads stage bytes to find its start
  const unsigned long long crlf = cr & ((lf >> 1) | ((unsigned long long)(stage[{H} + 64 * tid + 64] == '\\n') << 63));
  if (trailing) {{  // the last line has no terminator: a virtual one at n
    const long long r = n - tb;
    if (r >= 0 && r < 64) m |= 1ull << r;
  }}
  const int c = __popcll(m);
{scan_code}
  if (lane == 63) wtot[wave] = inc;
  if (wave == 0) {{
    // the terminator before the window's first line: nearest first, through the staged head
    long long found = -2;
    for (int k0 = 0; k0 < {H} && found == -2; k0 += 64) {{
      const long long q = wbase - 1 - k0 - lane;
      bool t = q < 0;
      if (q >= 0) {{
        const int sq = {H} - 1 - k0 - lane;
        const int ch = stage[sq];
        const bool pcr = q >= 1 && (sq >= 1 ? stage[sq - 1] : b[q - 1]) == '\\r';
        t = ch == '\\r' || (ch == '\\n' && !pcr);
      }}
      const unsigned long long bal = __ballot(t);
      if (bal) found = wbase - 1 - k0 - (long long)__builtin_ctzll(bal);
    }}
    for (long long q0 = wbase - 1 - {H}; found == -2; q0 -= 64) {{  // a line longer than the head
      const long long q = q0 - lane;
      bool t = q < 0;
      if (q >= 0) {{
        const int ch = b[q];
        t = ch == '\\r' || (ch == '\\n' && !(q >= 1 && b[q - 1] == '\\r'));
      }}
      const unsigned long long bal = __ballot(t);
      if (bal) found = q0 - (long long)__builtin_ctzll(bal);
    }}
    if (lane == 0) {{  // the window's first line starts after that terminator (and its LF)
      long long st0 = 0;
      if (found >= 0) {{
        st0 = found + 1;
        if (found + 1 < n) {{
          const bool ins = found >= sbase;
          const int c0 = ins ? stage[found - sbase] : b[found];
          const int c1 = ins ? stage[found + 1 - sbase] : b[found + 1];
          st0 += (c0 == '\\r' && c1 == '\\n') ? 1 : 0;
        }}
      }}
      sstart0 = st0;
    }}
  }}
  __syncthreads();
  int before = inc - c;
  for (int w = 0; w < wave; ++w) before += wtot[w];
  const int cnt = wtot[0] + wtot[1] + wtot[2] + wtot[3];
{_lookback(lookback) if not (abl & 4 or nolb) else "  const long long gl0 = 0;"}
{"  if (cnt + m == 7777777) dq_flag(vflag, (unsigned int)gl0 + (unsigned int)sstart0); return;" if abl & 8 else ""}
  if (cnt == 0) return;  // block-uniform
  double acc[{max(1, gram_width(gram) if gram else 1)}] = {{}};
  for (int R = 0; R < cnt; R += {CAP}) {{
    if (before + c > R - 1 && before < R + {CAP}) {{
      unsigned long long mm = m;
      int o = before;
      while (mm) {{
        const int bit = __builtin_ctzll(mm);
        mm &= mm - 1;
        if (o >= R - 1 && o < R + {CAP})
          lend[o - R + 1] = (unsigned short)(({H} + 64 * tid + bit) | ((unsigned int)((crlf >> bit) & 1ull) << 15));
        ++o;
      }}
    }}
    __syncthreads();
    const int nr = min(cnt - R, {CAP});
    for (int j = tid; j < nr; j += 256) {{
      const int jl = R + j;
      const long long end = sbase + (lend[j + 1] & 0x7FFFu);
      long long start = sstart0;
      if (jl != 0) {{
        const unsigned int w = lend[j];
        start = sbase + (w & 0x7FFFu) + 1 + (w >> 15);
      }}
      const long long li = gl0 + jl;
      if ({int(abl & 1)}) {{
        if (li == -7) dq_flag(vflag, (unsigned int)start);
      }} else if ({"false" if nolb else "li >= nalloc"}) {{
        dq_flag(vflag, 2u);
      }} else if (start >= sbase) {{
        const int s0 = (int)(start - sbase), e0 = (int)(end - sbase);  // 32-bit stage positions
        {"if (e0 - s0 <= 16) dq_row_swar(stage, s0, e0, li, p, vflag, acc); else " if swar else ""}dq_row(stage, 0, s0, e0, li, p, vflag, acc);
      }} else {{
        dq_row(b, 0ll, start, end, li, p, vflag, acc);
      }}
    }}
    __syncthreads();
  }}
{_gram_epilogue(gram, slots) if gram and not abl & 256 else ""}}}
""")


def _gram_epilogue(d: int, slots: dict) -> str:
    nv = gram_width(d)
    # DPP steps, the sum in lane 63 (no ds_bpermute round trips)
    red = "".join(f"""  {{
    const double t = dq_sum63(acc[{k}]);
    if (lane == 63) gred[wave][{k}] = t;
  }}
""" for k in range(nv))
    return f"""  // this window's statistics: wave sums, then the 4 waves in a fixed order (deterministic)
  __shared__ double gred[4][{nv}];
{red}  __syncthreads();
  if (tid < {nv})
    ((DQG double*)p[{slots['gpart']}])[blk * {nv} + tid] = gred[0][tid] + gred[1][tid] + gred[2][tid] + gred[3][tid];
"""


# ---------------------------------------------------------------------------------------------
# chain lowering over a not-yet-scanned relation + execution


class _ScanBase:
    """What ``dqvm.compile_chain`` reads of a base table, for a relation not scanned yet."""

    def __init__(self, schema, nrows: int, device):
        self.schema = schema
        self.columns = [None] * len(schema.fields)
        self.nrows = int(nrows)
        self.sel = None
        self.device = device


def _scan_gen(base: _ScanBase, nullable):
    from . import dqvm

    class _ScanGen(dqvm._Gen):
        """Base column c is the register pair (fzf<c>, fzm<c>) the kernel's parse defines — or
        (fzf<c>, true) for a column the earlier scan found null-free (verified in the kernel).
        The ``fz`` prefix keeps them apart from the generator's own temporaries (k<n>, m<n>, ...)."""

        def __init__(self):
            super().__init__(base, check_device=False)
            self.used = {}

        def load_col(self, idx: int):
            if idx not in self.col_cache:
                t = self.base.schema.fields[idx].dataType
                self.used[idx] = dqvm._ctype(t)
                self.col_cache[idx] = (f"fzf{idx}", f"fzm{idx}" if nullable[idx] else "true", t)
            return self.col_cache[idx]

    return _ScanGen()


class _ScanPlan:
    SCAN_SLOTS = ("buf", "offs", "nalloc", "trailing", "vflag")

    def __init__(self, src: str, g, outputs, refs, gram: int = 0):
        self.src = src
        self.recipe = list(g.recipe)
        self.has_raise = g.has_raise
        self.outs = [("new", o[1].dtype, o[2] is not None, o[3]) for o in outputs]
        self.refs = refs
        self.gram = gram

    def bind(self, nalloc: int, dev, scalars: dict, err: torch.Tensor):
        """Pointer slots; Gram mode allocates no row outputs (their slots are never stored to)."""
        g = self.gram
        outs = [(None if g else torch.empty(nalloc, dtype=o[1], device=dev),
                 torch.empty(nalloc, dtype=torch.bool, device=dev) if o[2] and not g else None) for o in self.outs]
        sel_out = None if g else torch.empty(nalloc, dtype=torch.bool, device=dev)
        ptrs = []
        for tag in self.recipe:
            k = tag[0]
            if k == "sel":
                v = 0
            elif k == "err":
                v = err.data_ptr()
            elif k in ("out", "outvalid", "selout") and g:
                v = 0
            elif k == "out":
                v = outs[tag[1]][0].data_ptr()
            elif k == "outvalid":
                v = outs[tag[1]][1].data_ptr()
            elif k == "selout":
                v = sel_out.data_ptr()
            elif k in scalars:
                x = scalars[k]
                v = x.data_ptr() if torch.is_tensor(x) else int(x)
            else:
                raise AssertionError(f"scan plan: unbound slot {tag}")
            ptrs.append(v)
        return ptrs, outs, sel_out


_CACHE: dict = {}
_streams: dict = {}


def _scan_stream(dev) -> torch.cuda.Stream:
    s = _streams.get(str(dev))
    if s is None:
        s = _streams[str(dev)] = torch.cuda.Stream(device=dev)
    return s


def _compile(nodes, rel, gram: int = 0):
    """The cached kernel plan of ``nodes`` fused into the scan of ``rel`` (None: not fusable,
    ``"vector"``: the chain ends in a VectorAssembler)."""
    from . import dqvm

    f = rel.fused
    if len(f["kinds"]) > 64 or f["mean_line"] > 64:
        return None  # one thread per line: wide rows take the cutter (ops/scancut.py) or scan eagerly
    (parts, udfs), refs = dqvm.nodes_key(nodes)
    head = head_bytes(f["mean_line"])
    lookback = os.environ.get("DQ4ML_SCAN_LOOKBACK", "1") != "0"
    # Gram mode stores no row, so it needs no global line numbering: no ticket, no look-back,
    # window = blockIdx.x (the line-count fact is a property of the same cached bytes)
    nolb = bool(gram) and lookback and os.environ.get("DQ4ML_SCAN_GRAM_NOLB", "1") != "0"
    ticket = ticket_mode()
    o = f["opts"]
    from .scancut import term_of

    tk = term_of(f) if os.environ.get("DQ4ML_SCAN_TERM1", "1") != "0" else None
    term_only = {(13, False): "cr", (10, False): "lf"}.get(tk)
    fast_only = (bool(f.get("fast_only")) and not o["null_value"] and not o["trim_lead"] and not o["trim_trail"]
                 and os.environ.get("DQ4ML_SCAN_FASTONLY", "1") != "0")
    key = (parts, udfs, tuple(rel.schema().names), tuple(f["kinds"]), tuple(f["nullable"]),
           repr(sorted(f["opts"].items())), f["strict"], head, lookback, fast_only, _wpe(fast_only),
           ticket, os.environ.get("DQ4ML_SCAN_ABL", "0"), gram, _scan_nt(), nolb, os.environ.get("DQ4ML_SCAN_P10"),
           term_only)
    cp = _CACHE.get(key)
    if cp is None and key not in _CACHE:
        base = _ScanBase(rel.schema(), 0, f["device"])
        g = _scan_gen(base, f["nullable"])
        try:
            _, g, outputs, _ = dqvm.compile_chain(nodes, base, False, gen=g)
            names = _ScanPlan.SCAN_SLOTS + (("gpart",) if gram else ())
            slots = {k: g.slot(None, (k,)) for k in names}
            src = kernel_source(g, f["kinds"], f["nullable"], g.used, f["opts"], f["strict"], head, slots, lookback,
                                fast_only, ticket, gram, nolb, term_only)
            cp = _ScanPlan(src, g, outputs, refs, gram)
            cp.lookback = lookback
        except dqvm.Unfusable as e:
            cp = "vector" if str(e) == "VectorAssembleExpr" else None
        except _GramNullable:  # Gram mode over nullable outputs: the row-storing scan instead
            cp = None
        if len(_CACHE) >= 64:
            _CACHE.clear()
        _CACHE[key] = cp
    return cp


def _launch(cp, nodes, rel, extra: dict, own_stream: bool = True):
    """One launch of ``cp`` over ``rel``'s cached bytes; returns (outs, sel_out, err, vflag,
    scan stream, compute stream) after checking a raised UDF error.  ``own_stream``: on the
    scan side stream (else on the compute stream, in order with the caller's work)."""
    from . import dqvm, native

    f = rel.fused
    h = native.hip()
    dev = f["device"]
    buf, n, nalloc = f["buf"], int(f["n"]), int(f["nlines"])
    # stage pipeline: the scan runs on its own stream and depends only on the
    # HBM-resident input bytes, so action k+1's scan overlaps action k's Gram / fit tail on the
    # compute stream; the compute stream waits for this scan's event before its consumers
    # (faststream: no per-call device resolution on this per-action path, profiles/r4_host_issue.md)
    cur = faststream.current(faststream.dev_index(dev))
    side = _scan_stream(dev) if own_stream and env(b"DQ4ML_SCAN_STREAM") != b"0" else cur
    with faststream.use(side):
        stream = side.cuda_stream
        nb = int(h.csv_count_blocks(n))
        # ONE zeroed scratch allocation: [offs | err, vflag | Gram partials]; offs is the
        # look-back status + ticket counters (single pass) or the per-window counts (two passes)
        no = nb + TICKET_WORDS if cp.lookback else nb + 1
        gw = gram_width(cp.gram) if cp.gram else 0
        z = torch.zeros(no + 1 + nb * gw, dtype=torch.int64, device=dev)
        offs = z[:no]
        if not cp.lookback:
            h.csv_line_ends(buf.data_ptr(), n, offs.data_ptr(), 0, stream, -1, 0)
        ev = z[no:no + 1].view(torch.int32)
        err, vflag = ev[0:1], ev[1:2]
        scalars = {"buf": buf, "offs": offs, "nalloc": nalloc, "trailing": int(f["trailing"]), "vflag": vflag}
        if cp.gram:
            extra["gpart"] = scalars["gpart"] = z[no + 1:].view(torch.float64).view(nb, gw)
        ptr_list, outs, sel_out = cp.bind(nalloc, dev, scalars, err)
        handle = dqvm.rtc_handle(h, cp, cp.src, ENTRY)
        with tracing.span("csv_scan_dq_fused"):
            dqvm.launch(h, handle, nb, ptr_list, n, stream)
    tracing.add_rows("csv_scan_dq_fused", nalloc)
    STATS["fused_scans"] += 1
    return outs, sel_out, err, vflag, side, cur


def _raise_message(nodes) -> str:
    """The message of the chain's raising rule (the last one found), or Spark's generic one."""
    from . import dqvm

    msg = "Failed to execute user defined function"
    for nd in nodes:
        for ex in getattr(nd, "exprs", []) + ([nd.cond] if hasattr(nd, "cond") else []):
            r = dqvm._find_raise(ex)
            if r is not None:
                msg = r.message
    return msg


def _udf_error_check(nodes, err):
    """A raising rule (``RaiseIfNull``: ``MinimumPriceDataQualityUdf``'s NPE on a null price,
    ``MinimumPriceDataQualityUdf.java:11-13``) as a deferred device check (``runtime/checks.py``):
    the action stays asynchronous and the SparkException surfaces with the first host read of
    its results — the job fails exactly as Spark's does, without a sync per action.  ``nodes``:
    the chain, or its precomputed ``_raise_message``."""
    from ..sql.expressions import SparkException

    msg = nodes if isinstance(nodes, str) else _raise_message(nodes)
    return defer(err, lambda: SparkException(msg))


def _fact_check(rel, vflag):
    # safety net: the earlier scan's facts (types, null-free columns, line count) are re-verified
    # by the kernel; a disagreement surfaces with the first host read of any output
    return defer(vflag, lambda: RuntimeError(
        f"fused CSV scan of {rel.label}: the input no longer matches the schema / line facts of its "
        f"earlier device scan"))


def try_fused_scan(nodes, rel, plan, session):
    """Run the Project/Filter chain ``nodes`` (bottom-up) fused into the scan of ``rel``.
    Returns the chain's Table, ``"vector"`` (the chain ends in a VectorAssembler: the assembler
    consumes the sub-chain instead) or None (not fusable: the caller scans, then runs the chain)."""
    from ..sql.table import ColumnData, Table

    if rel.fused.get("buf") is None:  # streamed input (§5g): rows are stored by the chunked eager scan
        return None
    cp = _compile(nodes, rel)
    if cp is None or cp == "vector":
        return cp
    outs, sel_out, err, vflag, side, cur = _launch(cp, nodes, rel, {})
    if side is not cur:
        cur.wait_stream(side)
        for t in [err, vflag, sel_out] + [x for o in outs for x in o if x is not None]:
            t.record_stream(cur)  # produced on the scan stream, consumed on the compute stream
    checks = [_fact_check(rel, vflag)] + ([_udf_error_check(nodes, err)] if cp.has_raise else [])
    checks = [c for c in checks if c is not None]
    schema = plan.schema()
    cols = [ColumnData(fd.dataType, oo[0], oo[1], dict(fd.metadata), list(checks))
            for fd, oo in zip(schema.fields, outs)]
    return Table(schema, cols, int(rel.fused["nlines"]), sel_out, rel.fused["device"])


class FusedGram:
    """``try_fused_gram``'s result: the f64 WLS statistics (``ops.device.gram_stats`` layout),
    the feature count, the pending fact check and the scanned line count."""

    def __init__(self, flat, d: int, checks: list, nrows: int):
        self.flat, self.d, self.checks, self.nrows = flat, d, checks, nrows


def try_fused_gram(plan, features_col: str, label_col: str, session, route_key=None) -> Optional[FusedGram]:
    """K1 + K3 + the VectorAssembler + the normal-equation Gram pass in ONE kernel: ``plan`` (pruned
    to the features and label) must be ``Project[VectorAssembler(inputs) AS features, label]`` over
    a Project/Filter chain over a not-yet-scanned CSV relation, with at most 8 numeric inputs, no
    weights and no nullable output.  The parsed rows never reach HBM: each block reduces the
    statistics of its live rows (``kernel_source(gram=d)``), a fixed-order column sum folds the
    per-window partials.  Spark runs this as one stage too — the assembler and the
    ``treeAggregate`` seqOp inside the scan's whole-stage-codegen pipeline
    (``DataQuality4MachineLearningApp.java:53-55, 68-90, 117-126``).  None: not this shape."""
    from ..models.feature import VectorAssembleExpr
    from ..sql.expressions import Alias, ColRef
    from ..sql.plan import CsvScanRelation, Filter, Project, output_name
    from ..sql.types import BooleanType, VectorUDT, is_numeric

    if os.environ.get("DQ4ML_SCAN_GRAM", "1") == "0" or session is None:
        return None
    if str(session.conf.get("dq4ml.fit.fuseScan", "true")).lower() not in ("1", "true", "yes"):
        return None
    if getattr(session, "device", None) is None or session.device.type != "cuda":
        return None
    nodes, p = [], plan
    while isinstance(p, (Project, Filter)) and p._memo is None:
        nodes.append(p)
        p = p.child
    if not nodes or not isinstance(nodes[0], Project):
        return None
    if not (isinstance(p, CsvScanRelation) and p._memo is None and p.fused is not None):
        return None
    top = nodes[0]
    by_name = {output_name(e): e for e in top.exprs}
    fe, le = by_name.get(features_col), by_name.get(label_col)
    if fe is None or le is None or not isinstance(fe, Alias) or not isinstance(fe.child, VectorAssembleExpr):
        return None
    va = fe.child
    cs = top.child.schema()
    d = len(va.inputs)
    if not 1 <= d <= 128:
        return None
    for c in va.inputs:
        t = ColRef(c).data_type(cs)
        if isinstance(t, VectorUDT) or not (is_numeric(t) or isinstance(t, BooleanType)):
            return None
    lexpr = le.child if isinstance(le, Alias) else le
    if not is_numeric(lexpr.data_type(cs)):
        return None
    gtop = Project(top.child, [Alias(ColRef(c), f"__gx{i}") for i, c in enumerate(va.inputs)] + [Alias(lexpr, "__gy")])
    chain = list(reversed(nodes[1:])) + [gtop]
    from . import scancut

    if p.fused.get("buf") is None:  # input not resident in HBM: the same kernels over a chunk ring
        return _streamed_gram(chain, p, d)
    ccp = scancut._compile(chain, p, d)  # the byte-parallel field cutter (wide rows, any d <= 128)
    if ccp is not None:
        route = _Route("cut", chain, ccp, d)
        _remember(route_key, route, session)
        return route.run(p)
    if d > 8:
        return None
    cp = _compile(chain, p, gram=d)
    if cp is None or cp == "vector":
        return None
    route = _Route("line", chain, cp, d)
    _remember(route_key, route, session)
    return route.run(p)


class _Route:
    """An action's lowered fused-scan fit: the compiled kernel (cutter or per-line) and the chain
    it was compiled from.  ``run(rel)`` launches it over a relation of the same structure (the
    action's fresh leaf: same cached bytes and facts)."""

    def __init__(self, kind, chain, cp, d):
        # the chain itself is not kept: its leaf is the first action's relation, whose fused
        # dict points at the cached HBM bytes (a remembered route must not keep them alive)
        self.kind, self.cp, self.d = kind, cp, d
        self.msg = _raise_message(chain)
        self.conf = None

    def run(self, p) -> "FusedGram":
        if self.kind == "cut":
            from . import scancut

            flat, err, vflag, ccp = scancut.launch_cut(self.cp, p, self.d)
            checks = [_fact_check(p, vflag)]
            if ccp.has_raise:
                checks.append(_udf_error_check(self.msg, err))
            STATS["fused_grams"] += 1
            return FusedGram(flat, self.d, [c for c in checks if c is not None], int(p.fused["nlines"]))
        return _run_line_gram(self.cp, self.msg, p, self.d)


_ROUTES: dict = {}
_ROUTE_ENV = ("DQ4ML_SCAN_GRAM", "DQ4ML_SCAN_CUT", "DQ4ML_CUT_MIN_LINE", "DQ4ML_SCAN_LOOKBACK", "DQ4ML_SCAN_GRAM_NOLB",
              "DQ4ML_SCAN_TERM1", "DQ4ML_SCAN_FASTONLY", "DQ4ML_SCAN_ABL", "DQ4ML_SCAN_P10", "DQ4ML_CUT_ABLATE",
              "DQ4ML_CUT_STAMPS", "DQ4ML_CUT_VSTRIP", "DQ4ML_SCAN_STREAM", "DQ4ML_SCAN_NT", "DQ4ML_SCAN_TICKET", "DQ4ML_SCAN_WPE",
              "DQ4ML_FUSE_ROUTES")


_ENV_DATA = getattr(os.environ, "_data", None)  # the process environment as bytes (CPython)
_ROUTE_ENV_B = tuple(k.encode() for k in _ROUTE_ENV)


def env(key: bytes):
    """``os.environ`` lookup of a bytes key without the str encode / decode round trip (the
    per-action knob reads of the replay path); None when unset."""
    if _ENV_DATA is None:
        v = os.environ.get(key.decode())
        return None if v is None else v.encode()
    return _ENV_DATA.get(key)


def route_key(plan_key, features_col: str, label_col: str, session):
    """Replay key of a fused-scan fit: the action's plan structure, the columns, the session conf
    and the scan knobs (None: not replayable)."""
    if plan_key is None or env(b"DQ4ML_FUSE_ROUTES") == b"0":
        return None
    return (plan_key, features_col, label_col, tuple(env(k) for k in _ROUTE_ENV_B),
            getattr(session, "device", None))


def window_fold(gpart, side):
    """The per-window partials [rows, gw] -> the flat gram_stats layout [n, Σw, Σw², Σwy, Σwy²,
    Σwx, Σwxy, packed-upper Σwxx] (unit weights: Σw = Σw² = n), fixed order, on ``side``."""
    from . import native

    with faststream.use(side):
        flat = torch.empty(gpart.shape[1] + 2, dtype=torch.float64, device=gpart.device)
        native.hip().gram_window_fold(gpart.data_ptr(), gpart.shape[0], gpart.shape[1], flat.data_ptr(),
                                      side.cuda_stream)
    return flat


_PLAN_CLASSES = []


def _plan_classes():
    """(CsvScanRelation, Filter, Project), imported once (sql.plan imports this package lazily)."""
    if not _PLAN_CLASSES:
        from ..sql.plan import CsvScanRelation, Filter, Project

        _PLAN_CLASSES.extend((CsvScanRelation, Filter, Project))
    return _PLAN_CLASSES


def replay(key, plan, session) -> Optional["FusedGram"]:
    """The remembered route of ``key`` launched over this action's leaf relation, or None."""
    r = _ROUTES.get(key) if key is not None else None
    if r is None or r.conf != session.conf._conf:
        return None
    CsvScanRelation, Filter, Project = _plan_classes()
    p = plan
    while isinstance(p, (Project, Filter)):
        if p._memo is not None:
            return None
        p = p.child
    if not isinstance(p, CsvScanRelation) or p._memo is not None or p.fused is None or p.fused.get("buf") is None:
        return None
    STATS["route_replays"] = STATS.get("route_replays", 0) + 1
    return r.run(p)


def _remember(key, route, session):
    if key is None:
        return
    route.conf = dict(session.conf._conf)
    if len(_ROUTES) >= 256:
        _ROUTES.clear()
    _ROUTES[key] = route


class _GramLaunch:
    """The per-action part of a Gram-mode per-line fused scan, resolved once per (plan, cached
    bytes): every pointer slot is either constant (the HBM-resident input, scalars, unused row
    outputs) or a fixed offset into the action's one zeroed scratch allocation, so an action is one
    allocation, one pointer-array fill, the kernel launch and the window fold (the host-issue path
    of a rebuilt lab action, ``profiles/r4_host_issue.md``)."""

    def __init__(self, cp, rel):
        import numpy as np

        from . import dqvm, native

        f = rel.fused
        self.h = h = native.hip()
        self.dev = f["device"]
        buf, n, nalloc = f["buf"], int(f["n"]), int(f["nlines"])
        self.key = (buf.data_ptr(), n, nalloc, bool(f["trailing"]))
        self.n, self.nb = n, int(h.csv_count_blocks(n))
        self.no = self.nb + TICKET_WORDS
        self.gw = gram_width(cp.gram)
        self.words = self.no + 1 + self.nb * self.gw
        scratch = {"offs": 0, "vflag": 8 * self.no + 4, "gpart": 8 * (self.no + 1)}
        tmpl, zi, zo = [], [], []
        for tag in cp.recipe:
            k = tag[0]
            if k in ("sel", "out", "outvalid", "selout"):
                v = 0
            elif k == "err":
                zi.append(len(tmpl))
                zo.append(8 * self.no)
                v = 0
            elif k in scratch:
                zi.append(len(tmpl))
                zo.append(scratch[k])
                v = 0
            elif k == "buf":
                v = buf.data_ptr()
            elif k == "nalloc":
                v = nalloc
            elif k == "trailing":
                v = int(f["trailing"])
            else:
                raise AssertionError(f"gram scan plan: unbound slot {tag}")
            tmpl.append(v)
        self.tmpl = np.asarray(tmpl, dtype=np.int64)
        self.zi, self.zo = np.asarray(zi, dtype=np.int64), np.asarray(zo, dtype=np.int64)
        # (the input's address is part of the key: the plan holds no reference to the bytes -- a
        # launch reads the bytes of the relation it is called for, which the file cache owns)
        self.handle = int(dqvm.rtc_handle(h, cp, cp.src, ENTRY))

    def __call__(self):
        """(flat statistics, err, vflag) of one launch on the current stream."""
        di = faststream.dev_index(self.dev)
        z = torch.empty(self.words, dtype=torch.int64, device=self.dev)
        arr = self.tmpl.copy()
        arr[self.zi] = self.zo + z.data_ptr()
        stream = faststream.raw(di)
        self.h.memset_async(z.data_ptr(), 0, 8 * self.words, stream)
        with tracing.span("csv_scan_dq_fused"):
            self.h.rtc_launch_args(self.handle, self.nb, 256, arr, self.n, stream)
        flat = torch.empty(self.gw + 2, dtype=torch.float64, device=self.dev)
        self.h.gram_window_fold(z.data_ptr() + 8 * (self.no + 1), self.nb, self.gw, flat.data_ptr(), stream)
        ev = z[self.no:self.no + 1].view(torch.int32)
        tracing.add_rows("csv_scan_dq_fused", int(self.key[2]))
        STATS["fused_scans"] += 1
        return flat, ev[0:1], ev[1:2]


def _run_line_gram(cp, chain, p, d) -> "FusedGram":
    gl = getattr(cp, "_gram_launch", None)
    f = p.fused
    if cp.gram and cp.lookback:
        key = (f["buf"].data_ptr(), int(f["n"]), int(f["nlines"]), bool(f["trailing"]))
        if gl is None or gl.key != key:
            gl = cp._gram_launch = _GramLaunch(cp, p)
        flat, err, vflag = gl()
        checks = [_fact_check(p, vflag)] + ([_udf_error_check(chain, err)] if cp.has_raise else [])
        STATS["fused_grams"] += 1
        return FusedGram(flat, d, [c for c in checks if c is not None], int(f["nlines"]))
    extra = {}
    # on the compute stream, after the previous action's fit tail: the one-workgroup solve
    # kernel co-running with a whole-GPU scan gets ~1/8 of a CU's issue slots (22 -> 727 us,
    # kernel trace) and holds the pipeline longer than running alone between two scans; with
    # nothing left to overlap, a side stream would only add cross-queue waits
    _, _, err, vflag, side, cur = _launch(cp, chain, p, extra, own_stream=False)
    flat = window_fold(extra["gpart"], side)
    if side is not cur:
        cur.wait_stream(side)
        for t in (err, flat):
            t.record_stream(cur)  # (err, vflag and the partials share one allocation)
    checks = [_fact_check(p, vflag)] + ([_udf_error_check(chain, err)] if cp.has_raise else [])
    STATS["fused_grams"] += 1
    return FusedGram(flat, d, [c for c in checks if c is not None], int(p.fused["nlines"]))


class _ChunkRel:
    """One row-aligned chunk of a streamed relation, as the fused-scan launchers see a relation:
    the relation's facts with the chunk's device bytes (``buf``, ``n``, ``trailing``)."""

    def __init__(self, rel, fused):
        self.fused, self.label, self._rel = fused, rel.label, rel

    def schema(self):
        return self._rel.schema()


def _streamed_gram(chain, rel, d: int) -> Optional[FusedGram]:
    """the fit's one fused pass over an input that does not stay resident in HBM.
    The relation's ``ChunkSource`` streams row-aligned chunks through a two-slot device ring (the
    H2D copy of chunk k+1 on the side stream overlaps the kernels of chunk k on the compute
    stream); every chunk runs the same compiled scan + DQ chain + assembler + Gram kernel as the
    resident path (the byte-parallel cutter, or the per-line kernel for d <= 8 short rows), and the
    chunks' f64 statistics sum into one accumulator on the device in chunk order (deterministic).
    Spark streams the partitions of ``DataQuality4MachineLearningApp.java:53-55`` through its
    iterators the same way, at constant memory."""
    from . import scancut

    f = rel.fused
    src = f["stream"]
    if not len(src):
        return None
    s0, e0 = src.spans[0]
    probe = _ChunkRel(rel, dict(f, buf=None, n=e0 - s0, trailing=False, stream=None))
    use_cut = scancut._compile(chain, probe, d) is not None
    cp = None
    if not use_cut:
        if d > 8:
            return None
        cp = _compile(chain, probe, gram=d)
        if cp is None or cp == "vector":
            return None
    acc, checks = None, []
    for buf, n, trailing in src.chunks():
        crel = _ChunkRel(rel, dict(f, buf=buf, n=n, trailing=trailing, stream=None))
        if use_cut:
            cut = scancut.try_cut_gram(chain, crel, d)
            if cut is None:
                raise RuntimeError("streamed fused Gram: the cutter plan did not apply to a chunk")
            flat, err, vflag, ccp = cut
            raising = ccp.has_raise
        else:
            extra = {}
            _, _, err, vflag, side, _cur = _launch(cp, chain, crel, extra, own_stream=False)
            flat = window_fold(extra["gpart"], side)
            raising = cp.has_raise
        acc = flat.clone() if acc is None else acc.add_(flat)
        checks.append(_fact_check(rel, vflag))
        if raising:
            checks.append(_udf_error_check(chain, err))
    STATS["fused_grams"] += 1
    STATS["streamed_grams"] = STATS.get("streamed_grams", 0) + 1
    return FusedGram(acc, d, [c for c in checks if c is not None], int(f["nlines"]))
