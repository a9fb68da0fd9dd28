"""Byte-parallel CSV field cutter with the DQ chain, the VectorAssembler and the normal-equation
Gram in ONE persistent hipRTC kernel per action (SURVEY.md K1 + K3 + K4 + K5).

The action is ``LinearRegression.fit`` over ``VectorAssembler`` over a DQ chain over a CSV re-read
(``DataQuality4MachineLearningApp.java:53-55, 68-90, 110-126``; Spark re-scans the file on every
action, S20).  ``scanfuse.py``'s per-line kernel gives each LINE to one lane, which then walks
its bytes serially: fine for the lab's 8-byte rows, latency-bound for a 300-byte row of 33
numeric fields.  Here the unit of parallel work is the FIELD:

1. a block stages a 16 KiB window plus a head (the row that straddles into it) in LDS with
   16-byte granule loads, and every lane builds the terminator and separator bitmasks of its 64
   window bytes with SWAR compares (4 bytes per 32-bit op);
2. the delimiter counts are prefix-summed across the block (wave ``shfl_up`` scans + one LDS
   word per wave) and each lane scatters its delimiter positions into an LDS position array —
   the cut: field f of the window spans (pos[f-1], pos[f]);
3. every lane converts its own field (fields ``tid + 256 k``, row and column advanced by constant
   steps): one 12-byte LDS frame ending at the field's delimiter and the 32-bit SWAR converter
   ``csv_num_r8q_w`` (digits and the dot by per-dword masks, the dot squeezed out by two
   ``v_perm_b32``, ``v_dot4`` digit combine, the quotient by the fma-corrected reciprocal of
   10^k; exact and bit-identical to the byte-walking fast path), the value stored once into an
   LDS row tile [row][column] (f64);
4. one thread per row runs the DQ chain (``ops/dqvm.py`` lowering, rule bodies and filters in
   registers) on its row of the tile, which gives the features, the label and the live flag;
5. the normal-equation statistics: for d <= 8 every row thread adds to f64 register sums (the
   per-line kernel's scheme); for wider rows the live rows' augmented vectors ``[x | 1 | y]`` go
   to a second LDS tile and 4 x 4 register blocks of the upper Gram accumulate over them (f64,
   every statistic exact to the input doubles).

Blocks are persistent (one per CU slot, windows ``blockIdx.x + k * gridDim.x``) and keep their
sums in registers across windows; one partial per block (and row group) is folded at the end in
a fixed order, so repeated actions are bitwise identical.  Nothing is stored per row.

Preconditions, all facts of the earlier device scan of the same cached bytes (Spark's schema
inference job at ``load()``): every field took the numeric fast path, no column holds nulls, no
empty line, every line has exactly the column count (separator count = lines x (columns - 1)),
int32 / double columns only, and the longest line fits the staged head.  The kernel re-verifies
the facts it relies on (field count per row, field classes) and raises the deferred data error
of ``runtime/checks.py`` if the bytes ever disagree.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from ..utils import diag

__all__ = ["applicable", "kernel_source", "try_cut_gram", "STATS", "ENTRY"]

ENTRY = "dq_scan_cut"
WINDOW = 16384
TILE_BYTES = 18432  # LDS of the row tiles (chain inputs + Gram rows) per round
TARGET_PER_CU = 4   # resident blocks per CU the LDS budget aims at
STATS = {"cut_grams": 0}
LAST_STAMPS: dict = {}  # diagnostic phase clocks of the last launch (DQ4ML_CUT_STAMPS=1)


def head_for(max_line: int) -> int:
    """Staged head: a power of two >= the longest line + 32 bytes, in [256, 4096] (None above)."""
    h = 256
    while h < max_line + 32:
        h *= 2
    return h if h <= 4096 else None


def applicable(f: dict) -> Optional[int]:
    """The head size when the cached relation's facts allow the cutter, else None."""
    if os.environ.get("DQ4ML_SCAN_CUT", "1") == "0":
        return None
    o = f["opts"]
    sep = o.get("sep", ",")
    if not (f.get("fast_only") or f.get("quoted_fast")) or f.get("strict") or any(f["nullable"]) \
            or f.get("empty_lines", 1) != 0:
        return None
    if not f.get("uniform_fields") or len(f["kinds"]) < 1 or any(int(k) not in (0, 1) for k in f["kinds"]):
        return None
    if o["null_value"] or o["trim_lead"] or o["trim_trail"] or int(o["comment"]) or len(sep) != 1:
        return None
    if sep in "0123456789.+-\r\n" or term_of(f) is None:
        return None
    return head_for(int(f.get("max_line", 1 << 30)))


def term_of(f: dict):
    """(terminator byte, CR LF) when every line of the cached bytes ends the same way — CR only
    (the reference data), LF only, or CR LF only — else None (mixed endings keep
    the per-line kernel)."""
    cr, lf, crlf = (list(f.get("term_kinds") or (1, 1, 0)) + [0, 0, 0])[:3]
    if lf == 0 and crlf == 0:
        return 13, False
    if cr == 0:
        return 10, False
    if lf == 0 and crlf == cr:
        return 13, True
    return None


def gram_width(d: int) -> int:
    return 3 + 2 * d + d * (d + 1) // 2


def _gram_index(i: int, j: int, d: int) -> Optional[int]:
    """Slot of augmented Gram entry (i <= j) of [x_0..x_{d-1}, 1, y] in the gram_width layout
    [count, Σy, Σy², Σx (d), Σxy (d), packed-upper Σxx]; None for padding."""
    if j >= d + 2:
        return None
    if j < d:
        return 3 + 2 * d + j * (j + 1) // 2 + i
    if j == d:
        return 3 + i if i < d else 0
    if i < d:
        return 3 + d + i
    return 1 if i == d else 2


def _tile_slot(sh, i: int, j: int):
    """gram_width slot of entry (i <= j) of the row tile's upper Gram.  The tile's columns are the
    augmented vector [x | 1 | y], or [x | y | 1] when ``sh.yfirst`` (the label column then sits
    right after the features, where the cutter stores the CSV's last column)."""
    d = sh.d
    if i > j:
        return None
    if sh.yfirst:
        sw = {d: d + 1, d + 1: d}
        i, j = sw.get(i, i), sw.get(j, j)
        i, j = min(i, j), max(i, j)
    return _gram_index(i, j, d)


def _passthrough(xs, used, d):
    """Feature columns when every feature is a bare column read (``fzf<c>``, each column at most
    once), else None."""
    import re

    cols = []
    for v in xs:
        m = re.fullmatch(r"\(*(?:\(double\))?\(*fzf(\d+)\)*", v.replace(" ", ""))
        if m is None:
            return None
        cols.append(int(m.group(1)))
    return cols if len(set(cols)) == len(cols) else None


class _Shape:
    """Compile-time sizes of one cutter kernel (shared by the codegen and the launcher)."""

    def __init__(self, C, d, H, min_line, ucols, feat):
        self.C, self.d, self.H = C, d, H
        self.W = WINDOW
        self.HG = (H // 16 + 2 + 255) // 256          # head + tail granules per thread
        rows_max = (H + self.W) // max(1, min_line) + 2  # rows that can end in one window
        self.DCAP = min((H + self.W) // 2 + 64, rows_max * C + 64)
        self.blocked = d > 8
        self.PP = (d + 2 + 3) // 4 * 4
        self.NB = self.PP // 4
        self.U = self.NB * (self.NB + 1) // 2
        self.RG = max(1, 256 // self.U) if self.blocked else 1
        # the MFMA Gram (v_mfma_f64_16x16x4_f64 over 16-feature tiles of the row tile): d + 2 <= 80;
        # waves split into G tile groups x (4 / G) row groups, <= 32 accumulator VGPRs per wave
        self.ucols = ucols                              # columns the chain reads, in vt order
        self.CU = max(1, len(ucols))
        self.feat = feat                                # passthrough feature columns (blocked only)
        # every CSV column has a row-tile slot: features 0..d-1 pass through and the last column
        # (the label's source) lands at slot d, so the converter stores each field straight into
        # the tile ([x | y | 1] order) and the chain reads its inputs from there
        self.yfirst = d > 8 and feat == list(range(d)) and C == d + 1
        self.mfma = self.blocked and d + 2 <= 80
        # the [y | 1] strip (sums of x y, x, y, y^2 and the count: 2 d + 3 of the gram_width slots)
        # on the VALU beside the MFMA tiles of x x^T: the strip's MFMA panel is mostly padding
        # (2 of 16 columns at d = 32, a third of the tiles)
        self.vstrip = self.mfma and self.yfirst and os.environ.get("DQ4ML_CUT_VSTRIP", "1") != "0"
        self.NT16 = (d + (0 if self.vstrip else 2) + 15) // 16
        self.tiles = [(I, J) for I in range(self.NT16) for J in range(I, self.NT16)]
        if self.mfma:
            self.G = next((g for g in (1, 2, 4) if -(-len(self.tiles) // g) * 8 <= 32), 4)
            self.RG = 4 // self.G
        per_row = 8 * (self.CU + (self.PP if self.blocked else 0))
        self.gw = gram_width(d)
        fixed = (16 + H + self.W + 32) + 2 * self.DCAP + 4 * C + 384 + (
            8 * (3 * self.PP + 16) if self.blocked else 32 * self.gw)
        # the row tiles take what keeps TARGET_PER_CU blocks resident per CU (40 KiB each at 4),
        # within [4 KiB, TILE_BYTES]: more rounds per window beat fewer resident blocks
        tile = max(4096, min(TILE_BYTES, (160 * 1024) // TARGET_PER_CU - fixed))
        self.RR = int(max(1, min(rows_max, tile // per_row)))
        # (fixed holds the row tile's 3 zero rows and 16 padding doubles; round 5 counted them twice,
        # which held d = 64 at 3 blocks per CU: 22.68 -> 20.96 ms at 5e7 x 64 with 4)
        self.lds = fixed + 8 * self.RR * self.CU + (8 * self.RR * self.PP if self.blocked else 0)
        if self.blocked and (not self.mfma or len(self.tiles) > 10):
            # 15 MFMA tiles (d > 64) or the VALU Gram: the accumulators spill at the 128 VGPRs of
            # 4 blocks per CU
            self.lds = max(self.lds, (160 * 1024) // 3)
        self.gw = gram_width(d)


def _valu_gram(sh, slots):
    """4 x 4 f64 register blocks of the upper augmented Gram per thread, rows of the tile in
    row groups (VALU FMAs; any d)."""
    d, PP, NB, U, RG, GW = sh.d, sh.PP, sh.NB, sh.U, sh.RG, sh.gw
    acc_decl = "  double acc[16];\n#pragma unroll\n  for (int k = 0; k < 16; ++k) acc[k] = 0.0;\n"
    acc_decl += f"""  const int gu = tid % {U}, grg = tid / {U};
  const bool gact = tid < {U * RG};
  int bi = 0, brem = gu;
  while (brem >= {NB} - bi) {{ brem -= {NB} - bi; ++bi; }}
  const int bj = bi + brem;
"""
    gram_phase = f"""      if (gact) {{
    for (int r = grg; r < nr; r += {RG}) {{
      const double* __restrict__ gr = gt + r * {PP};
      const f64x2 a01 = *reinterpret_cast<const f64x2*>(gr + 4 * bi), a23 = *reinterpret_cast<const f64x2*>(gr + 4 * bi + 2);
      const f64x2 b01 = *reinterpret_cast<const f64x2*>(gr + 4 * bj), b23 = *reinterpret_cast<const f64x2*>(gr + 4 * bj + 2);
      const double av[4] = {{a01[0], a01[1], a23[0], a23[1]}}, bv[4] = {{b01[0], b01[1], b23[0], b23[1]}};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[4 * u + v] = __builtin_fma(av[u], bv[v], acc[4 * u + v]);
    }}
  }}
"""
    # every (i <= j) entry of the augmented upper triangle sits in exactly one 4 x 4 block:
    # each row group writes a complete gram_width slab (no zero fill needed)
    idx_tab = []
    for bI in range(NB):
        for bJ in range(bI, NB):
            for u in range(4):
                for v in range(4):
                    i, j = 4 * bI + u, 4 * bJ + v
                    k = _tile_slot(sh, i, j)
                    idx_tab.append(-1 if k is None else k)
    epilogue = f"""  if (gact) {{
DQG double* __restrict__ gp = (DQG double*)p[{slots['gpart']}] + ((long long)blockIdx.x * {RG} + grg) * {GW};
#pragma unroll
for (int k = 0; k < 16; ++k) {{
  const int slot = DQ_GIDX[gu * 16 + k];
  if (slot >= 0) gp[slot] = acc[k];
}}
  }}
"""
    tables = f"__device__ const short DQ_GIDX[{U * 16}] = {{{', '.join(str(x) for x in idx_tab)}}};\n"
    return acc_decl, gram_phase, epilogue, tables


def _mfma_gram(sh, slots):
    """The augmented Gram of the row tile on the matrix cores: v_mfma_f64_16x16x4_f64 per upper
    16 x 16 feature tile, 4 rows per k-step.  Lane l holds row (l >> 4) of the k-step and feature
    16 X + (l & 15) of panel X — one conflict-free ds_read_b64 per panel — for both operands
    (A = tile rows, B = tile columns), and accumulates D[(l >> 4) + 4 e][l & 15] in f64.  The three
    rows past the tile's last row are zeroed by the row phase (stale LDS never enters); feature
    columns past d + 2 read the next row's bytes and only reach discarded (padding) entries.  Waves split into G tile groups x
    4/G row groups; each row group writes a complete gram_width slab."""
    d, PP, GW, G, RG = sh.d, sh.PP, sh.gw, sh.G, sh.RG
    tiles = sh.tiles
    groups = [tiles[g::G] for g in range(G)]
    TW = max(len(t) for t in groups)
    acc_decl = (f"  typedef double f64x4 __attribute__((ext_vector_type(4)));\n"
                f"  f64x4 gacc[{TW}];\n#pragma unroll\n  for (int t = 0; t < {TW}; ++t) gacc[t] = f64x4{{0.0, 0.0, 0.0, 0.0}};\n"
                f"  const int gtg = __builtin_amdgcn_readfirstlane(wave) % {G}, grg = __builtin_amdgcn_readfirstlane(wave) / {G};\n")
    bodies = []
    for g, tl in enumerate(groups):
        panels = sorted({x for t in tl for x in t})
        first = "".join(f"          double pv{x} = gr[{16 * x}];\n" for x in panels)
        reads = "".join(f"            const double qv{x} = gq[{16 * x}];\n" for x in panels)
        mf = "".join(f"            gacc[{k}] = __builtin_amdgcn_mfma_f64_16x16x4f64(pv{I}, pv{J}, gacc[{k}], 0, 0, 0);\n"
                     for k, (I, J) in enumerate(tl))
        shift = "".join(f"            pv{x} = qv{x};\n" for x in panels)
        # unconditional panel reads (rows nr .. nr + 2 of the tile are zeroed by the row phase, so
        # no per-row select, which compiled to exec-masked loads and branches); the next k-step's
        # reads are issued beside this step's MFMAs (the last step re-reads its own rows)
        bodies.append(f"""        if (gtg == {g}) {{{{
          const int ki = 4 * grg < nr ? 4 * grg : 0;
          const double* __restrict__ gr = gt + (ki + (lane >> 4)) * {PP} + (lane & 15);
{first}          for (int k0 = 4 * grg; k0 < nr; k0 += {4 * RG}) {{{{
/*SRD*/
            const int kn = k0 + {4 * RG} < nr ? k0 + {4 * RG} : k0;
            const double* __restrict__ gq = gt + (kn + (lane >> 4)) * {PP} + (lane & 15);
{reads}{mf}/*SFM*/
{shift}          }}}}
        }}}}
""")
    gram_phase = "".join(bodies).replace("{{", "{").replace("}}", "}")
    # (lane, e) -> gram_width slot of each tile (-1: lower half of a diagonal tile or padding;
    # with the VALU strip, also the tiles' y and 1 columns)
    tabs = []
    for I, J in tiles:
        for lane in range(64):
            for e in range(4):
                i, j = 16 * I + (lane >> 4) + 4 * e, 16 * J + (lane & 15)
                k = None if sh.vstrip and max(i, j) >= d else _tile_slot(sh, i, j)
                tabs.append(-1 if k is None else k)
    tables = f"__device__ const short DQ_TIDX[{len(tiles) * 256}] = {{{', '.join(str(x) for x in tabs)}}};\n"
    if sh.vstrip:
        # the strip: lane l of every wave owns sums s = l + 64 k (x_c y for s < d, x_c for
        # d <= s < 2 d) over the rows r = wave (mod 4) of every tile; the row phase sums y, y^2
        # and the live rows per thread; both reduce once at the end in a fixed order
        KS = -(-2 * d // 64)
        assert 4 * 64 * KS + 12 <= (sh.RR + 3) * PP + 16  # the epilogue's scratch (the tile array)
        acc_decl += "".join(f"  double sacc{k} = 0.0;\n  const int sc{k} = (lane + {64 * k}) % {d}, "
                            f"sw{k} = lane + {64 * k} < {d} ? {d} : {d + 1};\n" for k in range(KS))
        acc_decl += "  double sn_ = 0.0, sy_ = 0.0, syy_ = 0.0;\n"
        # 4 rows per trip with every read issued before the FMAs (one row per trip had waited on
        # each read pair); wave w takes rows 4 w .. 4 w + 3 (mod 16), so a trip never passes the
        # three zeroed rows past the tile
        rd = "".join(f"            const double a{k}{u} = gs[{u * PP} + sc{k}], b{k}{u} = gs[{u * PP} + sw{k}];\n"
                     for u in range(4) for k in range(KS))
        fm4 = "".join(f"            sacc{k} = __builtin_fma(a{k}{u}, b{k}{u}, sacc{k});\n" for u in range(4) for k in range(KS))
        if G == 1:
            # inside the MFMA k-loop: the wave's k-steps are its strip rows, and the strip's
            # reads and FMAs run beside the k-step's MFMAs
            gram_phase = gram_phase.replace("/*SRD*/\n", f"            const double* __restrict__ gs = gt + k0 * {PP};\n" + rd)
            gram_phase = gram_phase.replace("/*SFM*/\n", fm4)
        else:
            gram_phase += f"""        for (int r = 4 * __builtin_amdgcn_readfirstlane(wave); r < nr; r += 16) {{
          const double* __restrict__ gs = gt + r * {PP};
{rd}{fm4}        }}
"""
        sl = []
        for s_ in range(64 * KS):
            k = _tile_slot(sh, s_ % d, d if s_ < d else d + 1) if s_ < 2 * d else None
            sl.append(-1 if k is None else k)
        sl += [_tile_slot(sh, d + 1, d + 1), _tile_slot(sh, d, d + 1), _tile_slot(sh, d, d)]
        tables += f"__device__ const short DQ_SSLOT[{len(sl)}] = {{{', '.join(str(x) for x in sl)}}};\n"
        red = "".join(f"""    {{
      double t = {v};
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
      if (lane == 0) gt[{4 * 64 * KS} + wave * 3 + {j}] = t;
    }}
""" for j, v in enumerate(("sn_", "sy_", "syy_")))
        strip_ep = (f"""  __syncthreads();  // (the tile array is the reduction scratch from here)
  {{
""" + "".join(f"    gt[wave * {64 * KS} + {64 * k} + lane] = sacc{k};\n" for k in range(KS)) + red + f"""  }}
  __syncthreads();
  if (wave == 0) {{
    DQG double* __restrict__ g0 = (DQG double*)p[{slots['gpart']}] + (long long)blockIdx.x * {RG * GW};
    for (int s = lane; s < {64 * KS + 3}; s += 64) {{
      const int slot = DQ_SSLOT[s];
      const int b = s < {64 * KS} ? s : {4 * 64 * KS} + (s - {64 * KS});
      const int st = s < {64 * KS} ? {64 * KS} : 3;
      if (slot >= 0) g0[slot] = (gt[b] + gt[b + st]) + (gt[b + 2 * st] + gt[b + 3 * st]);
    }}
  }}
""")
    else:
        strip_ep = ""
    ep = []
    for g, tl in enumerate(groups):
        wr = "".join(f"""      for (int e = 0; e < 4; ++e) {{
        const int slot = DQ_TIDX[{tiles.index(t) * 256} + lane * 4 + e];
        if (slot >= 0) gp[slot] = gacc[{k}][e];
      }}
""" for k, t in enumerate(tl))
        ep.append(f"    if (gtg == {g}) {{\n{wr}    }}\n")
    epilogue = (f"  {{\n    DQG double* __restrict__ gp = (DQG double*)p[{slots['gpart']}] + "
                f"((long long)blockIdx.x * {RG} + grg) * {GW};\n" + "".join(ep) + "  }\n" + strip_ep)
    gram_phase = gram_phase.replace("/*SRD*/\n", "").replace("/*SFM*/\n", "")
    return acc_decl, gram_phase, epilogue, tables


def _conv_loop(C, CU, PP, FW, crlf, conv_call, frame_load, div_expr, int_ok, us_expr, feat_store, quote=0,
               one_store=False, tile_all=False):
    """The field-conversion loop: one field per lane per iteration (field fb, then fb + 256), its
    positions prefetched one iteration ahead and its frame + sign loads issued before any wait.
    The field's row and column advance by 256 fields per iteration (a constant quotient and
    remainder of C: no per-field division, and the tile row bases by additions, no multiply).
    ``quote`` (QUOTED build: some fields are quoted fast-path numbers, ``"12.5"``): a quoted
    field's bounds move inside its quotes and its wave takes the position-based converter.
    (Two or three fields per lane per iteration lost to register spills: profiles/r3_csv_cutter.md.)"""
    cr = 1 if crlf else 0
    dq, dr = 256 // C, 256 % C
    if tile_all:
        q_init = f"      int q_ga = ((f0 + tid) / {C} - R0) * {PP} + q_c;  // its row-tile slot\n"
        q_step = (f"        q_c += {dr};\n        q_ga += {dq * PP + dr};\n"
                  f"        if (q_c >= {C}) {{\n          q_c -= {C};\n          q_ga += {PP - C};\n        }}\n")
    else:
        q_init = (f"      int q_vb = ((f0 + tid) / {C} - R0) * {CU}, q_gb = ((f0 + tid) / {C} - R0) * {PP};"
                  f"  // its tile rows\n")
        q_step = (f"        q_c += {dr};\n        q_vb += {dq * CU};\n        q_gb += {dq * PP};\n"
                  f"        if (q_c >= {C}) {{\n          q_c -= {C};\n          q_vb += {CU};\n          q_gb += {PP};\n"
                  f"        }}\n")
    fl_ = (frame_load.replace("fw0", "q_w0").replace("fw1", "q_w1").replace("fw2", "q_w2")
           .replace("const int c0 =", "const int q_c0 =").replace("stage[start]", "stage[q_start]")
           .replace("fwp", "q_wp").replace("+ end", "+ q_end").replace("^ start", "^ q_start")
           .replace("+ f;", "+ fb;").replace("(f & 1)", "(fb & 1)"))
    cc = conv_call.replace(chr(10) + "        ", chr(10) + "          ")
    fs = (feat_store.replace(f"rr * {PP}", "q_gb").replace("        const int fs", "            const int fs")
          .replace("        if (fs >= 0)", "            if (fs >= 0)"))
    if tile_all:  # every column has its own row-tile slot ([x | y | 1] order): the field's tile address
        store = "          gt[q_ga] = dv;\n"
    elif one_store:  # every column goes to exactly one tile (or nowhere): one store through a selected address
        store = (f"          const int us = {us_expr};\n"
                 + fs.replace("            if (fs >= 0) gt[q_gb + fs] = dv;\n", "").replace("            const", "          const")
                 + "          *(fs >= 0 ? gt + q_gb + fs : (us >= 0 ? vt + q_vb + us : &dq_sink)) = dv;\n")
    else:
        store = f"          const int us = {us_expr};\n          if (us >= 0) vt[q_vb + us] = dv;\n{fs}"
    if quote:
        bounds = (f"const int qs_ = q_c0 == {quote}, qe_ = stage[q_end - 1] == {quote};\n"
                  f"          const bool qany = (qs_ | qe_) != 0;\n"
                  f"          const int end = q_end - qe_, start = q_start + qs_, len = end - start, c = q_c;")
    else:
        bounds = "const int end = q_end, start = q_start, len = end - start, c = q_c;"
    return f"""      // (the next iteration's positions are loaded while this one converts)
      int q_p = 0, q_e = 0;
      if (f0 + tid < f1) {{
        q_p = dposx[f0 + tid];
        q_e = dposx[f0 + tid + 1];
      }}
      int q_c = (f0 + tid) % {C};                            // the field's column
{q_init}
      for (int fb = f0 + tid; fb < f1; fb += 256) {{
        const int q_fn = fb + 256 < f1 ? fb + 256 : fb;
        const int q_pn = dposx[q_fn], q_en = dposx[q_fn + 1];
        const int q_end = q_e;
        const int q_start = q_p + 1 + ({cr} && q_c == 0 ? 1 : 0);
        q_p = q_pn;
        q_e = q_en;
        const int q_fsh = (q_end - 8) & 3;
        const unsigned* q_wp = reinterpret_cast<const unsigned*>(stage + (q_end - 8 - q_fsh));
        {fl_}
        asm volatile("" :: "v"(q_w0), "v"(q_w1), "v"(q_w2), "v"(q_c0));  // one wait for the frame (else it sinks past the branch)
        {{
          {bounds}
          const int fsh = q_fsh;
          const unsigned fw0 = q_w0, fw1 = q_w1, fw2 = q_w2;
          const int c0 = {"qany ? stage[start] : " if quote else ""}q_c0;
          const bool neg0 = c0 == '-';
          const int fl = len - ((c0 == '-' || c0 == '+') ? 1 : 0);
          unsigned m = 0u;
          int fr = 0;
          bool neg = neg0, dot = false, ok;
          {cc}
          const double v = {div_expr};  // fr = 0 without a dot: 10^0 = 1, exact
          double dv = neg ? -v : v;
          ok = ok && {int_ok};
          if (slowp && len > {FW}) {{  // (an 8-byte-frame field is exact whatever its sign makes len)
            int ps = start;
            long long lv = 0;
            int ty = C_NULL;
            ok = csv_field_fast(stage, 0, ps, end, O.sep, dv, lv, ty) && ty != C_NULL && csv_conforms(ty, DQ_KIND[c]);
          }}
          bad |= !ok;
{store}        }}
        // the next field: 256 fields on = {dq} rows and {dr} columns on
{q_step}
      }}
"""


def kernel_source(g, kinds, used, opts: dict, H: int, slots: dict, d: int, term: int = 13, crlf: bool = False,
                  min_line: int = 1, waves_per_simd: int = 0, max_line: int = 1 << 30, quoted: bool = False):
    """Source of the cutter kernel and its ``_Shape``.  ``term``: the file's one terminator byte
    (13 CR, 10 LF; ``crlf``: every CR is followed by LF, which then opens the next row and is
    skipped); ``min_line``: the shortest line, sizing the delimiter array and the row tile."""
    from .dqvm import ptr_struct
    from .scanfuse import _gram_code, header_text

    C = len(kinds)
    NS = len(g.ptrs)
    vals = {}
    for t, v, s in g.stores:
        tag = g.recipe[s]
        if tag[0] == "outvalid":
            from .scanfuse import _GramNullable

            raise _GramNullable("gram mode: nullable outputs")
        if tag[0] == "out":
            vals[tag[1]] = v
    xs, yv = [vals[i] for i in range(d)], vals[d]
    feat = _passthrough(xs, used, d) if d > 8 else None
    ucols = sorted(used)
    if feat is not None:  # features go straight from the converter to the Gram tile
        body_text = "\n".join(g.lines) + "\n" + yv
        import re

        ucols = [c for c in ucols if re.search(rf"\bfzf{c}\b", body_text)]
    sh = _Shape(C, d, H, min_line, ucols, feat)
    # the converter's frame: 8 bytes when no field can be longer (line minus terminator and the
    # other fields' >= 2 bytes each), else 16 (longer fields take the byte-walking fast path)
    FW = 8 if max_line - 1 - 2 * (C - 1) <= 8 else 16
    # diagnostic ablations (timing only, results are wrong): 1 no field conversion, 2 no Gram
    # phase (the compiler then also drops the feature conversions: nothing reads the tile), 4 no
    # row phase, 8 nothing after the cut (stage, masks, scans, scatter only)
    abl = diag.ablation("DQ4ML_CUT_ABLATE")  # (refused without DQ4ML_DIAG=1)
    # diagnostic phase clocks (DQ4ML_CUT_STAMPS=1): s_memtime after each block barrier, per-phase
    # sums of wave 0 of every block -> the dbg slot ([grid][8] u64: phases 0-5, windows)
    stamps = os.environ.get("DQ4ML_CUT_STAMPS", "0") == "1" and "dbg" in slots
    if stamps:
        stamp_decl = ("  unsigned long long dq_ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n"
                      "  unsigned long long dq_t = __builtin_amdgcn_s_memtime();\n"
                      "#define DQ_STAMP(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); "
                      "dq_ph[k] += t_ - dq_t; dq_t = t_; } while (0)\n")
        stamp_out = (f"  if (tid == 0) {{\n    dq_ph[6] = (unsigned long long)(w1 - w0);\n"
                     f"    unsigned long long* dg = (unsigned long long*)p[{slots.get('dbg', 0)}] + blockIdx.x * 8;\n"
                     "#pragma unroll\n    for (int k = 0; k < 8; ++k) dg[k] = dq_ph[k];\n  }\n")
    else:
        stamp_decl, stamp_out = "#define DQ_STAMP(k) do { } while (0)\n", ""
    # an int32 column must hold no dot (a double column takes both classes): VALU, no table load
    ints = [c for c, k in enumerate(kinds) if int(k) == 1]
    int_ok = "(" + " || ".join(f"c == {c}" for c in ints) + ") ? !dot : true" if 0 < len(ints) <= 8 else (
        "true" if not ints else "csv_conforms(dot ? C_DOUBLE : C_INT, DQ_KIND[c])")
    # the quotient's power-of-ten pair from an LDS table (the VALU select chain measured slower:
    # profiles/r3_csv_cutter.md)
    div_expr = "csv_div_pow10_fma((double)m, p10t[fr], ip10t[fr])"  # (both converters give fr <= 15)
    if abl & 16:  # (diagnostic) no table read: the quotient's LDS round trip
        div_expr = "csv_div_pow10_fma((double)m, 1.0 + fr, 1.0)"
    frame_load = ("const unsigned fw0 = fwp[0], fw1 = fwp[1], fw2 = fwp[2];\n        const int c0 = stage[start];"
                  if not abl & 32 else  # (diagnostic) no frame / sign reads
                  "const unsigned fw0 = 0x31323334u + end, fw1 = 0x2E353637u ^ start, fw2 = 0x38393031u + f;\n"
                  "        const int c0 = 0x30 + (f & 1);")
    # the next window's prefetch: right after this window's bytes are staged ("early"), or after
    # the field conversion of its first tile round ("late": the 20 prefetch VGPRs are not live
    # across the converter, and the loads still have the row, Gram and stage phases to land)
    pf_early = ""
    pf_late = "      if (R0 == 0 && blk + 1 < w1) dq_fetch(ab, a, n, blk + 1, tid, pg, ph);\n"
    pf_tail = ("    if ((cnt == 0 || " + ("true" if abl & 8 else "false") + ") && blk + 1 < w1) "
               "dq_fetch(ab, a, n, blk + 1, tid, pg, ph);  // no tile round ran\n")
    qb = int(opts.get("quote", 34)) if quoted else 0
    # slowp (wave-uniform): some field of the wave is longer than the 8-byte frame (or quoted);
    # only such a wave can hold a field for the byte-walking path
    conv_call = ("const bool slowp = false;\n        ok = true; m = (unsigned)len;" if abl & 1 else
                 f"""const bool slowp = __ballot(fl > 8{" || qany" if qb else ""}) != 0ull;
        if (!slowp) {{
          ok = csv_num_r8q_w(fw0, fw1, fw2, fsh, fl, m, fr, dot);
        }} else {{  // (re-reads its frame: no register array lives across the branch)
          ok = csv_num_r<{FW // 4}>(stage, end, len < {FW} ? len : {FW}, m, fr, neg, dot);
        }}""")
    W, HG, DCAP, RR, CU, PP, NB, U, RG, GW = sh.W, sh.HG, sh.DCAP, sh.RR, sh.CU, sh.PP, sh.NB, sh.U, sh.RG, sh.gw
    usl = {c: i for i, c in enumerate(ucols)}
    sep = ord(opts.get("sep", ","))
    sep4 = f"0x{sep:02X}{sep:02X}{sep:02X}{sep:02X}u"
    term4 = f"0x{term:02X}{term:02X}{term:02X}{term:02X}u"
    # carried row starts (every window but a run's first) count the head's separators in phase 0
    # from the head granule registers — one barrier and phase less per window — when the head's
    # granules all sit in wave 0 (H <= 1024)
    hf = H <= 1024
    if hf:
        hraw_code = f"""    unsigned int hraw16 = 0u;  // separators of this lane's head granule (wave 0, lanes < {H // 16})
    if (tid < {H // 16}) {{
      const csv_u32x4 v = ph[0];
#pragma unroll
      for (int w = 0; w < 4; w += 2) hraw16 |= dq_gather8(dq_eq80(v[w], {sep4}), dq_eq80(v[w + 1], {sep4})) << (4 * w);
    }}
"""
        hscan_code = f"""    const bool hfast = st0 >= 0;  // a carried row start (block-uniform)
    unsigned int hm16 = 0u;
    int hinc = 0;
    if (hfast && wave == 0) {{
      if (lane < {H // 16}) {{
        const int lo = st0 - 16 * lane;
        hm16 = lo >= 16 ? 0u : (lo > 0 ? (hraw16 & (0xFFFFu << lo)) : hraw16);
      }}
      int hsum;
      hinc = dq_wave_prefix<5>(__popc(hm16), hsum) + __popc(hm16);
      if (lane == 0) shtot = hsum;
    }}
"""
    else:
        hraw_code = ""
        hscan_code = "    const bool hfast = false;\n    unsigned int hm16 = 0u;\n    int hinc = 0;\n"
    o = (f"{{(unsigned char){sep}, (unsigned char){int(opts['quote'])}, (unsigned char){int(opts['escape'])}, "
         f"(unsigned char)0, (unsigned char)0, (unsigned char)0, (unsigned char)0, (unsigned char)0, "
         f"{{{', '.join('0' for _ in range(16))}}}}}")
    body = ("\n".join("      " + ln.strip() for ln in g.lines).replace("P[", "p[")
            .replace("atomicOr((int*)p[", "dq_flag((unsigned int*)p["))
    loads = "".join((f"      const {ct} fzf{c} = ({ct})(gt[r * {sh.PP} + {c}]);\n" if sh.yfirst else
                     f"      const {ct} fzf{c} = ({ct})(vt[rb + {usl[c]}]);\n")
                    for c, ct in sorted(used.items()) if c in usl)
    # per column: its vt slot (-1: the chain does not read it) and its feature slot in the Gram
    # tile (-1: not a passthrough feature)
    ctab = []
    for c in range(C):
        ctab.append(usl.get(c, -1))
        ctab.append(feat.index(c) if feat is not None and c in feat else -1)
    if sh.blocked:
        outs = f"      double* __restrict__ gr = gt + r * {PP};\n"
        if feat is None:
            outs += "".join(f"      gr[{i}] = live ? (double)({v}) : 0.0;\n" for i, v in enumerate(xs))
        else:
            outs += f"      if (!live) {{\n#pragma unroll\n        for (int i = 0; i < {d}; ++i) gr[i] = 0.0;\n      }}\n"
        if sh.vstrip:  # (+ the strip's y, y^2 and count sums of this thread's rows)
            outs += (f"      const double yv_ = live ? (double)({yv}) : 0.0;\n      gr[{d}] = yv_;\n"
                     f"      gr[{d + 1}] = live ? 1.0 : 0.0;\n      sn_ += live ? 1.0 : 0.0;\n"
                     f"      sy_ += yv_;\n      syy_ = __builtin_fma(yv_, yv_, syy_);\n")
        elif sh.yfirst:  # (gr[d] held the label column, read above as a chain input)
            outs += f"      gr[{d}] = live ? (double)({yv}) : 0.0;\n      gr[{d + 1}] = live ? 1.0 : 0.0;\n"
        else:
            outs += f"      gr[{d}] = live ? 1.0 : 0.0;\n      gr[{d + 1}] = live ? (double)({yv}) : 0.0;\n"
        # (the padding columns d + 2 .. PP - 1 are zeroed once at kernel start: nothing writes them)
        if sh.mfma:
            acc_decl, gram_phase, epilogue, tables = _mfma_gram(sh, slots)
        else:
            acc_decl, gram_phase, epilogue, tables = _valu_gram(sh, slots)
        # (+3 rows + 16: the MFMA Gram's k-step and padding-column reads stay inside the array)
        gt_decl = f"  __shared__ __attribute__((aligned(16))) double gt[{(RR + 3) * PP + 16}];\n"
        # the MFMA Gram's last k-step reads up to three rows past the tile's rows: zeros
        gt_zero = (f"      for (int i = tid; i < {3 * PP}; i += 256) gt[nr * {PP} + i] = 0.0;\n" if sh.mfma else "")
        gt_init = (f"  for (int i = tid; i < {(RR + 3) * PP + 16}; i += 256) gt[i] = 0.0;  // (padding columns stay 0)\n"
                   f"  __syncthreads();\n")
    else:
        outs = _gram_code(xs, yv).replace("    if (live)", "      if (live)")
        acc_decl = f"  double acc[{GW}];\n#pragma unroll\n  for (int k = 0; k < {GW}; ++k) acc[k] = 0.0;\n"
        gram_phase = ""
        red = "".join(f"""  {{
    double t = acc[{k}];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) gred[wave][{k}] = t;
  }}
""" for k in range(GW))
        epilogue = f"""  __shared__ double gred[4][{GW}];
{red}  __syncthreads();
  if (tid < {GW})
    ((DQG double*)p[{slots['gpart']}])[(long long)blockIdx.x * {GW} + tid] =
        (gred[0][tid] + gred[1][tid]) + (gred[2][tid] + gred[3][tid]);
"""
        tables = ""
        gt_decl = gt_zero = gt_init = ""
    # column -> vt slot / Gram-tile feature slot: VALU selects for the common shapes, else the
    # LDS table
    if len(ucols) <= 6:
        us_expr = "".join(f"c == {cc} ? {i} : " for i, cc in enumerate(ucols)) + "-1"
    else:
        us_expr = "ctab[2 * c]"
    feat_store = ""
    if sh.blocked and feat is not None:
        if feat == list(range(feat[0], feat[0] + d)):
            fs_expr = f"(c >= {feat[0]} && c < {feat[0] + d}) ? c - {feat[0]} : -1"
        else:
            fs_expr = "ctab[2 * c + 1]"
        feat_store = (f"        const int fs = {fs_expr};\n"
                      f"        if (fs >= 0) gt[rr * {PP} + fs] = dv;\n")
    # no barrier at the window top: phase 0 writes only the stage, the cut and the scan words,
    # which the previous window finished reading before its row-phase barrier, so the previous
    # window's Gram (reading the row tile, written again only after this window's cut barrier)
    # overlaps this window's staging
    top_sync = ""
    # one store per field when no column feeds both the chain and the Gram tile directly
    one_store = sh.blocked and feat is not None and not set(feat) & set(ucols)
    conv_loop = _conv_loop(C, CU, PP, FW, crlf, conv_call, frame_load, div_expr, int_ok, us_expr, feat_store,
                           quote=qb, one_store=one_store, tile_all=sh.yfirst)
    # the lane's two 32-byte halves one after the other, each with 32-bit steps (find-first,
    # clear, store): ~5 VALU per delimiter instead of the 64-bit find-first's ~10
    win_scatter = f"""    {{
      int idx = htot + before;
      unsigned int mm = (unsigned int)dm;
      const int pa = {H} + 64 * tid;
      while (mm) {{
        dcut[idx++] = (unsigned short)(pa + __builtin_ctz(mm));
        mm &= mm - 1u;
      }}
      mm = (unsigned int)(dm >> 32);
      while (mm) {{
        dcut[idx++] = (unsigned short)(pa + 32 + __builtin_ctz(mm));
        mm &= mm - 1u;
      }}
    }}
"""
    if sep < 0x80 and term < 0x80:
        delim_body = (f"  const unsigned int a = ((v ^ {sep4}) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;\n"
                      f"  const unsigned int t = ((v ^ {term4}) & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;\n"
                      f"  return ~((a & t) | v) & 0x80808080u;")
    else:
        delim_body = f"  return dq_eq80(v, {sep4}) | dq_eq80(v, {term4});"
    kind_tab = ", ".join(str(int(k)) for k in kinds)
    lb = f"__launch_bounds__(256, {waves_per_simd})" if waves_per_simd else "__launch_bounds__(256)"
    src = ("#define CSV_UDOT4(a, b, c) __builtin_amdgcn_udot4((a), (b), (c), false)\n"
           "#define CSV_MUL24(a, b) __umul24((a), (b))\n"
           "#define CSV_ALIGNBIT(a, b, s) __builtin_amdgcn_alignbit((a), (b), (s))\n"
           "#define CSV_PERM(a, b, s) __builtin_amdgcn_perm((a), (b), (s))\n"
           "#define CSV_OPAQUE(x) asm(\"\" : \"+v\"(x))\n") + header_text() + f"""
using namespace dq4ml_csv;
typedef unsigned int csv_u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
#define DQG __attribute__((address_space(1)))

__device__ __forceinline__ void dq_flag(unsigned int* f, unsigned int v) {{
  __hip_atomic_fetch_or((DQG unsigned int*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}}
__device__ const unsigned char DQ_KIND[{C}] = {{{kind_tab}}};
__device__ const short DQ_CTAB[{2 * C}] = {{{', '.join(str(x) for x in ctab)}}};
{tables}
// 0x80 in every byte of v equal to the byte of pat
__device__ __forceinline__ unsigned int dq_eq80(unsigned int v, unsigned int pat) {{
  const unsigned int x = v ^ pat;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}}
// exclusive prefix sum of c over the wave's 64 lanes, and the wave total: an inclusive DPP scan,
// row_shr 1, 2, 4, 8 within each 16-lane row (zero fill), then row_bcast 15 / 31 across rows --
// six DPP adds, the total from lane 63 (seven ballot bit planes with mbcnt measured 3 % slower
// over the whole action, profiles/r5_cutter.md)
template <int B>
__device__ __forceinline__ int dq_wave_prefix(int c, int& total) {{
  int v = c;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  total = __builtin_amdgcn_readlane(v, 63);
  return v - c;
}}
// 0x80 in every byte of v that is the separator or the terminator.  A byte's low seven bits
// differ from a pattern's iff bit 7 of ((x & 0x7F) + 0x7F) is set (x = byte ^ pattern); both
// patterns are ASCII, so a match also needs bit 7 of the byte clear: 6 ops for both patterns
__device__ __forceinline__ unsigned int dq_delim80(unsigned int v) {{
{delim_body}
}}
// the 0x80 flags of two consecutive dwords gathered to bits 0..7 in byte order by ONE multiply:
// z0's flags sit at bits 8k, z1's at 8k + 4, and every (flag, magic bit) product lands on its own
// bit (none collide below bit 29), so bits 21..28 are the eight flags in order
__device__ __forceinline__ unsigned int dq_gather8(unsigned int z0, unsigned int z1) {{
  return ((((z0 >> 7) | (z1 >> 3)) * 0x00204081u) >> 21) & 0xFFu;
}}
// one window's granules: 64 bytes per lane, then the head (the row straddling into the window)
// and two tail granules; zero outside [0, n)
__device__ __forceinline__ void dq_fetch(const DQG unsigned char* ab, long long a, long long n, long long blk, int tid,
                                         csv_u32x4 (&pg)[4], csv_u32x4 (&ph)[{HG}]) {{
  const long long wbase = blk * {W} - a, sbase = wbase - {H}, tb = wbase + 64 * tid;
#pragma unroll
  for (int j = 0; j < 4; ++j) {{
    const long long gi = tb + 16 * j;
    pg[j] = (gi < n && gi + 16 > 0) ? *reinterpret_cast<const DQG csv_u32x4*>(ab + gi + a) : csv_u32x4{{0u, 0u, 0u, 0u}};
  }}
#pragma unroll
  for (int i = 0; i < {HG}; ++i) {{
    const int gq = tid + 256 * i;
    const long long gi = gq < {H // 16} ? sbase + 16 * gq : wbase + {W} + 16 * (gq - {H // 16});
    ph[i] = (gq < {H // 16} + 2 && gi < n && gi + 16 > 0) ? *reinterpret_cast<const DQG csv_u32x4*>(ab + gi + a)
                                                          : csv_u32x4{{0u, 0u, 0u, 0u}};
  }}
}}

{ptr_struct(NS)}extern "C" __global__ {lb} void {ENTRY}(const DqPtrs P, long long n) {{
  void* p[{NS}];
#pragma unroll
  for (int i = 0; i < {NS}; ++i) p[i] = P.v[i];
  const DQG unsigned char* __restrict__ b = (const DQG unsigned char*)p[{slots['buf']}];
  const long long nwin = (long long)p[{slots['nwin']}];
  const bool trailing = (long long)p[{slots['trailing']}] != 0;
  unsigned int* vflag = (unsigned int*)p[{slots['vflag']}];
  __shared__ __attribute__((aligned(16))) unsigned char stage_raw[16 + {H} + {W} + 32];
  unsigned char* const stage = stage_raw + 16;  // 16 readable bytes below stage[0] (right-aligned reads)
  __shared__ unsigned short dpos[{DCAP} + 1];
  unsigned short* const dposx = dpos;  // dposx[0]: the delimiter before the window's first field
  unsigned short* const dcut = dpos + 1;  // the window's delimiters
  __shared__ __attribute__((aligned(16))) double vt[{RR * CU}];
{gt_decl}  __shared__ short ctab[{2 * C}];
  __shared__ int wtot[4], shtot, sst0;
  __shared__ double dq_sink;  // the store of a field no tile reads
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long a = (long long)(reinterpret_cast<unsigned long long>(b) & 15ull);
  const DQG unsigned char* ab = b - a;  // 16-byte aligned view
  const CsvOpts O = {o};
  bool bad = false;
{stamp_decl}  for (int i = tid; i < {2 * C}; i += 256) ctab[i] = DQ_CTAB[i];
  __shared__ double p10t[16], ip10t[16];  // 10^k and RN(10^-k) for the converter (k > 9: unused)
  if (tid < 16) {{
    p10t[tid] = tid <= 9 ? csv_pow10(tid) : 1.0;
    ip10t[tid] = tid <= 9 ? csv_inv_pow10(tid) : 1.0;
  }}
{acc_decl}{gt_init}
  // a CONTIGUOUS run of windows per block: the row start of window k+1 is carried from the cut
  // of window k (only the first window searches back for it), and window k+1's bytes are in
  // flight (registers) while window k is cut
  const long long w0 = nwin * blockIdx.x / gridDim.x, w1 = nwin * (blockIdx.x + 1) / gridDim.x;
  csv_u32x4 pg[4], ph[{HG}];
  if (w0 < w1) dq_fetch(ab, a, n, w0, tid, pg, ph);
  int st0 = -1;  // stage index of the window's first row (block-uniform; -1: search)
  for (long long blk = w0; blk < w1; ++blk) {{
    const long long wbase = blk * {W} - a;  // buffer index of window byte 0
    const long long sbase = wbase - {H};    // buffer index of stage[0]
    const long long tb = wbase + 64 * tid;  // this lane's 64 window bytes
{top_sync}    DQ_STAMP(5);
    unsigned int dlo = 0u, dhi = 0u;  // delimiter (separator or terminator) bits of the 64 bytes
#pragma unroll
    for (int j = 0; j < 4; ++j) {{
      const csv_u32x4 v = pg[j];
      *reinterpret_cast<csv_u32x4*>(stage + {H} + 64 * tid + 16 * j) = v;
#pragma unroll
      for (int w = 0; w < 4; w += 2) {{
        const unsigned int g8 = dq_gather8(dq_delim80(v[w]), dq_delim80(v[w + 1]));
        if (j < 2) dlo |= g8 << (16 * j + 4 * w);
        else dhi |= g8 << (16 * (j - 2) + 4 * w);
      }}
    }}
#pragma unroll
    for (int i = 0; i < {HG}; ++i) {{  // head granules + two tail granules
      const int gq = tid + 256 * i;
      if (gq < {H // 16} + 2)
        *reinterpret_cast<csv_u32x4*>(stage + (gq < {H // 16} ? 16 * gq : {H} + {W} + 16 * (gq - {H // 16}))) = ph[i];
    }}
{hraw_code}{pf_early}
    unsigned long long dm = ((unsigned long long)dhi << 32) | dlo;
    {{
      const long long lo = tb < 0 ? -tb : 0, hi = n - tb;
      if (lo > 0 || hi < 64) {{  // bytes before the buffer (aligned granule) or past its end
        const unsigned long long keep_lo = lo >= 64 ? 0ull : (~0ull << lo);
        const unsigned long long keep_hi = hi <= 0 ? 0ull : (hi >= 64 ? ~0ull : ((1ull << hi) - 1));
        dm &= keep_lo & keep_hi;
      }}
      if (trailing && hi >= 0 && hi < 64) dm |= 1ull << hi;  // the last line's virtual terminator at n
    }}
    const int cd = __popcll(dm);
    int wsum;
    const int inc = dq_wave_prefix<7>(cd, wsum) + cd;
    if (lane == 0) wtot[wave] = wsum;
{hscan_code}
    if (st0 < 0) __syncthreads();  // (block-uniform) wave 0 reads the other waves' head stores below
    if (st0 < 0 && wave == 0) {{
      // the first window of the run: the terminator before its first row, through the staged head
      long long found = -2;
      for (int k0 = 0; k0 < {H} && found == -2; k0 += 64) {{
        const long long q = wbase - 1 - k0 - lane;
        const bool t = q < 0 || stage[{H} - 1 - k0 - lane] == {term};
        const unsigned long long bal = __ballot(t);
        if (bal) found = wbase - 1 - k0 - (long long)__builtin_ctzll(bal);
      }}
      for (long long q0 = wbase - 1 - {H}; found == -2; q0 -= 64) {{  // longer than the head (fact violation)
        const long long q = q0 - lane;
        const bool t = q < 0 || b[q] == {term};
        const unsigned long long bal = __ballot(t);
        if (bal) found = q0 - (long long)__builtin_ctzll(bal);
      }}
      if (lane == 0) sst0 = (int)(found < 0 ? -sbase : found + 1 + {1 if crlf else 0} - sbase);
    }}
    __syncthreads();
    DQ_STAMP(0);
    if (st0 < 0) st0 = sst0;
    if (st0 < 0 || st0 > {H} + 1) {{  // a row longer than the head: the max-line fact is wrong
      bad = true;
      break;  // block-uniform
    }}
    int before = inc - cd;
    for (int w = 0; w < wave; ++w) before += wtot[w];
    const int dwin = (wtot[0] + wtot[1]) + (wtot[2] + wtot[3]);
    // separators of the first row's head part [st0, H) (no terminator can be there): for a
    // carried row start they were counted above from the head granule registers (H <= 1024)
    unsigned long long hm = 0ull;
    if (!hfast && tid < {H // 64}) {{
#pragma unroll
      for (int j = 0; j < 4; ++j) {{
        const csv_u32x4 v = *reinterpret_cast<const csv_u32x4*>(stage + 64 * tid + 16 * j);
#pragma unroll
        for (int w = 0; w < 4; w += 2)
          hm |= (unsigned long long)dq_gather8(dq_eq80(v[w], {sep4}), dq_eq80(v[w + 1], {sep4})) << (16 * j + 4 * w);
      }}
      const int lo = st0 - 64 * tid;
      hm = lo >= 64 ? 0ull : (lo > 0 ? (hm & (~0ull << lo)) : hm);
    }}
    if (!hfast) {{  // (block-uniform) the first window of the run
      hinc = __popcll(hm);
      if (wave == 0) {{
        int hsum;
        hinc += dq_wave_prefix<7>(hinc, hsum);
        if (lane == 0) shtot = hsum;
      }}
      __syncthreads();
    }}
    DQ_STAMP(1);
    const int htot = shtot;
    const int ftot = htot + dwin;      // delimiters from the first row's start on
    const int cnt = ftot / {C};        // complete rows (every row holds exactly {C} fields)
    if (ftot > {DCAP}) {{  // more delimiters than any window of valid lines holds
      bad = true;
      break;  // block-uniform
    }}
    // the cut: every delimiter's stage position, in byte order, after the sentinel (the
    // delimiter "before" the first field: its start minus one, minus the LF of a CR LF)
    if (tid == 0) dposx[0] = (unsigned short)(st0 - 1 - {1 if crlf else 0});
    if (hm) {{
      int idx = hinc - __popcll(hm);
      unsigned long long mm = hm;
      while (mm) {{
        const int bit = __builtin_ctzll(mm);
        mm &= mm - 1;
        dcut[idx++] = (unsigned short)(64 * tid + bit);
      }}
    }}
    if (hfast && hm16) {{
      int idx = hinc - __popc(hm16);
      unsigned int mm = hm16;
      while (mm) {{
        const int bit = __builtin_ctz(mm);
        mm &= mm - 1;
        dcut[idx++] = (unsigned short)(16 * tid + bit);
      }}
    }}
{win_scatter}
    __syncthreads();
    DQ_STAMP(2);
    // the next window's first row starts after this window's last complete row
    const int nst0 = cnt > 0 ? (int)dcut[cnt * {C} - 1] + 1 + {1 if crlf else 0} - {W} : st0 - {W};
    for (int R0 = 0; R0 < {"0" if abl & 8 else "cnt"}; R0 += {RR}) {{
      const int nr = min({RR}, cnt - R0), f0 = R0 * {C}, f1 = f0 + nr * {C};
      if (R0 > 0) __syncthreads();  // the previous round's Gram readers are done with the tiles
      // one field per lane: the sign byte, then the unsigned part through the 8-byte 64-bit SWAR
      // frame when every field of the wave fits it (wave-uniform branch), else the 16-byte frame;
      // fields longer than that take the byte-walking fast path (rare, divergent)
{conv_loop}
{pf_late}      __syncthreads();
      DQ_STAMP(3);
      for (int r = tid; r < nr; r += 256) {{  // one row per thread: the DQ chain and the assembler
        const int rb = r * {CU};
{loads}        const bool line = true;
        bool live = line;
{body if not abl & 4 else ""}
{outs if not abl & 4 else ""}      }}
{gt_zero}      __syncthreads();
      DQ_STAMP(4);
{gram_phase if not abl & 2 else ""}    }}
{pf_tail}    st0 = nst0;
  }}
  if (bad) dq_flag(vflag, 1u);
{stamp_out}
{epilogue}}}
"""
    return src, sh


# ---------------------------------------------------------------------------------------------
_CACHE: dict = {}


class _CutPlan:
    def __init__(self, src, g, refs, sh, per_cu):
        self.src, self.recipe, self.has_raise, self.refs = src, list(g.recipe), g.has_raise, refs
        self.sh, self.per_cu = sh, per_cu
        self.rg = sh.RG


def blocks_per_cu(lds: int) -> int:
    """Resident 256-thread blocks per CU the cutter is built for (160 KiB LDS, at most 4)."""
    return int(max(1, min(4, (160 * 1024) // max(lds, 1))))


# Below this mean line length (bytes) the per-line kernel (scanfuse.py) wins for d <= 8: a short
# row is one lane's few SWAR steps there, while the cutter pays its per-field cut and row-tile
# round trip (lab CSV, 9.2-byte rows: 1.60 vs 1.75 ms per action, same box).
MIN_MEAN_LINE = 24


def _compile(nodes, rel, d: int):
    from . import dqvm
    from .scanfuse import _GramNullable, _ScanBase, _scan_gen

    f = rel.fused
    H = applicable(f)
    if H is None:
        return None
    if d <= 8 and float(f.get("mean_line", 0.0)) < float(os.environ.get("DQ4ML_CUT_MIN_LINE", MIN_MEAN_LINE)):
        return None
    term, crlf = term_of(f)
    min_line = int(f.get("min_line", 1))
    (parts, udfs), refs = dqvm.nodes_key(nodes)
    # (diagnostic builds only: DQ4ML_CUT_ABLATE timing ablations, DQ4ML_CUT_STAMPS phase clocks;
    # the losing A/B alternatives of rounds 2-3 -- VALU powers of ten, early prefetch, slow head
    # scan, 2 fields per lane, top-of-window barrier, other tile sizes -- were removed in round 4;
    # round 5's -- lane-owned conversion without the position array, the split-half scatter --
    # are measured in profiles/r5_cutter.md and were not kept)
    quoted = not f.get("fast_only") and bool(f.get("quoted_fast"))
    key = (parts, udfs, tuple(rel.schema().names), tuple(f["kinds"]), repr(sorted(f["opts"].items())), H, d, term,
           crlf, min_line, int(f.get("max_line", 1 << 30)), quoted, os.environ.get("DQ4ML_CUT_ABLATE"),
           os.environ.get("DQ4ML_CUT_STAMPS"), os.environ.get("DQ4ML_CUT_VSTRIP"))
    if key in _CACHE:
        return _CACHE[key]
    base = _ScanBase(rel.schema(), 0, f["device"])
    g = _scan_gen(base, f["nullable"])
    cp = None
    try:
        _, g, outputs, _ = dqvm.compile_chain(nodes, base, False, gen=g)
        names = ("buf", "nwin", "trailing", "vflag", "gpart") + (
            ("dbg",) if os.environ.get("DQ4ML_CUT_STAMPS", "0") == "1" else ())
        slots = {k: g.slot(None, (k,)) for k in names}
        ml = int(f.get("max_line", 1 << 30))
        _, sh = kernel_source(g, f["kinds"], g.used, f["opts"], H, slots, d, term, crlf, min_line, 0, ml, quoted)
        per_cu = blocks_per_cu(sh.lds)
        src, sh = kernel_source(g, f["kinds"], g.used, f["opts"], H, slots, d, term, crlf, min_line, per_cu, ml,
                                quoted)
        cp = _CutPlan(src, g, refs, sh, per_cu)
    except (dqvm.Unfusable, _GramNullable):
        cp = None
    if len(_CACHE) >= 64:
        _CACHE.clear()
    _CACHE[key] = cp
    return cp


_grid_cache: dict = {}


def _grid(h, per_cu: int, nwin: int) -> int:
    dev = torch.cuda.current_device()
    cus = _grid_cache.get(dev)
    if cus is None:
        cus = _grid_cache[dev] = int(h.device_info()["multiProcessorCount"])
    return int(max(1, min(nwin, cus * per_cu)))


def n_windows(buf_ptr: int, n: int) -> int:
    """Windows covering buffer bytes [0, n] (byte n: the last line's virtual terminator); window
    k spans [k W - a, (k + 1) W - a) with a = the buffer's misalignment to 16 bytes."""
    return (n + (buf_ptr & 15)) // WINDOW + 1


def try_cut_gram(chain, rel, d: int):
    """Launch the cutter for the Gram action (``scanfuse.try_fused_gram``'s chain with the
    features as ``__gx<i>`` and the label as ``__gy``).  Returns (flat statistics, err, vflag,
    stream) or None when the facts / chain do not allow it."""
    cp = _compile(chain, rel, d)
    if cp is None:
        return None
    return launch_cut(cp, rel, d)


def launch_cut(cp, rel, d: int):
    """One launch of the compiled cutter ``cp`` over ``rel``'s device bytes (the part of
    ``try_cut_gram`` a replayed action repeats)."""
    from . import native
    from ..runtime import faststream
    from ..utils import tracing
    from .scanfuse import window_fold

    f = rel.fused
    h = native.hip()
    dev = f["device"]
    buf, n = f["buf"], int(f["n"])
    nwin = n_windows(buf.data_ptr(), n)
    grid = _grid(h, cp.per_cu, nwin)
    gw = gram_width(d)
    # one zeroed allocation: [err, vflag | per-block partials]
    z = torch.zeros(1 + grid * cp.rg * gw, dtype=torch.int64, device=dev)
    ev = z[:1].view(torch.int32)
    err, vflag = ev[0:1], ev[1:2]
    gpart = z[1:].view(torch.float64).view(grid * cp.rg, gw)
    scalars = {"buf": buf, "nwin": nwin, "trailing": int(f["trailing"]), "vflag": vflag, "gpart": gpart}
    if any(t[0] == "dbg" for t in cp.recipe):
        LAST_STAMPS["buf"] = scalars["dbg"] = torch.zeros(grid, 8, dtype=torch.int64, device=dev)
    ptrs = []
    for tag in cp.recipe:
        k = tag[0]
        if k == "err":
            ptrs.append(err.data_ptr())
        elif k in ("sel", "out", "outvalid", "selout"):
            ptrs.append(0)
        elif k in scalars:
            x = scalars[k]
            ptrs.append(x.data_ptr() if torch.is_tensor(x) else int(x))
        else:
            raise AssertionError(f"cut plan: unbound slot {tag}")
    from .dqvm import launch, rtc_handle

    handle = rtc_handle(h, cp, cp.src, ENTRY)
    stream = faststream.current(faststream.dev_index(dev))
    with tracing.span("csv_cut_gram"):
        launch(h, handle, grid, ptrs, n, stream.cuda_stream)
        flat = window_fold(gpart, stream)
    tracing.add_rows("csv_cut_gram", int(f["nlines"]))
    STATS["cut_grams"] += 1
    return flat, err, vflag, cp
