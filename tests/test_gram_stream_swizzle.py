"""LDS image of the streamed tall Gram kernels (ops/csrc/hip/gram_stream.hip), checked on the CPU.

Each 1-KiB LDS-DMA piece is lane-linear (lane l writes bytes [16 l, 16 l + 16) of the piece), so
the kernels permute the SOURCE chunk per lane: slot p of feature f holds chunk p ^ g(f).  These
tests re-derive, for every (storage dtype, tile width, stage rows) variant the kernels
instantiate, that

  * the DMA mapping covers every (feature, chunk) exactly once (no chunk lost or read twice);
  * every ds_read_b128 a lane issues for its rows is bank-conflict free under the gfx950 lane
    groups of ds_read_b128 (MI355X_MICROARCH.md §LDS: four 16-lane groups, one LDS cycle each);
  * the identity layout (no swizzle) WOULD conflict, i.e. the swizzle is load-bearing.
"""
import pytest

# ds_read_b128 lane groups on gfx950
_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
           list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
_GROUPS += [[l + 32 for l in g] for g in _GROUPS]


def swz16(f, cpl):  # f64 kernel (16-feature tiles), gram_stream.hip swz16<CPL>
    return f ^ (cpl if 4 <= f <= 11 else 0)


def swz32(f, cpl=4):  # f32-storage kernels (32-feature tiles), gram_stream.hip swz32<CPL>
    return f & 15 if cpl == 4 else (f >> 1) & 7


# (name, element bytes, tile features TF, stage rows RS)
VARIANTS = [("f64 storage, d<=32", 8, 16, 64), ("f64 storage, d>32", 8, 16, 32),
            ("f32 storage, f64 stats", 4, 16, 64), ("f32 storage, exact-f32 stats", 4, 32, 64),
            ("f32 storage, 64 features, 32-row stages", 4, 32, 32)]


def _geom(esz, tf, rs):
    feat_bytes = rs * esz
    cpf = feat_bytes // 16
    return feat_bytes, cpf, cpf // 4 if tf == 16 else cpf // 2


def _g(tf, cpl):
    # f32 kernels: the swizzle is keyed by chunks-per-feature / 4 (4 at 64 rows, 2 at 32 rows)
    return (lambda f: swz16(f, cpl)) if tf == 16 else (lambda f: swz32(f, cpl // 2))


def _lane_chunks(lane, tf, cpl):
    """(feature, chunk list) a lane reads in the MFMA phase."""
    if tf == 16:  # lane (f = l & 15, q = l >> 4): rows [q*E, q*E + E) = chunks [q*CPL, q*CPL + CPL)
        f, q = lane & 15, lane >> 4
    else:  # lane (f = l & 31, h = l >> 5): rows [32h, 32h + 32)
        f, q = lane & 31, lane >> 5
    return f, [q * cpl + i for i in range(cpl)]


@pytest.mark.parametrize("name,esz,tf,rs", VARIANTS)
def test_dma_mapping_is_a_bijection(name, esz, tf, rs):
    feat_bytes, cpf, cpl = _geom(esz, tf, rs)
    g = _g(tf, cpl)
    pieces = tf * feat_bytes // 1024
    seen = set()
    for k in range(pieces):
        for lane in range(64):
            slot = k * 64 + lane
            fl, p = divmod(slot, cpf)
            c = p ^ g(fl)
            assert 0 <= c < cpf
            seen.add((fl, c))
    assert len(seen) == tf * cpf


def _max_conflict(esz, tf, rs, g):
    feat_bytes, cpf, cpl = _geom(esz, tf, rs)
    worst = 1
    for i in range(cpl):
        for grp in _GROUPS:
            banks = {}
            for lane in grp:
                f, chunks = _lane_chunks(lane, tf, cpl)
                addr = f * feat_bytes + (chunks[i] ^ g(f)) * 16
                banks.setdefault((addr // 16) % 16, set()).add(addr)  # 16-B slot = 4 banks of 64
            worst = max(worst, max(len(v) for v in banks.values()))
    return worst


@pytest.mark.parametrize("name,esz,tf,rs", VARIANTS)
def test_reads_are_conflict_free(name, esz, tf, rs):
    _, _, cpl = _geom(esz, tf, rs)
    assert _max_conflict(esz, tf, rs, _g(tf, cpl)) == 1


@pytest.mark.parametrize("name,esz,tf,rs", VARIANTS)
def test_identity_layout_would_conflict(name, esz, tf, rs):
    assert _max_conflict(esz, tf, rs, lambda f: 0) > 1
