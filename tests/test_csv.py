"""CSV reader contract: host scanner on CPU, device scanner (K1/K2) on the MI355X."""
import numpy as np
import pytest
import torch

from conftest import data_path
from net.jgp.labs.sparkdq4ml_amd.ops import native
from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import merge_type_mask, shard_byte_range

CASES = {
    "cr_only": b"1,23.1\r2,30.0\r3,34.5",
    "lf_trailing": b"1,2.5\n-3,4e2\n7,-0.125\n",
    "crlf": b"10,1\r\n20,2\r\n30,3.75\r\n",
    "empty_lines": b"1,2\n\n3,4\n\n",
    "short_rows": b"1,2,3\n4,5\n6\n",
    "long_ints": b"1,3000000000\n2,-5\n",
    "nulls": b"1,,3\n,2.5,\n",
    "bools": b"true,1\nFALSE,2\n",
    "special": b"NaN,1\n-Infinity,2\n1.5d,3\n",
    # the parser's one-walk fast path ([+-]digits[.digits], <= 9 digits) and its edges
    "fast_path_edges": b"-0,+5,007\n.5,5.,-.5\n123456789,1234567890,0.000000001\n-0.0,99999.9999,-123.456789\n",
    "fast_path_strings": b"-,1\n+,2\n",
    "fast_path_dots": b"1..2,3\n4,5\n",
}


def _fuzz_numeric(seed=11, rows=3000):
    """Random numeric tokens around the fast path's limits (digit counts 1..15, signs, dots,
    exponents, leading zeros) — all inside the device parser's exact range, so no host fallback —
    checked against the host scanner."""
    import random

    rnd = random.Random(seed)

    def tok():
        nd = rnd.choice([1, 2, 3, 8, 9, 10, 12, 15])
        digits = "".join(rnd.choice("0123456789") for _ in range(nd))
        sign = rnd.choice(["", "", "-", "+"])
        k = rnd.random()
        if k < 0.35:
            return sign + digits
        if k < 0.85:
            d = rnd.randint(0, nd)
            return sign + digits[:d] + "." + digits[d:] if nd > 0 else sign + "0.5"
        return sign + digits[:3] + "e" + str(rnd.randint(-7, 7))

    return "\n".join(",".join(tok() for _ in range(3)) for _ in range(rows)).encode()


CASES["fuzz_numeric"] = _fuzz_numeric()


def _host(data, infer=True):
    n, cols = native.host().csv_scan(data, infer=infer)
    return n, [(c[0], c[1], c[2], c[3]) for c in cols]


def test_type_lattice():
    h = native.host()
    assert h.csv_infer_field("12") == 1 and h.csv_infer_field("3000000000") == 2
    assert h.csv_infer_field("123456789012345678901234") == 3 and h.csv_infer_field("1.5") == 4
    assert h.csv_infer_field("true") == 5 and h.csv_infer_field("abc") == 6 and h.csv_infer_field("") == 0
    assert h.csv_merge_types(1, 4) == 4 and h.csv_merge_types(1, 2) == 2 and h.csv_merge_types(5, 1) == 6
    assert merge_type_mask(0b10010) == 4 and merge_type_mask(0b100000) == 5 and merge_type_mask(0b100010) == 6


def test_host_cases():
    n, cols = _host(CASES["cr_only"])
    assert n == 3 and [c[1] for c in cols] == [1, 4]
    n, cols = _host(CASES["empty_lines"])
    assert n == 2
    n, cols = _host(CASES["short_rows"])
    assert n == 3 and list(cols[2][3]) == [1, 0, 0] and list(cols[1][3]) == [1, 1, 0]
    n, cols = _host(CASES["long_ints"])
    assert cols[1][1] == 2
    n, cols = _host(CASES["nulls"])
    assert list(cols[0][3]) == [1, 0] and list(cols[1][3]) == [0, 1]
    n, cols = _host(b'"a,b",1\n"c""d",2\n')
    assert cols[0][1] == 6 and cols[0][2] == ["a,b", 'c"d']


def test_reader_schema_and_options(cpu_session, tmp_path):
    df = cpu_session.read().format("csv").option("inferSchema", "true").option("header", "false") \
        .load(data_path("dataset-full.csv"))
    assert [(f.name, f.dataType.simpleString()) for f in df.schema.fields] == [("_c0", "int"), ("_c1", "double")]
    assert df.count() == 1040
    p = tmp_path / "h.csv"
    p.write_bytes(b"a;b\n1;x\n2;y\n")
    df = cpu_session.read().option("header", "true").option("sep", ";").csv(str(p))
    assert df.columns == ["a", "b"] and [r.b for r in df.collect()] == ["x", "y"]
    df = cpu_session.read().schema("a double, b string").option("sep", ";").option("header", "true").csv(str(p))
    assert df.schema.fields[0].dataType.simpleString() == "double"
    # no inferSchema: all strings
    df = cpu_session.read().csv(data_path("dataset-small.csv"))
    assert df.dtypes == [("_c0", "string"), ("_c1", "string")]


def test_shard_byte_range_covers_rows():
    data = open(data_path("dataset-full.csv"), "rb").read()
    for world in (2, 3, 8):
        spans = [shard_byte_range(data, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == len(data)
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        rows = sum(_host(data[lo:hi])[0] for lo, hi in spans)
        assert rows == 1040


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES) + ["dataset-small.csv", "dataset-abstract.csv", "dataset-full.csv"])
def test_device_scan_matches_host(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    data = CASES[name] if name in CASES else open(data_path(name), "rb").read()
    t = csvscan.scan_device(data, device="cuda")
    n, cols = _host(data)
    if any(c[1] == 3 for c in cols):
        assert t is None  # decimals go to the host scanner
        return
    assert t is not None and t.nrows == n
    for (name_, code, vals, valid), c in zip(cols, t.columns):
        v = c.valid_mask().cpu().numpy()
        assert list(v.astype(int)) == list(valid.astype(int))
        if code == 6:  # a device string column (field spans; text built on the host)
            assert [x for x, ok in zip(c.values, valid) if ok] == [x for x, ok in zip(vals, valid) if ok]
            continue
        got = c.values.cpu().numpy()
        ref = np.asarray(vals)
        if code == 5:
            ref = ref.astype(bool)
        np.testing.assert_array_equal(np.where(valid.astype(bool), got.astype(np.float64), 0),
                                      np.where(valid.astype(bool), ref.astype(np.float64), 0))


@pytest.mark.gpu
def test_device_scan_types_hint():
    """A correct types_hint stores typed columns directly (same table); a wrong one is caught by
    the inference masks and the scan re-runs unhinted."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    data = b"1,2.5,true\n-3,4,false\n\n5,,TRUE\n,1e3,false"
    ref = csvscan.scan_device(data, device="cuda")
    codes = [csvscan.type_code_of(f.dataType) for f in ref.schema.fields]
    assert codes == [csvscan.CT_INT, csvscan.CT_DOUBLE, csvscan.CT_BOOL]
    for hint in (codes, [csvscan.CT_INT, csvscan.CT_INT, csvscan.CT_BOOL]):
        before = csvscan.STATS.get("hint_misses", 0)
        t = csvscan.scan_device(data, device="cuda", types_hint=hint)
        assert t.schema == ref.schema and t.nrows == ref.nrows == 4
        for a, b in zip(t.columns, ref.columns):
            assert a.values.dtype == b.values.dtype
            assert torch.equal(a.valid_mask(), b.valid_mask())
            m = a.valid_mask()
            assert torch.equal(a.values[m], b.values[m])
        assert csvscan.STATS.get("hint_misses", 0) - before == (0 if hint == codes else 1)


@pytest.mark.gpu
def test_device_scan_through_reader(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    rng = np.random.default_rng(0)
    n = 200_000
    a = rng.integers(-1000, 1000, n)
    b = np.round(rng.normal(size=n), 4)
    p = tmp_path / "big.csv"
    p.write_text("\n".join(f"{int(x)},{float(y)!r}" for x, y in zip(a, b)))
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", 0).getOrCreate()
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    before = csvscan.STATS["device_scans"]
    df = spark.read().option("inferSchema", "true").csv(str(p))
    assert csvscan.STATS["device_scans"] == before + 1
    t = df._table()
    assert t.columns[0].values.is_cuda and df.dtypes == [("_c0", "int"), ("_c1", "double")]
    np.testing.assert_array_equal(t.columns[0].values.cpu().numpy(), a)
    np.testing.assert_array_equal(t.columns[1].values.cpu().numpy(), b)
    spark.stop()


def test_chunk_bounds_are_row_aligned():
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import chunk_bounds

    data = open(data_path("dataset-full.csv"), "rb").read() + b"\r\n1,2\n3,4.5"
    for cb in (7, 100, 1000, len(data) + 5):
        b = chunk_bounds(data, cb)
        assert b[0] == 0 and b[-1] == len(data) and all(x < y for x, y in zip(b, b[1:]))
        assert all(data[x - 1] in (10, 13) for x in b[1:-1])  # every cut follows a terminator
        assert all(not (data[x - 1] == 13 and data[x] == 10) for x in b[1:-1])  # never inside CRLF
        assert sum(_host(data[x:y])[0] for x, y in zip(b, b[1:])) == _host(data)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [997, 64 << 10])
def test_device_chunked_scan_matches_one_shot(chunk):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    rng = np.random.default_rng(1)
    n = 50_000
    lines = [f"{int(x)},{float(y)!r},{int(z)}" for x, y, z in
             zip(rng.integers(-99, 99, n), np.round(rng.normal(size=n), 3), rng.integers(0, 2**40, n))]
    lines[1234] = "7,,"  # nulls
    lines[40000] = "3,2.5,12.75"  # widens the third column to double late in the file
    data = ("\r\n".join(lines[:30000]) + "\n\n" + "\n".join(lines[30000:])).encode()
    one = csvscan.scan_device(data, device="cuda")
    before = csvscan.STATS["chunks"]
    many = csvscan.scan_device(data, device="cuda", chunk_bytes=chunk)
    assert csvscan.STATS["chunks"] - before > 1
    assert one.nrows == many.nrows == n
    assert [c.dtype.simpleString() for c in many.columns] == ["int", "double", "double"]
    for a, b in zip(one.columns, many.columns):
        assert torch.equal(a.values, b.values)
        assert torch.equal(a.valid_mask(), b.valid_mask())


@pytest.mark.gpu
def test_pinned_file_cache_chunked_reader_and_file_change(tmp_path):
    """Large single files go through the pinned host file cache (runtime.filecache) and the
    chunked ring with direct DMA; a rewritten file must not be served from a stale copy."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    rng = np.random.default_rng(5)
    n = 120_000
    g = rng.integers(1, 36, n)
    pr = np.round(rng.uniform(3, 199, n), 2)
    p = tmp_path / "lab.csv"
    p.write_bytes("\r".join(f"{int(x)},{float(y)!r}" for x, y in zip(g, pr)).encode())  # CR-only, no final CR
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", 0) \
        .config("dq4ml.chunkBytes", 64 << 10).config("dq4ml.csv.deviceCache", "false").getOrCreate()
    before = csvscan.STATS["chunks"]
    for _ in range(2):  # second action: cached pinned copy, chunks DMA'd through the ring
        t = spark.read().option("inferSchema", "true").csv(str(p))._table()
        np.testing.assert_array_equal(t.columns[0].values.cpu().numpy(), g)
        np.testing.assert_array_equal(t.columns[1].values.cpu().numpy(), pr)
    assert csvscan.STATS["chunks"] - before > 4
    spark.conf.set("dq4ml.csv.deviceCache", "true")
    for _ in range(2):  # HBM-resident input bytes
        t = spark.read().option("inferSchema", "true").csv(str(p))._table()
        np.testing.assert_array_equal(t.columns[0].values.cpu().numpy(), g)
        np.testing.assert_array_equal(t.columns[1].values.cpu().numpy(), pr)
    pf = filecache.open_pinned(str(p))
    assert pf.host.is_pinned() and pf is filecache.open_pinned(str(p))
    import os
    import time

    time.sleep(0.01)
    p.write_bytes(b"1,2.5\r3,4.25")
    os.utime(p, ns=(time.time_ns(), time.time_ns()))
    t = spark.read().option("inferSchema", "true").csv(str(p))._table()
    assert t.nrows == 2 and t.columns[1].values.cpu().tolist() == [2.5, 4.25]
    filecache.clear()
    spark.stop()


@pytest.mark.gpu
def test_file_larger_than_pinned_cache_streams_from_a_map(tmp_path, monkeypatch):
    """A file above filecache.MAX_BYTES is never copied whole: a read-only map is streamed
    through the pinned staging ring, and nothing enters the pinned cache."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    filecache.clear()
    rng = np.random.default_rng(9)
    n = 50_000
    g = rng.integers(1, 36, n)
    pr = np.round(rng.uniform(3, 199, n), 2)
    p = tmp_path / "big.csv"
    p.write_bytes("\r".join(f"{int(x)},{float(y)!r}" for x, y in zip(g, pr)).encode())
    monkeypatch.setattr(filecache, "MAX_BYTES", 1 << 16)
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", 0) \
        .config("dq4ml.chunkBytes", 64 << 10).getOrCreate()
    t = spark.read().option("inferSchema", "true").csv(str(p))._table()
    np.testing.assert_array_equal(t.columns[0].values.cpu().numpy(), g)
    np.testing.assert_array_equal(t.columns[1].values.cpu().numpy(), pr)
    assert not filecache._cache
    spark.stop()


def test_shard_range_matches_in_memory_sharding(tmp_path):
    """runtime.filecache.shard_range (windowed reads around the cut points) must give exactly the
    byte ranges of ops.csvscan.shard_byte_range (the whole-buffer Hadoop-split rule)."""
    import random

    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import shard_byte_range
    from net.jgp.labs.sparkdq4ml_amd.runtime.filecache import shard_range

    rnd = random.Random(7)
    p = tmp_path / "s.csv"
    for trial in range(25):
        parts = []
        for i in range(rnd.randint(1, 200)):
            parts.append(b"%d,%d" % (rnd.randint(0, 10 ** rnd.randint(0, 8)), i))
            parts.append(rnd.choice([b"\n", b"\r", b"\r\n"]))
        if rnd.random() < 0.5:
            parts.pop()
        data = b"".join(parts)
        p.write_bytes(data)
        for world in (1, 2, 3, 8):
            for r in range(world):
                assert shard_range(str(p), r, world) == shard_byte_range(data, r, world), (trial, world, r)


def test_filecache_keeps_other_ranges_of_unchanged_file(tmp_path, monkeypatch):
    """Two byte ranges of one unchanged file stay cached side by side; a rewrite evicts both."""
    import os
    import time

    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache

    class _Dummy:
        def __init__(self, path, lo, hi):
            self.nbytes = hi - lo

    monkeypatch.setattr(filecache, "PinnedFile", _Dummy)
    filecache.clear()
    p = tmp_path / "a.csv"
    p.write_bytes(b"1,2\r3,4\r5,6")
    a, b = filecache.open_pinned(str(p), 0, 4), filecache.open_pinned(str(p), 4, 11)
    assert filecache.open_pinned(str(p), 0, 4) is a and filecache.open_pinned(str(p), 4, 11) is b
    p.write_bytes(b"1,2\r3,4\r5,7")
    os.utime(p, ns=(time.time_ns() + 10**9, time.time_ns() + 10**9))
    a2 = filecache.open_pinned(str(p), 0, 4)
    assert a2 is not a and len(filecache._cache) == 1
    filecache.clear()


def _fuzz_csv(rng, n, header, null_tok, spaces, comment):
    lines = []
    if comment:
        lines.append("# a comment line before the header")
    if header:
        lines.append(" id , price,ok,big " if spaces else "id,price,ok,big")
    for i in range(n):
        r = rng.random()
        if comment and r < 0.02:
            lines.append("#" + "skip me,1,2")
            continue
        if r < 0.03:
            lines.append("")
            continue
        f = [str(int(rng.integers(-10**6, 10**6))), repr(round(float(rng.normal()) * 100, 3)),
             "true" if rng.random() < 0.5 else "FALSE", str(int(rng.integers(-2**40, 2**40)))]
        for k in range(4):
            u = rng.random()
            if u < 0.05:
                f[k] = null_tok
            elif u < 0.07:
                f[k] = ""
        if spaces:
            f = [(" " * int(rng.integers(0, 3))) + x + ("\t" if rng.random() < 0.3 else "") for x in f]
        lines.append(",".join(f))
    return "\n".join(lines).encode()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["header", "header_schema", "null_value", "whitespace", "comment", "schema_bad"])
def test_device_reader_options_match_host(tmp_path, case):
    """Reader options on the device scanner (header, user schema, nullValue, whitespace trims,
    comment lines): same rows, types and names as the host scanner, and the device path is
    actually taken."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    import zlib

    rng = np.random.default_rng(zlib.crc32(case.encode()) % 1000)  # (hash() is salted per process)
    opts = {"inferSchema": "true"}
    schema = None
    header = case in ("header", "header_schema", "whitespace", "comment")
    null_tok = "NA" if case == "null_value" else ""
    data = _fuzz_csv(rng, 5000, header, null_tok, case == "whitespace", case == "comment")
    if header:
        opts["header"] = "true"
    if case == "null_value":
        opts["nullValue"] = "NA"
    if case == "whitespace":
        opts["ignoreLeadingWhiteSpace"] = "true"
        opts["ignoreTrailingWhiteSpace"] = "true"
    if case == "comment":
        opts["comment"] = "#"
    if case in ("header_schema", "schema_bad"):
        schema = "a INT, b DOUBLE, c BOOLEAN, d LONG"
        if case == "schema_bad":  # values the schema's types do not accept -> all-null records
            data = data + b"\n1.5,2,true,3\nx,1,false,2\n7,8,maybe,9\n3,4,true,99999999999999999"
    p = tmp_path / f"{case}.csv"
    p.write_bytes(data)

    def read(threshold):
        s = SparkSession.getActiveSession()
        if s is not None:
            s.stop()
        spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes",
                                                                  threshold).getOrCreate()
        r = spark.read()
        for k, v in opts.items():
            r = r.option(k, v)
        if schema:
            r = r.schema(schema)
        before = csvscan.STATS["device_scans"]
        df = r.csv(str(p))
        took = csvscan.STATS["device_scans"] - before
        out = (df.dtypes, [tuple(x) for x in df.collect()], took)
        spark.stop()
        return out

    dev_types, dev_rows, took = read(0)
    host_types, host_rows, _ = read(1 << 40)
    assert took == 1, "the device scanner did not take the read"
    assert dev_types == host_types
    assert len(dev_rows) == len(host_rows)

    def same(a, b):
        if a is None or b is None:
            return a is b
        if isinstance(a, float) and a != a:
            return b != b
        return a == b

    for ra, rb in zip(dev_rows, host_rows):
        assert all(same(a, b) for a, b in zip(ra, rb)), (ra, rb)


def test_device_column_count_skips_empty_and_comment_lines():
    # Spark drops empty lines (and comment lines) before it tokenizes the first record; the device
    # scanner's column count follows (a leading empty line used to give one column)
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import _ncols_of

    assert _ncols_of(b"\n\na,b,c\n1,2,3", ",") == 3
    assert _ncols_of(b"\r\r1,2\r", ",") == 2
    assert _ncols_of(b"a,b\r\n1,2", ",") == 2
    assert _ncols_of(b"#x,y\na,b,c,d\n", ",", ord("#")) == 4
    assert _ncols_of(b"1,2,3", ",") == 3
    assert _ncols_of(b"", ",") == 1 and _ncols_of(b"\n\n", ",") == 1
    big = b"\n" * 5 + b"x" * (1 << 17) + b",y\n"  # the first real line runs past the first head window
    assert _ncols_of(big, ",") == 2


def _quoted(data: bytes, frac: float, seed: int, sep_inside: bool = False) -> bytes:
    """``data`` with a fraction of its fields wrapped in quotes (CR / LF terminators kept)."""
    rng = np.random.default_rng(seed)
    out = []
    for line in data.replace(b"\r\n", b"\n").replace(b"\r", b"\n").split(b"\n"):
        fs = line.split(b",")
        fs = [b'"' + f + b'"' if f and rng.random() < frac else f for f in fs]
        out.append(b",".join(fs))
    return b"\r".join(out)


def test_split_record_matches_host_tokenizer():
    """``ops.csvscan.split_record`` (the host-side header splitter, mirror of the device parser's
    quoting) against the native univocity-style tokenizer on quoted / escaped records."""
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import _count_fields, split_record

    lines = [b'1,"2.5",3', b'"a,b",c', b'"x""y",z', b'"p\\"q",1', b'a\\"b,2', b'"",7', b'"1",,""', b'"u"v,w']
    for line in lines:
        n, cols = _host(line + b"\n" + line, infer=True)
        fields = split_record(line, ord(","), 34, 92)
        assert len(fields) == len(cols) == _count_fields(line, ord(","), 34, 92), line
        h = native.host()
        for (t, null), c in zip(fields, cols):
            cls = 0 if null else h.csv_infer_field(t.decode())
            if cls != 0:  # (an all-null column's type is the host's default)
                assert c[1] == cls, (line, t, c[1], cls)


@pytest.mark.gpu
@pytest.mark.parametrize("name,frac", [("dataset-full.csv", 1.0), ("dataset-full.csv", 0.4),
                                       ("dataset-abstract.csv", 0.5), ("fuzz_numeric", 0.5)])
def test_device_scan_of_quoted_fields_matches_host(name, frac):
    """quoted numeric fields parse on the device (no host fallback) and equal the
    host scanner's values and types."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    data = CASES[name] if name in CASES else open(data_path(name), "rb").read()
    q = _quoted(data, frac, 3)
    before = csvscan.STATS["fallbacks"]
    t = csvscan.scan_device(q, device="cuda")
    assert t is not None and csvscan.STATS["fallbacks"] == before, "quoted numeric fields fell back to the host"
    n, cols = _host(q)
    assert t.nrows == n
    for (name_, code, vals, valid), c in zip(cols, t.columns):
        assert list(c.valid_mask().cpu().numpy().astype(int)) == list(valid.astype(int))
        got, ref = c.values.cpu().numpy().astype(np.float64), np.asarray(vals).astype(np.float64)
        np.testing.assert_array_equal(np.where(valid.astype(bool), got, 0), np.where(valid.astype(bool), ref, 0))


@pytest.mark.gpu
def test_device_reader_quoted_header_and_large_quoted_file(tmp_path):
    """A quoted header and a 1e6-row quoted numeric file through the reader: device scan taken,
    no fallback, same rows as the host scanner."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    rng = np.random.default_rng(5)
    n = 1_000_000
    g = rng.integers(1, 36, n)
    pr = np.round(5.0 * g + 20 + rng.normal(0, 3, n), 2)
    body = "\r".join(f'"{a}","{b:.2f}"' for a, b in zip(g.tolist(), pr.tolist()))
    p = tmp_path / "q.csv"
    p.write_bytes(('"guest","price"\r' + body).encode())
    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    b0, f0 = csvscan.STATS["device_scans"], csvscan.STATS["fallbacks"]
    df = spark.read().option("header", "true").option("inferSchema", "true").csv(str(p))
    assert df.columns == ["guest", "price"]
    assert [t for _, t in df.dtypes] == ["int", "double"]
    assert csvscan.STATS["device_scans"] == b0 + 1 and csvscan.STATS["fallbacks"] == f0
    assert df.count() == n
    got = np.asarray([r[1] for r in df.limit(1000).collect()])
    np.testing.assert_allclose(got, pr[:1000], rtol=0, atol=1e-9)
    spark.stop()


def _span_ref(line: bytes, pos: int, sep: int, quote: int, escape: int):
    """Python mirror of the device's ``csv_field_span`` (csv_parse_dev.h): (fs, fe, raw, next pos)."""
    n, c, raw = len(line), pos, False
    if c < n and line[c] == quote:
        raw, c = True, c + 1
        while c < n:
            ch = line[c]
            if escape != quote and ch == escape and c + 1 < n and line[c + 1] in (quote, escape):
                c += 2
            elif ch == quote:
                if c + 1 < n and line[c + 1] == quote:
                    c += 2
                else:
                    c += 1
                    break
            else:
                c += 1
    while c < n and line[c] != sep:
        raw |= line[c] == escape
        c += 1
    return pos, c, raw, c + 1


def _string_fuzz(rng, rows: int, ncols: int = 4) -> list:
    """Records of string-ish fields: separators / doubled quotes / escapes inside quotes, quoted
    empties, unquoted quotes, escape-led tokens, unicode, spaces."""
    toks = ['a', 'plain text', '"a,b"', '"x""y"', '"p\\"q"', '"\\\\"', '""', '', 'u"v', '\\N', '\\"w',
            '"1,5"', '"abc"tail', ' pad ', '"  sp  "', 'café', '"niño, s.a."', '7', '-3.5', '"12"', 'true']
    out = []
    for _ in range(rows):
        out.append(",".join(toks[int(rng.integers(0, len(toks)))] for _ in range(ncols)).encode())
    return out


@pytest.mark.parametrize("trim", [False, True])
def test_csv_strings_materializer_matches_tokenizer(trim):
    """The host half of the device string columns: spans cut the device's way (``_span_ref``),
    packed like the kernel stores them, then ``csv_strings`` builds the text -- equal to what the
    univocity tokenizer (``split_record``) yields for every field."""
    from net.jgp.labs.sparkdq4ml_amd.ops.csvscan import split_record

    rng = np.random.default_rng(3)
    lines = _string_fuzz(rng, 3000, 5)
    data = b"\n".join(lines)
    spans, valid, want = [], [], []
    base = 0
    for line in lines:
        pos = 0
        fields = split_record(line, ord(","), 34, 92, b"", trim, trim)
        for text, null in fields:
            fs, fe, raw, pos = _span_ref(line, pos, ord(","), 34, 92)
            spans.append(((base + fs) << 25) | (int(raw) << 24) | (fe - fs))
            quoted = line[fs:fs + 1] == b'"'
            valid.append(0 if (not quoted and fe == fs) else 1)
            want.append(None if null else text.decode("utf-8"))
        assert pos == len(line) + 1  # the spans cover the record exactly as the tokenizer splits it
        base += len(line) + 1
    got = native.host().csv_strings(data, np.array(spans, dtype=np.int64), np.array(valid, dtype=np.uint8),
                                    ignore_leading_ws=trim, ignore_trailing_ws=trim)
    assert got == want


TS_CASES = {  # token -> expected datetime (None: not a timestamp)
    "2019-01-01": (2019, 1, 1), "2019-1-5": (2019, 1, 5), "2019-02-30": (2019, 3, 2),  # Date.valueOf is lenient
    "2019-01-01 10:20:30": (2019, 1, 1, 10, 20, 30), "2019-01-01 10:20:30.5": (2019, 1, 1, 10, 20, 30, 500000),
    "2019-01-01 1:2:3": (2019, 1, 1, 1, 2, 3), "2019-01-01 10:20:30.123456789": (2019, 1, 1, 10, 20, 30, 123000),
    "2019-01-01T10:20:30": (2019, 1, 1, 10, 20, 30), "2019-01-01T10:20:30Z": (2019, 1, 1, 10, 20, 30),
    "2019-01-01T10:20:30.25+01:00": (2019, 1, 1, 9, 20, 30, 250000), "2020-02-29T23:59:59-00:30": (2020, 3, 1, 0, 29, 59),
    "1970-01-01": (1970, 1, 1), "1600-03-01": (1600, 3, 1), "9999-12-31 23:59:59": (9999, 12, 31, 23, 59, 59),
    "2019-1-01T10:20:30": None, "2019-02-30T00:00:00": None, "1599-12-31": None, "20190101": None,
    "2019-13-01": None, "2019-01-01 10:20": None, "2019-01-01x": None, "2019-01-01 10:20:30.": None,
    "2019-01-01T10:20:30+1:00": None, "2019-01-01T24:00:00": None, "2019-01-32": None, "2019/01/01": None,
    "2019-01-01  10:20:30": None, "T10:20:30": None,
}


def test_timestamp_parser_and_inference():
    """SURVEY S03's lattice step double -> timestamp -> boolean: Spark 2.4's fallback timestamp
    parsers (Date.valueOf, Timestamp.valueOf, xsd:dateTime) in the host scanner, UTC, millisecond
    precision; a timestamp merges only with timestamps."""
    import datetime

    h = native.host()
    for tok, want in TS_CASES.items():
        got = h.csv_parse_timestamp(tok)
        if want is None:
            assert got is None, tok
        else:
            ref = datetime.datetime(*want) - datetime.datetime(1970, 1, 1)
            assert got == (ref.days * 86400 + ref.seconds) * 1_000_000 + ref.microseconds, tok
            assert h.csv_infer_field(tok) == 7, tok
    assert h.csv_merge_types(7, 7) == 7 and h.csv_merge_types(7, 0) == 7
    assert h.csv_merge_types(7, 4) == 6 and h.csv_merge_types(1, 7) == 6 and h.csv_merge_types(7, 5) == 6
    assert merge_type_mask((1 << 7) | 1) == 7 and merge_type_mask((1 << 7) | (1 << 4)) == 6
    n, cols = _host(b"2019-01-01,1\n2019-02-01 10:00:00.5,2019-01-01\n,x")
    assert [c[1] for c in cols] == [7, 6]
    assert list(cols[0][3]) == [1, 1, 0]


def test_timestamp_column_collect_and_show(cpu_session, tmp_path):
    """A timestamp column through the reader (host scanner on CPU): collect() gives datetimes,
    show() prints Spark's ``yyyy-MM-dd HH:mm:ss[.fff]``."""
    import datetime

    p = tmp_path / "ts.csv"
    p.write_bytes(b"2019-01-01,1\r2019-06-15 08:30:00.25,2\r,3")
    df = cpu_session.read().option("inferSchema", "true").csv(str(p))
    assert df.dtypes == [("_c0", "timestamp"), ("_c1", "int")]
    rows = df.collect()
    assert rows[0][0] == datetime.datetime(2019, 1, 1) and rows[2][0] is None
    assert rows[1][0] == datetime.datetime(2019, 6, 15, 8, 30, 0, 250000)
    out = df._show_string(20, 20) if hasattr(df, "_show_string") else None
    if out is None:
        from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import _cell_str

        assert _cell_str(rows[1][0]) == "2019-06-15 08:30:00.25" and _cell_str(rows[0][0]) == "2019-01-01 00:00:00"
    else:
        assert "2019-06-15 08:30:00.25" in out and "2019-01-01 00:00:00|" in out


@pytest.mark.gpu
def test_device_timestamps_match_host():
    """The device parser's timestamps (csv_parse_dev.h csv_parse_ts) equal the host scanner's:
    every TS_CASES token's class, a 5000-row column of mixed formats (inferred, then under a user
    schema), values in microseconds."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan

    for tok in TS_CASES:
        data = f"{tok},1\n{tok},2".encode()
        t = csvscan.scan_device(data, device="cuda")
        _, cols = _host(data)
        assert t is not None and csvscan.type_code_of(t.schema.fields[0].dataType) == cols[0][1], tok
    valid = [t for t, w in TS_CASES.items() if w is not None]
    data = "\n".join(f"{valid[i % len(valid)]},{i}" if i % 7 else f",{i}" for i in range(5000)).encode()
    _, cols = _host(data)
    assert cols[0][1] == csvscan.CT_TIMESTAMP
    for t in (csvscan.scan_device(data, device="cuda"),
              csvscan.scan_device(data, device="cuda", user_types=[csvscan.CT_TIMESTAMP, csvscan.CT_INT])):
        assert t is not None and csvscan.type_code_of(t.schema.fields[0].dataType) == csvscan.CT_TIMESTAMP
        c = t.columns[0]
        ok = cols[0][3].astype(bool)
        assert np.array_equal(c.valid_mask().cpu().numpy(), ok)
        np.testing.assert_array_equal(c.values.cpu().numpy()[ok], np.asarray(cols[0][2])[ok])


def test_device_string_column_moves_spans_until_read():
    """``DeviceStringColumn`` (the device scan's string column): row selections move only the
    spans, the validity mask needs no text, and the strings are built once, on first read."""
    from net.jgp.labs.sparkdq4ml_amd.sql.table import DeviceStringColumn, Table
    from net.jgp.labs.sparkdq4ml_amd.sql.types import StringType, StructField, StructType

    data = b'ab,"c,d",x""y,\xc3\xa9'
    fields = [(0, 2, 0), (3, 5, 1), (9, 4, 0), (14, 2, 0)]  # (fs, len, raw)
    spans = torch.tensor([(fs << 25) | (raw << 24) | ln for fs, ln, raw in fields], dtype=torch.int64)
    col = DeviceStringColumn(spans, None, data, {"quote": '"', "escape": "\\"})
    assert col.n == 4 and bool(col.valid_mask().all()) and not col.materialized
    sub = col.index(torch.tensor([3, 1]))
    assert isinstance(sub, DeviceStringColumn) and not col.materialized
    assert sub.values == ["é", "c,d"]
    assert col.slice(0, 2).values == ["ab", "c,d"] and not col.materialized
    assert col.values == ["ab", "c,d", 'x""y', "é"]  # (x""y is unquoted: its bytes as they stand)
    t = Table(StructType([StructField("s", StringType(), True)]), [col], 4, torch.tensor([True, False, True, True]))
    assert [r[0] for r in t.to_rows()] == ["ab", 'x""y', "é"]


def test_string_equality_filter_keeps_device_strings_lazy(monkeypatch):
    """``filter(col = 'text')`` over a device string column: the engine's planning (the fused
    chain's structural key, the filter, the projection) never builds the column's strings; the
    comparison itself is ``eq_literal`` (here a CPU stand-in for the HBM span compare)."""
    from net.jgp.labs.sparkdq4ml_amd import SparkSession, col
    from net.jgp.labs.sparkdq4ml_amd.sql.dataframe import DataFrame
    from net.jgp.labs.sparkdq4ml_amd.sql.plan import LocalRelation
    from net.jgp.labs.sparkdq4ml_amd.sql.table import ColumnData, DeviceStringColumn, Table
    from net.jgp.labs.sparkdq4ml_amd.sql.types import IntegerType, StringType, StructField, StructType

    data = b"ab,x,ab,abc"
    fields = [(0, 2), (3, 1), (5, 2), (8, 3)]
    spans = torch.tensor([(fs << 25) | ln for fs, ln in fields], dtype=torch.int64)

    def eq_literal(self, lit):
        b = lit.encode()
        out = []
        for v in self.spans.tolist():
            fs, ln = v >> 25, v & 0xFFFFFF
            out.append(data[fs:fs + ln] == b)
        return torch.tensor(out, dtype=torch.bool)

    monkeypatch.setattr(DeviceStringColumn, "eq_literal", eq_literal)
    s = DeviceStringColumn(spans, None, data, {"quote": '"', "escape": "\\"})
    ids = ColumnData(IntegerType(), torch.arange(4, dtype=torch.int32))
    schema = StructType([StructField("i", IntegerType(), False), StructField("s", StringType(), True)])
    spark = SparkSession.builder().master("local[*]").getOrCreate()
    df = DataFrame(LocalRelation(Table(schema, [ids, s], 4)), spark)
    assert [r[0] for r in df.filter(col("s") == "ab").select("i").collect()] == [0, 2]
    assert df.filter(col("s") != "ab").count() == 2
    from net.jgp.labs.sparkdq4ml_amd.ops import dqvm

    dqvm._chain_key([df.filter(col("s") == "ab")._plan], df._plan.table)  # (the GPU executor's key)
    assert not s.materialized


def test_mapped_input_string_check(tmp_path):
    """Strings of a device scan over a file MAP (inputs above the pinned cache) are built from the
    file's own pages: a changed file raises instead of yielding other bytes (or a SIGBUS)."""
    from net.jgp.labs.sparkdq4ml_amd.runtime import filecache
    from net.jgp.labs.sparkdq4ml_amd.sql.readwriter import _map_check

    p = tmp_path / "m.csv"
    p.write_bytes(b"a,1\nb,2\n")
    mf = filecache.open_mapped(str(p))
    chk = _map_check(mf)
    chk()
    class Owned:  # a pinned-cache entry: an owned host copy
        host = object()

    assert _map_check(Owned()) is None and _map_check(None) is None
    import os
    import time

    time.sleep(0.01)
    p.write_bytes(b"a,1\nb,2\nc,3\n")
    os.utime(p)
    with pytest.raises(RuntimeError, match="changed after it was scanned"):
        chk()
    filecache.clear()


def test_timestamp_casts(cpu_session, tmp_path):
    """Spark 2.4 casts around TimestampType: to string (``yyyy-MM-dd HH:mm:ss[.f]``), to long
    (whole seconds, floor) and double (fractional seconds), from strings (the reader's parser;
    null when it does not parse) and from seconds."""
    import datetime

    p = tmp_path / "ts.csv"
    p.write_bytes(b"1969-12-31 23:59:59.5,2019-06-15\r2019-06-15 08:30:00.25,bad\r")
    df = cpu_session.read().option("inferSchema", "true").csv(str(p))
    assert df.dtypes == [("_c0", "timestamp"), ("_c1", "string")]
    df.createOrReplaceTempView("t")
    rows = cpu_session.sql("SELECT CAST(_c0 AS STRING) s, CAST(_c0 AS LONG) l, CAST(_c0 AS DOUBLE) d, "
                           "CAST(_c1 AS TIMESTAMP) t2, CAST(CAST(_c0 AS LONG) AS TIMESTAMP) t3 FROM t").collect()
    assert [tuple(r) for r in rows] == [
        ("1969-12-31 23:59:59.5", -1, -0.5, datetime.datetime(2019, 6, 15), datetime.datetime(1969, 12, 31, 23, 59, 59)),
        ("2019-06-15 08:30:00.25", 1560587400, 1560587400.25, None, datetime.datetime(2019, 6, 15, 8, 30)),
    ]


def test_timestamp_comparisons(cpu_session, tmp_path):
    """A timestamp compared with a string literal: Spark 2.4's ``findCommonTypeForBinaryComparison``
    maps (timestamp, string) to string, so the timestamp is printed (``yyyy-MM-dd HH:mm:ss[.f]``)
    and the two compare as text (Spark 3.0 would cast the string to a timestamp instead)."""
    p = tmp_path / "ts.csv"
    p.write_bytes(b"2019-01-01,1\r2019-06-15 08:30:00,2\r2020-02-29T12:00:00Z,3\r")
    df = cpu_session.read().option("inferSchema", "true").csv(str(p))
    df.createOrReplaceTempView("t")
    got = [r[0] for r in cpu_session.sql("SELECT _c1 FROM t WHERE _c0 >= '2019-06-15 08:30:00'").collect()]
    assert got == [2, 3]
    got = [r[0] for r in cpu_session.sql("SELECT _c1 FROM t WHERE _c0 < '2019-03-01'").collect()]
    assert got == [1]
    # the rules differ on date-only literals: a midnight timestamp prints as '2019-01-01 00:00:00',
    # which is neither equal to nor <= the text '2019-01-01' (3.0's instant rule gives row 1 both times)
    assert cpu_session.sql("SELECT _c1 FROM t WHERE _c0 = '2019-01-01'").collect() == []
    assert cpu_session.sql("SELECT _c1 FROM t WHERE _c0 <= '2019-01-01'").collect() == []
    got = [r[0] for r in cpu_session.sql("SELECT _c1 FROM t WHERE _c0 > '2019'").collect()]
    assert got == [1, 2, 3]  # text order: every '2019-…' / '2020-…' string sorts after '2019'
    got = [r[0] for r in cpu_session.sql("SELECT _c1 FROM t WHERE '2019-06-15 08:30:00' = _c0").collect()]
    assert got == [2]


def test_timestamp_csv_write_round_trip(cpu_session, tmp_path):
    """The CSV writer prints timestamps in the source's default ``timestampFormat``
    (``yyyy-MM-dd'T'HH:mm:ss.SSSXXX``); reading them back gives the same instants."""
    p = tmp_path / "ts.csv"
    p.write_bytes(b"2019-06-15 08:30:00.25,1\r1999-12-31,2\r")
    df = cpu_session.read().option("inferSchema", "true").csv(str(p))
    out = str(tmp_path / "out")
    df.write().csv(out)
    text = open(tmp_path / "out" / "part-00000.csv").read()
    assert text.splitlines()[0] == "2019-06-15T08:30:00.250Z,1"
    back = cpu_session.read().option("inferSchema", "true").csv(out)
    assert back.dtypes == df.dtypes
    assert [tuple(r) for r in back.collect()] == [tuple(r) for r in df.collect()]
