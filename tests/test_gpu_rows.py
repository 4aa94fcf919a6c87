"""Query-time compaction and span assembly on the GPU (rows.hip, through the
C-ABI) against the oracle's restatement (or_compact_row / or_span_assemble,
pinned by the TestCompactionQueue / TestRowSeq vectors) and against the
reference's own known answers: bit-exact bytes, same exceptions.  Needs an
MI355X."""
import numpy as np
import pytest

from opentsdb_amd import core, storage
from oracle import pyoracle
from tests import datasets, kat, rows_fuzz

pytestmark = pytest.mark.gpu

EXC = {"IllegalDataException": core.IllegalDataException,
       "IllegalArgumentException": core.IllegalArgumentException}
STATUS_EXC = {1: core.IllegalDataException, 3: core.IllegalArgumentException,
              5: core.UnsupportedOperationException}


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _gpu_compact(engine, rows, fix=True, with_ts=True):
    """rows: [(series, base, [(q, v, ts)])] -> [(series, base, q, v)]"""
    raw = storage.HostRawRows(rows, with_ts=with_ts).to_device()
    return storage.cells_rows(storage.compact_rows_device(engine, raw, fix))


def test_compaction_queue_kats(engine):
    """Every TestCompactionQueue vector with an answer, one row each, in one
    call: the kept rows' bytes are the asserted column."""
    cases = [c for c in kat.load_cases("compact") if "error" not in c]
    rows = []
    for i, c in enumerate(cases):
        cols = [(bytes.fromhex(q), bytes.fromhex(v), j)
                for j, (q, v) in enumerate(c["columns"])]
        assert c["fix_duplicates"]
        rows.append((i, 1356998400, cols))
    got = {s: (q, v) for s, _, q, v in _gpu_compact(engine, rows)}
    for i, c in enumerate(cases):
        if c["expect"] is None:
            assert i not in got, c["name"]
        else:
            assert got[i][0].hex() == c["expect"][0], c["name"]
            assert got[i][1].hex() == c["expect"][1], c["name"]


@pytest.mark.parametrize("c", [c for c in kat.load_cases("compact")
                               if "error" in c], ids=lambda c: c["name"])
def test_compaction_queue_errors(engine, c):
    cols = [(bytes.fromhex(q), bytes.fromhex(v), j)
            for j, (q, v) in enumerate(c["columns"])]
    with pytest.raises(EXC[c["error"]]):
        _gpu_compact(engine, [(0, 1356998400, cols)], c["fix_duplicates"])


def _oracle_rows(rows, fix):
    out = []
    for s, b, cols in rows:
        r = pyoracle.compact_row([(q, v) for q, v, _ in cols],
                                 [t for _, _, t in cols], fix)
        if r is not None:
            out.append((s, b, r[0], r[1]))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_compaction_fuzz_matches_oracle(engine, seed):
    """Random rows (single cells, compacted columns in and out of time
    order, appends, duplicates across columns, annotations, legacy fix-ups),
    fix_duplicates on: every row's bytes equal the oracle's."""
    rng = np.random.default_rng(seed)
    rows, s = [], 0
    while len(rows) < 400:
        cols = rows_fuzz.random_row(rng)
        if rows_fuzz.heap_with_append(cols):
            continue
        try:
            pyoracle.compact_row([(q, v) for q, v, _ in cols],
                                 [t for _, _, t in cols], True)
        except pyoracle.OracleError:
            continue  # corrupt inputs are covered below
        rows.append((s, rows_fuzz.BASE + 3600 * (s % 5), cols))
        s += 1
    got = _gpu_compact(engine, rows)
    ref = _oracle_rows(rows, True)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert g == r, (g, r)


@pytest.mark.parametrize("seed", [11, 12])
def test_compaction_fuzz_errors_match_oracle(engine, seed):
    """Corrupt and duplicate-with-different-value rows, fix_duplicates off:
    the GPU raises the oracle's exception (one row per call), or returns its
    bytes."""
    rng = np.random.default_rng(seed)
    n_err = n_ok = 0
    for i in range(60):
        cols = rows_fuzz.random_row(rng, corrupt=0.5)
        if rows_fuzz.heap_with_append(cols):
            continue
        try:
            ref = pyoracle.compact_row([(q, v) for q, v, _ in cols],
                                       [t for _, _, t in cols], False)
            err = None
        except pyoracle.OracleError as e:
            err = e.status
        if err is None:
            got = _gpu_compact(engine, [(0, rows_fuzz.BASE, cols)], fix=False)
            assert got == ([] if ref is None else
                           [(0, rows_fuzz.BASE, ref[0], ref[1])])
            n_ok += 1
        else:
            with pytest.raises(STATUS_EXC[err]):
                _gpu_compact(engine, [(0, rows_fuzz.BASE, cols)], fix=False)
            n_err += 1
    assert n_err > 5 and n_ok > 5


def _uniform_rows(rng, n_rows):
    """Single-column rows of compacted columns, mostly what a TSD compaction
    writes (one qualifier width, strictly increasing offsets, meta 0) — the
    k_rows_plan fast path — and near misses it must hand to the exact walk:
    a meta byte of 1, a repeated offset, two offsets swapped, one ms point in
    a seconds column, a value byte too many; long ms columns (thousands of
    points, several 1 KB qualifier passes) and short ones."""
    rows = []
    for i in range(n_rows):
        ms = rng.random() < 0.4
        n = int(rng.choice([2, 3, 7, 8, 9, 63, 64, 65, 360, 511, 512, 513,
                            2000, 4100])) if ms else int(rng.integers(2, 361))
        if ms:
            offs = np.sort(rng.choice(3600000, size=n, replace=False))
        else:
            offs = np.sort(rng.choice(3600, size=n, replace=False)) * 1000
        kind = int(rng.integers(0, 6))
        cs = [rows_fuzz.cell(rng, int(o), ms, rows_fuzz.enc_value(rng, kind))
              for o in offs]
        miss = int(rng.integers(0, 8))
        meta = None
        if miss == 1:
            meta = 1
        elif miss == 2 and n > 2:
            cs[2] = rows_fuzz.cell(rng, int(offs[1]), ms, rows_fuzz.enc_value(rng, kind))
        elif miss == 3 and n > 3:
            cs[1], cs[2] = cs[2], cs[1]
        elif miss == 4 and not ms and n > 4:
            cs[3] = rows_fuzz.cell(rng, int(offs[3]) + 1, True,
                                   rows_fuzz.enc_value(rng, kind))
        q, v = rows_fuzz.compacted(cs, meta)
        if miss == 5:
            v = v[:-1] + b"\x07" + v[-1:]
        rows.append((i, rows_fuzz.BASE + 3600 * (i % 7), [(q, v, 0)]))
    return rows


@pytest.mark.parametrize("seed", [21, 22])
def test_compaction_uniform_columns(engine, seed):
    """Compacted single-column rows through the fast uniform check and the
    exact walk (fix_duplicates on, and off on rows without a repeated
    offset): the bytes equal the oracle's, or both raise."""
    rng = np.random.default_rng(seed)
    rows = _uniform_rows(rng, 300)
    for fix in (True, False):
        ok, bad = [], []
        for r in rows:
            try:
                _oracle_rows([r], fix)
                ok.append(r)
            except pyoracle.OracleError:
                bad.append(r)
        got = _gpu_compact(engine, ok, fix)
        assert got == _oracle_rows(ok, fix)
        for r in bad[:20]:
            with pytest.raises((core.IllegalDataException,
                                core.IllegalArgumentException)):
                _gpu_compact(engine, [r], fix)


@pytest.mark.parametrize("breaker", [None, "annotation", "merge"])
def test_query_from_storage_rows_aliasing(engine, breaker):
    """Storage rows of back-to-back single compacted columns (what a scan of
    compacted data returns): the compacted output aliases the input pools
    and no value byte moves; with an annotation column in between, or one
    row that needs a merge, it is packed instead.  Either way the query
    equals the oracle's over the same points."""
    import torch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare
    from tests.test_gpu_decode import _device_batch, _result_points
    from tests import cells as C
    rng = np.random.default_rng(5)
    hb = datasets.random_batch(47, n_series=24, n_groups=4, span_ms=5 * 3600000,
                               cadence_ms=10000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    rows = []
    for s in range(hb.n_series):
        a, b = hb.offsets[s], hb.offsets[s + 1]
        for base, q, v in C.encode_series(hb.ts[a:b], hb.val[a:b],
                                          hb.is_float[a:b]):
            cols = [(q, v, 0)]
            if breaker == "annotation" and len(rows) == 40:
                cols = [(bytes([1, 0, 0]), b'{"a":1}', 1)] + cols
            rows.append((s, base, cols))
    if breaker == "merge":  # split one row into two columns
        s, base, cols = rows[40]
        pts = rows_fuzz.split_points(cols[0][0], cols[0][1])
        h = len(pts) // 2
        rows[40] = (s, base, [rows_fuzz.compacted(pts[:h]) + (0,),
                              rows_fuzz.compacted(pts[h:]) + (1,)])
    raw = storage.HostRawRows(rows, with_ts=True).to_device()
    raw.n_series = hb.n_series
    db = _device_batch(hb, "float")
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 5 * 3600000
    spec = core.make_spec(t0, t1, core.Aggregators.get("sum"),
                          core.DownsamplingSpecification("1m-avg"), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    storage.run_raw_device(engine, spec, raw, db, res)
    compare(_result_points(res, db.n_groups), ref, False,
            where="alias/%s" % breaker)


def _stage_calls(engine):
    """How many times each engine stage ran since the last read
    (otsdb_prof_read; stage 5 = query-time compaction)."""
    import ctypes as C
    ms = (C.c_double * 8)()
    n = (C.c_int64 * 8)()
    engine.lib.otsdb_prof_read(engine.ctx, ms, n, 8, 1)
    return list(n)


@pytest.mark.parametrize("breaker", [None, "unsorted", "repeat", "repeat-nofix",
                                     "length", "ms-row", "window"])
def test_query_from_storage_rows_verbatim(engine, breaker):
    """Storage rows of single compacted columns over a whole-range window:
    the query takes the rows as stored (no compaction pass: k_rows_shape,
    then the cells fold checks every point's order as it streams).  A column
    compaction would change — offsets out of order or repeated, value bytes
    that do not add up, an ms row in a seconds series — or a window that
    does not stream every point sends the query through the full path:
    either way the result (or the error) is the oracle's."""
    import torch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare
    from tests.test_gpu_decode import _device_batch, _result_points
    from tests import cells as C
    hb = datasets.random_batch(48, n_series=24, n_groups=4, span_ms=5 * 3600000,
                               cadence_ms=10000, outside=False)
    hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    rows = []
    for s in range(hb.n_series):
        a, b = hb.offsets[s], hb.offsets[s + 1]
        for base, q, v in C.encode_series(hb.ts[a:b], hb.val[a:b],
                                          hb.is_float[a:b]):
            rows.append((s, base, [(q, v, 0)]))
    fix = breaker != "repeat-nofix"
    k = 30
    s_k, base_k, cols = rows[k]
    pts = rows_fuzz.split_points(cols[0][0], cols[0][1])
    if breaker == "unsorted":
        pts[3], pts[4] = pts[4], pts[3]
        rows[k] = (s_k, base_k, [rows_fuzz.compacted(pts) + (0,)])
    elif breaker in ("repeat", "repeat-nofix"):
        pts.insert(5, (pts[5][0], pts[4][1]))  # offset 5 again, other bytes
        rows[k] = (s_k, base_k, [rows_fuzz.compacted(pts) + (0,)])
    elif breaker == "length":
        q, v = cols[0][0], cols[0][1]
        rows[k] = (s_k, base_k, [(q, v[:-2] + v[-1:], 0)])  # a byte short
    elif breaker == "ms-row":
        ms = [(rows_fuzz.ms_qual(((qq[0] << 8 | qq[1]) >> 4) * 1000,
                                 qq[1] & 0xF), vv) for qq, vv in pts]
        rows[k] = (s_k, base_k, [rows_fuzz.compacted(ms) + (0,)])
    raw = storage.HostRawRows(rows, with_ts=True).to_device()
    raw.n_series = hb.n_series
    db = _device_batch(hb, "float")
    lo, hi = int(hb.ts.min()), int(hb.ts.max())
    if breaker == "window":
        lo += 600000
    spec = core.make_spec(lo, hi, core.Aggregators.get("sum"),
                          core.DownsamplingSpecification("1m-avg"), lo, hi)
    # the oracle over the points the full path compacts from the rows
    try:
        crow = _oracle_rows(rows, fix)
        ref_err = None
    except pyoracle.OracleError as e:
        ref_err = e.status
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    engine.lib.otsdb_prof_enable(engine.ctx, 1)
    _stage_calls(engine)
    try:
        if ref_err is not None:
            with pytest.raises(core.OpenTSDBException):
                storage.run_raw_device(engine, spec, raw, db, res,
                                       fix_duplicates=fix)
            return
        storage.run_raw_device(engine, spec, raw, db, res, fix_duplicates=fix)
        calls = _stage_calls(engine)
    finally:
        engine.lib.otsdb_prof_enable(engine.ctx, 0)
    assert (calls[5] == 0) == (breaker is None), calls  # compaction ran?
    from tests.cells import batch_from_rows
    ref = pyoracle.group_by(spec, batch_from_rows(crow, hb))
    compare(_result_points(res, db.n_groups), ref, False,
            where="verbatim/%s" % breaker)


def test_compaction_first_failing_row_decides(engine):
    """The first failing row in row order decides the exception (the
    scanner compacts rows in order)."""
    bad_arg = (bytes([5, 0, 0, 0, 0]), b"", 0)
    bad_data = (rows_fuzz.sec_qual(7, 0xB), b"\1\0\0\0\0\0\0\1", 0)
    ok = (rows_fuzz.sec_qual(1, 0x7), b"\0" * 7 + b"\1", 0)
    rows = [(0, rows_fuzz.BASE, [ok]), (1, rows_fuzz.BASE, [bad_data]),
            (2, rows_fuzz.BASE, [bad_arg])]
    with pytest.raises(core.IllegalDataException):
        _gpu_compact(engine, rows)
    rows[1], rows[2] = (1, rows_fuzz.BASE, [bad_arg]), (2, rows_fuzz.BASE, [bad_data])
    with pytest.raises(core.IllegalArgumentException):
        _gpu_compact(engine, rows)


def test_compaction_uncompacted_hour(engine):
    """A row never compacted: 3600 single-second cells in column (qualifier)
    order, plus a few repeats with newer HBase timestamps and equal bytes —
    the LDS sort path at its size."""
    rng = np.random.default_rng(5)
    pts = [rows_fuzz.cell(rng, 1000 * k, False) for k in range(3600)]
    cols = [(q, v, k) for k, (q, v) in enumerate(pts)]
    for k in rng.integers(0, 3600, size=20):
        cols.append((pts[k][0], pts[k][1], 5000 + int(k)))
    got = _gpu_compact(engine, [(0, rows_fuzz.BASE, cols)])
    q, v = rows_fuzz.compacted(pts)
    assert got == [(0, rows_fuzz.BASE, q, v)]


def test_compaction_large_ms_row(engine):
    """An hour of millisecond points written as single cells (100,000
    columns, past the LDS caps: the global-memory merge of rows.hip), with
    repeats under newer and older HBase timestamps, next to ordinary rows in
    the same call: bit-exact with or_compact_row."""
    rng = np.random.default_rng(61)
    offs = np.sort(rng.choice(3600 * 1000, size=100000, replace=False))
    pts = [rows_fuzz.cell(rng, int(o), True) for o in offs]
    cols = [(q, v, int(t)) for (q, v), t in
            zip(pts, rng.integers(0, 1 << 40, size=len(pts)))]
    for k in rng.integers(0, len(pts), size=300):  # equal-byte repeats
        cols.append((pts[k][0], pts[k][1], int(rng.integers(0, 1 << 40))))
    order = rng.permutation(len(cols))
    big = [cols[i] for i in order]
    small = rows_fuzz.random_row(np.random.default_rng(62))
    while rows_fuzz.heap_with_append(small):
        small = rows_fuzz.random_row(np.random.default_rng(63))
    # a 12,000-column row the oracle merges in seconds
    mid = [c for c in big if (int.from_bytes(c[0], "big") >> 6) % 9 == 0][:12000]
    rows = [(0, rows_fuzz.BASE, small), (1, rows_fuzz.BASE, big),
            (2, rows_fuzz.BASE + 3600, small), (3, rows_fuzz.BASE, mid)]
    got = _gpu_compact(engine, rows)
    ref = _oracle_rows([rows[0], rows[2], rows[3]], True)
    assert len(got) == 4
    assert [got[0], got[2], got[3]] == ref
    # the 100,000-point row: every offset once, in time order, the repeats
    # (equal bytes) dropped (CompactionQueue.java:549-584); the oracle's heap
    # takes ~40 s on it, so the expectation is the column it must build
    q, v = rows_fuzz.compacted(pts)
    assert got[1] == (1, rows_fuzz.BASE, q, v)


def test_compaction_large_merged_columns(engine):
    """Two compacted columns of 5,000 ms points each (10,000 cells to
    merge) plus an append column and second-resolution cells: the large-row
    merge keeps the heap order (newer column first on equal offsets) and the
    mixed-resolution meta byte, bit-exact with the oracle; fix_duplicates
    off raises IllegalDataException on a differing duplicate."""
    rng = np.random.default_rng(6)
    a = rows_fuzz.compacted([rows_fuzz.cell(rng, 2 * k, True)
                             for k in range(5000)])
    b = rows_fuzz.compacted([rows_fuzz.cell(rng, 2 * k + 1, True)
                             for k in range(5000)])
    app = b"".join(q + v for q, v in [rows_fuzz.cell(rng, 20000 + 7 * k, True)
                                      for k in range(40)])
    sec = [rows_fuzz.cell(rng, 1000 * k, False) for k in range(30, 60)]
    cols = [a + (3,), b + (1,), (bytes([5, 0, 0]), app, 2)]
    cols += [(q, v, 9) for q, v in sec]
    rows = [(0, rows_fuzz.BASE, cols)]
    got = _gpu_compact(engine, rows)
    assert got == _oracle_rows(rows, True)
    # a repeated offset with different bytes
    dup = rows_fuzz.cell(rng, 4, True, value=(0x7, b"\0" * 7 + b"\x05"))
    cols2 = cols + [(dup[0], dup[1], 99)]
    try:
        ref = _oracle_rows([(0, rows_fuzz.BASE, cols2)], False)
        err = None
    except pyoracle.OracleError as e:
        err = e.status
    if err is None:
        assert _gpu_compact(engine, [(0, rows_fuzz.BASE, cols2)], fix=False) == ref
    else:
        with pytest.raises(STATUS_EXC[err]):
            _gpu_compact(engine, [(0, rows_fuzz.BASE, cols2)], fix=False)


@pytest.mark.parametrize("fix", [True, False])
def test_compaction_large_row_out_of_order(engine, fix):
    """Large rows (past the LDS caps) holding compacted columns whose offsets
    go back in time (never written by the write path or compaction): the
    heap's pop order is replayed over the in-order columns' merged cells and
    each unsorted column (CompactionQueue.java:549-584) — the bytes equal
    the oracle's heap merge, or both raise."""
    rng = np.random.default_rng(7)
    offs = list(range(0, 20000, 2))
    offs[10], offs[11] = offs[11], offs[10]
    a = rows_fuzz.compacted([rows_fuzz.cell(rng, o, True) for o in offs])
    b = rows_fuzz.compacted([rows_fuzz.cell(rng, o + 1, True)
                             for o in range(0, 20000, 2)])
    # a second unsorted column (a stretch reversed, repeating offsets of a)
    c_offs = list(range(500, 1500, 4))
    c_offs[20:40] = c_offs[20:40][::-1]
    c = rows_fuzz.compacted([rows_fuzz.cell(rng, o, True) for o in c_offs])
    singles = [rows_fuzz.cell(rng, 1000 * k, False) for k in range(3, 9)]
    rows = [(0, rows_fuzz.BASE, [a + (0,), b + (1,)]),
            (1, rows_fuzz.BASE, [c + (5,), a + (3,)] +
             [(q, v, 9) for q, v in singles]),
            (2, rows_fuzz.BASE, [b + (0,)])]
    for r in rows:
        try:
            ref = _oracle_rows([r], fix)
            err = None
        except pyoracle.OracleError as e:
            err = e.status
        if err is None:
            assert _gpu_compact(engine, [r], fix) == ref
        else:
            with pytest.raises(STATUS_EXC[err]):
                _gpu_compact(engine, [r], fix)
    if fix:
        assert _gpu_compact(engine, rows, fix) == _oracle_rows(rows, fix)


def test_row_seq_kats(engine):
    """TestRowSeq's merge vectors: the span's rows decode to the asserted
    points."""
    cases = kat.load_cases("span")
    rows = []
    for i, c in enumerate(cases):
        for b, q, v in c["rows"]:
            rows.append((i, b, bytes.fromhex(q), bytes.fromhex(v)))
    got = _gpu_span(engine, rows, len(cases))
    for i, c in enumerate(cases):
        pts = []
        for s, b, q, v in got:
            if s != i:
                continue
            for p in pyoracle.decode_row(q, v, b):
                pts.append([int(p["ts"]), kat.point_value(p["bits"], p["is_int"])])
        assert pts == c["expect"], c["name"]


def _gpu_span(engine, rows, n_series):
    """rows: [(series, base, q, v)] in arrival order -> span rows"""
    import torch
    from opentsdb_amd.workload import DeviceCells
    qo = np.cumsum([0] + [len(r[2]) for r in rows]).astype(np.int64)
    vo = np.cumsum([0] + [len(r[3]) for r in rows]).astype(np.int64)
    t = dict(row_series=np.asarray([r[0] for r in rows], np.int64),
             row_base_s=np.asarray([r[1] for r in rows], np.int64),
             qual_off=qo, val_off=vo,
             qual=np.frombuffer(b"".join(r[2] for r in rows) + b"\0" * 16,
                                np.uint8),
             val=np.frombuffer(b"".join(r[3] for r in rows) + b"\0" * 16,
                               np.uint8))
    t = {k: torch.from_numpy(np.ascontiguousarray(x)).cuda() for k, x in t.items()}
    cells = DeviceCells(t, n_series)
    return storage.cells_rows(storage.span_assemble_device(engine, cells))


@pytest.mark.parametrize("seed", [21, 22])
def test_span_fuzz_matches_oracle(engine, seed):
    """Series whose rows arrive in any order, with repeated row keys
    (overlapping and disjoint in time): the span rows' bytes equal the
    oracle's Span.addRow replay; in-order series pass through unchanged."""
    rng = np.random.default_rng(seed)
    rows, ref = [], []
    S = 120
    for s in range(S):
        n = int(rng.integers(1, 7))
        if s % 3 == 0:  # the scanner's order: strictly increasing bases
            bases = sorted(rng.choice(24, size=n, replace=False))
        else:
            bases = list(rng.integers(0, 4, size=n))
        rs = []
        for b in bases:
            q, v = rows_fuzz.random_compacted_row(rng, pool_s=600)
            rs.append((rows_fuzz.BASE + 3600 * int(b), q, v))
        rows += [(s, b, q, v) for b, q, v in rs]
        ref += [(s, b, q, v) for b, q, v in pyoracle.span_assemble(rs)]
    got = _gpu_span(engine, rows, S)
    assert got == ref


def _raw_from_hb(rng, hb, split=0.3):
    """Storage rows holding exactly hb's points, scattered over columns the
    way uncompacted / partially compacted / appended rows hold them, some
    hours split over two rows of the same key arriving in either order."""
    from tests import cells as C
    rows = []
    isf = hb.is_float
    for s in range(hb.n_series):
        a, b = hb.offsets[s], hb.offsets[s + 1]
        f = isf[a:b] if isf is not None else np.ones(b - a, np.uint8)
        for base, q, v in C.encode_series(hb.ts[a:b], hb.val[a:b], f):
            pts = rows_fuzz.split_points(q, v)
            if len(pts) > 3 and rng.random() < split:
                m = rng.random() < 0.5  # interleaved or consecutive halves
                p1 = pts[0::2] if m else pts[:len(pts) // 2]
                p2 = pts[1::2] if m else pts[len(pts) // 2:]
                parts = [p1, p2] if rng.random() < 0.5 else [p2, p1]
            else:
                parts = [pts]
            for p in parts:
                rows.append((s, base, rows_fuzz.scatter_row(rng, p)))
    return rows


@pytest.mark.parametrize("agg,ds", [("sum", "1m-avg"), ("zimsum", "5m-sum"),
                                    ("max", "1m-first"), ("p99", "1m-avg")])
@pytest.mark.parametrize("kind", ["float", "int"])
def test_query_from_storage_rows(engine, agg, ds, kind):
    """otsdb_agg_run_raw_device: storage rows (cells, compacted pieces,
    appends, repeats, split row keys) -> compaction -> spans -> the fused
    query equals the oracle's query over the same points."""
    import torch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_parity import compare, cancel_floor
    from tests.test_gpu_decode import _device_batch, _result_points
    rng = np.random.default_rng(hash((agg, ds, kind)) % 2**31)
    hb = datasets.random_batch(41, n_series=30, n_groups=3, span_ms=3 * 3600000,
                               value_kind=kind, cadence_ms=10000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    isf = 1 if kind == "float" else 0
    hb.is_float = np.full(len(hb.ts), isf, np.uint8)
    raw = storage.HostRawRows(_raw_from_hb(rng, hb), with_ts=True).to_device()
    raw.n_series = hb.n_series
    db = _device_batch(hb, kind)
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1)
    ref = pyoracle.group_by(spec, hb)
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    storage.run_raw_device(engine, spec, raw, db, res)
    got = _result_points(res, db.n_groups)
    exact = ds.endswith(("max", "first")) and agg in ("max", "p99")
    compare(got, ref, exact, where="raw/%s/%s" % (agg, ds),
            floor=cancel_floor(hb, 60) if kind == "int" else 0.0)


def test_query_from_storage_rows_host_entry(engine):
    """otsdb_agg_run_raw (host buffers, the JNI entry) = the device entry."""
    import torch
    from opentsdb_amd.engine import DeviceResult
    from tests.test_gpu_decode import _device_batch, _result_points
    rng = np.random.default_rng(3)
    hb = datasets.random_batch(43, n_series=20, n_groups=4, span_ms=2 * 3600000,
                               cadence_ms=10000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    rows = _raw_from_hb(rng, hb)
    hraw = storage.HostRawRows(rows, with_ts=True)
    hraw.n_series = hb.n_series
    draw = hraw.to_device()
    draw.n_series = hb.n_series
    db = _device_batch(hb, "float")
    spec = core.make_spec(datasets.T0, datasets.T0 + 2 * 3600000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    storage.run_raw_device(engine, spec, draw, db, res)
    dev = _result_points(res, db.n_groups)
    offs, ts, val, isi = storage.run_raw(engine, spec, hraw, hb.group_offsets,
                                         hb.group_members, 4 * len(hb.ts) + 64)
    for g in range(db.n_groups):
        a, b = offs[g], offs[g + 1]
        assert np.array_equal(dev[g].ts, ts[a:b])
        assert np.array_equal(dev[g].bits, val[a:b])
        assert np.array_equal(dev[g].is_int, isi[a:b])


@pytest.mark.parametrize("c", kat.load_cases("decode"), ids=lambda c: c["name"])
def test_decode_kats(engine, c):
    """TestInternal's compacted columns through otsdb_decode_cells_device."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.workload import DeviceCells
    q, v = bytes.fromhex(c["qual"]), bytes.fromhex(c["val"])
    t = dict(row_series=np.zeros(1, np.int64),
             row_base_s=np.asarray([c["base"]], np.int64),
             qual_off=np.asarray([0, len(q)], np.int64),
             val_off=np.asarray([0, len(v)], np.int64),
             qual=np.frombuffer(q + b"\0" * 16, np.uint8).copy(),
             val=np.frombuffer(v + b"\0" * 16, np.uint8).copy())
    cells = DeviceCells({k: torch.from_numpy(x).cuda() for k, x in t.items()}, 1)
    if "error" in c:
        with pytest.raises(EXC[c["error"]]):
            workload.decode_cells_device(engine, cells)
        return
    offs, ts, val, isf = workload.decode_cells_device(engine, cells)
    got = [[int(a), int(b)] for a, b in zip(ts.cpu().numpy(), val.cpu().numpy())]
    assert got == c["expect"] and not isf.any()


@pytest.mark.parametrize("agg,ds", [("sum", "1m-avg"), ("max", "5m-max"),
                                    ("p95", "1m-avg"), ("zimsum", None)])
def test_host_cells_entry_matches_oracle(engine, agg, ds):
    """otsdb_agg_run_cells (host buffers: what GpuAggregation.java passes
    through the JNI shim) against the oracle on the same points."""
    from opentsdb_amd.engine import DataPoints
    from tests import cells as CC
    from tests.test_gpu_parity import compare
    hb = datasets.random_batch(47, n_series=25, n_groups=5, span_ms=3 * 3600000,
                               cadence_ms=10000)
    hb.ts[:] = hb.ts - hb.ts % 1000
    hb.is_float = np.ones(len(hb.ts), np.uint8)
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
    d = core.DownsamplingSpecification(ds) if ds else None
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg), d, t0, t1)
    ref = pyoracle.group_by(spec, hb)
    offs, ts, val, isi = storage.run_cells(
        engine, spec, CC.encode_batch(hb), hb.n_series, hb.group_offsets,
        hb.group_members, 8 * len(hb.ts) + 64)
    got = [DataPoints(ts[offs[g]:offs[g + 1]], val[offs[g]:offs[g + 1]],
                      isi[offs[g]:offs[g + 1]]) for g in range(len(offs) - 1)]
    compare(got, ref, agg in ("max",) and ds == "5m-max", where="host-cells")


@pytest.mark.parametrize("c", kat.load_cases("rows_query"), ids=lambda c: c["name"])
def test_rows_query_kats(engine, c):
    """TestTsdbQueryQueries' multi-compaction rows (compacted columns, and
    single cells between them, in one storage row) through the storage-row
    query (otsdb_agg_run_raw: query-time compaction, span assembly, the raw
    group-by): the points the test asserts, as longs."""
    from opentsdb_amd.batch import groups_from_ids
    cols = [(bytes.fromhex(q), bytes.fromhex(v), j)
            for j, (q, v) in enumerate(c["columns"])]
    hraw = storage.HostRawRows([(0, c["base"], cols)], with_ts=True)
    hraw.n_series = 1
    g_off, members = groups_from_ids(np.zeros(1, np.int64), 1)
    spec = core.make_spec(1356998400000, 1357045200000, core.Aggregators.SUM,
                          None, 1356998400000, 1357041600000)
    offs, ts, val, isi = storage.run_raw(engine, spec, hraw, g_off, members, 64)
    got = [[int(t), int(v)] for t, v in zip(ts[offs[0]:offs[1]],
                                            val[offs[0]:offs[1]])]
    assert got == c["expect"]
    assert isi[offs[0]:offs[1]].all()
