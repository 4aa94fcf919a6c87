"""Pins the CPU oracle against the reference's own JUnit known answers
(transcribed in tests/golden/kat_reference.json).  CPU only."""
import math

import numpy as np
import pytest

from opentsdb_amd import core
from oracle import pyoracle
from tests import kat

EXC = {"IllegalStateException": 2, "IllegalDataException": 1}


@pytest.mark.parametrize("c", kat.load_cases("agg_long"), ids=lambda c: c["name"])
def test_agg_long(c):
    agg = core.Aggregators.get(c["agg"]).id
    if "error" in c:
        with pytest.raises(pyoracle.OracleError) as ei:
            pyoracle.run_long(agg, c["values"])
        assert ei.value.status == EXC[c["error"]]
        return
    got = pyoracle.run_long(agg, c["values"])
    assert abs(got - c["expect"]) <= c["tol"], (got, c["expect"])


@pytest.mark.parametrize("c", kat.load_cases("agg_double"), ids=lambda c: c["name"])
def test_agg_double(c):
    agg = core.Aggregators.get(c["agg"]).id
    got = pyoracle.run_double(agg, [kat.dec(v) for v in c["values"]])
    e = kat.dec(c["expect"])
    if isinstance(e, float) and math.isnan(e):
        assert math.isnan(got)
    else:
        assert abs(got - e) <= c["tol"], (got, e)


@pytest.mark.parametrize("c", kat.load_cases("view"), ids=lambda c: c["name"])
def test_view(c):
    pts = c["points"]
    edges = None
    cover = None
    if kat.is_fill_calendar(c["spec"]):
        cover = pts[-1][0] if pts else None
    elif c["spec"].get("ds_string", "").split("-")[0].endswith("c"):
        edges = kat.view_cal_edges(c["spec"], pts, c.get("seek"))
    spec = kat.spec_from_case(c["spec"], edges, cover)
    ts = [p[0] for p in pts]
    bits = [np.float64(kat.dec(p[1])).view(np.int64) if p[2] else int(p[1])
            for p in pts]
    isf = [p[2] for p in pts]
    if "error" in c:
        with pytest.raises(pyoracle.OracleError) as ei:
            pyoracle.view_stream(spec, ts, bits, isf, c.get("seek"))
        assert ei.value.status == EXC[c["error"]]
        return
    got = pyoracle.view_stream(spec, ts, bits, isf, c.get("seek"))
    if c.get("prefix"):  # the test asserts only the first point(s)
        got = got[:len(c["expect"])]
    kat.check_points(got, c["expect"], c["tol"], c["name"],
                     c.get("check_from", 0))


@pytest.mark.parametrize("c", kat.load_cases("group_by"), ids=lambda c: c["name"])
def test_group_by(c):
    spec = kat.spec_from_case(c["spec"])
    batch = kat.batch_from_case(c)
    got = pyoracle.group_by(spec, batch)
    if c.get("post"):
        got = [kat.post_downsample(g, c["post"]) for g in got]
    for g, exp in enumerate(c["expect"]):
        kat.check_points(got[g], exp, c["tol"], "%s/g%d" % (c["name"], g))
        if c.get("check_ts_mod"):
            assert all(int(t) % c["check_ts_mod"] == 0 for t in got[g]["ts"])


@pytest.mark.parametrize("c", kat.load_cases("scan_bounds"), ids=lambda c: c["name"])
def test_scan_bounds(c):
    ds = core.DownsamplingSpecification(
        interval_ms=c["interval_ms"], function=core.Aggregators.SUM)
    assert core.get_scan_start_time_seconds(c["start"], ds) == c["expect"][0]
    assert core.get_scan_end_time_seconds(c["end"], ds) == c["expect"][1]


def test_percentile_double_weibull_crosscheck():
    """Double-path LEGACY percentile vs numpy 'weibull' (same formula; SURVEY
    §8c: agrees to <= 1 ulp).  The only pin available for the double path."""
    rng = np.random.default_rng(7)
    v = rng.normal(size=777)
    for name, p in (("p50", 50), ("p99", 99), ("p999", 99.9), ("p95", 95)):
        got = pyoracle.run_double(core.Aggregators.get(name).id, v)
        ref = np.percentile(v, p, method="weibull")
        assert abs(got - ref) <= 4 * np.spacing(abs(ref)), (name, got, ref)


def test_decode_row_seconds_and_ms():
    """RowSeq decode: 2-byte second qualifiers, 4-byte ms qualifiers,
    1/2/4/8-byte ints, 4/8-byte floats (RowSeq.java:552-643)."""
    base = 1356998400
    # second qualifier: offset 10s, int 1 byte -> (10<<4)|0
    q = bytes([0x00, 0xA0])
    q += bytes([0x01, 0x41])                   # offset 20, int 2 bytes
    q += bytes([0x01, 0xEB])                   # offset 30, float 4 bytes
    ms = (0xF << 28) | (1500 << 6) | 0x7       # ms offset 1500, int 8 bytes
    q += ms.to_bytes(4, "big")
    v = bytes([0xFE]) + (300).to_bytes(2, "big", signed=True)
    v += np.float32(2.5).tobytes()[::-1]
    v += (-7).to_bytes(8, "big", signed=True) + b"\x00"  # meta byte
    got = pyoracle.decode_row(q, v, base)
    assert [int(t) for t in got["ts"]] == [
        (base + 10) * 1000, (base + 20) * 1000, (base + 30) * 1000,
        base * 1000 + 1500]
    assert [kat.point_value(b, i) for b, i in zip(got["bits"], got["is_int"])] \
        == [-2, 300, 2.5, -7]


@pytest.mark.parametrize("c", kat.load_cases("prev_interval"),
                         ids=lambda c: c["name"])
def test_previous_interval(c):
    """The calendar-grid anchor (host side of calendar downsampling) against
    DateTime.previousInterval's own known answers."""
    from opentsdb_amd import jcalendar
    got = jcalendar.previous_interval(c["ts"], c["interval"], c["unit"],
                                      c["tz"])
    assert got == c["expect"], (got, c["expect"])


@pytest.mark.parametrize("c", kat.load_cases("compact"), ids=lambda c: c["name"])
def test_compact_row(c):
    """Query-time compaction of one storage row (CompactionQueue.compact via
    Span's scanner path) against TestCompactionQueue's asserted cells.  The
    JUnit KeyValues carry increasing HBase timestamps (makekv, :1537), so the
    column index is the cell timestamp."""
    cols = [(bytes.fromhex(q), bytes.fromhex(v)) for q, v in c["columns"]]
    ts = list(range(len(cols)))
    if "error" in c:
        with pytest.raises(pyoracle.OracleError) as ei:
            pyoracle.compact_row(cols, ts, c["fix_duplicates"])
        assert ei.value.status == EXC[c["error"]]
        return
    got = pyoracle.compact_row(cols, ts, c["fix_duplicates"])
    if c["expect"] is None:
        assert got is None
    else:
        assert got is not None
        assert got[0].hex() == c["expect"][0]
        assert got[1].hex() == c["expect"][1]


@pytest.mark.parametrize("c", kat.load_cases("span"), ids=lambda c: c["name"])
def test_span_assemble(c):
    """Span/RowSeq.addRow merge of one series' rows in arrival order, then
    the iteration the span yields, against TestRowSeq's asserted points."""
    rows = [(b, bytes.fromhex(q), bytes.fromhex(v)) for b, q, v in c["rows"]]
    got = []
    for base, q, v in pyoracle.span_assemble(rows):
        for p in pyoracle.decode_row(q, v, base):
            got.append([int(p["ts"]), kat.point_value(p["bits"], p["is_int"])])
    assert got == c["expect"]


@pytest.mark.parametrize("c", kat.load_cases("decode"), ids=lambda c: c["name"])
def test_decode_kat(c):
    """Compacted columns broken down point by point (RowSeq.Iterator,
    Internal.extractDataPoints) against TestInternal's asserted cells."""
    q, v = bytes.fromhex(c["qual"]), bytes.fromhex(c["val"])
    if "error" in c:
        with pytest.raises(pyoracle.OracleError) as ei:
            pyoracle.decode_row(q, v, c["base"])
        assert ei.value.status == EXC[c["error"]]
        return
    got = pyoracle.decode_row(q, v, c["base"])
    assert [[int(p["ts"]), kat.point_value(p["bits"], p["is_int"])]
            for p in got] == c["expect"]


@pytest.mark.parametrize("c", kat.load_cases("rows_query"), ids=lambda c: c["name"])
def test_rows_query(c):
    """One storage row's columns compacted at query time and decoded
    (CompactionQueue + RowSeq), the series read back by a TsdbQuery: the
    points the test asserts."""
    cols = [(bytes.fromhex(q), bytes.fromhex(v)) for q, v in c["columns"]]
    q, v = pyoracle.compact_row(cols, list(range(len(cols))), c["fix_duplicates"])
    got = pyoracle.decode_row(q, v, c["base"])
    assert [[int(p["ts"]), kat.point_value(p["bits"], p["is_int"])]
            for p in got] == c["expect"]
