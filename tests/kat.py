"""Shared helpers: turn the transcribed reference KATs
(tests/golden/kat_reference.json) into engine/oracle inputs and check outputs.
"""
import json
import math
import os

import numpy as np

from opentsdb_amd import core
from opentsdb_amd.batch import HostBatch

HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases(kind=None):
    with open(os.path.join(HERE, "golden", "kat_reference.json")) as f:
        cases = json.load(f)["cases"]
    return [c for c in cases if kind is None or c["kind"] == kind]


def dec(x):
    if isinstance(x, str):
        return {"NaN": math.nan, "Infinity": math.inf,
                "-Infinity": -math.inf}[x]
    return x


def view_cal_edges(d, points, seek=None):
    """Calendar grid of a lone Downsampler over one series: anchored at its
    first point (the seek position when seeked), Downsampler.java:330-345;
    a FillingDownsampler's grid from its start to its end as well
    (FillingDownsampler.java:113-135)."""
    from opentsdb_amd import jcalendar as J
    ds = core.DownsamplingSpecification(d["ds_string"])
    n, unit = ds.calendar_interval()
    lo = [p[0] for p in points[:1]]
    hi = [p[0] for p in points[-1:]]
    if seek is not None:
        lo.append(seek)
    if d.get("fill") or "-" in d["ds_string"][d["ds_string"].index("-") + 1:]:
        lo.append(d["start_ms"])
        hi.append(d["end_ms"])
    if not lo:  # no points, no filling grid: any table (nothing is read)
        lo, hi = [0], [0]
    return J.bucket_edges_for_series(min(lo), max(hi), n, unit, d.get("tz"))


def is_fill_calendar(d):
    """A FillingDownsampler view over a calendar grid: its spec takes the
    query's own tables (make_spec: one edge table, or anchored chains when
    the grid depends on the series), so the filling grid ends at
    previousInterval(end) even when that is no edge of the series' chain
    (FillingDownsampler.java:121-131)."""
    ds = d.get("ds_string") or ""
    parts = ds.split("-")
    return (len(parts) == 3 and parts[0].endswith("c") and "all" not in parts[0]
            and parts[2] != "none")


def spec_from_case(d, cal_edges=None, cover_ms=None):
    ds = None
    if d.get("ds_string"):
        ds = core.DownsamplingSpecification(d["ds_string"])
        if d.get("tz"):
            ds.setTimezone(d["tz"])
    elif d.get("ds_interval_ms"):
        ds = core.DownsamplingSpecification(
            interval_ms=d["ds_interval_ms"],
            function=core.Aggregators.get(d["ds_agg"]),
            fill_policy=core.FillPolicy.fromString(d.get("fill", "none")))
    ro = core.RateOptions(d.get("counter", False),
                          d.get("counter_max", core.LONG_MAX),
                          d.get("reset_value", 0), d.get("drop_resets", False))
    interp = d.get("interp")
    return core.make_spec(
        d.get("start_ms", 0), d.get("end_ms", core.LONG_MAX // 2),
        core.Aggregators.get(d.get("agg", "sum")), ds,
        d.get("query_start_ms", 0), d.get("query_end_ms", 0),
        d.get("rate", False), ro,
        None if interp is None else core.Interpolation[interp],
        cal_edges=cal_edges, cal_cover_ms=cover_ms)


def batch_from_case(c):
    groups = [[[(p[0], dec(p[1]), p[2]) for p in span] for span in g]
              for g in c["groups"]]
    return HostBatch.from_groups(groups)


def point_value(bits, is_int):
    return int(bits) if is_int else float(np.int64(bits).view(np.float64))


def check_points(got, expect, tol, where, check_from=0):
    """got: structured array (ts, bits, is_int); expect: [[ts, v, is_float]]"""
    assert len(got) == len(expect), "%s: %d points, expected %d" % (
        where, len(got), len(expect))
    for i, (g, e) in enumerate(zip(got, expect)):
        if i < check_from:
            continue
        assert int(g["ts"]) == e[0], "%s[%d]: ts %d != %d" % (
            where, i, g["ts"], e[0])
        ev = dec(e[1])
        gv = point_value(g["bits"], g["is_int"])
        if not e[2]:
            assert g["is_int"], "%s[%d]: expected a long" % (where, i)
        t = e[3] if len(e) > 3 else tol  # a point's own tolerance
        if isinstance(ev, float) and math.isnan(ev):
            assert math.isnan(gv), "%s[%d]: %r not NaN" % (where, i, gv)
        else:
            assert abs(gv - ev) <= t, "%s[%d]: %r != %r (tol %g)" % (
                where, i, gv, ev, t)


def post_downsample(got, post):
    """A Downsampler over an AggregationIterator's output (a test that
    downsamples after aggregating): the oracle's view over those points."""
    from oracle import pyoracle
    spec = spec_from_case(post)
    return pyoracle.view_stream(spec, got["ts"], got["bits"],
                                (got["is_int"] == 0).astype(np.uint8))


def view_as_query(c):
    """A view KAT (one Downsampler / FillingDownsampler / RateSpan chain over
    one series) as the query the engine runs: one group of that one span,
    `sum` across it, the AggregationIterator seeked to the view's seek (or a
    calendar grid's first edge).  Where the query path differs from the lone
    view (the junk first rate is not emitted, the iterator ends at the
    window's end, empty spans are dropped) the oracle's group_by says so."""
    from opentsdb_amd.batch import HostBatch
    pts = c["points"]
    d = dict(c["spec"])
    d["agg"] = "sum"
    if "start_ms" not in d:
        # the iterator window: from the first bucket start (or the seek,
        # which the iterator's seek rounds up the way Downsampler.seek does)
        # to the last point — tight, so the engine's grid stays small
        d["start_ms"] = c.get("seek") or 0
        d["end_ms"] = pts[-1][0] if pts else 1
        iv = 0
        if d.get("ds_interval_ms"):
            iv = d["ds_interval_ms"]
        elif d.get("ds_string") and not d["ds_string"].split("-")[0].endswith(
                ("c", "all")):
            iv = core.DownsamplingSpecification(d["ds_string"]).getInterval()
        if iv and not c.get("seek") and pts:
            d["start_ms"] = pts[0][0] - pts[0][0] % iv
        elif not c.get("seek") and pts and not d.get("ds_string"):
            d["start_ms"] = pts[0][0]
    elif c.get("seek"):
        d["start_ms"] = c["seek"]
    edges = cover = None
    if is_fill_calendar(d):
        cover = pts[-1][0] if pts else None
    elif d.get("ds_string", "").split("-")[0].endswith("c"):
        edges = view_cal_edges(d, pts, c.get("seek"))
        if not c.get("seek") and "start_ms" not in c["spec"]:
            d["start_ms"] = edges[0]
    spec = spec_from_case(d, edges, cover)
    batch = HostBatch.from_groups([[[(p[0], dec(p[1]), p[2]) for p in pts]]])
    return spec, batch
