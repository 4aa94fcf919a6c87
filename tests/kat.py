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
    first point (the seek position when seeked), Downsampler.java:330-345."""
    from opentsdb_amd import jcalendar as J
    ds = core.DownsamplingSpecification(d["ds_string"])
    n, unit = ds.calendar_interval()
    first = points[0][0] if seek is None else min(seek, points[0][0])
    return J.bucket_edges_for_series(first, points[-1][0], n, unit,
                                     d.get("tz"))


def spec_from_case(d, cal_edges=None):
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
        cal_edges=cal_edges)


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
        if isinstance(ev, float) and math.isnan(ev):
            assert math.isnan(gv), "%s[%d]: %r not NaN" % (where, i, gv)
        else:
            assert abs(gv - ev) <= tol, "%s[%d]: %r != %r (tol %g)" % (
                where, i, gv, ev, tol)
