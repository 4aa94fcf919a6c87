"""Writes tests/golden/kat_reference.json: known-answer vectors transcribed
from the reference's own JUnit tests (the only way to pin the oracle: the Java
reference cannot be compiled or run in this image).

Every case cites the test it is transcribed from (paths under
/root/reference).  Inputs and expected outputs are DATA copied from the test's
literals (expressions like `40.0 / 1356998400` are evaluated here with the
same double arithmetic Java uses); tolerances are the test's own deltas.

Case kinds:
  agg_long / agg_double   Aggregator.runLong / runDouble over a sequence
  view                    a Downsampler/FillingDownsampler/RateSpan chain over
                          one MockSeekableView, iterated directly
  group_by                AggregationIterator over several spans (optionally
                          downsampled / rate), or a whole TsdbQuery run
  scan_bounds             TsdbQuery.getScanStartTimeSeconds/EndTimeSeconds

Run:  python tests/golden/make_kats.py
"""
import json
import math
import os

LMAX = 2**63 - 1
NAN = float("nan")
BASE = 1356998400000  # TestAggregationIterator/TestDownsampler BASE_TIME


def L(ts, v):
    return [int(ts), int(v), 0]      # long point: [ts, value, is_float]


def D(ts, v):
    return [int(ts), float(v), 1]    # double point


cases = []


def add(**kw):
    cases.append(kw)


# ---------------------------------------------------------------- Aggregators
# test/core/TestAggregators.java:81-95 testStdDevKnownValues (runLong, +-1.0)
add(kind="agg_long", name="dev_0_9999", agg="dev", values=list(range(10000)),
    expect=2886.7513315143719, tol=1.0,
    cite="test/core/TestAggregators.java:81-95")
# :110-116 testStdDevNoDeviation
add(kind="agg_long", name="dev_no_deviation", agg="dev", values=[3, 3, 3],
    expect=0, tol=1.0, cite="test/core/TestAggregators.java:110-116")
# :118-124 testStdDevFewDataInputs (expected 0.5 within max(0, 1.0))
add(kind="agg_long", name="dev_few", agg="dev", values=[1, 2], expect=0.5,
    tol=1.0, cite="test/core/TestAggregators.java:118-124")
# :148-176 testPercentiles (runLong on 1..1000, exact)
_p = {"p50": 500, "p75": 750, "p90": 900, "p95": 950, "p99": 990, "p999": 999}
for est in ("", "r3", "r7"):
    for k, v in _p.items():
        name = k if not est else "e" + k + est
        add(kind="agg_long", name="pct_" + name, agg=name,
            values=list(range(1, 1001)), expect=v, tol=0,
            cite="test/core/TestAggregators.java:148-176")
# :178-195 testFirst ; :197-214 testLast
add(kind="agg_long", name="first_long", agg="first", values=list(range(10)),
    expect=0, tol=0, cite="test/core/TestAggregators.java:178-195")
add(kind="agg_double", name="first_double", agg="first",
    values=[0.5 + i for i in range(10)], expect=0.5, tol=0.0001,
    cite="test/core/TestAggregators.java:178-195")
add(kind="agg_long", name="last_long", agg="last", values=list(range(10)),
    expect=9, tol=0, cite="test/core/TestAggregators.java:197-214")
add(kind="agg_double", name="last_double", agg="last",
    values=[0.5 + i for i in range(10)], expect=9.5, tol=0.0001,
    cite="test/core/TestAggregators.java:197-214")
# :216-244 testMedian
add(kind="agg_long", name="median_5", agg="median", values=[5, 2, -1, 400, 3],
    expect=3, tol=0, cite="test/core/TestAggregators.java:216-244")
add(kind="agg_long", name="median_6", agg="median",
    values=[5, 2, -1, 400, 3, -42], expect=3, tol=0,
    cite="test/core/TestAggregators.java:216-244")
add(kind="agg_long", name="median_1", agg="median", values=[42], expect=42,
    tol=0, cite="test/core/TestAggregators.java:216-244")
add(kind="agg_long", name="median_empty", agg="median", values=[],
    error="IllegalStateException", cite="test/core/TestAggregators.java:216-244")
add(kind="agg_double", name="median_d5", agg="median",
    values=[5.1, 2.434, -1.99, 400.69487, 3.15168], expect=3.15168,
    tol=0.0001, cite="test/core/TestAggregators.java:216-244")
add(kind="agg_double", name="median_d6", agg="median",
    values=[5.1, 2.434, -1.99, 400.69487, 3.15168, -42], expect=3.15168,
    tol=0.0001, cite="test/core/TestAggregators.java:216-244")
add(kind="agg_double", name="median_d1", agg="median", values=[42.5],
    expect=42.5, tol=0.0001, cite="test/core/TestAggregators.java:216-244")
add(kind="agg_double", name="median_dempty", agg="median", values=[],
    expect="NaN", tol=0, cite="test/core/TestAggregators.java:216-244")
# :255-264 testSquareSumFewDataInputs
add(kind="agg_long", name="squaresum_few", agg="squareSum", values=[1, 2],
    expect=5, tol=0, cite="test/core/TestAggregators.java:255-264")

# ------------------------------------------------- AggregationIterator (raw)
DP1 = [L(BASE, 40), L(BASE + 10000, 50), L(BASE + 30000, 70)]
DP2 = [L(BASE + 10000, 37), L(BASE + 20000, 48)]
SPEC_AI = dict(start_ms=BASE, end_ms=1356998500 * 1000, agg="sum")
# test/core/TestAggregationIterator.java:73-88 testAggregate_singleSpan
add(kind="group_by", name="ai_single_span", spec=dict(SPEC_AI),
    groups=[[DP1]], expect=[[L(BASE, 40), L(BASE + 10000, 50),
                             L(BASE + 30000, 70)]], tol=0, filter=False,
    cite="test/core/TestAggregationIterator.java:73-88")
# :90-113 testAggregate_doubleSpans (LERP: 60 interpolated)
add(kind="group_by", name="ai_double_spans", spec=dict(SPEC_AI),
    groups=[[DP1, DP2]],
    expect=[[L(BASE, 40), L(BASE + 10000, 87), L(BASE + 20000, 108),
             L(BASE + 30000, 70)]], tol=0, filter=False,
    cite="test/core/TestAggregationIterator.java:90-113")
# :219-234 testAggregate_emptySpan
add(kind="group_by", name="ai_empty_span", spec=dict(SPEC_AI),
    groups=[[[], DP1]], expect=[DP1], tol=0, filter=False,
    cite="test/core/TestAggregationIterator.java:219-234")
# :290-318 pfsum (PREV interpolation)
add(kind="group_by", name="ai_pfsum",
    spec=dict(start_ms=BASE, end_ms=1356998500 * 1000, agg="sum", interp="PREV"),
    groups=[[[L(BASE, 40), L(BASE + 30000, 70)], DP2]],
    expect=[[L(BASE, 40), L(BASE + 10000, 77), L(BASE + 20000, 88),
             L(BASE + 30000, 70)]], tol=0, filter=False,
    cite="test/core/TestAggregationIterator.java:290-318")
# :116-148 testAggregate_manySpansWithDownsampling (7 spans, 10s-avg, sum)
DATA_5SEC = [D(BASE + t, 1) for t in
             (0, 7000, 10000, 15000, 20000, 25000, 30000, 35000, 40000, 45000,
              50000)]
add(kind="group_by", name="ai_many_spans_downsampled",
    spec=dict(start_ms=BASE + 1000, end_ms=BASE + 100000, agg="sum",
              ds_interval_ms=10000, ds_agg="avg"),
    groups=[[DATA_5SEC] * 7],
    expect=[[D(BASE + 10000 * i, 7) for i in range(1, 6)]], tol=0,
    filter=False, cite="test/core/TestAggregationIterator.java:116-148")

# ----------------------------------------------------------- Downsampler
DS_DATA = [L(BASE, 40), L(BASE + 2000000, 50), L(BASE + 3600000, 40),
           L(BASE + 3605000, 50), L(BASE + 7200000, 40),
           L(BASE + 9200000, 50)]
# test/core/TestDownsampler.java:81-104 testDownsampler ("1000s-avg")
add(kind="view", name="ds_1000s_avg",
    spec=dict(ds_interval_ms=1000000, ds_agg="avg", query_start_ms=0,
              query_end_ms=LMAX), points=DS_DATA,
    expect=[D(BASE - 400000, 40), D(BASE + 1600000, 50),
            D(BASE + 3600000, 45), D(BASE + 6600000, 40),
            D(BASE + 8600000, 50)], tol=1e-7,
    cite="test/core/TestDownsampler.java:81-104")
P10 = [D(BASE + 5000 * i, 2 ** i) for i in range(11)]
# :155-183 testDownsampler_10seconds ("10s-sum")
add(kind="view", name="ds_10s_sum",
    spec=dict(ds_interval_ms=10000, ds_agg="sum", query_start_ms=0,
              query_end_ms=LMAX), points=P10,
    expect=[D(BASE, 3), D(BASE + 10000, 12), D(BASE + 20000, 48),
            D(BASE + 30000, 192), D(BASE + 40000, 768),
            D(BASE + 50000, 1024)], tol=1e-7,
    cite="test/core/TestDownsampler.java:155-183")
P15 = [L(BASE + 5000, 1), L(BASE + 15000, 2), L(BASE + 25000, 4),
       L(BASE + 35000, 8), L(BASE + 45000, 16), L(BASE + 55000, 32)]
# :212-237 testDownsampler_15seconds ("15s-sum")
add(kind="view", name="ds_15s_sum",
    spec=dict(ds_interval_ms=15000, ds_agg="sum", query_start_ms=0,
              query_end_ms=LMAX), points=P15,
    expect=[D(BASE, 1), D(BASE + 15000, 6), D(BASE + 30000, 8),
            D(BASE + 45000, 48)], tol=1e-7,
    cite="test/core/TestDownsampler.java:212-237")

# ----------------------------------------------------- FillingDownsampler
B5 = 500
FD = [D(B5 + 25 * k, 1.0) for k in (4, 5, 7, 12, 15, 24, 25, 26, 27)]
# test/core/TestFillingDownsampler.java:45-75 testNaNMissingInterval
add(kind="view", name="fill_nan_missing",
    spec=dict(start_ms=B5, end_ms=B5 + 36 * 25, ds_interval_ms=100,
              ds_agg="sum", fill="nan", query_start_ms=0, query_end_ms=0),
    points=FD,
    expect=[D(B5 + 100 * i, v) for i, v in enumerate(
        [NAN, 3, NAN, 2, NAN, NAN, 4, NAN, NAN])], tol=0,
    cite="test/core/TestFillingDownsampler.java:45-75")
# :77-107 testZeroMissingInterval
add(kind="view", name="fill_zero_missing",
    spec=dict(start_ms=B5, end_ms=B5 + 36 * 25, ds_interval_ms=100,
              ds_agg="sum", fill="zero", query_start_ms=0, query_end_ms=0),
    points=FD,
    expect=[D(B5 + 100 * i, v) for i, v in enumerate(
        [0, 3, 0, 2, 0, 0, 4, 0, 0])], tol=0,
    cite="test/core/TestFillingDownsampler.java:77-107")
# :110-137 testWithoutMissingIntervals
B1 = 1000
add(kind="view", name="fill_no_missing",
    spec=dict(start_ms=B1, end_ms=B1 + 12 * 25, ds_interval_ms=100,
              ds_agg="sum", fill="nan", query_start_ms=0, query_end_ms=0),
    points=[D(B1 + 25 * k, 12 - k) for k in range(12)],
    expect=[D(B1, 42), D(B1 + 100, 26), D(B1 + 200, 10)], tol=0,
    cite="test/core/TestFillingDownsampler.java:110-137")
BO = 1425335895000
OOB = [D(BO - 60000 * 5 + 320, 53), D(BO - 60000 * 2 + 8839, 16),
       D(BO + 849, 9), D(BO + 3849, 8), D(BO + 6210, 7), D(BO + 42216, 6),
       D(BO + 60000 + 167, 5), D(BO + 60000 + 28593, 4),
       D(BO + 120000 + 30384, 37), D(BO + 240000 + 1530, 86)]
# :140-168 testWithOutOfBoundsData
add(kind="view", name="fill_out_of_bounds",
    spec=dict(start_ms=BO, end_ms=BO + 120000, ds_interval_ms=60000,
              ds_agg="sum", fill="nan", query_start_ms=0, query_end_ms=0),
    points=OOB, expect=[D(1425335880000, 30), D(1425335940000, 9)], tol=0,
    cite="test/core/TestFillingDownsampler.java:140-168")
# :170-185 testWithOutOfBoundsDataEarly
add(kind="view", name="fill_oob_early",
    spec=dict(start_ms=BO, end_ms=BO + 120000, ds_interval_ms=60000,
              ds_agg="sum", fill="nan", query_start_ms=0, query_end_ms=0),
    points=OOB[:2],
    expect=[D(1425335880000, NAN), D(1425335940000, NAN)], tol=0,
    cite="test/core/TestFillingDownsampler.java:170-185")
# :187-202 testWithOutOfBoundsDataLate
add(kind="view", name="fill_oob_late",
    spec=dict(start_ms=BO, end_ms=BO + 120000, ds_interval_ms=60000,
              ds_agg="sum", fill="nan", query_start_ms=0, query_end_ms=0),
    points=OOB[-2:],
    expect=[D(1425335880000, NAN), D(1425335940000, NAN)], tol=0,
    cite="test/core/TestFillingDownsampler.java:187-202")

# --------------------------------------------------------------- RateSpan
RD = [D(1356998400000, 40.0), L(1356998400000 + 2000000, 50),
      L(1357002000000, 40), D(1357002000000 + 5000, 50.0),
      L(1357005600000, 40), D(1357005600000 + 2000000, 50.0)]
RATES = [D(1356998400000, 40.0 / 1356998400),
         D(1356998400000 + 2000000, 10.0 / 2000.0),
         D(1357002000000, -10.0 / (1357002000 - 1356998400 - 2000)),
         D(1357002000000 + 5000, 10.0 / 5.0),
         D(1357005600000, -10.0 / (1357005600 - 1357002005)),
         D(1357005600000 + 2000000, 10.0 / 2000.0)]
# test/core/TestRateSpan.java:93-107 testNext_iterateAll
add(kind="view", name="rate_iterate_all", spec=dict(rate=True), points=RD,
    expect=RATES, tol=1e-7, cite="test/core/TestRateSpan.java:93-107")
# :129-144 testSeek
add(kind="view", name="rate_seek", spec=dict(rate=True), points=RD,
    seek=1357002000000,
    expect=[D(1357002000000, 40.0 / 1357002000)] + RATES[3:], tol=1e-7,
    cite="test/core/TestRateSpan.java:129-144")
# :146-155 testNext_decreasingTimestamps
add(kind="view", name="rate_decreasing_ts", spec=dict(rate=True),
    points=[L(1357002000000 + 5000, 50), L(1357002000000 + 4000, 50)],
    error="IllegalStateException",
    cite="test/core/TestRateSpan.java:146-155")
# :157-167 testMoveToNextRate_duplicatedTimestamps
add(kind="view", name="rate_duplicated_ts", spec=dict(rate=True),
    points=[L(1356998400000, 40), L(1356998400000 + 2000000, 50),
            L(1356998400000 + 2000000, 50)],
    error="IllegalStateException",
    cite="test/core/TestRateSpan.java:157-167")
# :169-183 testCalculateDelta_bigLongValues (second rate = 0.8 exactly)
add(kind="view", name="rate_big_longs", spec=dict(rate=True),
    points=[L(1356998400000, LMAX - 100), L(1356998500000, LMAX - 20)],
    expect=[D(1356998400000, (LMAX - 100) / 1356998400.0),
            D(1356998500000, 0.8)], tol=0, check_from=1,
    cite="test/core/TestRateSpan.java:169-183")
# :185-201 testNext_counter (COUNTER_MAX = 70)
add(kind="view", name="rate_counter",
    spec=dict(rate=True, counter=True, counter_max=70, reset_value=0),
    points=RD,
    expect=[D(1356998400000, 40.0 / 1356998400),
            D(1356998400000 + 2000000, 10.0 / 2000.0),
            D(1357002000000, (40.0 + 20) / 1600.0),
            D(1357002000000 + 5000, 10.0 / 5.0),
            D(1357005600000, (40.0 + 20) / 3595),
            D(1357005600000 + 2000000, 10.0 / 2000.0)], tol=1e-7,
    cite="test/core/TestRateSpan.java:185-201")
# :203-227 testNext_counterLongMax
add(kind="view", name="rate_counter_long_max",
    spec=dict(rate=True, counter=True, counter_max=LMAX, reset_value=0),
    points=[L(1356998430000, LMAX - 55), L(1356998460000, LMAX - 25),
            L(1356998490000, 5)],
    expect=[D(1356998430000, (LMAX - 55) / 1356998430.0),
            D(1356998460000, 1), D(1356998490000, 1)], tol=1e-7,
    cite="test/core/TestRateSpan.java:203-227")
# :229-256 testNext_counterWithResetValue (RESET_VALUE = 1)
add(kind="view", name="rate_counter_reset_value",
    spec=dict(rate=True, counter=True, counter_max=70, reset_value=1),
    points=[L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40)],
    expect=[D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10),
            D(1356998402000, 0)], tol=1e-7,
    cite="test/core/TestRateSpan.java:229-256")
# :258-286 testNext_counterDroResets
add(kind="view", name="rate_counter_drop_resets",
    spec=dict(rate=True, counter=True, counter_max=70, reset_value=1,
              drop_resets=True),
    points=[L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40),
            L(1356998403000, 50)],
    expect=[D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10),
            D(1356998403000, 10)], tol=1e-7,
    cite="test/core/TestRateSpan.java:258-286")
# :288-313 testNext_counterDroResetsNothingAfter
add(kind="view", name="rate_counter_drop_resets_nothing_after",
    spec=dict(rate=True, counter=True, counter_max=70, reset_value=1,
              drop_resets=True),
    points=[L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40)],
    expect=[D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10)],
    tol=1e-7, cite="test/core/TestRateSpan.java:288-313")

# ------------------------------------------------ TsdbQuery (integration)
# BaseTsdbTest.storeLongTimeSeriesSeconds(two_metrics, offset=False):
# web01: ts 1356998430 + 30*(i-1), value i (1..300); longs.
WEB01 = [L((1356998400 + 30 * i) * 1000, i) for i in range(1, 301)]
# test/core/TestTsdbQueryDownsample.java:136-167 runLongSingleTSDownsample:
# query [1356998400, 1357041600] s, 60000-avg, sum; scan window from
# getScanStart/EndTimeSeconds = [1356998400, 1357045200] s.
exp = []
for i in range(151):
    v = 1.0 if i == 0 else (300.0 if i >= 150 else i * 2 + 0.5)
    exp.append(D(1356998400000 + 60000 * i, v))
add(kind="group_by", name="tsdb_single_ts_downsample",
    spec=dict(start_ms=1356998400000, end_ms=1357045200000,
              query_start_ms=1356998400000, query_end_ms=1357041600000,
              agg="sum", ds_interval_ms=60000, ds_agg="avg"),
    groups=[[WEB01]], expect=[exp], tol=0.00001, check_ts_mod=60000,
    cite="test/core/TestTsdbQueryDownsample.java:136-167")
# :204-238 runLongSingleTSDownsampleAndRate
exp = []
for i in range(150):
    v = 0.025 if (i == 0 or i >= 149) else 2.0 / 60
    exp.append(D(1356998460000 + 60000 * i, v))
add(kind="group_by", name="tsdb_single_ts_downsample_rate",
    spec=dict(start_ms=1356998400000, end_ms=1357045200000,
              query_start_ms=1356998400000, query_end_ms=1357041600000,
              agg="sum", ds_interval_ms=60000, ds_agg="avg", rate=True),
    groups=[[WEB01]], expect=[exp], tol=0.001,
    cite="test/core/TestTsdbQueryDownsample.java:204-238")

# ------------------------------------------------------ scan bounds
# test/core/TestTsdbQueryDownsample.java:49-120
add(kind="scan_bounds", name="scan_fully_aligned", interval_ms=60000,
    start=1356998400, end=1357041600, expect=[1356998400, 1357045200],
    cite="test/core/TestTsdbQueryDownsample.java:49-63")
add(kind="scan_bounds", name="scan_unaligned", interval_ms=900000,
    start=1427415547 - 43200, end=1427415547,
    expect=[1427371200, 1427418000],
    cite="test/core/TestTsdbQueryDownsample.java:65-84")
add(kind="scan_bounds", name="scan_weirdly", interval_ms=86400000,
    start=1427415547 - 43200, end=1427415547,
    expect=[1427328000, 1427500800],
    cite="test/core/TestTsdbQueryDownsample.java:86-104")
add(kind="scan_bounds", name="scan_ms", interval_ms=60000,
    start=1356998400000, end=1357041600000,
    expect=[1356998400, 1357045200],
    cite="test/core/TestTsdbQueryDownsample.java:106-126")


# ------------------------------------------------- calendar downsampling
# test/core/TestDownsampler.java:390-1180, :1368-1400.  Each reference test
# iterates `while (downsampler.hasNext())` and asserts every emitted point
# against a sequence its loop computes; the loops are transcribed below as
# generators (_seq_*).  The number of points is not asserted by most of those
# tests: it is taken from bucketing the test's points on the calendar grid,
# and the generator must agree with that bucketing on every point (checked
# here at generation time) — so both the sequences and the counts are
# pinned to the reference's literals.
DST_TS = 1450137600000
TZ_AF, TZ_TV, TZ_FJ = "Asia/Kabul", "Pacific/Funafuti", "Pacific/Fiji"


def _cal_case(name, ds, tz, points, seq, cite, seek=None, n=None):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))
    from opentsdb_amd import jcalendar as J
    iv, unit = J.parse_calendar_interval(ds.split("-")[0][:-1])
    first = points[0][0] if seek is None else seek
    edges = J.bucket_edges_for_series(min(first, points[0][0]),
                                      points[-1][0], iv, unit, tz)
    lo = 0
    if seek is not None:
        k = J.edge_index(edges, seek)
        if seek > edges[k]:
            k += 1
        lo = edges[k]
    sums = {}
    for t, v, _ in points:
        if t < lo:
            continue
        k = J.edge_index(edges, t)
        sums[edges[k]] = sums.get(edges[k], 0) + v
    got = sorted(sums.items())
    if n is not None:
        assert len(got) == n, (name, got)
    exp = []
    it = seq()
    for _ in got:
        exp.append(next(it))
    assert [(t, float(v)) for t, v in got] == [(t, float(v)) for t, v in exp], (
        name, got, exp)
    add(kind="view", name=name,
        spec=dict(ds_string=ds, tz=tz, query_start_ms=0, query_end_ms=LMAX),
        points=points, seek=seek,
        expect=[D(t, v) for t, v in exp], tol=1e-3, cite=cite)


P6 = [L(BASE + 5000, 1), L(BASE + 15000, 2), L(BASE + 25000, 4),
      L(BASE + 35000, 8), L(BASE + 45000, 16), L(BASE + 55000, 32)]


def _seq_const(ts, v):
    def g():
        while True:
            yield ts, v
    return g


# :390-416 testDownsampler_calendar (asserts exactly 1 point)
_cal_case("cal_1dc_denver", "1dc-sum", "America/Denver", P6,
          _seq_const(1356937200000, 63), "test/core/TestDownsampler.java:390-416",
          n=1)
PH = [L(BASE, 1), L(BASE + 1800000, 2), L(BASE + 3599000, 3),
      L(BASE + 3600000, 4), L(BASE + 5400000, 5), L(BASE + 7199000, 6)]


def _seq_hour_tv():
    ts, v = BASE, 6
    while True:
        yield ts, v
        ts += 3600000
        v = 15


def _seq_hour_af():
    ts, v = 1356996600000, 1
    while True:
        yield ts, v
        ts += 3600000
        v = 9 if v == 1 else 11


_cal_case("cal_1hc_tv", "1hc-sum", TZ_TV, PH, _seq_hour_tv,
          "test/core/TestDownsampler.java:418-441")
_cal_case("cal_1hc_af", "1hc-sum", TZ_AF, PH, _seq_hour_af,
          "test/core/TestDownsampler.java:443-463")
_cal_case("cal_4hc_af", "4hc-sum", TZ_AF, PH,
          _seq_const(1356996600000, 21), "test/core/TestDownsampler.java:465-477")
PD = [L(DST_TS, 1), L(DST_TS + 86399000, 2), L(DST_TS + 126001000, 3),
      L(DST_TS + 172799000, 4), L(DST_TS + 172800000, 5),
      L(DST_TS + 242999000, 6)]


def _seq_day(ts, vals):
    def g():
        t, i = ts, 0
        while True:
            yield t, vals[min(i, len(vals) - 1)]
            t += 86400000
            i += 1
    return g


_cal_case("cal_1dc_utc", "1dc-sum", None, PD, _seq_day(DST_TS, [3, 7, 11]),
          "test/core/TestDownsampler.java:480-506")
_cal_case("cal_1dc_tv", "1dc-sum", TZ_TV, PD,
          _seq_day(1450094400000, [1, 5, 9, 6]),
          "test/core/TestDownsampler.java:508-530")
_cal_case("cal_1dc_fj", "1dc-sum", TZ_FJ, PD,
          _seq_day(1450090800000, [1, 2, 12, 6]),
          "test/core/TestDownsampler.java:532-553")
_cal_case("cal_1dc_af", "1dc-sum", TZ_AF, PD,
          _seq_day(1450121400000, [1, 5, 15]),
          "test/core/TestDownsampler.java:555-574")
_cal_case("cal_3dc_af", "3dc-sum", TZ_AF, PD, _seq_const(1450121400000, 21),
          "test/core/TestDownsampler.java:576-589")
PW = [L(DST_TS, 1), L(DST_TS + 86400000 * 7, 2), L(1451129400000, 3),
      L(DST_TS + 86400000 * 21, 4), L(1452367799000, 5)]


def _seq_week_utc():
    ts, v = 1449964800000, 1
    while True:
        yield ts, v
        ts = 1451779200000 if ts == 1450569600000 else ts + 86400000 * 7
        v = 5 if v == 1 else 9


def _seq_week_tv():
    ts, v = 1449921600000, 1
    while True:
        yield ts, v
        ts = 1451736000000 if ts == 1450526400000 else ts + 86400000 * 7
        v = 5 if v == 1 else (4 if v == 5 else 5)


def _seq_week_fj():
    ts, v = 1449918000000, 1
    while True:
        yield ts, v
        ts += 86400000 * 7
        v += 1


def _seq_week_af():
    ts, v = 1449948600000, 1
    while True:
        yield ts, v
        ts = 1450553400000 if ts == 1449948600000 else 1451763000000
        v = 5 if v == 1 else 9


def _seq_2week_af():
    ts, v = 1449948600000, 6
    while True:
        yield ts, v
        ts, v = 1451158200000, 9


_cal_case("cal_1wc_utc", "1wc-sum", None, PW, _seq_week_utc,
          "test/core/TestDownsampler.java:591-626")
_cal_case("cal_1wc_tv", "1wc-sum", TZ_TV, PW, _seq_week_tv,
          "test/core/TestDownsampler.java:628-653")
_cal_case("cal_1wc_fj", "1wc-sum", TZ_FJ, PW, _seq_week_fj,
          "test/core/TestDownsampler.java:655-670")
_cal_case("cal_1wc_af", "1wc-sum", TZ_AF, PW, _seq_week_af,
          "test/core/TestDownsampler.java:672-695")
_cal_case("cal_2wc_af", "2wc-sum", TZ_AF, PW, _seq_2week_af,
          "test/core/TestDownsampler.java:697-713")
DEC1 = 1448928000000
PM = [L(DEC1, 1), L(1451559600000, 2), L(1451606400000, 3),
      L(1454284800000, 4), L(1456704000000, 5), L(1456772400000, 6)]


def _seq_month_utc():
    ts, v = DEC1, 3
    while True:
        yield ts, v
        if ts == 1448928000000:
            ts = 1451606400000
        else:
            ts, v = 1454284800000, 15


def _seq_month_tv():
    ts, v = 1448884800000, 3
    while True:
        yield ts, v
        if ts == 1448884800000:
            ts = 1451563200000
        elif ts == 1451563200000:
            v, ts = 9, 1454241600000
        else:
            ts, v = 1456747200000, 6


def _seq_month_af():
    ts, v = 1448911800000, 3
    while True:
        yield ts, v
        if ts == 1448911800000:
            ts = 1451590200000
        else:
            ts, v = 1454268600000, 15


def _seq_3month_tv():
    ts, v = 1443614400000, 3
    while True:
        yield ts, v
        ts, v = 1451563200000, 18


_cal_case("cal_1nc_utc", "1nc-sum", None, PM, _seq_month_utc,
          "test/core/TestDownsampler.java:715-742")
_cal_case("cal_1nc_tv", "1nc-sum", TZ_TV, PM, _seq_month_tv,
          "test/core/TestDownsampler.java:744-766")
_cal_case("cal_1nc_af", "1nc-sum", TZ_AF, PM, _seq_month_af,
          "test/core/TestDownsampler.java:791-808")
_cal_case("cal_3nc_tv", "3nc-sum", TZ_TV, PM, _seq_3month_tv,
          "test/core/TestDownsampler.java:810-824")


def _seq_pairs(ts_list, npts):
    """(1 << j++) + (1 << j++) per bucket over the given bucket starts."""
    def g():
        j = 0
        for t in ts_list:
            yield t, float((1 << j) + (1 << (j + 1)))
            j += 2
    return g


def _month_points(t0_list):
    """testDownsampler_1month's data: two points per bucket, at the bucket
    start and half way to the next start (+1 for the UTC case)."""
    pts = []
    for i, (a, b) in enumerate(zip(t0_list, t0_list[1:])):
        pts.append(L(a, 1 << (2 * i)))
        pts.append(L(a + (b - a) // 2, 1 << (2 * i + 1)))
    return pts


# :937-960 testDownsampler_1month (UTC; bucket starts = Calendar month
# starts from Jan 2013; the second point sits at (start + (next+1)) / 2)
_M13 = [1356998400000, 1359676800000, 1362096000000, 1364774400000,
        1367366400000, 1370044800000, 1372636800000, 1375315200000,
        1377993600000, 1380585600000, 1383264000000, 1385856000000,
        1388534400000]
_pts = []
for _i in range(12):
    _a, _b = _M13[_i], _M13[_i + 1] + 1
    _pts.append(L(_a, 1 << (2 * _i)))
    _pts.append(L(_a + (_b - _a) // 2, 1 << (2 * _i + 1)))
_cal_case("cal_1nc_utc_12", "1nc-sum", None, _pts, _seq_pairs(_M13[:12], 24),
          "test/core/TestDownsampler.java:937-960", n=12)
# :1110-1135 testDownsampler_1year (UTC, 2 buckets)
_Y = [1356998400000, 1388534400000, 1420070400000]
_cal_case("cal_1yc_utc", "1yc-sum", None, _month_points(_Y),
          _seq_pairs(_Y[:2], 4), "test/core/TestDownsampler.java:1110-1135",
          n=2)
# :1368-1400 testSeek_useCalendar (second half: "1yc-sum", seek one ms past
# 2015-01-01 -> only 2016's bucket)
PY = [L(1356998400000, 1), L(1388534400000, 2), L(1420070400000, 4),
      L(1451606400000, 8)]
_cal_case("cal_seek_1yc", "1yc-sum", None, PY, _seq_const(1451606400000, 8),
          "test/core/TestDownsampler.java:1387-1397", seek=1420070400001, n=1)


def _seq_seek_exact():
    yield 1420070400000, 4
    yield 1451606400000, 8


_cal_case("cal_seek_1yc_exact", "1yc-sum", None, PY, _seq_seek_exact,
          "test/core/TestDownsampler.java:1368-1386", seek=1420070400000, n=2)


# --------------------------------------- DateTime.previousInterval KATs
# test/utils/TestDateTime.java:548-963 (assertEquals(expected,
# previousInterval(ts, interval, unit[, tz]))), transcribed as data.
# Units as DateTime.unitsToCalendarType names them ("w" = DAY_OF_WEEK);
# WEEK_OF_YEAR is not reachable from a downsampling spec and is skipped.
_D, _N = 1450152145123, 1431699673432   # DST_TS, NON_DST_TS
_AF, _NZ, _TV, _FJ = "Asia/Kabul", "Pacific/Chatham", "Pacific/Funafuti", \
    "Pacific/Fiji"
_PI = [
    # previousIntervalMilliseconds :548-589
    (_D, 1, "ms", None, _D), (_N, 1, "ms", None, _N),
    (_D, 100, "ms", None, 1450152145100), (1450152145000, 100, "ms", None,
                                           1450152145000),
    (_D, 799, "ms", None, 1450152144769),
    (_D, 100, "ms", _AF, 1450152145100), (_N, 100, "ms", _AF, 1431699673400),
    (_D, 100, "ms", _NZ, 1450152145100), (_N, 100, "ms", _NZ, 1431699673400),
    (_D, 100, "ms", _TV, 1450152145100), (_N, 100, "ms", _TV, 1431699673400),
    (_D, 100, "ms", _FJ, 1450152145100), (_N, 100, "ms", _FJ, 1431699673400),
    (_D, 60000, "ms", None, 1450152120000), (_N, 60000, "ms", None,
                                             1431699660000),
    # previousIntervalSeconds :591-636
    (_D, 1, "s", None, 1450152145000), (_N, 1, "s", None, 1431699673000),
    (_D, 30, "s", None, 1450152120000), (_N, 30, "s", None, 1431699660000),
    (1450152120000, 30, "s", None, 1450152120000),
    (_N, 29, "s", None, 1431699647000), (_D, 29, "s", None, 1450152145000),
    (_D, 30, "s", _AF, 1450152120000), (_N, 30, "s", _AF, 1431699660000),
    (_D, 30, "s", _NZ, 1450152120000), (_N, 30, "s", _NZ, 1431699660000),
    (_D, 30, "s", _TV, 1450152120000), (_N, 30, "s", _TV, 1431699660000),
    (_D, 30, "s", _FJ, 1450152120000), (_N, 30, "s", _FJ, 1431699660000),
    (_D, 60000, "s", None, 1450152000000), (_N, 60000, "s", None,
                                            1431698400000),
    # previousIntervalMinutes :638-690
    (_D, 1, "m", None, 1450152120000), (_N, 1, "m", None, 1431699660000),
    (_D, 30, "m", None, 1450152000000), (_N, 30, "m", None, 1431698400000),
    (1431698400000, 30, "m", None, 1431698400000),
    (_N, 29, "m", None, 1431698460000), (_D, 29, "m", None, 1450151520000),
    (_D, 30, "m", _AF, 1450152000000), (_N, 30, "m", _AF, 1431698400000),
    (_D, 15, "m", _AF, 1450152000000), (_N, 15, "m", _AF, 1431699300000),
    (_D, 30, "m", _NZ, 1450151100000), (_N, 30, "m", _NZ, 1431699300000),
    (_D, 30, "m", _TV, 1450152000000), (_N, 30, "m", _TV, 1431698400000),
    (_D, 30, "m", _FJ, 1450152000000), (_N, 30, "m", _FJ, 1431698400000),
    (_D, 120, "m", None, 1450152000000), (_N, 120, "m", None, 1431698400000),
    # previousIntervalHours :692-739
    (_D, 1, "h", None, 1450152000000), (_N, 1, "h", None, 1431698400000),
    (_D, 12, "h", None, 1450137600000), (_N, 12, "h", None, 1431691200000),
    (1450137600000, 12, "h", None, 1450137600000),
    (_N, 15, "h", None, 1431680400000), (_D, 15, "h", None, 1450116000000),
    (_D, 12, "h", _AF, 1450121400000), (_N, 12, "h", _AF, 1431675000000),
    (_D, 12, "h", _NZ, 1450131300000), (_N, 12, "h", _NZ, 1431688500000),
    (_D, 12, "h", _TV, 1450137600000), (_N, 12, "h", _TV, 1431691200000),
    (_D, 12, "h", _FJ, 1450134000000), (_N, 12, "h", _FJ, 1431691200000),
    (_D, 36, "h", None, 1450094400000), (_N, 36, "h", None, 1431604800000),
    # previousIntervalDays :741-787
    (_D, 1, "d", None, 1450137600000), (_N, 1, "d", None, 1431648000000),
    (_D, 7, "d", None, 1449705600000), (_N, 7, "d", None, 1431561600000),
    (1449705600000, 7, "d", None, 1449705600000),
    (1330516800000, 1, "d", None, 1330473600000),
    (_D, 1, "d", _AF, 1450121400000), (_N, 1, "d", _AF, 1431631800000),
    (_D, 1, "d", _NZ, 1450088100000), (_N, 1, "d", _NZ, 1431688500000),
    (_D, 1, "d", _TV, 1450094400000), (_N, 1, "d", _TV, 1431691200000),
    (_D, 1, "d", _FJ, 1450090800000), (_N, 1, "d", _FJ, 1431691200000),
    (_D, 60, "d", None, 1445990400000), (_N, 60, "d", None, 1430438400000),
    # previousIntervalWeeks :789-833 (Locale.US: weeks start on Sunday)
    (_D, 1, "w", None, 1449964800000), (_N, 1, "w", None, 1431216000000),
    (_D, 2, "w", None, 1449964800000), (_N, 2, "w", None, 1431216000000),
    (1435795200000, 2, "w", None, 1435449600000),
    (_D, 1, "w", _AF, 1449948600000), (_N, 1, "w", _AF, 1431199800000),
    (_D, 1, "w", _NZ, 1449915300000), (_N, 1, "w", _NZ, 1431170100000),
    (_D, 1, "w", _TV, 1449921600000), (_N, 1, "w", _TV, 1431172800000),
    (_D, 1, "w", _FJ, 1449918000000), (_N, 1, "w", _FJ, 1431172800000),
    (_D, 104, "w", None, 1449964800000), (_N, 104, "w", None, 1431216000000),
    # previousIntervalMonths :878-925
    (_D, 1, "n", None, 1448928000000), (_N, 1, "n", None, 1430438400000),
    (_D, 3, "n", None, 1443657600000), (_N, 3, "n", None, 1427846400000),
    (1443657600000, 3, "n", None, 1443657600000),
    (_D, 5, "n", None, 1446336000000), (_N, 5, "n", None, 1420070400000),
    (_D, 1, "n", _AF, 1448911800000), (_N, 1, "n", _AF, 1430422200000),
    (_D, 1, "n", _NZ, 1448878500000), (_N, 1, "n", _NZ, 1430392500000),
    (_D, 1, "n", _TV, 1448884800000), (_N, 1, "n", _TV, 1430395200000),
    (_D, 1, "n", _FJ, 1448881200000), (_N, 1, "n", _FJ, 1430395200000),
    (_D, 24, "n", None, 1420070400000), (_N, 24, "n", None, 1420070400000),
    # previousIntervalYears :927-962
    (_D, 1, "y", None, 1420070400000), (_N, 1, "y", None, 1420070400000),
    (_D, 5, "y", None, 1420070400000), (_N, 5, "y", None, 1420070400000),
    (1420070400000, 5, "y", None, 1420070400000),
    (_D, 1, "y", _AF, 1420054200000), (_N, 1, "y", _AF, 1420054200000),
    (_D, 1, "y", _NZ, 1420020900000), (_N, 1, "y", _NZ, 1420020900000),
    (_D, 1, "y", _TV, 1420027200000), (_N, 1, "y", _TV, 1420027200000),
    (_D, 1, "y", _FJ, 1420023600000), (_N, 1, "y", _FJ, 1420023600000),
]
for _k, (_t, _iv, _u, _tz, _e) in enumerate(_PI):
    add(kind="prev_interval", name="prev_%d_%s%s_%s" % (_k, _iv, _u, _tz),
        ts=_t, interval=_iv, unit=_u, tz=_tz, expect=_e,
        cite="test/utils/TestDateTime.java:548-963")


# ------------------------------------------- TsdbQuery over BaseTsdbTest data
# test/core/BaseTsdbTest.java:612-700 datasets (what tsdb.addPoint writes,
# read back as one span per series) and the expectation loops of
# test/core/TestTsdbQueryAggregators.java:44-1117 and
# test/core/TestTsdbQueryQueries.java:1358-1519, transcribed loop for loop.
# Every query is setStartTime(1356998400) / setEndTime(1357041600) with no
# group-by tag: one group {web01, web02} in SpanCmp order.  The SpanGroup
# window is getScanStart/EndTimeSeconds in ms (pinned by the scan_bounds
# KATs above): [1356998400, 1357045200] s with or without a 1 s downsample.
Q_WIN = dict(start_ms=1356998400000, end_ms=1357045200000,
             query_start_ms=1356998400000, query_end_ms=1357041600000)


def _long_seconds(offset):
    """storeLongTimeSeriesSeconds(false, offset) :612-639"""
    a, ts = [], 1356998400
    for i in range(1, 301):
        ts += 30
        a.append(L(ts * 1000, i))
    b, ts = [], (1356998415 if offset else 1356998400)
    for i in range(300, 0, -1):
        ts += 30
        b.append(L(ts * 1000, i))
    return [a, b]


def _f32_steps(start, stop_incl, step, up):
    """Java `for (float i = start; up ? i <= stop : i > stop; i += step)`
    (0.25 multiples are exact in float: the loop values are exact doubles)"""
    out, i = [], start
    while (i <= stop_incl) if up else (i > stop_incl):
        out.append(i)
        i = i + step if up else i - step
    return out


def _float_seconds(offset):
    """storeFloatTimeSeriesSeconds(false, offset) :679-706 (4-byte floats)"""
    a, ts = [], 1356998400
    for v in _f32_steps(1.25, 76.0, 0.25, True):
        ts += 30
        a.append(D(ts * 1000, v))
    b, ts = [], (1356998415 if offset else 1356998400)
    for v in _f32_steps(75.0, 0.0, 0.25, False):
        ts += 30
        b.append(D(ts * 1000, v))
    return [a, b]


def _missing_data():
    """storeLongTimeSeriesWithMissingData() :649-676"""
    a, ts = [], 1356998400
    for i in range(300):
        if i % 3 != 0:
            a.append(L(ts * 1000, i + 1))
        ts += 10
    b, ts = [], 1356998400
    for i in range(300, 0, -1):
        if i % 2 != 0:
            b.append(L(ts * 1000, i))
        ts += 10
    return [b, a][::-1]


def _q(name, agg, groups, expect, tol, cite, **extra):
    spec = dict(Q_WIN, agg=agg)
    spec.update(extra)
    add(kind="group_by", name=name, spec=spec, groups=[groups],
        expect=[expect], tol=tol, cite=cite)


TQA = "test/core/TestTsdbQueryAggregators.java"


def _seq(n, step, f, ts0=1356998430000):
    return [f(k, ts0 + step * k) for k in range(n)]


# runZimSum :44-61, runZimSumFloat :63-81
_q("tq_zimsum", "zimsum", _long_seconds(False),
   _seq(300, 30000, lambda k, t: L(t, 301)), 0, TQA + ":44-61")
_q("tq_zimsum_float", "zimsum", _float_seconds(False),
   _seq(300, 30000, lambda k, t: D(t, 76.25)), 0.001, TQA + ":63-81")


def _alt(v1, v2, d1, d2, mk, n=600, step=15000):
    """counter % 2 == 0 -> v1 (then v1 += d1) else v2 (v2 += d2)"""
    out = []
    ts = 1356998430000
    for c in range(n):
        if c % 2 == 0:
            out.append(mk(ts, v1))
            v1 += d1
        else:
            out.append(mk(ts, v2))
            v2 += d2
        ts += step
    return out


# runZimSumOffset :83-111, runZimSumFloatOffset :113-141
_q("tq_zimsum_offset", "zimsum", _long_seconds(True),
   _alt(1, 300, 1, -1, L), 0, TQA + ":83-111")
_q("tq_zimsum_float_offset", "zimsum", _float_seconds(True),
   _alt(1.25, 75.0, 0.25, -0.25, D), 0.001, TQA + ":113-141")


# runZimSumWithMissingData :143-199
def _exp_missing():
    out, i, ts = [], 0, 1356998400000
    while len(out) < 250:
        offset = i % 6
        if offset == 0:
            ts += 10000
            i += 1
            offset += 1
        if offset in (1, 5):
            v = 301
        elif offset in (2, 4):
            v = i + 1
        else:
            v = 300 - i
        out.append(L(ts, v))
        ts += 10000
        i += 1
    return out


_q("tq_zimsum_missing", "zimsum", _missing_data(), _exp_missing(), 0,
   TQA + ":143-199")


def _updown(v, step, dec, turn, reset, mk, n=300, ts_step=30000, cmp="eq"):
    """the min/max/dev/mimmin/mimmax loops: assert v, step it, and flip the
    direction when it crosses `turn` (then set it to `reset`)"""
    out, ts = [], 1356998430000
    for _ in range(n):
        out.append(mk(ts, v))
        ts += ts_step
        v = v - step if dec else v + step
        hit = {"eq": v == turn, "gt": v > turn, "lt": v < turn}[cmp]
        if hit:
            v = reset
            dec = not dec
    return out


# runMin :201-232 / runMimMin :718-749 (v == 151 -> 150, decrement)
for nm, agg, cite in (("min", "min", ":201-232"), ("mimmin", "mimmin", ":718-749")):
    _q("tq_" + nm, agg, _long_seconds(False),
       _updown(1, 1, False, 151, 150, L), 0, TQA + cite)
# runMinFloat :234-265 / runMimMinFloat :782-813 (v > 38 -> 38.0)
for nm, agg, cite in (("min", "min", ":234-265"), ("mimmin", "mimmin", ":782-813")):
    _q("tq_%s_float" % nm, agg, _float_seconds(False),
       _updown(1.25, 0.25, False, 38, 38.0, D, cmp="gt"), 0.0001, TQA + cite)
# runMax :334-365 / runMimMax :846-877 (v == 150 -> 151, increment)
for nm, agg, cite in (("max", "max", ":334-365"), ("mimmax", "mimmax", ":846-877")):
    _q("tq_" + nm, agg, _long_seconds(False),
       _updown(300, 1, True, 150, 151, L), 0, TQA + cite)
# runMaxFloat :367-398 / runMimMaxFloat :879-910 (v < 38.25 -> 38.25)
for nm, agg, cite in (("max", "max", ":367-398"), ("mimmax", "mimmax", ":879-910")):
    _q("tq_%s_float" % nm, agg, _float_seconds(False),
       _updown(75.0, 0.25, True, 38.25, 38.25, D, cmp="lt"), 0.001, TQA + cite)


# runMinOffset :267-300
def _exp_min_offset():
    out, v, ts, counter, dec = [], 1, 1356998430000, 0, False
    while len(out) < 600:
        out.append(L(ts, v))
        ts += 15000
        if counter % 2 != 0:
            v = v - 1 if dec else v + 1
        elif v == 151:
            v = 150
            dec = True
            counter -= 1
        counter += 1
    return out


_q("tq_min_offset", "min", _long_seconds(True), _exp_min_offset(), 0,
   TQA + ":267-300")


# runMinFloatOffset :302-332
def _exp_min_float_offset():
    out, v, ts, dec = [], 1.25, 1356998430000, False
    for _ in range(600):
        out.append(D(ts, v))
        ts += 15000
        v = v - 0.125 if dec else v + 0.125
        if v > 38.125:
            v = 38.125
            dec = True
    return out


_q("tq_min_float_offset", "min", _float_seconds(True),
   _exp_min_float_offset(), 0.001, TQA + ":302-332")


# runMaxOffset :400-439
def _exp_max_offset():
    out, v, ts, counter, dec = [], 1, 1356998430000, 0, True
    for _ in range(600):
        out.append(L(ts, v))
        t = ts
        ts += 15000
        if v == 1:
            v = 300
        elif t == 1357007400000:
            v = 1
        elif counter % 2 == 0:
            v = v - 1 if dec else v + 1
        if v == 150:
            v = 151
            dec = False
            counter -= 1
        counter += 1
    return out


_q("tq_max_offset", "max", _long_seconds(True), _exp_max_offset(), 0,
   TQA + ":400-439")


# runMaxFloatOffset :441-477
def _exp_max_float_offset():
    out, v, ts, dec = [], 1.25, 1356998430000, True
    for _ in range(600):
        out.append(D(ts, v))
        t = ts
        ts += 15000
        if v == 1.25:
            v = 75.0
        elif t == 1357007400000:
            v = 0.25
        else:
            v = v - 0.125 if dec else v + 0.125
            if v < 38.25:
                v = 38.25
                dec = False
    return out


_q("tq_max_float_offset", "max", _float_seconds(True),
   _exp_max_float_offset(), 0.0001, TQA + ":441-477")

# runAvg :479-497, runAvgFloat :499-517
_q("tq_avg", "avg", _long_seconds(False),
   _seq(300, 30000, lambda k, t: L(t, 150)), 0, TQA + ":479-497")
_q("tq_avg_float", "avg", _float_seconds(False),
   _seq(300, 30000, lambda k, t: D(t, 38.125)), 0.001, TQA + ":499-517")


# runAvgOffset :519-547
def _exp_avg_offset():
    out, v, ts = [], 1, 1356998430000
    for _ in range(600):
        out.append(L(ts, v))
        t = ts
        ts += 15000
        if v == 1:
            v = 150
        elif t == 1357007400000:
            v = 1
        elif v == 150:
            v = 151
        else:
            v = 150
    return out


_q("tq_avg_offset", "avg", _long_seconds(True), _exp_avg_offset(), 0,
   TQA + ":519-547")


# runAvgFloatOffset :549-573
def _exp_avg_float_offset():
    out, v, ts = [], 1.25, 1356998430000
    for _ in range(600):
        out.append(D(ts, v))
        t = ts
        ts += 15000
        if v == 1.25:
            v = 38.1875
        elif t == 1357007400000:
            v = 0.25
    return out


_q("tq_avg_float_offset", "avg", _float_seconds(True),
   _exp_avg_float_offset(), 0.0001, TQA + ":549-573")

# runDev :575-606 (v < 0 -> 0, increment), runDevFloat :608-639
_q("tq_dev", "dev", _long_seconds(False),
   _updown(149, 1, True, 0, 0, L, cmp="lt"), 0, TQA + ":575-606")
_q("tq_dev_float", "dev", _float_seconds(False),
   _updown(36.875, 0.25, True, 0.125, 0.125, D, cmp="lt"), 0.001,
   TQA + ":608-639")


# runDevOffset :641-679
def _exp_dev_offset():
    out, v, ts, counter, dec = [], 0, 1356998430000, 0, True
    for _ in range(600):
        out.append(L(ts, v))
        t = ts
        ts += 15000
        if t == 1356998430000:
            v = 149
        elif t == 1357007400000:
            v = 0
        elif counter % 2 == 0:
            v = v - 1 if dec else v + 1
            if v < 0:
                v = 0
                dec = False
                counter += 1
        counter += 1
    return out


_q("tq_dev_offset", "dev", _long_seconds(True), _exp_dev_offset(), 0,
   TQA + ":641-679")


# runDevFloatOffset :681-716
def _exp_dev_float_offset():
    out, v, ts, dec = [], 0.0, 1356998430000, True
    for _ in range(600):
        out.append(D(ts, v))
        t = ts
        ts += 15000
        if t == 1356998430000:
            v = 36.8125
        elif t == 1357007400000:
            v = 0.0
        else:
            v = v - 0.125 if dec else v + 0.125
            if v < 0.0625:
                v = 0.0625
                dec = False
    return out


_q("tq_dev_float_offset", "dev", _float_seconds(True),
   _exp_dev_float_offset(), 0.0001, TQA + ":681-716")

# runMimMinOffset :751-780, runMimMinFloatOffset :815-844,
# runMimMaxOffset :912-941, runMimMaxFloatOffset :943-972
_q("tq_mimmin_offset", "mimmin", _long_seconds(True),
   _alt(1, 300, 1, -1, L), 0, TQA + ":751-780")
_q("tq_mimmin_float_offset", "mimmin", _float_seconds(True),
   _alt(1.25, 75.0, 0.25, -0.25, D), 0.001, TQA + ":815-844")
_q("tq_mimmax_offset", "mimmax", _long_seconds(True),
   _alt(1, 300, 1, -1, L), 0, TQA + ":912-941")
_q("tq_mimmax_float_offset", "mimmax", _float_seconds(True),
   _alt(1.25, 75.0, 0.25, -0.25, D), 0.001, TQA + ":943-972")

# runPercentiles :974-996 + testPercentile :1099-1116 (value 150, delta 150:
# the test pins the constructor path and the emission grid, not precision)
for _p in ("p50", "p75", "p90", "p95", "p99", "p999", "ep50r3", "ep75r3",
           "ep90r3", "ep95r3", "ep99r3", "ep999r3", "ep50r7", "ep75r7",
           "ep90r7", "ep95r7", "ep99r7", "ep999r7"):
    _q("tq_pct_" + _p, _p, _long_seconds(True),
       _seq(600, 15000, lambda k, t: L(t, 150)), 150, TQA + ":974-996,1099-1116")

# runCount :998-1013, runCountFloat :1015-1030 (doubleValue: a long
# result read as a double), runCountOffset :1032-1053,
# runCountFloatOffset :1055-1076
_q("tq_count", "count", _long_seconds(False),
   _seq(300, 30000, lambda k, t: L(t, 2)), 0, TQA + ":998-1013")
_q("tq_count_float", "count", _float_seconds(False),
   _seq(300, 30000, lambda k, t: [t, 2.0, 1]), 0.001, TQA + ":1015-1030")
_q("tq_count_offset", "count", _long_seconds(True),
   _seq(600, 15000, lambda k, t: L(t, 1 if k in (0, 599) else 2)), 0,
   TQA + ":1032-1053")
_q("tq_count_float_offset", "count", _float_seconds(True),
   _seq(600, 15000, lambda k, t: [t, 1.0 if k in (0, 599) else 2.0, 1]),
   0.0001, TQA + ":1055-1076")

TQQ = "test/core/TestTsdbQueryQueries.java"


# runInterpolationSeconds :1357-1392 (LERP, long): the offset dataset
def _exp_interp_seconds():
    out, v, ts = [], 1, 1356998430000
    for _ in range(600):
        out.append(L(ts, v))
        t = ts
        ts += 15000
        if t == 1357007400000:
            v = 1
        elif v == 1 or v == 302:
            v = 301
        else:
            v = 302
    return out


_q("tq_interp_seconds", "sum", _long_seconds(True), _exp_interp_seconds(), 0,
   TQQ + ":1357-1392")


# runInterpolationMs :1394-1429
def _ms_series(t0, step, vals):
    out, t = [], t0
    for v in vals:
        t += step
        out.append(L(t, v))
    return out


def _exp_interp_ms():
    out, v, ts = [], 1, 1356998400500
    for _ in range(600):
        out.append(L(ts, v))
        t = ts
        ts += 250
        if t == 1356998550000:
            v = 1
        elif v == 1 or v == 302:
            v = 301
        else:
            v = 302
    return out


_q("tq_interp_ms", "sum",
   [_ms_series(1356998400000, 500, range(1, 301)),
    _ms_series(1356998400250, 500, range(300, 0, -1))],
   _exp_interp_ms(), 0, TQQ + ":1394-1429")


# runInterpolationMsDownsampled :1431-1519 (1 s sum downsample, LERP of
# the downsampled points, tolerance 1e-7)
def _ds_ts1():
    out, t = [], 1356998400000
    for i in range(1, 121):
        t += 500 if i <= 100 else 5000
        out.append(L(t, i))
    return out


def _exp_interp_ms_ds():
    out = []
    ts = 1356998400000
    for i in range(151):
        if i == 0:
            v = 301.0
        elif i < 50:
            v = 602.0
        else:
            v = 701 + (i - 50) * 0.2 - i * 4
        out.append(D(ts, v))
        ts += 1000
    return out


_q("tq_interp_ms_downsampled", "sum",
   [_ds_ts1(), _ms_series(1356998400250, 500, range(300, 0, -1))],
   _exp_interp_ms_ds(), 0.0000001, TQQ + ":1431-1519",
   ds_interval_ms=1000, ds_agg="sum")


# ------------------------------------------ query-time compaction (bytes)
# test/core/TestCompactionQueue.java: each test's KeyValues (makekv stamps
# them with increasing HBase timestamps, :1537-1539: the later cell is the
# newer one) and the compacted column it asserts.  fix_duplicates is true
# (:95-97) unless the test turns it off.  Hex strings.
import struct as _st


def _Lb(x):
    return _st.pack(">q", x)


def _Ib(x):
    return _st.pack(">I", x & 0xFFFFFFFF)


_ZB = b"\x00"
_NOTE_Q = bytes([1, 0, 0])
_NOTE = (b'{"tsuid":"ABCD","description":"Description","notes":"Notes",'
         b'"custom":null,"endTime":1328140801,"startTime":1328140800}')
_APPQ = bytes([0x05, 0x00, 0x00])
TCQ = "test/core/TestCompactionQueue.java"


def _cq(name, cols, expect, cite, fix=True, error=None):
    c = dict(kind="compact", name=name,
             columns=[[q.hex(), v.hex()] for q, v in cols],
             fix_duplicates=fix, cite=TCQ + cite)
    if error:
        c["error"] = error
    else:
        c["expect"] = None if expect is None else [expect[0].hex(),
                                                   expect[1].hex()]
    add(**c)


_q1, _q2 = bytes([0, 7]), bytes([0, 0x17])
_cq("emptyRow", [], None, ":134-146")
_cq("oneCellRow", [(_q1, _Lb(42))], (_q1, _Lb(42)), ":148-164")
_cq("oneCellAppend", [(_APPQ, _q1 + _Lb(42))], (_q1, _Lb(42)), ":166-183")
_cq("oneCellRowWAnnotation", [(_NOTE_Q, _NOTE), (_q1, _Lb(42))],
    (_q1, _Lb(42)), ":185-203")
_cq("oneCellAppendWAnnotation", [(_NOTE_Q, _NOTE), (_APPQ, _q1 + _Lb(42))],
    (_q1, _Lb(42)), ":205-224")
_cq("oneCellRowBadLength", [(bytes([0, 3]), _Lb(42))],
    (bytes([0, 7]), _Lb(42)), ":246-262")
_qm = bytes([0xF0, 0, 0, 7])
_cq("oneCellRowMS", [(_qm, _Lb(42))], (_qm, _Lb(42)), ":264-280")
_cq("twoCellRow", [(_q1, _Lb(4)), (_q2, _Lb(5))],
    (_q1 + _q2, _Lb(4) + _Lb(5) + _ZB), ":282-302")
_cq("twoCellAppend", [(_APPQ, _q1 + _Lb(42) + _q2 + _Lb(5))],
    (_q1 + _q2, _Lb(42) + _Lb(5) + _ZB), ":304-323")
_cq("twoCellRowWAnnotation", [(_NOTE_Q, _NOTE), (_q1, _Lb(4)), (_q2, _Lb(5))],
    (_q1 + _q2, _Lb(4) + _Lb(5) + _ZB), ":325-347")
_cq("twoCellAppendWAnnotations",
    [(_NOTE_Q, _NOTE), (_APPQ, _q1 + _Lb(42) + _q2 + _Lb(5))],
    (_q1 + _q2, _Lb(42) + _Lb(5) + _ZB), ":349-370")
_fq = [_st.pack(">H", ((i << 4) | 0x07) & 0xFFFF) for i in range(3600)]
_cq("fullRowSeconds", [(_fq[i], _Lb(i)) for i in range(3600)],
    (b"".join(_fq), b"".join(_Lb(i) for i in range(3600)) + _ZB), ":372-397")
_mq1, _mq2 = bytes([0xF0, 0, 0, 7]), bytes([0xF0, 0, 1, 7])
_cq("twoCellRowMS", [(_mq1, _Lb(4)), (_mq2, _Lb(5))],
    (_mq1 + _mq2, _Lb(4) + _Lb(5) + _ZB), ":425-445")
_sq2, _sq3 = bytes([0xF0, 0, 2, 7]), bytes([0xF0, 0, 1, 7])
_cq("sortMsAndS", [(_q1, _Lb(4)), (_sq2, _Lb(5)), (_sq3, _Lb(5))],
    (_q1 + _sq3 + _sq2, _Lb(4) + _Lb(5) + _Lb(5) + b"\x01"), ":447-473")
_o1, _o2, _o3 = bytes([2, 7]), bytes([0, 7]), bytes([1, 7])
_cq("secondsOutOfOrder", [(_o1, _Lb(4)), (_o2, _Lb(5)), (_o3, _Lb(6))],
    (_o2 + _o3 + _o1, _Lb(5) + _Lb(6) + _Lb(4) + _ZB), ":475-501")
_m1, _m2, _m3 = (bytes([0xF0, 0, 2, 7]), bytes([0xF0, 0, 0, 7]),
                 bytes([0xF0, 0, 1, 7]))
_cq("msOutOfOrder", [(_m1, _Lb(4)), (_m2, _Lb(5)), (_m3, _Lb(6))],
    (_m2 + _m3 + _m1, _Lb(5) + _Lb(6) + _Lb(4) + _ZB), ":503-530")
_cq("secondAndMs", [(_q1, _Lb(4)), (_mq2, _Lb(5))],
    (_q1 + _mq2, _Lb(4) + _Lb(5) + b"\x01"), ":532-553")
_cq("secondAndMsWAnnotation", [(_NOTE_Q, _NOTE), (_q1, _Lb(4)), (_mq2, _Lb(5))],
    (_q1 + _mq2, _Lb(4) + _Lb(5) + b"\x01"), ":555-578")
_cq("msSameAsSecond", [(_q1, _Lb(4)), (_mq1, _Lb(5))], None, ":580-593",
    fix=False, error="IllegalDataException")
_cq("msSameAsSecondFix", [(_q1, _Lb(4)), (_mq1, _Lb(5))], (_mq1, _Lb(5)),
    ":595-614")
_cq("fixQualifierFlags", [(bytes([0, 3]), _Lb(4)), (_q2, _Lb(5))],
    (bytes([0, 7]) + _q2, _Lb(4) + _Lb(5) + _ZB), ":616-639")
_f42 = _st.unpack(">i", _st.pack(">f", 4.2))[0]
_cq("fixFloatingPoint", [(_q1, _Lb(4)), (bytes([0, 0x1B]), _Lb(_f42))],
    (_q1 + bytes([0, 0x1B]), _Lb(4) + _Ib(_f42) + _ZB), ":641-666")
_cq("overlappingDataPoints", [(_q1, _Lb(4)), (bytes([0, 3]), _Ib(4))], None,
    ":668-682", fix=False, error="IllegalDataException")
_cq("overlappingDataPointsFix", [(_q1, _Lb(4)), (bytes([0, 3]), _Ib(4))],
    (bytes([0, 3]), _Ib(4)), ":684-704")
_cq("failedCompactNoop",
    [(_q1, _Lb(4)), (_q2, _Lb(5)), (_q1 + _q2, _Lb(4) + _Lb(5) + _ZB)],
    (_q1 + _q2, _Lb(4) + _Lb(5) + _ZB), ":706-731")
_cq("annotationOnly", [(_NOTE_Q, _NOTE)], None, ":733-747")
_cq("annotationsOnly", [(_NOTE_Q, _NOTE), (bytes([1, 0, 1]), _NOTE)], None,
    ":749-766")
_w2, _w3 = bytes([0, 0x27]), bytes([0, 0x17])
_cq("weirdOverlappingCompactedCells",
    [(_q1, _Lb(4)), (_q1 + _w2, _Lb(4) + _Lb(5) + _ZB),
     (_q1 + _w3, _Lb(4) + _Lb(6) + _ZB), (_w3, _Lb(6)), (_w2, _Lb(5))],
    (_q1 + _w3 + _w2, _Lb(4) + _Lb(6) + _Lb(5) + _ZB), ":1065-1101")
_t = [bytes([0, (k << 4) | 7]) for k in (0, 2, 3, 4, 5, 6)]
_tv = [_Lb(x) for x in (4, 5, 6, 7, 8, 9)]
_cq("tripleCompacted",
    [(_t[0] + _t[1], _tv[0] + _tv[1] + _ZB), (_t[2] + _t[3], _tv[2] + _tv[3] + _ZB),
     (_t[4] + _t[5], _tv[4] + _tv[5] + _ZB)],
    (b"".join(_t), b"".join(_tv) + _ZB), ":1103-1144")
_cq("tripleCompactedOutOfOrder",
    [(_t[0] + _t[1], _tv[0] + _tv[1] + _ZB), (_t[4] + _t[5], _tv[4] + _tv[5] + _ZB),
     (_t[2] + _t[3], _tv[2] + _tv[3] + _ZB)],
    (b"".join(_t), b"".join(_tv) + _ZB), ":1146-1187")
_tm = [bytes([0xF0, 0, 0, 7]), bytes([0, 0x27]), bytes([0, 0x37]),
       bytes([0xF0, 0x04, 0x65, 0x07]), bytes([0xF0, 0x05, 0x5F, 0x07]),
       bytes([0, 0x67])]
_cq("tripleCompactedSecondsAndMs",
    [(_tm[0] + _tm[1], _tv[0] + _tv[1] + _ZB),
     (_tm[2] + _tm[3], _tv[2] + _tv[3] + _ZB),
     (_tm[4] + _tm[5], _tv[4] + _tv[5] + _ZB)],
    (b"".join(_tm), b"".join(_tv) + b"\x01"), ":1189-1232")
_a = [bytes([0, (k << 4) | 7]) for k in range(6)]
_av = [_Lb(x) for x in (42, 5, 3, 2, 1, 0)]
_cq("appendsAndLaterPuts",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]), (_a[2], _av[2]), (_a[3], _av[3])],
    (b"".join(_a[:4]), b"".join(_av[:4]) + _ZB), ":1234-1261")
_cq("appendsAndEarlierPuts",
    [(_a[0], _av[0]), (_a[1], _av[1]), (_APPQ, _a[2] + _av[2] + _a[3] + _av[3])],
    (b"".join(_a[:4]), b"".join(_av[:4]) + _ZB), ":1263-1290")
_cq("appendsAndInterspersedPuts",
    [(_a[0], _av[0]), (_a[2], _av[2]), (_APPQ, _a[1] + _av[1] + _a[3] + _av[3])],
    (b"".join(_a[:4]), b"".join(_av[:4]) + _ZB), ":1292-1319")
_cq("doubleAppends",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]),
     (_APPQ, _a[2] + _av[2] + _a[3] + _av[3])],
    (b"".join(_a[:4]), b"".join(_av[:4]) + _ZB), ":1321-1348")
_cq("tripleAppends",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]),
     (_APPQ, _a[2] + _av[2] + _a[3] + _av[3]),
     (_APPQ, _a[4] + _av[4] + _a[5] + _av[5])],
    (b"".join(_a), b"".join(_av) + _ZB), ":1350-1383")
_cq("doubleAppendsAndPuts",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]), (_a[2], _av[2]), (_a[3], _av[3]),
     (_APPQ, _a[4] + _av[4] + _a[5] + _av[5])],
    (b"".join(_a), b"".join(_av) + _ZB), ":1385-1418")
_cq("appendsAndCompacted",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]),
     (_a[2] + _a[3], _av[2] + _av[3] + _ZB)],
    (b"".join(_a[:4]), b"".join(_av[:4]) + _ZB), ":1420-1447")
_cq("appendsAndCompactedAndPuts",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]),
     (_a[2] + _a[3], _av[2] + _av[3] + _ZB), (_a[4], _av[4]), (_a[5], _av[5])],
    (b"".join(_a), b"".join(_av) + _ZB), ":1449-1482")
_cq("appendsDuplicatePuts",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]), (_a[0], _av[0]), (_a[1], _av[1])],
    (_a[0] + _a[1], _av[0] + _av[1] + _ZB), ":1484-1505")
_cq("appendsDuplicateCompacted",
    [(_APPQ, _a[0] + _av[0] + _a[1] + _av[1]),
     (_a[0] + _a[1], _av[0] + _av[1] + _ZB)],
    (_a[0] + _a[1], _av[0] + _av[1] + _ZB), ":1507-1530")

# TestInternal.extractDataPoints (test/core/TestInternal.java:43-286): the
# per-cell fix-ups and breakdown it asserts, restated as the compaction of
# the same columns (distinct, increasing offsets: the compacted column is
# the asserted cells concatenated, meta byte 1 iff seconds and ms mix).
TIN = "test/core/TestInternal.java"
_B = 1356998400


def _ci(name, cols, cells, cite, error=None):
    if error:
        add(kind="compact", name=name, columns=[[q.hex(), v.hex()] for q, v in cols],
            fix_duplicates=True, error=error, cite=TIN + cite)
        return
    mixed = len({len(q) for q, _ in cells}) > 1
    q = b"".join(c[0] for c in cells)
    v = b"".join(c[1] for c in cells) + (bytes([1 if mixed else 0])
                                        if len(cells) > 1 else b"")
    add(kind="compact", name=name, columns=[[a.hex(), b.hex()] for a, b in cols],
        fix_duplicates=True, expect=[q.hex(), v.hex()], cite=TIN + cite)


_ci("extractDataPointsFixQualifierFlags",
    [(bytes([0, 0x07]), _Lb(4)), (bytes([0, 0x27]), _Ib(5)),
     (bytes([0, 0x43]), _Lb(6))],
    [(bytes([0, 0x07]), _Lb(4)), (bytes([0, 0x23]), _Ib(5)),
     (bytes([0, 0x47]), _Lb(6))], ":43-64")
_ci("extractDataPointsFixFloatingPointValue",
    [(bytes([0, 0x0F]), bytes(7) + b"\1"), (bytes([0, 0x2B]), bytes(7) + b"\1"),
     (bytes([0, 0x4B]), bytes(3) + b"\1")],
    [(bytes([0, 0x0F]), bytes(7) + b"\1"), (bytes([0, 0x2B]), bytes(3) + b"\1"),
     (bytes([0, 0x4B]), bytes(3) + b"\1")], ":67-88")
_ci("extractDataPointsFixFloatingPointValueCorrupt",
    [(bytes([0, 0x0F]), bytes(7) + b"\1"),
     (bytes([0, 0x2B]), b"\0\2" + bytes(5) + b"\1"),
     (bytes([0, 0x4B]), bytes(3) + b"\1")], None, ":91-105",
    error="IllegalDataException")
_ci("extractDataPointsMixSecondsMs",
    [(bytes([0, 0x27]), _Lb(4)), (bytes([1, 0, 2]), b"Annotation"),
     (bytes([0, 0x47]), _Lb(6))],
    [(bytes([0, 0x27]), _Lb(4)), (bytes([0, 0x47]), _Lb(6))], ":108-125")
_ms2 = bytes([0xF0, 0, 2, 7])
_ci("extractDataPointsWithNonDataColumns",
    [(bytes([0, 0x07]), _Lb(4)), (_ms2, _Lb(5)), (bytes([0, 0x47]), _Lb(6))],
    [(bytes([0, 0x07]), _Lb(4)), (_ms2, _Lb(5)), (bytes([0, 0x47]), _Lb(6))],
    ":128-147")
_ci("extractDataPointsWithNonDataColumnsSort",
    [(bytes([0, 0x47]), _Lb(6)), (_ms2, _Lb(5)), (bytes([0, 0x07]), _Lb(4))],
    [(bytes([0, 0x07]), _Lb(4)), (_ms2, _Lb(5)), (bytes([0, 0x47]), _Lb(6))],
    ":150-169")

# compacted columns broken down by the decode (RowSeq / extractDataPoints
# agree on a sorted column): points (ts ms, long value) or the exception
def _dk(name, q, v, expect, cite, error=None):
    c = dict(kind="decode", name=name, qual=q.hex(), val=v.hex(), base=_B,
             cite=TIN + cite)
    if error:
        c["error"] = error
    else:
        c["expect"] = expect
    add(**c)


_dk("extractDataPointsCompactSeconds", bytes([0, 7, 0, 0x27, 0, 0x47]),
    _Lb(4) + _Lb(5) + _Lb(6) + _ZB,
    [[_B * 1000, 4], [_B * 1000 + 2000, 5], [_B * 1000 + 4000, 6]], ":172-193")
_dk("extractDataPointsCompactMs",
    bytes([0xF0, 0, 0, 7, 0xF0, 0, 2, 7, 0xF0, 0, 7, 7]),
    _Lb(4) + _Lb(5) + _Lb(6) + _ZB,
    [[_B * 1000, 4], [_B * 1000 + 8, 5], [_B * 1000 + 28, 6]], ":220-244")
_dk("extractDataPointsCompactSecAndMs",
    bytes([0, 7, 0xF0, 0, 2, 7, 0, 0x47]), _Lb(4) + _Lb(5) + _Lb(6) + _ZB,
    [[_B * 1000, 4], [_B * 1000 + 8, 5], [_B * 1000 + 4000, 6]], ":247-269")
_dk("extractDataPointsCompactCorrupt",
    bytes([0, 7, 0xF0, 0, 2, 7, 0, 0x41]), _Lb(4) + _Lb(5) + _Lb(6) + _ZB,
    None, ":272-286", error="IllegalDataException")

# ----------------------------------------------------- span assembly (bytes)
# test/core/TestRowSeq.java:122-508: rows of one series handed to the span
# in this order (setRow + addRow), and the data points the series yields
# (timestamps, long values).  Base time 1356998400 (KEY).
TRS = "test/core/TestRowSeq.java"
_B = 1356998400


def _sp(name, rows, expect, cite):
    add(kind="span", name=name,
        rows=[[b, q.hex(), v.hex()] for b, q, v in rows],
        expect=[[t, x] for t, x in expect], cite=TRS + cite)


def _sq(*ks):
    return b"".join(bytes([0, (k << 4) | 7]) for k in ks)


def _sv(*xs):
    return b"".join(_Lb(x) for x in xs) + _ZB


_E4 = [(1356998400000, 4), (1356998402000, 5), (1356998403000, 6),
       (1356998404000, 7)]
_sp("addRowMergeLater", [(_B, _sq(0, 2), _sv(4, 5)), (_B, _sq(3, 4), _sv(6, 7))],
    _E4, ":122-150")
_sp("addRowMergeEarlier", [(_B, _sq(3, 4), _sv(6, 7)), (_B, _sq(0, 2), _sv(4, 5))],
    _E4, ":187-215")
_sp("addRowMergeMiddle",
    [(_B, _sq(0, 2), _sv(4, 5)), (_B, _sq(5, 6), _sv(8, 9)),
     (_B, _sq(3, 4), _sv(6, 7))],
    _E4 + [(1356998405000, 8), (1356998406000, 9)], ":252-292")
_sp("addRowMergeDuplicateLater",
    [(_B, _sq(0, 2, 3), _sv(4, 5, 6)), (_B, _sq(3, 4), _sv(6, 7))], _E4,
    ":342-370")
_sp("addRowMergeDuplicateEarlier",
    [(_B, _sq(2, 3, 4), _sv(5, 6, 7)), (_B, _sq(0, 2), _sv(4, 5))], _E4,
    ":372-400")
_msq = lambda *ms: b"".join(_Ib((0xF << 28) | (m << 6) | 7) for m in ms)  # noqa
_sp("addRowMergeMs",
    [(_B, _msq(0, 8), _sv(4, 5)), (_B, _msq(28, 36), _sv(6, 7))],
    [(1356998400000, 4), (1356998400008, 5), (1356998400028, 6),
     (1356998400036, 7)], ":447-475")
_sp("addRowMergeSecAndMs",
    [(_B, _sq(0) + _msq(8), _Lb(4) + _Lb(5) + b"\x01"),
     (_B, _sq(3) + _msq(1060), _Lb(6) + _Lb(7) + b"\x01")],
    [(1356998400000, 4), (1356998400008, 5), (1356998403000, 6),
     (1356998401060, 7)], ":477-507")
# timestamp / iterate tests :523-696 (one row)
_sp("timestamp", [(_B, _sq(0, 2), _sv(4, 5))],
    [(1356998400000, 4), (1356998402000, 5)], ":523-538")
_sp("timestampMs", [(_B, _msq(0, 8), _sv(4, 5))],
    [(1356998400000, 4), (1356998400008, 5)], ":575-590")
_sp("timestampMixedNormalized", [(_B, _sq(0) + _msq(8), _sv(4, 5))],
    [(1356998400000, 4), (1356998400008, 5)], ":592-607")


# ------------------------------------------- round 6: the remaining in-scope
# TestDownsampler / TestFillingDownsampler tests (rollup tests excluded: out
# of scope).  Same conventions as above; `prefix` marks a test
# that asserts only the first point(s) after a seek.
TDS = "test/core/TestDownsampler.java"
TFD = "test/core/TestFillingDownsampler.java"
DS6 = [L(BASE + 5000, 1), L(BASE + 15000, 2), L(BASE + 25000, 4),
       L(BASE + 35000, 8), L(BASE + 45000, 16), L(BASE + 55000, 32)]
# testDownsamplerDeprecated :108-132 (Downsampler(source, 1000 s, avg):
# query_start = query_end = 0, Downsampler.java:76-91)
add(kind="view", name="ds_deprecated_1000s_avg",
    spec=dict(ds_interval_ms=1000000, ds_agg="avg", query_start_ms=0,
              query_end_ms=0), points=DS_DATA,
    expect=[D(BASE - 400000, 40), D(BASE + 1600000, 50),
            D(BASE + 3600000, 45), D(BASE + 6600000, 40),
            D(BASE + 8600000, 50)], tol=1e-7, cite=TDS + ":108-132")
# testDownsamplerDeprecated_10seconds :134-173 (10000 ms sum)
add(kind="view", name="ds_deprecated_10s_sum",
    spec=dict(ds_interval_ms=10000, ds_agg="sum", query_start_ms=0,
              query_end_ms=0), points=P10,
    expect=[D(BASE, 3), D(BASE + 10000, 12), D(BASE + 20000, 48),
            D(BASE + 30000, 192), D(BASE + 40000, 768),
            D(BASE + 50000, 1024)], tol=1e-7, cite=TDS + ":134-173")
# testDownsamplerDeprecated_15seconds :217-247
add(kind="view", name="ds_deprecated_15s_sum",
    spec=dict(ds_interval_ms=15000, ds_agg="sum", query_start_ms=0,
              query_end_ms=0), points=P15,
    expect=[D(BASE, 1), D(BASE + 15000, 6), D(BASE + 30000, 8),
            D(BASE + 45000, 48)], tol=1e-7, cite=TDS + ":217-247")
# testDownsampler_allFullRange :282-308 ("0all-sum", [0, Long.MAX])
add(kind="view", name="ds_all_full_range",
    spec=dict(ds_string="0all-sum", query_start_ms=0, query_end_ms=LMAX),
    points=DS6, expect=[D(0, 63)], tol=1e-7, cite=TDS + ":282-308")
# testDownsampler_allFilterOnQuery :310-336 (query [BASE+15 s, BASE+45 s])
add(kind="view", name="ds_all_filter_on_query",
    spec=dict(ds_string="0all-sum", query_start_ms=BASE + 15000,
              query_end_ms=BASE + 45000),
    points=DS6, expect=[D(BASE + 15000, 14)], tol=1e-7, cite=TDS + ":310-336")
# testDownsampler_allFilterOnQueryOutOfRangeEarly :338-362
add(kind="view", name="ds_all_out_of_range_early",
    spec=dict(ds_string="0all-sum", query_start_ms=BASE + 65000,
              query_end_ms=BASE + 75000),
    points=DS6, expect=[], tol=0, cite=TDS + ":338-362")
# testDownsampler_allFilterOnQueryOutOfRangeLate :364-388
add(kind="view", name="ds_all_out_of_range_late",
    spec=dict(ds_string="0all-sum", query_start_ms=BASE - 15000,
              query_end_ms=BASE - 5000),
    points=DS6, expect=[], tol=0, cite=TDS + ":364-388")
# testDownsampler_noData :833-840, testDownsampler_noDataCalendar :842-849
add(kind="view", name="ds_no_data",
    spec=dict(ds_string="1d-sum", query_start_ms=0, query_end_ms=LMAX),
    points=[], expect=[], tol=0, cite=TDS + ":833-840")
add(kind="view", name="ds_no_data_calendar",
    spec=dict(ds_string="1mc-sum", query_start_ms=0, query_end_ms=LMAX),
    points=[], expect=[], tol=0, cite=TDS + ":842-849")
# testDownsampler_1day :851-872 (fixed 86,400,000 ms grid, sum)
add(kind="view", name="ds_1day_fixed",
    spec=dict(ds_interval_ms=86400000, ds_agg="sum", query_start_ms=0,
              query_end_ms=0),
    points=[L(BASE, 1), L(BASE + 43200000, 2), L(BASE + 86400000, 4),
            L(BASE + 129600000, 8)],
    expect=[D(BASE, 3), D(1357084800000, 12)], tol=1e-6, cite=TDS + ":851-872")
EST = "EST"


def _seq_two(t0, v0, t1, v1):
    def g():
        yield t0, v0
        while True:
            yield t1, v1
    return g


# testDownsampler_1day_timezone :874-898 (1dc in EST)
_cal_case("cal_1dc_est", "1dc-sum", EST,
          [L(1357016400000, 1), L(1357059600000, 2), L(1357102800000, 4),
           L(1357146000000, 8)],
          _seq_two(1357016400000, 3, 1357102800000, 12), TDS + ":874-898")
# testDownsampler_1week :900-924 (1wc UTC, Sunday weeks)
_cal_case("cal_1wc_utc_b", "1wc-sum", None,
          [L(1356825600000, 1), L(1357128000000, 2), L(1357430400000, 4),
           L(1357732800000, 8)],
          _seq_two(1356825600000, 3, 1357430400000, 12), TDS + ":900-924")
# testDownsampler_1week_timezone :926-950 (1wc EST)
_cal_case("cal_1wc_est", "1wc-sum", EST,
          [L(1356843600000, 1), L(1357146000000, 2), L(1357448400000, 4),
           L(1357750800000, 8)],
          _seq_two(1356843600000, 3, 1357448400000, 12), TDS + ":926-950")


def _fixed_month_starts(y, m, n, off_h):
    """n local month starts from (y, m) in a fixed-offset zone (UTC,
    EST = UTC-5 with no DST), as UTC ms: what Calendar.add(MONTH, 1) steps
    through from previousInterval's first-of-month midnight."""
    import datetime as dt
    out = []
    for k in range(n):
        yy, mm = y + (m - 1 + k) // 12, (m - 1 + k) % 12 + 1
        out.append(int(dt.datetime(yy, mm, 1, tzinfo=dt.timezone.utc)
                       .timestamp()) * 1000 + off_h * 3600000)
    return out


def _pair_points(starts, plus1=False):
    """the 1month / 2months / 1year tests' data: two points per step, at its
    start and half way to the next start (+1 ms on the next start for the
    UTC 1month test)"""
    pts = []
    for i in range(len(starts) - 1):
        a, b = starts[i], starts[i + 1] + (1 if plus1 else 0)
        pts.append(L(a, 1 << (2 * i)))
        pts.append(L(a + (b - a) // 2, 1 << (2 * i + 1)))
    return pts


# testDownsampler_1month_alt :989-1038: one point a month (04:00 / 05:00
# UTC), 1dc buckets: each month's first day at UTC midnight, value 1
_ALT = [1380600000000, 1383278400000, 1385874000000, 1388552400000,
        1391230800000, 1393650000000, 1396324800000, 1398916800000,
        1401595200000, 1404187200000, 1406865600000, 1409544000000]
_alt_days = _fixed_month_starts(2013, 10, 12, 0)


def _seq_list(pairs):
    def g():
        for t, v in pairs:
            yield t, v
    return g


_cal_case("cal_1dc_month_alt", "1dc-sum", None, [L(t, 1) for t in _ALT],
          _seq_list([(t, 1) for t in _alt_days]), TDS + ":989-1038", n=12)
# testDownsampler_2months :1040-1077 (2nc over 24 points, 4 a bucket)
_M13b = _fixed_month_starts(2013, 1, 13, 0)
assert _M13b == _M13
_cal_case("cal_2nc_utc", "2nc-sum", None, _pair_points(_M13b),
          _seq_list([(_M13b[2 * k], float(sum(1 << (4 * k + i) for i in range(4))))
                     for k in range(6)]), TDS + ":1040-1077", n=6)
# testDownsampler_1month_timezone :1079-1113 (1nc in EST)
_MEST = _fixed_month_starts(2013, 1, 13, 5)
assert _MEST[0] == 1357016400000
_cal_case("cal_1nc_est", "1nc-sum", EST, _pair_points(_MEST),
          _seq_pairs(_MEST[:12], 24), TDS + ":1079-1113", n=12)
# testDownsampler_1year_timezone :1150-1185 (1yc in EST)
_YEST = [_fixed_month_starts(y, 1, 1, 5)[0] for y in (2013, 2014, 2015)]
_cal_case("cal_1yc_est", "1yc-sum", EST, _pair_points(_YEST),
          _seq_pairs(_YEST[:2], 4), TDS + ":1150-1185", n=2)
# testSeek :1344-1365 (1000 s avg, seek to BASE + 3,600,000: aligned)
_SEEK3 = [D(BASE + 3600000, 45), D(BASE + 6600000, 40), D(BASE + 8600000, 50)]
add(kind="view", name="ds_seek", seek=BASE + 3600000,
    spec=dict(ds_interval_ms=1000000, ds_agg="avg", query_start_ms=0,
              query_end_ms=0), points=DS_DATA, expect=_SEEK3, tol=1e-7,
    cite=TDS + ":1344-1365")
# testSeek_skipPartialInterval :1407-1432 (seek BASE + 3,800,000 is not on
# the 1000 s grid: the interval holding it is abandoned, Downsampler.java:431)
add(kind="view", name="ds_seek_skip_partial", seek=BASE + 3800000,
    spec=dict(ds_interval_ms=1000000, ds_agg="avg", query_start_ms=0,
              query_end_ms=0), points=DS_DATA,
    expect=[D(BASE + 6600000, 40), D(BASE + 8600000, 50)], tol=1e-7,
    cite=TDS + ":1407-1432")
# testSeek_doubleIteration :1434-1457 (a full iteration, then the seek:
# the view is re-read from the seek, as a fresh seek)
add(kind="view", name="ds_seek_double_iteration", seek=BASE + 3600000,
    spec=dict(ds_interval_ms=1000000, ds_agg="avg", query_start_ms=0,
              query_end_ms=0), points=DS_DATA, expect=_SEEK3, tol=1e-7,
    cite=TDS + ":1434-1457")
# testSeek_abandoningIncompleteInterval :1459-1495 (10 s sum; the first
# point after each seek: seek(BASE) -> (BASE, 400); every later seek inside
# [BASE+1 s, BASE+10.1 s) -> (BASE + 10 s, 40))
_AB = [L(BASE + 100 + 1000 * i, 40) for i in range(11)]
add(kind="view", name="ds_seek_abandon_0", seek=BASE, prefix=True,
    spec=dict(ds_interval_ms=10000, ds_agg="sum", query_start_ms=0,
              query_end_ms=0), points=_AB, expect=[D(BASE, 400)], tol=1e-7,
    cite=TDS + ":1459-1495")
for _k in range(1, 11):
    add(kind="view", name="ds_seek_abandon_%d" % _k, seek=BASE + 1000 * _k,
        prefix=True,
        spec=dict(ds_interval_ms=10000, ds_agg="sum", query_start_ms=0,
                  query_end_ms=0), points=_AB, expect=[D(BASE + 10000, 40)],
        tol=1e-7, cite=TDS + ":1459-1495")

# ------------------------------------------------ FillingDownsampler
# testDownsampler_allFullRange :212-230, allFilterOnQuery :232-250,
# ...OutOfRangeEarly :252-268, ...OutOfRangeLate :270-286 ("0all-sum-nan":
# one point, or none when the query window misses every point)
for _nm, _q0, _q1, _exp, _c in (
        ("all_full_range", 0, LMAX, [D(0, 63)], ":212-230"),
        ("all_filter_on_query", BASE + 15000, BASE + 45000,
         [D(BASE + 15000, 14)], ":232-250"),
        ("all_out_of_range_early", BASE + 65000, BASE + 75000, [], ":252-268"),
        ("all_out_of_range_late", BASE - 15000, BASE - 5000, [], ":270-286")):
    add(kind="view", name="fill_" + _nm,
        spec=dict(ds_string="0all-sum-nan", start_ms=BASE + 5000,
                  end_ms=BASE + 55000, query_start_ms=_q0, query_end_ms=_q1),
        points=DS6, expect=_exp, tol=1e-7, cite=TFD + _c)
# testDownsampler_noData :792-804 (1m-sum-nan over two minutes: two NaNs),
# testDownsampler_noDataCalendar :806-818 (1mc)
for _nm, _ds, _c in (("fill_no_data", "1m-sum-nan", ":792-804"),
                     ("fill_no_data_calendar", "1mc-sum-nan", ":806-818")):
    add(kind="view", name=_nm,
        spec=dict(ds_string=_ds, start_ms=BASE, end_ms=BASE + 120000,
                  query_start_ms=0, query_end_ms=0),
        points=[], expect=[D(BASE, NAN), D(BASE + 60000, NAN)], tol=0,
        cite=TFD + _c)


def _fcal_case(name, ds, tz, start, end, points, seq, cite):
    """FillingDownsampler over a calendar grid: the reference test asserts
    every emitted point against its loop (transcribed as `seq`); how many it
    emits is the filling grid's bucket count, from previousInterval(start)
    to previousInterval(end) advanced once when the two coincide
    (FillingDownsampler.java:113-135, :154-163) — previousInterval is pinned
    by the TestDateTime KATs above."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))
    from opentsdb_amd import jcalendar as J
    iv, unit = J.parse_calendar_interval(ds.split("-")[0][:-1])
    a = J.previous_interval(start, iv, unit, tz)
    b = J.previous_interval(end, iv, unit, tz)
    edges = J.bucket_edges_for_series(a, max(end, b) + 1, iv, unit, tz)
    if b == a:
        b = edges[edges.index(a) + 1]
    n = sum(1 for e in edges if a <= e < b)
    it = seq()
    exp = [next(it) for _ in range(n)]
    add(kind="view", name=name,
        spec=dict(ds_string=ds, tz=tz, start_ms=start, end_ms=end,
                  query_start_ms=0, query_end_ms=LMAX),
        points=points, expect=[D(t, v) for t, v in exp], tol=1e-3, cite=cite)


def _fseq(ts0, step_ms, vals, tail=NAN):
    """ts advances by a fixed step; values from a list, then `tail`"""
    def g():
        t, i = ts0, 0
        while True:
            yield t, (vals[i] if i < len(vals) else tail)
            t += step_ms
            i += 1
    return g


def _fseq_ts(pairs, tail_step=None):
    """explicit (ts, value) pairs, then (the last ts + tail_step k, NaN)"""
    def g():
        for t, v in pairs:
            yield t, v
        t = pairs[-1][0]
        while True:
            t = t + tail_step if tail_step else t
            yield t, NAN
    return g


H = 3600000
# testDownsampler_calendarHour :292-360
_fcal_case("fcal_1hc_tv", "1hc-sum-nan", TZ_TV, BASE, BASE + 3 * H, PH,
           _fseq(BASE, H, [6, 15]), TFD + ":292-328")
_fcal_case("fcal_1hc_af", "1hc-sum-nan", TZ_AF, 1356996600000,
           1356996600000 + 4 * H, PH, _fseq(1356996600000, H, [1, 9, 11]),
           TFD + ":330-342")
_fcal_case("fcal_4hc_af", "4hc-sum-nan", TZ_AF, 1356996600000,
           1356996600000 + 8 * H, PH,
           _fseq_ts([(1356996600000, 21), (1357011000000, NAN)]),
           TFD + ":344-360")
DY = 86400000
# testDownsampler_calendarDay :362-492 (the "1d" control: fixed grid)
add(kind="view", name="fill_1d_control",
    spec=dict(ds_string="1d-sum-nan", start_ms=DST_TS, end_ms=DST_TS + 4 * DY,
              query_start_ms=0, query_end_ms=LMAX), points=PD,
    expect=[D(DST_TS + DY * i, v) for i, v in enumerate([3, 7, 11, NAN])],
    tol=1e-3, cite=TFD + ":362-392")
_fcal_case("fcal_1dc_tv", "1dc-sum-nan", TZ_TV, 1450094400000 - DY,
           DST_TS + 5 * DY, PD, _fseq(1450094400000 - DY, DY, [NAN, 1, 5, 9, 6]),
           TFD + ":394-419")
_fcal_case("fcal_1dc_fj", "1dc-sum-nan", TZ_FJ, 1450094400000,
           DST_TS + 5 * DY, PD, _fseq(1450090800000, DY, [1, 2, 12, 6]),
           TFD + ":421-444")
_fcal_case("fcal_1dc_af", "1dc-sum-nan", TZ_AF, 1450121400000,
           DST_TS + 4 * DY, PD, _fseq(1450121400000, DY, [1, 5, 15]),
           TFD + ":446-467")
_fcal_case("fcal_3dc_af", "3dc-sum-nan", TZ_AF, 1450121400000,
           DST_TS + 6 * DY, PD, _fseq(1450121400000, 3 * DY, [21]),
           TFD + ":469-484")
WK = 7 * DY
# testDownsampler_calendarWeek :487-616 (sequences: the tests' if-chains)


def _cycle(first, rest):
    """value after `first`: the test's if/else chain as a function"""
    def g():
        v = first
        while True:
            yield v
            v = rest(v)
    return g


def _wk_ctrl(v):
    if v == 1:
        return 5
    if v == 5:
        return NAN
    if v != v:
        return 9
    return NAN


def _fseq_fn(ts0, step_ms, vals_gen):
    def g():
        t = ts0
        for v in vals_gen():
            yield t, v
            t += step_ms
    return g


_fcal_case("fcal_1wc_utc", "1wc-sum-nan", None, 1449964800000,
           DST_TS + 35 * DY, PW, _fseq_fn(1449964800000, WK, _cycle(1, _wk_ctrl)),
           TFD + ":487-509")


def _wk_tv(v):
    if v == 1:
        return 5
    if v == 5:
        return NAN
    if v != v:
        return 4
    return 5


_fcal_case("fcal_1wc_tv", "1wc-sum-nan", TZ_TV, 1449964800000,
           DST_TS + 35 * DY, PW, _fseq_fn(1449921600000, WK, _cycle(1, _wk_tv)),
           TFD + ":511-534")
_fcal_case("fcal_1wc_fj", "1wc-sum-nan", TZ_FJ, 1449964800000,
           DST_TS + 35 * DY, PW,
           _fseq_fn(1449918000000, WK, _cycle(1, lambda v: v + 1)),
           TFD + ":536-551")
_fcal_case("fcal_1wc_af", "1wc-sum-nan", TZ_AF, 1449964800000,
           DST_TS + 35 * DY, PW, _fseq_fn(1449948600000, WK, _cycle(1, _wk_ctrl)),
           TFD + ":553-576")
_fcal_case("fcal_2wc_af", "2wc-sum-nan", TZ_AF, 1449964800000,
           DST_TS + 35 * DY, PW,
           _fseq_fn(1449948600000, 2 * WK, _cycle(6, lambda v: 9 if v == 6 else NAN)),
           TFD + ":578-598")
# testDownsampler_calendarMonth :618-760 ("1n" control: fixed 30-day grid)
DEC1 = 1448928000000
add(kind="view", name="fill_1n_control",
    spec=dict(ds_string="1n-sum-nan", start_ms=DEC1,
              end_ms=DEC1 + 2592000000 * 5, query_start_ms=0,
              query_end_ms=LMAX), points=PM,
    expect=[D(DEC1 + 2592000000 * i, v) for i, v in
            enumerate([1, 5, 4, 11, NAN])], tol=1e-3, cite=TFD + ":618-648")
_fcal_case("fcal_1nc_tv", "1nc-sum-nan", TZ_TV, DEC1, DEC1 + 2592000000 * 6,
           PM, _fseq_ts([(1448884800000, 3), (1451563200000, 3),
                         (1454241600000, 9), (1456747200000, 6),
                         (1459425600000, NAN)]), TFD + ":650-676")
_fcal_case("fcal_1nc_fj", "1nc-sum-nan", TZ_FJ, DEC1, DEC1 + 2592000000 * 6,
           PM, _fseq_ts([(1448881200000, 1), (1451559600000, 5),
                         (1454241600000, 9), (1456747200000, 6),
                         (1459425600000, NAN)]), TFD + ":678-704")
_fcal_case("fcal_1nc_af", "1nc-sum-nan", TZ_AF, DEC1, DEC1 + 2592000000 * 5,
           PM, _fseq_ts([(1448911800000, 3), (1451590200000, 3),
                         (1454268600000, 15), (1456774200000, NAN)]),
           TFD + ":706-729")
_fcal_case("fcal_3nc_tv", "3nc-sum-nan", TZ_TV, DEC1, DEC1 + 2592000000 * 9,
           PM, _fseq_ts([(1443614400000, 3), (1451563200000, 18),
                         (1459425600000, NAN)]), TFD + ":731-752")
# testDownsampler_calendarSkipSomePoints :762-790
_fcal_case("fcal_skip_some", "1hc-sum-nan", TZ_TV, 1356998400000,
           1357009200000, [L(BASE, 1), L(BASE + 1800000, 2), L(BASE + 7200000, 6)],
           _fseq(BASE, H, [3, NAN, 6]), TFD + ":762-790")


# --------------------------------------------- TestTsdbQueryDownsample (rest)
# (single series web01 — the tests' tags select it; query [1356998400,
# 1357041600] s: the SpanGroup window is the scan bounds, Q_WIN).  A point's
# optional 4th element is its own tolerance (tests assert the ends and the
# middle with different deltas; float literals as Java's `F` constants).
TQD = "test/core/TestTsdbQueryDownsample.java"


def F32(x):
    import struct as st
    return st.unpack("<f", st.pack("<f", x))[0]


def _long_ms_web01():
    """storeLongTimeSeriesMs (BaseTsdbTest.java:641-659): web01"""
    return [L(1356998400000 + 500 * i, i) for i in range(1, 301)]


def _float_steps_web01(step_ms, t0):
    return [D(t0 + step_ms * (k + 1), v)
            for k, v in enumerate(_f32_steps(1.25, 76.0, 0.25, True))]


_FS = _float_steps_web01(30000, 1356998400000)   # storeFloatTimeSeriesSeconds
_FMS = _float_steps_web01(500, 1356998400000)    # storeFloatTimeSeriesMs
_QD = dict(Q_WIN, agg="sum")


def _ds_avg_exp(n, step, first, last, mid):
    return [D(1356998400000 + step * i,
              first if i == 0 else (last if i >= n - 1 else mid(i)))
            for i in range(n)]


# runLongSingleTSDownsampleMs :174-209 (1000 ms avg)
add(kind="group_by", name="tsdb_single_ts_downsample_ms",
    spec=dict(_QD, ds_interval_ms=1000, ds_agg="avg"), groups=[[_long_ms_web01()]],
    expect=[_ds_avg_exp(151, 1000, 1.0, 300.0, lambda i: i * 2 + 0.5)],
    tol=0.00001, check_ts_mod=1000, cite=TQD + ":174-209")
# runLongSingleTSDownsampleAndRateMs :250-285
add(kind="group_by", name="tsdb_single_ts_downsample_rate_ms",
    spec=dict(_QD, ds_interval_ms=1000, ds_agg="avg", rate=True),
    groups=[[_long_ms_web01()]],
    expect=[[[1356998401000 + 1000 * i, F32(1.5) if i == 0 else
              (1.5 if i >= 149 else F32(2.0)), 1,
              0.001 if i == 0 else (0.00001 if i >= 149 else 0.001)]
             for i in range(150)]],
    tol=0.001, check_ts_mod=1000, cite=TQD + ":250-285")
# runFloatSingleTSDownsample :286-322 (60 s avg over storeFloatTimeSeriesSeconds)
add(kind="group_by", name="tsdb_float_downsample",
    spec=dict(_QD, ds_interval_ms=60000, ds_agg="avg"), groups=[[_FS]],
    expect=[_ds_avg_exp(151, 60000, 1.25, 76.0, lambda i: (i + 2.25) / 2)],
    tol=0.00001, check_ts_mod=60000, cite=TQD + ":286-322")
# runFloatSingleTSDownsampleMs :323-359
add(kind="group_by", name="tsdb_float_downsample_ms",
    spec=dict(_QD, ds_interval_ms=1000, ds_agg="avg"), groups=[[_FMS]],
    expect=[_ds_avg_exp(151, 1000, 1.25, 76.0, lambda i: (i + 2.25) / 2)],
    tol=0.00001, check_ts_mod=1000, cite=TQD + ":323-359")
# runFloatSingleTSDownsampleAndRate :360-399
add(kind="group_by", name="tsdb_float_downsample_rate",
    spec=dict(_QD, ds_interval_ms=60000, ds_agg="avg", rate=True), groups=[[_FS]],
    expect=[[[1356998460000 + 60000 * i,
              F32(0.00625) if (i == 0 or i >= 149) else F32(0.00833), 1,
              0.000001 if (i == 0 or i >= 149) else 0.00001]
             for i in range(150)]],
    tol=0.00001, check_ts_mod=60000, cite=TQD + ":360-399")
# runFloatSingleTSDownsampleAndRateMs :400-435
add(kind="group_by", name="tsdb_float_downsample_rate_ms",
    spec=dict(_QD, ds_interval_ms=1000, ds_agg="avg", rate=True), groups=[[_FMS]],
    expect=[[[1356998401000 + 1000 * i,
              F32(0.375) if (i == 0 or i >= 149) else F32(0.5), 1,
              0.000001 if (i == 0 or i >= 149) else 0.00001]
             for i in range(150)]],
    tol=0.00001, check_ts_mod=1000, cite=TQD + ":400-435")
# runLongSingleTSDownsampleCount :436-463 (60 s count)
add(kind="group_by", name="tsdb_downsample_count",
    spec=dict(_QD, ds_interval_ms=60000, ds_agg="count"), groups=[[WEB01]],
    expect=[[D(1356998400000 + 60000 * i, 1 if i in (0, 150) else 2)
             for i in range(151)]],
    tol=0.00001, cite=TQD + ":436-463")
# runFloatSingleTSDownsampleAndRateAndCount :563-599 (60 s count, rate)
add(kind="group_by", name="tsdb_float_downsample_count_rate",
    spec=dict(_QD, ds_interval_ms=60000, ds_agg="count", rate=True),
    groups=[[_FS]],
    expect=[[D(1356998460000 + 60000 * i,
               F32(0.016666) if i == 0 else (F32(-0.016666) if i == 149 else 0.0))
             for i in range(150)]],
    tol=0.00001, check_ts_mod=60000, cite=TQD + ":563-599")


def _scan_ms(start_s, end_s):
    """TsdbQuery.getScanStart/EndTimeSeconds with a 0-interval ("all")
    downsampler, in ms (TsdbQuery.java:1573-1675; pinned by scan_bounds)"""
    a = start_s - start_s % 3600
    b = end_s + (3600 - end_s % 3600)
    return a * 1000, b * 1000


# runLongSingleTSDownsampleAll :464-495, AllSubSet :497-528, AllNoEnd
# :530-561 (TSQuery "0all-sum": one point at the query start; no end: "now",
# any instant past the data)
for _nm, _s0, _s1, _v, _c in (("all", 1356998400, 1357041600, 45150, ":464-495"),
                              ("all_subset", 1356998500, 1356998600, 15,
                               ":497-528"),
                              ("all_no_end", 1356998400, 1500000000, 45150,
                               ":530-561")):
    _a, _b = _scan_ms(_s0, _s1)
    add(kind="group_by", name="tsdb_downsample_" + _nm,
        spec=dict(start_ms=_a, end_ms=_b, query_start_ms=_s0 * 1000,
                  query_end_ms=_s1 * 1000, agg="sum", ds_string="0all-sum"),
        groups=[[WEB01]], expect=[[D(_s0 * 1000, _v)]], tol=0.00001,
        cite=TQD + _c)


# runTSDownsampleWithMissingData :859-907 and its six callers :677-857:
# {web01, web02} of storeLongTimeSeriesWithMissingData, 30 s downsample
# with a fill policy, 1,560 points: the first 100 by the test's validator
# (transcribed as generators), the rest its missing value (NaN or 0).
def _v_const(c):
    def g():
        while True:
            yield c
    return g


def _v_alt(even0, even_step, odd):
    def g():
        e = even0
        while True:
            e += even_step
            yield e
            yield odd
    return g


def _v_minmin():
    e, ec, o, oc = -4.0, 6.0, -1.0, 6.0
    while True:
        e += ec
        if e == 152.0:
            e, ec = 149.0, -6.0
        yield e
        o += oc
        if o == 155.0:
            o, oc = 145.0, -6.0
        yield o


def _v_minsum():
    e, ec, o, oc = -7.0, 12.0, -1.0, 12.0
    while True:
        e += ec
        if e == 209.0:
            e, ec = 197.0, -6.0
        yield e
        o += oc
        if o == 311.0:
            o, oc = 292.0, -12.0
        yield o


def _v_summin():
    while True:
        yield 301.0
        yield 300.0


for _nm, _agg, _dsa, _fill, _val, _c in (
        ("sum_avg", "sum", "avg", "nan", _v_const(301.5), ":677-689"),
        ("avg_sum", "avg", "sum", "nan", _v_alt(149.0, 3.0, 301.5), ":691-712"),
        ("avg_avg", "avg", "avg", "zero", _v_const(150.75), ":714-726"),
        ("sum_sum", "sum", "sum", "nan", _v_alt(298.0, 6.0, 603.0), ":728-750"),
        ("min_min", "min", "min", "zero", _v_minmin, ":752-793"),
        ("min_sum", "min", "sum", "nan", _v_minsum, ":795-837"),
        ("sum_min", "sum", "min", "nan", _v_summin, ":839-857")):
    _it = _val()
    _miss = NAN if _fill == "nan" else 0.0
    _exp = [D(1356998400000 + 30000 * i, next(_it) if i < 100 else _miss)
            for i in range(1560)]
    add(kind="group_by", name="tsdb_wnulls_" + _nm,
        spec=dict(Q_WIN, agg=_agg, ds_interval_ms=30000, ds_agg=_dsa,
                  fill=_fill),
        groups=[_missing_data()], expect=[_exp], tol=0.0001,
        cite=TQD + _c + ",859-907")

# ------------------------------------------- TestTsdbQueryQueries (rate)
# runRateCounterDefault :1130-1154 .. runRateCounterAnomallyDrop :1229-1251
# (one series, 30 s cadence from 1356998430 s, counter rates; the junk
# first rate is not emitted)
_T = [1356998430000 + 30000 * k for k in range(4)]
for _nm, _vals, _ro, _exp, _c in (
        ("default", [LMAX - 55, LMAX - 25, 5], dict(counter_max=LMAX, reset_value=0),
         [(_T[1], 1.0), (_T[2], 1.0)], ":1130-1154"),
        ("default_noop", [30, 60, 90], dict(counter_max=LMAX, reset_value=0),
         [(_T[1], 1.0), (_T[2], 1.0)], ":1156-1178"),
        ("max_set", [45, 75, 5], dict(counter_max=100, reset_value=0),
         [(_T[1], 1.0), (_T[2], 1.0)], ":1180-1202"),
        ("anomaly", [45, 75, 25], dict(counter_max=10000, reset_value=35),
         [(_T[1], 1.0), (_T[2], 0.0)], ":1204-1227"),
        ("anomaly_drop", [45, 75, 25, 55],
         dict(counter_max=10000, reset_value=35, drop_resets=True),
         [(_T[1], 1.0), (_T[3], 1.0)], ":1229-1251")):
    add(kind="group_by", name="tq_rate_counter_" + _nm,
        spec=dict(Q_WIN, agg="sum", rate=True, counter=True, **_ro),
        groups=[[[L(t, v) for t, v in zip(_T, _vals)]]],
        expect=[[D(t, v) for t, v in _exp]], tol=0.001, cite=TQQ + _c)

# runMultiCompact :1253-1302, runMultiCompactAndSingles :1304-1355: one
# storage row of compacted columns (and single cells), compacted at query
# time, decoded, one series: points 1..6 at 1 s steps (longs)
_mq = [bytes([0, (k << 4) | 7]) for k in range(1, 7)]
_mv = [_Lb(k) for k in range(1, 7)]
_MC = [(_mq[0] + _mq[1], _mv[0] + _mv[1] + _ZB),
       (_mq[2] + _mq[3], _mv[2] + _mv[3] + _ZB),
       (_mq[4] + _mq[5], _mv[4] + _mv[5] + _ZB)]
_MCS = [_MC[0], (_mq[2], _mv[2]), (_mq[3], _mv[3]), _MC[2]]
for _nm, _cols, _c in (("multi_compact", _MC, ":1253-1302"),
                       ("multi_compact_singles", _MCS, ":1304-1355")):
    add(kind="rows_query", name="tq_" + _nm, base=1356998400,
        columns=[[q.hex(), v.hex()] for q, v in _cols], fix_duplicates=True,
        expect=[[1356998401000 + 1000 * k, k + 1] for k in range(6)],
        cite=TQQ + _c)

# ------------------------------------------- TestAggregationIterator (rest)
TAI = "test/core/TestAggregationIterator.java"
# testAggregate_seek :189-207 (one span, seeked once to the start: its
# points unchanged)
add(kind="group_by", name="ai_seek", spec=dict(SPEC_AI), groups=[[DP1]],
    expect=[DP1], tol=0, filter=False, cite=TAI + ":189-207")
# testDownsample_afterAggregation :150-187 (seven 10 s-avg spans summed,
# then a 15 s-sum Downsampler over the aggregate)
add(kind="group_by", name="ai_downsample_after_aggregation",
    spec=dict(start_ms=BASE + 1000, end_ms=BASE + 100000, agg="sum",
              ds_interval_ms=10000, ds_agg="avg"),
    groups=[[DATA_5SEC] * 7],
    post=dict(ds_interval_ms=15000, ds_agg="sum", query_start_ms=0,
              query_end_ms=0),
    expect=[[D(BASE, 7), D(BASE + 15000, 7), D(BASE + 30000, 14),
             D(BASE + 45000, 7)]], tol=0, filter=False, cite=TAI + ":150-187")

def _enc(x):
    if isinstance(x, float):
        if math.isnan(x):
            return "NaN"
        if math.isinf(x):
            return "Infinity" if x > 0 else "-Infinity"
    if isinstance(x, list):
        return [_enc(y) for y in x]
    if isinstance(x, dict):
        return {k: _enc(v) for k, v in x.items()}
    return x


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "kat_reference.json")
    with open(out, "w") as f:
        json.dump({"source": "transcribed from /root/reference/test/core "
                             "JUnit literals (see 'cite')",
                   "cases": _enc(cases)}, f, indent=0)
    print("wrote", out, len(cases), "cases")
