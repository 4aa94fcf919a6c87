"""Seeded random-query sweep against the oracle: aggregator x downsampler x
fill x interpolation override x rate x window x batch shape, drawn from the
reference's surface (Aggregators, DownsamplingSpecification, FillPolicy,
RateOptions).  Exercises the paths' interplay the parity matrix crosses only
partly: multi-window and narrowed folds, 32-member tiles, the row path for
rate and percentiles, fills, windows cut inside buckets."""
import numpy as np
import pytest

from opentsdb_amd import core
from tests import datasets
from tests.test_gpu_parity import check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()

AGGS = ["sum", "zimsum", "pfsum", "avg", "min", "max", "mimmin", "mimmax",
        "dev", "count", "first", "last", "diff", "mult", "squareSum",
        "median", "p50", "p95", "p99", "ep90r3", "ep99r7"]
DSF = ["avg", "sum", "min", "max", "count", "first", "last", "dev",
       "zimsum", "mimmax", "median", "p90"]
FILLS = ["none", "none", "nan", "null", "zero"]
INTERVALS = ["30s", "1m", "2m", "5m", "7m", "13m", "1h"]
# downsamplers computed bit-identically to the reference: order-free ones,
# and dev (one sequential Welford pass per bucket, in point order)
EXACT_DS = ("min", "max", "count", "first", "last", "mimmax", "median", "p90",
            "dev")
# cross-series: order-free ones, and dev (one sequential chain per (group,
# bucket) in SpanCmp order) and diff (last - first) over exact inputs
EXACT_AGG = ("min", "max", "mimmin", "mimmax", "count", "first", "last",
             "median", "p50", "p95", "p99", "ep90r3", "ep99r7", "dev", "diff")


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    kind = ["float", "int", "mixed"][int(rng.integers(0, 3))]
    rate = bool(rng.random() < 0.2)
    n_series = int(rng.integers(1, 90))
    b = datasets.random_batch(
        5000 + seed, n_series=n_series,
        n_groups=int(rng.integers(1, max(1, n_series // 3) + 1)),
        span_ms=int(rng.integers(1, 7)) * 3600 * 1000,
        cadence_ms=int(rng.choice([1000, 7000, 10000, 60000])),
        value_kind="int" if rate else kind,
        nan_frac=0.03 if kind == "float" and not rate else 0.0,
        counter=rate, big_group=bool(rng.random() < 0.15))
    agg = AGGS[int(rng.integers(0, len(AGGS)))]
    ds = DSF[int(rng.integers(0, len(DSF)))]
    fill = "none" if rate else FILLS[int(rng.integers(0, len(FILLS)))]
    iv = INTERVALS[int(rng.integers(0, len(INTERVALS)))]
    t0 = datasets.T0 + int(rng.integers(0, 3600)) * 1000
    t1 = t0 + int(rng.integers(1800, 6 * 3600)) * 1000
    interp = None
    if rng.random() < 0.25:
        interp = int(rng.integers(0, 5))  # LERP ZIM MAX MIN PREV
    ro = core.RateOptions(True, core.LONG_MAX, 0) if rate else None
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification("%s-%s-%s" % (iv, ds, fill)),
                          t0, t1, rate, ro, interp)
    # order-free downsamplers feeding order-free aggregators: bit-exact,
    # rate queries included (one RateSpan division of exact values)
    exact = ds in EXACT_DS and agg in EXACT_AGG
    return b, spec, exact, "%d:%s:%s-%s-%s%s%s" % (
        seed, agg, iv, ds, fill, ":rate" if rate else "",
        "" if interp is None else ":i%d" % interp)


@pytest.mark.parametrize("seed", range(120))
def test_random_query_sweep(engine, seed):
    b, spec, exact, where = _case(seed)
    # 1e-12 relative; an absolute 1e-12 x sum|contributions| only at points
    # whose contributions have both signs (contribution_floor)
    check(engine, spec, b, exact, where=where, floor="contributions")


@pytest.mark.parametrize("seed", [5266])
def test_sweep_regressions(engine, seed):
    """Seeds sweep_many.py found diverging.  5266: `mult` of 4 series' 5 m
    `dev` of counter rates (increments of 0-1,000 on ~3e9 every 10 s) — the
    dev buckets were merged in a lane tree (Chan's formula) where the
    reference runs one sequential Welford pass; on such offset data the two
    orders differ at ~1e-10 (now replayed in point order: bit-exact)."""
    b, spec, exact, where = _case(seed)
    check(engine, spec, b, exact, where=where, floor="contributions")


def _rate_case(seed):
    """Rate queries only: counter options (dropResets, counterMax,
    resetValue — RateOptions.java:27-176) x downsampler (percentiles take the
    k_ds_select path) x window; the generator's outages and counter resets
    put kept rates past windows and resets next to bucket edges."""
    rng = np.random.default_rng(7000 + seed)
    n_series = int(rng.integers(1, 60))
    b = datasets.random_batch(
        9000 + seed, n_series=n_series,
        n_groups=int(rng.integers(1, max(1, n_series // 3) + 1)),
        span_ms=int(rng.integers(1, 7)) * 3600 * 1000,
        cadence_ms=int(rng.choice([1000, 10000, 60000])),
        value_kind="int", counter=True, big_group=bool(rng.random() < 0.15))
    agg = AGGS[int(rng.integers(0, len(AGGS)))]
    ds = DSF[int(rng.integers(0, len(DSF)))]
    iv = INTERVALS[int(rng.integers(0, len(INTERVALS)))]
    t0 = datasets.T0 + int(rng.integers(0, 3 * 3600)) * 1000
    t1 = t0 + int(rng.integers(600, 4 * 3600)) * 1000
    drop = bool(rng.random() < 0.5)
    cmax = core.LONG_MAX if rng.random() < 0.7 else int(2**40)
    reset = 0 if rng.random() < 0.6 else int(rng.integers(1, 10**6))
    ro = core.RateOptions(True, cmax, reset, drop)
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification("%s-%s" % (iv, ds)),
                          t0, t1, True, ro)
    exact = ds in EXACT_DS and agg in EXACT_AGG
    return b, spec, exact, "%d:%s:%s-%s:drop=%s:max=%d:reset=%d" % (
        seed, agg, iv, ds, drop, cmax, reset)


@pytest.mark.parametrize("seed", range(60))
def test_random_rate_sweep(engine, seed):
    b, spec, exact, where = _rate_case(seed)
    check(engine, spec, b, exact, where=where, floor="contributions")


@pytest.mark.parametrize("seed", range(60))
def test_random_cells_sweep(engine, seed):
    """The general sweep's queries over the same points stored as RowSeq
    bytes: storage rows (otsdb_agg_run_raw_device — columns scattered,
    appended, split row keys: compaction, span assembly) and, when every
    series has one value type, device-encoded compacted cells
    (otsdb_agg_run_cells_device).  Whole-second data takes the cells fold
    (one window, several, narrowed ones), ms data rows of mixed qualifier
    widths and the generic decode; rate and percentile downsampling the row
    kernel.  Against the oracle on the same points."""
    import torch
    from opentsdb_amd import storage, workload
    from opentsdb_amd.engine import DeviceResult
    from oracle import pyoracle
    from tests.test_gpu_decode import _device_batch, _result_points
    from tests.test_gpu_parity import compare, contribution_floor
    from tests.test_gpu_rows import _raw_from_hb
    b, spec, exact, where = _case(seed)
    rng = np.random.default_rng(3000 + seed)
    if rng.random() < 0.7:  # whole seconds: 2-byte qualifiers
        ts2 = b.ts - b.ts % 1000
        if all((np.diff(ts2[b.offsets[s]:b.offsets[s + 1]]) > 0).all()
               for s in range(b.n_series)):
            b.ts[:] = ts2
    try:
        ref = pyoracle.group_by(spec, b)
    except pyoracle.OracleError:
        return  # a rejected query: covered by the columnar sweep
    fl = contribution_floor(spec, b, ref)
    db = None
    types = [np.unique(b.is_float[b.offsets[s]:b.offsets[s + 1]])
             for s in range(b.n_series)]
    if all(len(t) <= 1 for t in types):
        kinds = {int(t[0]) for t in types if len(t)}
        if len(kinds) <= 1:
            kind = "float" if kinds != {0} else "int"
            db = _device_batch(b, kind)
            cells = workload.encode_cells_device(engine, db)
            res = DeviceResult(torch, b.n_groups, 4 * len(b.ts) + 4096, "cuda")
            workload.run_cells_device(engine, spec, cells, db, res)
            compare(_result_points(res, b.n_groups), ref, exact,
                    where="cells/" + where, floor=fl)
    raw = storage.HostRawRows(_raw_from_hb(rng, b), with_ts=True).to_device()
    raw.n_series = b.n_series
    if db is None:
        db = _device_batch(b, "float")  # groups only: the rows hold the types
    res = DeviceResult(torch, b.n_groups, 4 * len(b.ts) + 4096, "cuda")
    storage.run_raw_device(engine, spec, raw, db, res)
    compare(_result_points(res, b.n_groups), ref, exact, where="rows/" + where,
            floor=fl)
