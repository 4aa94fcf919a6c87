"""`dev` in the reference's order, bit for bit (Needs an MI355X).

StdDev.runDouble is one sequential Welford pass (Aggregators.java:547-568).
On offset data — counters near 2^32 that move by < 10^4 inside a bucket, a
gauge of ~3e9 across many series — that pass is ill-conditioned: its own
result lies ~1e-11 from the exact standard deviation, and any other order
(a lane tree merged with Chan's formula, even in exact arithmetic) lands
~1e-11 from the reference's (tests/test_dev_conditioning_cpu.py shows it on
the CPU).  So the engine does not merge Welford runs inside a downsample
bucket (reduce_step's ordered chain hands the state from lane to lane in
point order), and reduces a group's members in one sequential chain per
(group, bucket) while the group fits one chain (fold tiles of 256 members,
row-path chains of 16,384).  Everything here compares BIT-EXACTLY with the
oracle: no tolerance, no floor."""
import numpy as np
import pytest

from opentsdb_amd import core
from tests import datasets
from tests.test_gpu_parity import RATES, _spec, check

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("cadence_ms", [1000, 10000])
@pytest.mark.parametrize("interval", ["30s", "1m", "5m", "1h"])
def test_dev_downsample_counters(engine, interval, cadence_ms):
    """Downsample `dev` over raw counters (start U[0, 2^32), +0..999 a step,
    resets): the buckets span 3 to 3,600 points, i.e. up to 7 steps of 512
    points with every lane of a step in one bucket (the longest chains)."""
    b = datasets.random_batch(5266 + cadence_ms // 1000, n_series=24,
                              n_groups=4, counter=True, cadence_ms=cadence_ms,
                              span_ms=2 * 3600 * 1000)
    end = datasets.T0 + 2 * 3600 * 1000
    for agg in ("sum", "min", "dev", "mult"):
        spec = _spec(agg, "dev", end=end, interval=interval)
        # sum / dev / mult over the group's members are fed in SpanCmp order
        # (groups of <= 256 members: one fold tile)
        check(engine, spec, b, True, where="dev/%s/%s/%d" % (agg, interval,
                                                             cadence_ms))


@pytest.mark.parametrize("ri", [0, 1, 3])
def test_dev_downsample_counter_rates(engine, ri):
    """`sum:5m-dev:rate` and the sweep's failing shape (`mult` of 5 m `dev`
    buckets of counters, rate): RateSpan differences the bit-exact buckets."""
    b = datasets.random_batch(5300 + ri, n_series=30, n_groups=5, counter=True)
    for agg in ("sum", "mult", "dev", "max"):
        spec = _spec(agg, "dev", rate=True, ro=RATES[ri], interval="5m")
        check(engine, spec, b, True, where="devrate%d/%s" % (ri, agg))


@pytest.mark.parametrize("kind", ["offset", "float", "int"])
@pytest.mark.parametrize("n_series", [100, 300, 5000])
def test_cross_series_dev_offset_members(engine, n_series, kind):
    """Cross-series `dev` over > 64 and > 256 members of one group: one fold
    tile (100), the row path's one chain per bucket (300, 5,000) — fed in
    SpanCmp order, so bit-exact, on gauge values ~3e9 +- 1e4 too."""
    b = datasets.random_batch(5400 + n_series, n_series=n_series,
                              big_group=True, span_ms=3600 * 1000,
                              cadence_ms=30000, value_kind=kind)
    end = datasets.T0 + 3600 * 1000
    for ds in ("max", "dev", "first"):
        for fill in ("none", "nan"):
            spec = _spec("dev", ds, fill, end=end)
            check(engine, spec, b, True,
                  where="xdev%d/%s/%s/%s" % (n_series, kind, ds, fill))


def test_cross_series_dev_rate_chain(engine):
    """Rate queries take the row path: a 2,000-member group of counter rates
    reduced by `dev` in one chain per bucket."""
    b = datasets.random_batch(5501, n_series=2000, big_group=True,
                              counter=True, span_ms=3600 * 1000,
                              cadence_ms=10000)
    spec = _spec("dev", "sum", rate=True, ro=RATES[1],
                 end=datasets.T0 + 3600 * 1000)
    check(engine, spec, b, True, where="xdevrate")


def test_dev_cells_fold(engine):
    """The same counters stored as compacted cells: the cells fold (one
    window, and narrowed windows) and the row kernel (rate) replay the
    buckets in point order too."""
    import torch
    from opentsdb_amd import workload
    from opentsdb_amd.engine import DeviceResult
    from oracle import pyoracle
    from tests.test_gpu_decode import _device_batch, _result_points
    from tests.test_gpu_parity import compare
    b = datasets.random_batch(5600, n_series=40, n_groups=4, counter=True,
                              span_ms=3 * 3600 * 1000)
    b.ts[:] = b.ts - b.ts % 1000  # whole seconds: 2-byte qualifiers
    db = _device_batch(b, "int")
    cells = workload.encode_cells_device(engine, db)
    for agg, interval, rate in (("sum", "5m", False), ("dev", "1m", False),
                                ("mult", "1h", False), ("sum", "5m", True)):
        spec = _spec(agg, "dev", interval=interval, rate=rate,
                     ro=RATES[1] if rate else None)
        ref = pyoracle.group_by(spec, b)
        res = DeviceResult(torch, b.n_groups, 4 * len(b.ts) + 4096, "cuda")
        workload.run_cells_device(engine, spec, cells, db, res)
        compare(_result_points(res, b.n_groups), ref, True,
                where="cellsdev/%s/%s/%s" % (agg, interval, rate))
