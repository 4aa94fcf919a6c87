"""The production boundary as GpuAggregation.java drives it (Needs an
MI355X): integration/jni/otsdb_agg_jni.c, compiled against the fake JNIEnv
of tests/jni_fake (the image has no JDK), called through its
Java_net_opentsdb_core_GpuAggregation_* natives with Java-like arrays —
packed spec, compacted cells as HBase returns them, group offsets — on the
real engine.  Results against the oracle; the status / exception mapping
GpuAggregation relies on (CAPACITY retry with the needed size, UNSUPPORTED
returned without an exception, corrupt cells -> IllegalDataException)."""
import numpy as np
import pytest

from opentsdb_amd import core
from opentsdb_amd.batch import HostBatch
from oracle import pyoracle
from tests import cells, datasets
from tests import jni_fake_lib as J
from tests.test_gpu_parity import cancel_floor, compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def shim():
    lib = J.load()
    ctx = lib.fj_ctx_create(0)
    assert ctx != 0 and J.pending(lib) is None
    yield lib, ctx
    lib.fj_ctx_destroy(ctx)


def _data(seed, kind, ms):
    rng = np.random.default_rng(seed)
    b = datasets.random_batch(seed, n_series=24, n_groups=3, value_kind=kind,
                              cadence_ms=7000)
    if ms:
        b.ts = b.ts + rng.integers(0, 999, len(b.ts)) * (rng.random(len(b.ts)) < 0.5)
        for s in range(b.n_series):
            a, z = b.offsets[s], b.offsets[s + 1]
            b.ts[a:z] = np.sort(b.ts[a:z])
    else:
        b.ts = b.ts - b.ts % 1000
    enc = cells.encode_batch(b)
    ts, bits, isint = [], [], []
    for r in range(len(enc["row_series"])):
        q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
        v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
        p = pyoracle.decode_row(q.tobytes(), v.tobytes(), enc["row_base_s"][r])
        ts.append(p["ts"])
        bits.append(p["bits"])
        isint.append(p["is_int"])
    hb = HostBatch(b.offsets, np.concatenate(ts).astype(np.int64),
                   np.concatenate(bits).astype(np.int64),
                   (np.concatenate(isint) == 0).astype(np.uint8), None,
                   b.group_offsets, b.group_members)
    return enc, hb


def _points(offs, ts, val, isint, G):
    from opentsdb_amd.engine import DataPoints
    return [DataPoints(ts[offs[g]:offs[g + 1]].copy(),
                       val[offs[g]:offs[g + 1]].copy(),
                       isint[offs[g]:offs[g + 1]].copy()) for g in range(G)]


CASES = [("sum", "1m-avg", False, "float", False),
         ("max", "5m-max", False, "int", True),
         ("dev", "10m-dev-nan", False, "float", True),
         ("zimsum", "1m-sum", True, "int", False),
         ("p99", "5m-avg", False, "float", False),
         ("sum", "0all-sum", False, "float", True)]


@pytest.mark.parametrize("agg,ds,rate,kind,ms", CASES)
def test_run_cells_through_the_shim(shim, agg, ds, rate, kind, ms):
    lib, ctx = shim
    enc, hb = _data(61, kind, ms)
    t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
    ro = core.RateOptions(True, core.LONG_MAX, 0) if rate else None
    spec = core.make_spec(t0, t1, core.Aggregators.get(agg),
                          core.DownsamplingSpecification(ds), t0, t1, rate, ro)
    ref = pyoracle.group_by(spec, hb)
    G = len(hb.group_offsets) - 1
    st, offs, ts, val, isint = J.run_cells(
        lib, ctx, spec, enc, hb.n_series, hb.group_offsets, hb.group_members,
        4 * len(hb.ts) + 64)
    assert st == 0 and J.pending(lib) is None, (st, J.pending(lib))
    got = _points(offs, ts, val, isint, G)
    exact = agg in ("max", "dev") and ds.split("-")[1] in ("max", "dev")
    fl = cancel_floor(hb, 400) if kind == "int" else 0.0
    compare(got, ref, exact, floor=fl, where="jni/%s/%s" % (agg, ds))


def test_capacity_then_retry(shim):
    """Too small an output: OTSDB_E_CAPACITY back to Java without an
    exception, the offsets carrying the size needed; the retry succeeds."""
    lib, ctx = shim
    enc, hb = _data(62, "float", False)
    t0, t1 = datasets.T0, datasets.T0 + 3 * 3600000
    spec = core.make_spec(t0, t1, core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"), t0, t1)
    G = len(hb.group_offsets) - 1
    st, offs, *_ = J.run_cells(lib, ctx, spec, enc, hb.n_series,
                               hb.group_offsets, hb.group_members, 8)
    assert st == 7 and J.pending(lib) is None
    need = int(offs[G])
    assert need > 8
    st, offs, ts, val, isint = J.run_cells(lib, ctx, spec, enc, hb.n_series,
                                           hb.group_offsets, hb.group_members,
                                           need)
    assert st == 0 and int(offs[G]) == need
    compare(_points(offs, ts, val, isint, G), pyoracle.group_by(spec, hb),
            False, where="jni/retry")


def test_corrupt_cells_throw_illegal_data(shim):
    lib, ctx = shim
    enc, hb = _data(63, "float", False)
    enc["val_off"] = enc["val_off"].copy()
    enc["val_off"][2:] -= 1  # row 1 loses a value byte
    spec = core.make_spec(datasets.T0, datasets.T0 + 3600000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    st, *_ = J.run_cells(lib, ctx, spec, enc, hb.n_series, hb.group_offsets,
                         hb.group_members, 1 << 16)
    exc = J.pending(lib)
    assert st == 1 and exc[0] == "net/opentsdb/core/IllegalDataException", exc
    assert "Corrupted value" in exc[1]


def test_unsupported_returns_without_exception(shim):
    """A calendar spec without its table: UNSUPPORTED goes back to Java
    (GpuAggregation keeps the reference iterators), nothing thrown."""
    lib, ctx = shim
    enc, hb = _data(64, "float", False)
    spec = core.make_spec(datasets.T0, datasets.T0 + 3600000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    sa = J.pack_spec(spec)
    sa[J.SPEC_FIELDS.index("use_calendar")] = 1
    st, *_ = J.run_cells(lib, ctx, spec, enc, hb.n_series, hb.group_offsets,
                         hb.group_members, 1 << 16, spec_arr=sa)
    assert st == 5 and J.pending(lib) is None
