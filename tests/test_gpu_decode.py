"""Compacted-cell decode on the GPU (RowSeq semantics) against the oracle's
RowSeq.Iterator restatement, and decode -> aggregate against the columnar
path."""
import ctypes as C

import numpy as np
import pytest

from opentsdb_amd import abi, core
from opentsdb_amd.engine import Engine
from oracle import pyoracle
from tests import cells, datasets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = Engine(0)
    yield e
    e.close()


def decode_gpu(engine, enc, S):
    import torch
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda()
         for k, v in enc.items()}
    cs = abi.Cells(len(enc["row_series"]), d["row_series"].data_ptr(),
                   d["row_base_s"].data_ptr(), d["qual_off"].data_ptr(),
                   d["qual"].data_ptr(), d["val_off"].data_ptr(),
                   d["val"].data_ptr())
    offs = torch.zeros(S + 1, dtype=torch.int64, device="cuda")
    engine._check(engine.lib.otsdb_decode_cells_device(
        engine.ctx, C.byref(cs), S, offs.data_ptr(), None, None, None, 0,
        None))
    n = int(offs[-1].item())
    ts = torch.empty(max(n, 2), dtype=torch.int64, device="cuda")
    val = torch.empty(max(n, 2), dtype=torch.int64, device="cuda")
    isf = torch.empty(max(n, 2), dtype=torch.uint8, device="cuda")
    engine._check(engine.lib.otsdb_decode_cells_device(
        engine.ctx, C.byref(cs), S, offs.data_ptr(), ts.data_ptr(),
        val.data_ptr(), isf.data_ptr(), n, None))
    torch.cuda.synchronize()
    return (offs.cpu().numpy(), ts[:n].cpu().numpy(), val[:n].cpu().numpy(),
            isf[:n].cpu().numpy())


@pytest.mark.parametrize("kind,f4,ms", [("float", 0.0, 0.0), ("int", 0, 0.0),
                                        ("mixed", 0.3, 0.2), ("float", 0, 1.0)])
def test_decode_roundtrip_and_oracle(engine, kind, f4, ms):
    rng = np.random.default_rng(5)
    b = datasets.random_batch(3, n_series=20, n_groups=2, value_kind=kind,
                              cadence_ms=7000 if ms else 10000)
    if ms:  # millisecond timestamps
        b.ts = b.ts + rng.integers(0, 999, len(b.ts))
        b.ts.sort()  # keep rows sorted
        for s in range(b.n_series):
            a, z = b.offsets[s], b.offsets[s + 1]
            b.ts[a:z] = np.sort(b.ts[a:z])
    enc = cells.encode_batch(b, rng, f4, ms)
    offs, ts, val, isf = decode_gpu(engine, enc, b.n_series)
    # oracle: RowSeq.Iterator row by row
    ref_ts, ref_bits, ref_int = [], [], []
    for r in range(len(enc["row_series"])):
        q = enc["qual"][enc["qual_off"][r]:enc["qual_off"][r + 1]]
        v = enc["val"][enc["val_off"][r]:enc["val_off"][r + 1]]
        p = pyoracle.decode_row(q.tobytes(), v.tobytes(), enc["row_base_s"][r])
        ref_ts.append(p["ts"])
        ref_bits.append(p["bits"])
        ref_int.append(p["is_int"])
    assert np.array_equal(ts, np.concatenate(ref_ts))
    assert np.array_equal(val, np.concatenate(ref_bits))
    assert np.array_equal(isf == 0, np.concatenate(ref_int).astype(bool))
    assert np.array_equal(offs, b.offsets)
    if f4 == 0:  # lossless encoding: the columns come back exactly
        assert np.array_equal(ts, b.ts)
        assert np.array_equal(val, b.val)


def test_decode_corrupt_column(engine):
    b = datasets.random_batch(4, n_series=3, n_groups=1, empty_frac=0)
    enc = cells.encode_batch(b)
    enc["val_off"] = enc["val_off"].copy()
    enc["val_off"][1] -= 1  # first row loses a value byte
    with pytest.raises(core.IllegalDataException):
        decode_gpu(engine, enc, b.n_series)


def test_cells_to_aggregate_matches_columns(engine):
    """decode -> aggregate == aggregate of the original columns."""
    from opentsdb_amd.batch import HostBatch
    b = datasets.random_batch(8, n_series=30, n_groups=3, value_kind="mixed")
    enc = cells.encode_batch(b)
    offs, ts, val, isf = decode_gpu(engine, enc, b.n_series)
    hb = HostBatch(offs, ts, val, isf, None, b.group_offsets, b.group_members)
    spec = core.make_spec(datasets.T0, datasets.T0 + 3 * 3600 * 1000,
                          core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))
    got = engine.run(spec, hb)
    ref = engine.run(spec, b)
    for g, r in zip(got, ref):
        assert np.array_equal(g.ts, r.ts) and np.array_equal(g.bits, r.bits)
