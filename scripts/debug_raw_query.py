"""GPU-box debugging aid: the storage-row query against the cells query on
the same points, stage by stage."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from opentsdb_amd import core, storage, workload  # noqa: E402
from opentsdb_amd.engine import DeviceResult, Engine  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import datasets  # noqa: E402
from tests.test_gpu_decode import _device_batch, _result_points  # noqa: E402
from tests.test_gpu_rows import _raw_from_hb  # noqa: E402

e = Engine(0)
rng = np.random.default_rng(7)
hb = datasets.random_batch(41, n_series=30, n_groups=3, span_ms=3 * 3600000,
                           value_kind="float", cadence_ms=10000)
hb.ts[:] = hb.ts - hb.ts % 1000
hb.is_float = np.ones(len(hb.ts), np.uint8)
split = float(sys.argv[1]) if len(sys.argv) > 1 else 0.3
rows = _raw_from_hb(rng, hb, split=split)
raw = storage.HostRawRows(rows, with_ts=True).to_device()
raw.n_series = hb.n_series
db = _device_batch(hb, "float")
t0, t1 = datasets.T0 + 600000, datasets.T0 + 3 * 3600000
spec = core.make_spec(t0, t1, core.Aggregators.SUM,
                      core.DownsamplingSpecification("1m-avg"), t0, t1)
ref = pyoracle.group_by(spec, hb)


def diff(tag, got):
    bad = 0
    for g in range(db.n_groups):
        a = np.asarray(got[g].bits).view(np.float64)
        r = ref[g]["bits"].view(np.float64)
        if len(a) != len(r) or not np.allclose(a, r, rtol=1e-9, equal_nan=True):
            bad += 1
    print(tag, "groups differing:", bad)


res = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
storage.run_raw_device(e, spec, raw, db, res)
diff("raw query", _result_points(res, db.n_groups))
cells = storage.compact_rows_device(e, raw, True)
diff_rows = cells.n_rows
sp = storage.span_assemble_device(e, cells)
res2 = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
workload.run_cells_device(e, spec, sp, db, res2)
diff("cells query on compact+span", _result_points(res2, db.n_groups))
res3 = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
workload.run_cells_device(e, spec, cells, db, res3)
diff("cells query on compact only", _result_points(res3, db.n_groups))
enc = workload.encode_cells_device(e, db)
res4 = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
workload.run_cells_device(e, spec, enc, db, res4)
diff("cells query on encoder", _result_points(res4, db.n_groups))
off, ts, val, isf = workload.decode_cells_device(e, sp)
print("decode of spans: points", int(off[-1]), "vs", len(hb.ts),
      "ts equal", np.array_equal(ts.cpu().numpy(), hb.ts),
      "val equal", np.array_equal(val.cpu().numpy(), hb.val))
print("rows: compact", diff_rows, "span", sp.n_rows, "encoder", enc.n_rows)

# experiment: the encoder's rows, each split in two rows of the same base
from tests import cells as CC  # noqa: E402
from opentsdb_amd.workload import DeviceCells  # noqa: E402
from tests.rows_fuzz import compacted, split_points  # noqa: E402


def to_cells(rows, S):
    qo = np.cumsum([0] + [len(r[2]) for r in rows]).astype(np.int64)
    vo = np.cumsum([0] + [len(r[3]) for r in rows]).astype(np.int64)
    t = dict(row_series=np.asarray([r[0] for r in rows], np.int64),
             row_base_s=np.asarray([r[1] for r in rows], np.int64),
             qual_off=qo, val_off=vo,
             qual=np.frombuffer(b"".join(r[2] for r in rows) + b"\0" * 64, np.uint8).copy(),
             val=np.frombuffer(b"".join(r[3] for r in rows) + b"\0" * 64, np.uint8).copy())
    t = {k: torch.from_numpy(x).cuda() for k, x in t.items()}
    return DeviceCells(t, S)


for mode in ("whole", "halves", "firstpoint"):
    rr = []
    for s in range(hb.n_series):
        a, b = hb.offsets[s], hb.offsets[s + 1]
        for base, q, v in CC.encode_series(hb.ts[a:b], hb.val[a:b], hb.is_float[a:b]):
            pts = split_points(q, v)
            if mode == "whole" or len(pts) < 4:
                rr.append((s, base) + compacted(pts))
            elif mode == "halves":
                h = len(pts) // 2
                rr.append((s, base) + compacted(pts[:h]))
                rr.append((s, base) + compacted(pts[h:]))
            else:
                rr.append((s, base) + compacted(pts[:1]))
                rr.append((s, base) + compacted(pts[1:]))
    cc = to_cells(rr, hb.n_series)
    r5 = DeviceResult(torch, db.n_groups, 4 * len(hb.ts) + 64, "cuda")
    workload.run_cells_device(e, spec, cc, db, r5)
    diff("experiment " + mode, _result_points(r5, db.n_groups))

# per-series view: one group per series
from opentsdb_amd.batch import groups_from_ids  # noqa: E402
g_off, members = groups_from_ids(np.arange(hb.n_series))
hb1 = datasets.random_batch(41, n_series=30, n_groups=3, span_ms=3 * 3600000,
                            value_kind="float", cadence_ms=10000)
hb1.ts[:] = hb1.ts - hb1.ts % 1000
hb1.is_float = np.ones(len(hb1.ts), np.uint8)
hb1.group_offsets, hb1.group_members = g_off, members
db1 = _device_batch(hb1, "float")
ref1 = pyoracle.group_by(spec, hb1)
rr = []
for s in range(hb1.n_series):
    a, b = hb1.offsets[s], hb1.offsets[s + 1]
    for base, q, v in CC.encode_series(hb1.ts[a:b], hb1.val[a:b], hb1.is_float[a:b]):
        pts = split_points(q, v)
        h = len(pts) // 2 if len(pts) >= 4 else len(pts)
        rr.append((s, base) + compacted(pts[:h]))
        if h < len(pts):
            rr.append((s, base) + compacted(pts[h:]))
cc = to_cells(rr, hb1.n_series)
r6 = DeviceResult(torch, db1.n_groups, 4 * len(hb1.ts) + 64, "cuda")
workload.run_cells_device(e, spec, cc, db1, r6)
got = _result_points(r6, db1.n_groups)
shown = 0
for g in range(db1.n_groups):
    a = np.asarray(got[g].bits).view(np.float64)
    r = ref1[g]["bits"].view(np.float64)
    if len(a) != len(r):
        print("series", g, "len", len(a), len(r))
        shown += 1
    else:
        bad = np.nonzero(~np.isclose(a, r, rtol=1e-9, equal_nan=True))[0]
        if len(bad):
            print("series", g, "bad buckets", bad[:8], "ts", np.asarray(got[g].ts)[bad[:4]],
                  "got", a[bad[:4]], "ref", r[bad[:4]])
            shown += 1
    if shown > 6:
        break
print("rows per series:", [sum(1 for x in rr if x[0] == s) for s in range(6)])
print("bases s0:", [x[1] for x in rr if x[0] == 0], "t0", t0, "t1", t1)
