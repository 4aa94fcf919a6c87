"""GPU-box debugging aid: replays the row-test generators and prints the
first row where the GPU compaction / span assembly and the oracle differ."""
import sys

import numpy as np

sys.path.insert(0, ".")
from opentsdb_amd import storage  # noqa: E402
from opentsdb_amd.engine import Engine  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import datasets, rows_fuzz  # noqa: E402
from tests.test_gpu_rows import _gpu_compact, _gpu_span, _raw_from_hb  # noqa: E402


def show(cols):
    for q, v, t in cols:
        print("   q=%s v=%s ts=%d" % (q.hex(), v.hex(), t))


e = Engine(0)
for seed in (11, 12):
    rng = np.random.default_rng(seed)
    for i in range(60):
        cols = rows_fuzz.random_row(rng, corrupt=0.5)
        if rows_fuzz.heap_with_append(cols):
            continue
        try:
            ref = pyoracle.compact_row([(q, v) for q, v, _ in cols],
                                       [t for _, _, t in cols], False)
            err = None
        except pyoracle.OracleError as ex:
            err = ex.status
        try:
            got = _gpu_compact(e, [(0, rows_fuzz.BASE, cols)], fix=False)
            gerr = None
        except Exception as ex:  # noqa: BLE001
            got, gerr = None, repr(ex)
        if (err is None) != (gerr is None) or (err is None and got != (
                [] if ref is None else [(0, rows_fuzz.BASE, ref[0], ref[1])])):
            print("MISMATCH seed", seed, "row", i, "oracle", err, ref, "gpu", gerr, got)
            show(cols)
            break

# end-to-end rows: compaction and span bytes vs the oracle
rng = np.random.default_rng(7)
hb = datasets.random_batch(41, n_series=30, n_groups=3, span_ms=3 * 3600000,
                           value_kind="float", cadence_ms=10000)
hb.ts[:] = hb.ts - hb.ts % 1000
hb.is_float = np.ones(len(hb.ts), np.uint8)
rows = _raw_from_hb(rng, hb)
got = _gpu_compact(e, rows)
ref = []
for s, b, cols in rows:
    r = pyoracle.compact_row([(q, v) for q, v, _ in cols], [t for _, _, t in cols], True)
    if r is not None:
        ref.append((s, b, r[0], r[1]))
print("compact rows", len(got), len(ref), "equal", got == ref)
for k, (g, r) in enumerate(zip(got, ref)):
    if g != r:
        print("first diff at", k, "\n gpu", g[0], g[1], g[2].hex(), g[3].hex(),
              "\n ref", r[0], r[1], r[2].hex(), r[3].hex())
        show(rows[k][2])
        break
sp = _gpu_span(e, ref, hb.n_series)
sref = []
for s in range(hb.n_series):
    sref += [(s, b, q, v) for b, q, v in pyoracle.span_assemble(
        [(b, q, v) for ss, b, q, v in ref if ss == s])]
print("span rows", len(sp), len(sref), "equal", sp == sref)
# points of the spans vs hb
for s in range(hb.n_series):
    pts = []
    for ss, b, q, v in sref:
        if ss == s:
            pts += [int(p["ts"]) for p in pyoracle.decode_row(q, v, b)]
    a, bb = hb.offsets[s], hb.offsets[s + 1]
    if pts != [int(x) for x in hb.ts[a:bb]]:
        print("series", s, "points differ", len(pts), bb - a)
        break
