"""Print the GPU and oracle timestamps of one group of a sweep case, plus
the same query over that group alone.  Usage: debug_sweep_case.py seed:g ..."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from opentsdb_amd.engine import Engine  # noqa: E402
from opentsdb_amd.batch import HostBatch, groups_from_ids  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import datasets  # noqa: E402
from tests.test_gpu_sweep import _case  # noqa: E402

T0 = datasets.T0


def sub_batch(b, members):
    offs, ts, val, isf = [0], [], [], []
    for s in members:
        a, e = b.offsets[s], b.offsets[s + 1]
        ts.append(b.ts[a:e])
        val.append(b.val[a:e])
        if b.is_float is not None:
            isf.append(b.is_float[a:e])
        else:
            f = 1 if b.series_float is None else int(b.series_float[s])
            isf.append(np.full(e - a, f, np.uint8))
        offs.append(offs[-1] + e - a)
    g_off, mem = groups_from_ids(np.zeros(len(members), np.int64), 1)
    return HostBatch(np.array(offs, np.int64), np.concatenate(ts),
                     np.concatenate(val), np.concatenate(isf), None, g_off, mem)


def show(e, spec, b, g, tag):
    got = e.run(spec, b)
    ref = pyoracle.group_by(spec, b)
    gt = (np.asarray(got[g].ts) - T0) // 1000
    rt = (ref[g]["ts"] - T0) // 1000
    print(tag, "gpu", len(gt), "oracle", len(rt))
    print("  gpu-only", np.setdiff1d(gt, rt)[:40])
    print("  oracle-only", np.setdiff1d(rt, gt)[:80])


def main():
    e = Engine(0)
    for arg in sys.argv[1:]:
        seed, g = map(int, arg.split(":"))
        b, spec, exact, where = _case(seed)
        print("==", where, "window", (spec.start_ms - T0) // 1000,
              (spec.end_ms - T0) // 1000)
        show(e, spec, b, g, "full")
        m = b.group_members[b.group_offsets[g]:b.group_offsets[g + 1]]
        for s in m:
            t = (b.ts[b.offsets[s]:b.offsets[s + 1]] - T0) // 1000
            print("  member", s, len(t), (t[0], t[-1]) if len(t) else None)
        show(e, spec, sub_batch(b, m), 0, "alone")
        g0 = -(-spec.start_ms // spec.ds_interval_ms) * spec.ds_interval_ms
        stop = spec.end_ms // spec.ds_interval_ms * spec.ds_interval_ms
        empty = [s for s in m if not ((b.ts[b.offsets[s]:b.offsets[s + 1]] >= g0)
                                      & (b.ts[b.offsets[s]:b.offsets[s + 1]] < stop)).any()]
        full = [s for s in m if s not in empty]
        print("  empty-in-grid members", empty)
        if empty and full:
            show(e, spec, sub_batch(b, full), 0, "without empty")
            show(e, spec, sub_batch(b, full[:1]), 0, "first full alone")
            show(e, spec, sub_batch(b, full[:1] + empty[:1]), 0, "full+empty")
            show(e, spec, sub_batch(b, empty[:1] + full[:1]), 0, "empty+full")
            show(e, spec, sub_batch(b, empty[:1]), 0, "empty alone")
    e.close()


if __name__ == "__main__":
    main()
