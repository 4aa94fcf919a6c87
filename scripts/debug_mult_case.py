"""One failing product case of the sweep: each member of the group alone
(the downsampled rate devs that the product multiplies), GPU vs oracle, and
the worst bucket's factors.  Usage: debug_mult_case.py seed g"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from opentsdb_amd import core  # noqa: E402
from opentsdb_amd.engine import Engine  # noqa: E402
from oracle import pyoracle  # noqa: E402
from scripts.debug_sweep_case import sub_batch  # noqa: E402
from tests.test_gpu_parity import _vals  # noqa: E402
from tests.test_gpu_sweep import _case  # noqa: E402


def main():
    seed, g = int(sys.argv[1]), int(sys.argv[2])
    b, spec, exact, where = _case(seed)
    print(where, "exact", exact, flush=True)
    e = Engine(0)
    members = list(b.group_members[b.group_offsets[g]:b.group_offsets[g + 1]])
    print("members", members, flush=True)
    for s in members:
        sb = sub_batch(b, [s])
        got = e.run(spec, sb)
        ref = pyoracle.group_by(spec, sb)
        if not ref or len(ref[0]) == 0:
            print("series", s, "no points")
            continue
        va = _vals(got[0].bits, got[0].is_int)
        vr = _vals(ref[0]["bits"], ref[0]["is_int"])
        ok = ~np.isnan(vr)
        rel = np.abs(va - vr)[ok] / np.maximum(np.abs(vr[ok]), 1e-300)
        i = int(np.argmax(rel)) if rel.size else 0
        print("series %d: %d pts, max rel %.3g at %r vs %r, bits equal %d/%d" % (
            s, len(vr), rel.max() if rel.size else 0, va[ok][i], vr[ok][i],
            int((np.asarray(got[0].bits) == ref[0]["bits"]).sum()), len(vr)),
            flush=True)


if __name__ == "__main__":
    main()
