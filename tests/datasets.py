"""Seeded synthetic query batches for parity tests (small enough for the
oracle to finish in seconds).  Shapes follow BaseTsdbTest's datasets
(BaseTsdbTest.java:612-791) in spirit: regular cadences with missing points,
offsets, late/early series, long and double values, plus the edge cases the
reference tests cover (empty spans, points outside the window, NaNs)."""
import numpy as np

from opentsdb_amd.batch import HostBatch, groups_from_ids

T0 = 1356998400000  # BaseTsdbTest base time, ms


def random_batch(seed, n_series=40, n_groups=5, span_ms=3 * 3600 * 1000,
                 cadence_ms=10000, value_kind="float", nan_frac=0.0,
                 empty_frac=0.05, outside=True, counter=False,
                 big_group=False, t0=T0):
    rng = np.random.default_rng(seed)
    offs = [0]
    tss, vals, isf = [], [], []
    for s in range(n_series):
        if rng.random() < empty_frac:
            offs.append(offs[-1])
            continue
        n = span_ms // cadence_ms
        phase = int(rng.integers(0, cadence_ms))
        t = t0 + phase + cadence_ms * np.arange(n, dtype=np.int64)
        keep = rng.random(n) > 0.05
        # an outage
        if rng.random() < 0.4:
            a = int(rng.integers(0, n))
            keep[a:a + int(rng.integers(1, n // 3 + 2))] = False
        # late start / early end
        if rng.random() < 0.2:
            keep[:int(rng.integers(0, n // 2))] = False
        if rng.random() < 0.2:
            keep[n - int(rng.integers(0, n // 2)):] = False
        if outside and rng.random() < 0.3:
            # points before the window start and after the end
            t = t - int(rng.integers(0, 2 * 3600 * 1000))
        t = t[keep]
        m = len(t)
        if counter:
            inc = rng.integers(0, 1000, m)
            v = np.cumsum(inc) + int(rng.integers(0, 2**32))
            rs = rng.random(m) < 0.02
            for i in np.nonzero(rs)[0]:
                v[i:] -= v[i]
            f = np.zeros(m, np.uint8)
            bits = v.astype(np.int64)
        elif value_kind == "float":
            v = rng.random(m) * 100.0
            if nan_frac:
                v[rng.random(m) < nan_frac] = np.nan
            bits = v.view(np.int64)
            f = np.ones(m, np.uint8)
        elif value_kind == "offset":
            # large values with a small spread (a gauge of ~3e9 moving by
            # < 1e4): Welford's result depends on its order at ~1e-11
            v = 3.0e9 + rng.random(m) * 1.0e4
            bits = v.view(np.int64)
            f = np.ones(m, np.uint8)
        elif value_kind == "int":
            bits = rng.integers(-50, 100, m).astype(np.int64)
            f = np.zeros(m, np.uint8)
        else:  # mixed
            f = (rng.random(m) < 0.5).astype(np.uint8)
            fv = (rng.random(m) * 100.0).view(np.int64)
            iv = rng.integers(0, 100, m).astype(np.int64)
            bits = np.where(f == 1, fv, iv)
        tss.append(t)
        vals.append(bits)
        isf.append(f)
        offs.append(offs[-1] + m)
    ts = np.concatenate(tss) if tss else np.zeros(0, np.int64)
    val = np.concatenate(vals) if vals else np.zeros(0, np.int64)
    isf = np.concatenate(isf) if isf else np.zeros(0, np.uint8)
    if big_group:
        gid = np.zeros(n_series, np.int64)
    else:
        gid = rng.integers(0, n_groups, n_series)
        gid[:n_groups] = np.arange(n_groups)  # every group non-empty
    g_off, members = groups_from_ids(gid, n_groups if not big_group else 1)
    return HostBatch(np.array(offs, np.int64), ts, val, isf, None, g_off,
                     members)
