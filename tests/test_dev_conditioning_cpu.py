"""Why `dev` must be replayed in the reference's order (CPU only).

StdDev.runDouble (Aggregators.java:547-568) is one sequential Welford pass.
On offset data its result carries the pass's own rounding, ~1e-11 relative
from the exact standard deviation; a different order of the same values —
lanes merged with Chan's formula, even with the merge done in EXACT rational
arithmetic (what double-double partials approximate) — carries a different
~1e-11.  The north star's 1e-12 bar for dev therefore cannot be met by a
more accurate merge, only by the same order; tests/test_gpu_dev_order.py
checks the engine does that (bit-exact).  Conversely, on well-conditioned
data (cpu% gauges, C4's rates of counters across series: mean / sigma < 100)
any order lands within ~1e-14: the chunk and rank merges of groups too large
for one chain stay far inside the bar there."""
import math
from fractions import Fraction

import numpy as np


def java_welford(xs):
    """StdDev.runDouble, line for line (Aggregators.java:547-568)."""
    old_mean = xs[0]
    n = 2
    m2 = 0.0
    for x in xs[1:]:
        new_mean = old_mean + (x - old_mean) / n
        m2 += (x - old_mean) * (x - new_mean)
        old_mean = new_mean
        n += 1
    return 0.0 if n == 2 else math.sqrt(m2 / (n - 1)), (n - 1, old_mean, m2)


def exact_dev(xs):
    fs = [Fraction(x) for x in xs]
    m = sum(fs) / len(fs)
    return math.sqrt(float(sum((f - m) ** 2 for f in fs) / len(fs)))


def exact_chan(parts):
    """Chan et al.'s merge of Welford runs in exact arithmetic."""
    n, mean, m2 = 0, Fraction(0), Fraction(0)
    for pn, pm, pm2 in parts:
        pm, pm2 = Fraction(pm), Fraction(pm2)
        if n == 0:
            n, mean, m2 = pn, pm, pm2
            continue
        d = pm - mean
        tot = n + pn
        m2 = m2 + pm2 + d * d * n * pn / tot
        mean = mean + d * pn / tot
        n = tot
    return math.sqrt(float(m2 / n))


def _rel(a, b):
    return abs(a - b) / abs(b)


def test_offset_data_needs_the_reference_order():
    rng = np.random.default_rng(5266)
    worst_ref, worst_chan = 0.0, 0.0
    for _ in range(40):
        # one 5 m bucket of a counter near 2^32 (30 points, +0..999 a step)
        xs = [float(x) for x in
              int(rng.integers(0, 2**32)) + np.cumsum(rng.integers(0, 1000, 30))]
        ref, _ = java_welford(xs)
        ex = exact_dev(xs)
        # the lane tree: runs of 8 points, merged exactly
        parts = [java_welford(xs[i:i + 8])[1] if len(xs[i:i + 8]) > 1 else
                 (1, xs[i], 0.0) for i in range(0, 30, 8)]
        worst_ref = max(worst_ref, _rel(ref, ex))
        worst_chan = max(worst_chan, _rel(exact_chan(parts), ref))
    # the reference itself is ~1e-11 from the exact value, and so an exact
    # merge of the lane runs misses the reference by far more than 1e-12
    assert worst_ref > 1e-12
    assert worst_chan > 1e-12


def test_well_conditioned_data_any_order():
    rng = np.random.default_rng(7)
    for mean, sd in ((50.0, 29.0), (600.0, 8.0)):  # cpu %, C4's rate sums
        xs = list(rng.normal(mean, sd, 3000))
        ref, _ = java_welford(xs)
        parts = [java_welford(xs[i:i + 256])[1] for i in range(0, 3000, 256)]
        assert _rel(exact_chan(parts), ref) < 1e-13
