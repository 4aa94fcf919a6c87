"""The qualifier-start logic of k_requal (decode.hip), restated in Python
and checked against RowSeq's sequential walk (RowSeq.java:552-643: a
qualifier whose first byte has the 0xF nibble is 4 bytes, else 2) on
random unit streams.  What the kernel computes per 16-unit lane:
  m      ms-looking units (high nibble 0xF),
  S1     the starts if the lane is entered on a start: non-starts are
         a+1, a+3, ... for each run of ms-looking units starting at a, runs
         labelled by the parity of a with one add,
  flip   the units whose start state depends on the entry state (up to
         and including the first non-ms unit),
and the entry state of a lane is the exit state of the nearest lane below
holding a non-ms unit (lanes of 16 ms-looking units flip 16 times)."""
import numpy as np

M32 = (1 << 32) - 1


def sequential_starts(ms):
    s, out = 1, []
    for b in ms:
        out.append(s)
        s = int(not (s and b))
    return out


def lane(ms_bits, nu):
    m = sum(1 << i for i in range(nu) if ms_bits[i])
    vm = 0xFFFF if nu >= 16 else (1 << nu) - 1
    edges = m & ~(m << 1) & M32
    x = (m + (edges & 0x55555555)) & M32
    ns = ((((m & ~x) << 1) & 0xAAAAAAAA) | (((m & x) << 1) & 0x55555555)) & M32
    s1 = ~ns & vm
    nz = ~m & vm
    d = nz != 0
    fixed_out = int(not ((ns >> nu) & 1))
    flip = ((2 << ((nz & -nz).bit_length() - 1)) - 1) if d else vm
    return s1, flip, d, fixed_out


def wave_starts(ms):
    units = len(ms)
    out, cs = [0] * units, 1
    for u0 in range(0, units, 1024):
        lanes = []
        for ln in range(64):
            ub = u0 + 16 * ln
            nu = 0 if ub >= units else min(16, units - ub)
            lanes.append(lane([ms[ub + i] if i < nu else 0 for i in range(16)],
                              nu) + (nu, ub))
        cin = []
        for ln in range(64):
            below = [k for k in range(ln) if lanes[k][2]]
            cin.append(lanes[below[-1]][3] if below else cs)
        for ln in range(64):
            s1, flip, d, fo, nu, ub = lanes[ln]
            s = s1 if cin[ln] else s1 ^ flip
            for i in range(nu):
                out[ub + i] = (s >> i) & 1
        s1, flip, d, fo, nu, ub = lanes[63]
        cs = fo if d else cin[63]
    return out


def test_requal_starts_match_the_sequential_walk():
    rng = np.random.default_rng(7)
    for t in range(600):
        units = int(rng.integers(1, 2600))
        p = [0.05, 0.5, 0.9, 0.99, 1.0][t % 5]
        ms = [int(x) for x in (rng.random(units) < p)]
        assert wave_starts(ms) == sequential_starts(ms), (t, units, p)
