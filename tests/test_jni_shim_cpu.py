"""The JNI shim (integration/jni/otsdb_agg_jni.c) compiled against the fake
JNIEnv (tests/jni_fake) — the calls that need no GPU: Aggregator names to
ids, and the argument checks that throw before the engine runs
(IllegalArgumentException, as GpuAggregation.java expects)."""
import numpy as np

from opentsdb_amd import core
from tests import jni_fake_lib as J


def _lib():
    J.build()
    return J.load()


def test_agg_ids_match_the_abi():
    """nativeAggId maps Aggregator.toString() onto the engine's ids."""
    lib = _lib()
    for name in ("sum", "zimsum", "avg", "dev", "p99", "ep999r7", "none",
                 "mult", "first", "mimmax", "median"):
        agg = core.Aggregators.get(name)
        assert lib.fj_agg_id(str(agg).encode()) == agg.id, name
    assert lib.fj_agg_id(b"nope") == -1
    assert J.pending(lib) is None


def _spec():
    return core.make_spec(0, 3600 * 1000, core.Aggregators.SUM,
                          core.DownsamplingSpecification("1m-avg"))


def _enc():
    z = np.zeros(1, np.int64)
    return dict(row_series=z[:0], row_base_s=z[:0], qual_off=z, qual=np.zeros(1, np.uint8),
                val_off=z, val=np.zeros(1, np.uint8))


def test_bad_arguments_throw_illegal_argument():
    """Checks the shim makes before any engine call (ctx 0 is never used)."""
    lib = _lib()
    goff = np.array([0, 0], np.int64)
    # spec shorter than SPEC_LEN
    st, *_ = J.run_cells(lib, 0, _spec(), _enc(), 0, goff, goff[:0], 4,
                         spec_arr=np.zeros(3, np.int64))
    assert st == 3 and J.pending(lib)[0] == "java/lang/IllegalArgumentException"
    # output offsets shorter than groups + 1
    st, *_ = J.run_cells(lib, 0, _spec(), _enc(), 0, goff, goff[:0], 4,
                         ooff_len=1)
    assert st == 3 and J.pending(lib)[0] == "java/lang/IllegalArgumentException"
    # values / is_int shorter than the timestamps
    st, *_ = J.run_cells(lib, 0, _spec(), _enc(), 0, goff, goff[:0], 4,
                         oval_len=2)
    assert st == 3 and J.pending(lib)[0] == "java/lang/IllegalArgumentException"
