"""ctypes access to the JNI shim compiled against the fake JNIEnv
(tests/jni_fake: harness.c + its jni.h test double), so tests drive
integration/jni/otsdb_agg_jni.c's Java_net_opentsdb_core_GpuAggregation_*
natives the way GpuAggregation.java does.  Tests only."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "opentsdb_amd", "_build", "libotsdb_agg_jni_fake.so")

# GpuAggregation.SPEC_* (integration/java/.../GpuAggregation.java:132-136)
SPEC_FIELDS = ("start_ms", "end_ms", "query_start_ms", "query_end_ms",
               "agg_id", "interp", "ds_interval_ms", "ds_agg_id", "fill",
               "run_all", "use_calendar", "rate", "counter", "drop_resets",
               "counter_max", "reset_value")


def build():
    """make -C tests/jni_fake (a no-op when up to date)."""
    subprocess.check_call(["make", "-s", "-C",
                           os.path.join(ROOT, "tests", "jni_fake")])


def load():
    if not os.path.exists(LIB):
        build()
    # the engine first, through abi.load(): it imports torch so that
    # libotsdb_agg.so (the shim's dependency) binds to torch's HIP runtime —
    # the shim pulling in the system one first would start a second runtime
    # in the process and leave torch without devices
    from opentsdb_amd import abi
    abi.load()
    lib = C.CDLL(LIB)
    lib.fj_exception_class.restype = C.c_char_p
    lib.fj_exception_message.restype = C.c_char_p
    lib.fj_ctx_create.restype = C.c_int64
    lib.fj_ctx_create.argtypes = [C.c_int32]
    lib.fj_ctx_destroy.argtypes = [C.c_int64]
    lib.fj_agg_id.restype = C.c_int32
    lib.fj_agg_id.argtypes = [C.c_char_p]
    lib.fj_run_cells.restype = C.c_int32
    lib.fj_run_cells.argtypes = [C.c_int64, C.c_int32, C.POINTER(C.c_void_p),
                                 C.POINTER(C.c_int64)]
    return lib


def pending(lib):
    """(exception class, message) ThrowNew left pending, or None."""
    cls = lib.fj_exception_class().decode()
    return (cls, lib.fj_exception_message().decode()) if cls else None


def pack_spec(spec):
    """otsdb_query_spec -> the long[] GpuAggregation packs."""
    return np.array([int(getattr(spec, f)) for f in SPEC_FIELDS], np.int64)


def run_cells(lib, ctx, spec, enc, n_series, goff, gmem, cap, cal=None,
              spec_arr=None, ooff_len=None, oval_len=None):
    """nativeRunCells over Java-like arrays; returns (status, offsets, ts,
    val bits, is_int).  Arrays given as None are Java nulls."""
    lib.fj_clear()
    G = len(goff) - 1
    sa = pack_spec(spec) if spec_arr is None else spec_arr
    outs = [np.zeros(G + 1 if ooff_len is None else ooff_len, np.int64),
            np.zeros(cap, np.int64),
            np.zeros(cap if oval_len is None else oval_len, np.int64),
            np.zeros(cap, np.uint8)]
    arrs = [sa, cal, None, None,
            enc["row_series"], enc["row_base_s"], enc["qual_off"],
            enc["qual"].view(np.int8), enc["val_off"],
            enc["val"].view(np.int8), goff, gmem] + outs
    keep = [None if a is None else np.ascontiguousarray(a) for a in arrs]
    ptrs = (C.c_void_p * 16)(*[0 if a is None else a.ctypes.data for a in keep])
    lens = (C.c_int64 * 16)(*[-1 if a is None else len(a) for a in keep])
    st = lib.fj_run_cells(ctx, n_series, ptrs, lens)
    return st, keep[12], keep[13], keep[14], keep[15]
