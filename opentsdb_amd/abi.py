"""ctypes mirror of include/otsdb_agg.h and the loader of libotsdb_agg.so.

The product path ALWAYS goes through the native library; there is no
Python/CPU fallback.  `load()` raises if the HIP extension is missing.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libotsdb_agg.so")
# tuning runs (scripts/ab_bucketize.py) point this at the variants build
if os.environ.get("OTSDB_LIB"):
    LIB_PATH = os.environ["OTSDB_LIB"]

# otsdb_status
OK = 0
E_ILLEGAL_DATA = 1
E_ILLEGAL_STATE = 2
E_ILLEGAL_ARGUMENT = 3
E_NO_SUCH_ELEMENT = 4
E_UNSUPPORTED = 5
E_DEVICE = 6
E_CAPACITY = 7


class QuerySpec(C.Structure):
    _fields_ = [
        ("start_ms", C.c_int64),
        ("end_ms", C.c_int64),
        ("query_start_ms", C.c_int64),
        ("query_end_ms", C.c_int64),
        ("agg_id", C.c_int32),
        ("interp", C.c_int32),
        ("ds_interval_ms", C.c_int64),
        ("ds_agg_id", C.c_int32),
        ("fill", C.c_int32),
        ("run_all", C.c_int32),
        ("use_calendar", C.c_int32),
        ("rate", C.c_int32),
        ("counter", C.c_int32),
        ("drop_resets", C.c_int32),
        ("flags", C.c_int32),  # OTSDB_SPEC_* (ABI 5)
        ("counter_max", C.c_int64),
        ("reset_value", C.c_int64),
        ("cal_edges", C.c_void_p),
        ("n_cal_edges", C.c_int64),
        ("cal_anchors", C.c_void_p),
        ("cal_anchor_edge", C.c_void_p),
        ("n_cal_anchors", C.c_int64),
    ]


class Batch(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("n_points", C.c_int64),
        ("offsets", C.c_void_p),
        ("ts_ms", C.c_void_p),
        ("val", C.c_void_p),
        ("is_float", C.c_void_p),
        ("series_float", C.c_void_p),
        ("n_groups", C.c_int64),
        ("group_offsets", C.c_void_p),
        ("group_members", C.c_void_p),
        ("group_offsets_host", C.c_void_p),
    ]


class Result(C.Structure):
    _fields_ = [
        ("capacity", C.c_int64),
        ("offsets", C.c_void_p),
        ("ts", C.c_void_p),
        ("val", C.c_void_p),
        ("is_int", C.c_void_p),
    ]


class Sizes(C.Structure):
    _fields_ = [
        ("n_buckets", C.c_int64),
        ("max_out_points", C.c_int64),
        ("workspace_bytes", C.c_int64),
    ]


class Partial(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double),
                ("w", C.c_int64)]


class Cells(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("row_series", C.c_void_p),
        ("row_base_s", C.c_void_p),
        ("qual_off", C.c_void_p),
        ("qual", C.c_void_p),
        ("val_off", C.c_void_p),
        ("val", C.c_void_p),
    ]


class CellsOut(C.Structure):
    _fields_ = [("row_series", C.c_void_p), ("row_base_s", C.c_void_p),
                ("qual_off", C.c_void_p), ("qual", C.c_void_p),
                ("val_off", C.c_void_p), ("val", C.c_void_p)]


class RawRows(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64),
        ("row_series", C.c_void_p),
        ("row_base_s", C.c_void_p),
        ("row_col_off", C.c_void_p),
        ("col_qual_off", C.c_void_p),
        ("qual", C.c_void_p),
        ("col_val_off", C.c_void_p),
        ("val", C.c_void_p),
        ("col_ts", C.c_void_p),
    ]


class GenSpec(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("t0_ms", C.c_int64),
        ("duration_ms", C.c_int64),
        ("cadence_ms", C.c_int64),
        ("kind", C.c_int32),
        ("flags", C.c_int32),
    ]


SPEC_EXACT_ORDER = 1  # otsdb_query_spec.flags


EXPORTS = [
    "otsdb_abi_version", "otsdb_ctx_create", "otsdb_ctx_destroy",
    "otsdb_last_error", "otsdb_agg_lookup", "otsdb_agg_name",
    "otsdb_agg_interpolation", "otsdb_agg_plan", "otsdb_agg_run",
    "otsdb_agg_run_device", "otsdb_agg_partials_device",
    "otsdb_agg_partials_chained_device", "otsdb_agg_finalize_device",
    "otsdb_gen_counts_device",
    "otsdb_gen_fill_device", "otsdb_prof_enable", "otsdb_prof_read",
    "otsdb_ctx_counters", "otsdb_test_set_compact_epoch",
    "otsdb_decode_cells_device", "otsdb_sel_prepare_device",
    "otsdb_sel_hist_device", "otsdb_sel_hist_wait", "otsdb_sel_pick_device",
    "otsdb_sel_finish_device",
    "otsdb_encode_cells_device", "otsdb_agg_run_cells_device",
    "otsdb_compact_rows_device", "otsdb_span_assemble_device",
    "otsdb_agg_run_raw_device", "otsdb_agg_run_raw", "otsdb_agg_run_cells",
]

_lib = None


def load(path=None):
    """Loads libotsdb_agg.so (built by __graft_entry__.build()).  Raises
    RuntimeError when the HIP extension is missing — never falls back."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            "libotsdb_agg.so not built (%s): run __graft_entry__.build(); the "
            "aggregation path has no CPU fallback" % p)
    try:
        # torch ships its own HIP runtime under the same SONAME; loading it
        # first makes libotsdb_agg.so bind to that one copy instead of
        # starting a second runtime in the process.
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(p)
    vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
    lib.otsdb_abi_version.restype = C.c_int
    lib.otsdb_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    lib.otsdb_ctx_create.restype = C.c_int
    lib.otsdb_ctx_destroy.argtypes = [vp]
    lib.otsdb_ctx_destroy.restype = None
    lib.otsdb_last_error.restype = C.c_char_p
    lib.otsdb_agg_lookup.argtypes = [C.c_char_p, C.POINTER(i32)]
    lib.otsdb_agg_lookup.restype = C.c_int
    lib.otsdb_agg_name.argtypes = [i32]
    lib.otsdb_agg_name.restype = C.c_char_p
    lib.otsdb_agg_interpolation.argtypes = [i32]
    lib.otsdb_agg_interpolation.restype = i32
    PS, PB, PR = C.POINTER(QuerySpec), C.POINTER(Batch), C.POINTER(Result)
    lib.otsdb_agg_plan.argtypes = [vp, PS, PB, C.POINTER(Sizes)]
    lib.otsdb_agg_plan.restype = C.c_int
    lib.otsdb_agg_run.argtypes = [vp, PS, PB, PR]
    lib.otsdb_agg_run.restype = C.c_int
    lib.otsdb_agg_run_device.argtypes = [vp, PS, PB, PR, vp]
    lib.otsdb_agg_run_device.restype = C.c_int
    lib.otsdb_agg_partials_device.argtypes = [vp, PS, PB, vp, vp, vp]
    lib.otsdb_agg_partials_device.restype = C.c_int
    lib.otsdb_agg_partials_chained_device.argtypes = [vp, PS, PB, vp, vp, vp,
                                                      vp, vp]
    lib.otsdb_agg_partials_chained_device.restype = C.c_int
    lib.otsdb_agg_finalize_device.argtypes = [vp, PS, i64, i64, i32, vp, vp,
                                              PR, vp]
    lib.otsdb_agg_finalize_device.restype = C.c_int
    PG = C.POINTER(GenSpec)
    lib.otsdb_gen_counts_device.argtypes = [vp, PG, i64, i64, vp, vp]
    lib.otsdb_gen_counts_device.restype = C.c_int
    lib.otsdb_gen_fill_device.argtypes = [vp, PG, i64, i64, vp, vp, vp, vp]
    lib.otsdb_gen_fill_device.restype = C.c_int
    lib.otsdb_decode_cells_device.argtypes = [vp, C.POINTER(Cells), i64, vp,
                                              vp, vp, vp, i64, vp]
    lib.otsdb_decode_cells_device.restype = C.c_int
    lib.otsdb_sel_prepare_device.argtypes = [vp, PS, PB, vp, vp, vp, vp]
    lib.otsdb_sel_prepare_device.restype = C.c_int
    lib.otsdb_sel_hist_device.argtypes = [vp, i32, vp, vp, vp, vp, vp,
                                          C.POINTER(C.c_int32), vp]
    lib.otsdb_sel_hist_device.restype = C.c_int
    lib.otsdb_sel_hist_wait.argtypes = [vp, vp]
    lib.otsdb_sel_hist_wait.restype = C.c_int
    lib.otsdb_sel_pick_device.argtypes = [vp, vp, vp]
    lib.otsdb_sel_pick_device.restype = C.c_int
    lib.otsdb_sel_finish_device.argtypes = [vp, vp, PR, vp]
    lib.otsdb_sel_finish_device.restype = C.c_int
    lib.otsdb_encode_cells_device.argtypes = [vp, PB, vp, vp, vp,
                                              C.POINTER(CellsOut), vp]
    lib.otsdb_encode_cells_device.restype = C.c_int
    lib.otsdb_agg_run_cells_device.argtypes = [vp, PS, C.POINTER(Cells), PB,
                                               PR, vp]
    lib.otsdb_agg_run_cells_device.restype = C.c_int
    PW, PC, PCO = C.POINTER(RawRows), C.POINTER(Cells), C.POINTER(CellsOut)
    lib.otsdb_compact_rows_device.argtypes = [vp, PW, i32, PCO, i64, i64,
                                              C.POINTER(i64), vp]
    lib.otsdb_compact_rows_device.restype = C.c_int
    lib.otsdb_span_assemble_device.argtypes = [vp, PC, i64, PCO, i64, i64,
                                               C.POINTER(i64), vp]
    lib.otsdb_span_assemble_device.restype = C.c_int
    lib.otsdb_agg_run_raw_device.argtypes = [vp, PS, PW, i32, PB, PR, vp]
    lib.otsdb_agg_run_raw_device.restype = C.c_int
    lib.otsdb_agg_run_raw.argtypes = [vp, PS, PW, i32, PB, PR]
    lib.otsdb_agg_run_raw.restype = C.c_int
    lib.otsdb_agg_run_cells.argtypes = [vp, PS, PC, PB, PR]
    lib.otsdb_agg_run_cells.restype = C.c_int
    lib.otsdb_prof_enable.argtypes = [vp, C.c_int]
    lib.otsdb_prof_enable.restype = C.c_int
    lib.otsdb_prof_read.argtypes = [vp, vp, vp, C.c_int, C.c_int]
    lib.otsdb_prof_read.restype = C.c_int
    if hasattr(lib, "otsdb_ctx_counters"):  # (diagnostics; A/B of old builds)
        lib.otsdb_ctx_counters.argtypes = [vp, vp, C.c_int]
        lib.otsdb_ctx_counters.restype = C.c_int
    if hasattr(lib, "otsdb_test_set_compact_epoch"):  # (test hook)
        lib.otsdb_test_set_compact_epoch.argtypes = [vp, C.c_uint32]
        lib.otsdb_test_set_compact_epoch.restype = C.c_int
    if path is None:
        _lib = lib
    return lib
