"""ctypes binding of libqe_hip.so (include/qe_hip.h).

This is the Python twin of the JNI shim described in INTEGRATION.md: the reference's
``Expression.evaluate`` / ``HashAggregateExec.execute`` (kquerydiy/src/Main.kt:448-450,
:615-651) call into these entry points with plain device pointers. Device buffers come from
torch (plumbing only); no torch type crosses the C ABI.

There is deliberately NO CPU fallback: if the HIP library is missing or no GPU is present,
every call raises. The CPU restatement lives in ``oracle/`` and is test infrastructure only.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

_ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB_PATH = _ROOT / "lib" / "libqe_hip.so"

# ---- constants (qe_hip.h) -----------------------------------------------------------------
QE_OK = 0
QE_ERR_INVALID_ARG = -1
QE_ERR_UNSUPPORTED = -2
QE_ERR_OOM = -3
QE_ERR_DEVICE = -4
QE_ERR_CAPACITY = -5
QE_ERR_COMM = -6
COMM_ID_BYTES = 128

TYPE_INT64 = 1
TYPE_FLOAT64 = 2
TYPE_BOOL = 3
TYPE_UTF8 = 4
TYPE_INT32 = 5
TYPE_UINT8 = 6
TYPE_DATE32 = 7

GEN_MOD = 1
GEN_RAW = 2
GEN_UNIT53 = 3
GEN_MOD_F64 = 4

OP_ADD, OP_SUB, OP_MUL, OP_DIV = 1, 2, 3, 4
OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE = 10, 11, 12, 13, 14, 15
OP_AND, OP_OR, OP_NOT, OP_IS_NULL, OP_IS_NOT_NULL = 20, 21, 22, 23, 24

AGG_SUM, AGG_MIN, AGG_MAX, AGG_COUNT, AGG_COUNT_STAR, AGG_AVG = 1, 2, 3, 4, 5, 6

MAX_KEYS, MAX_AGGS, MAX_COLS, MAX_TERMS, MAX_TOKENS = 4, 8, 8, 8, 16
TOK_COL, TOK_LIT, TOK_ADD, TOK_SUB, TOK_MUL, TOK_DIV = 1, 2, 3, 4, 5, 6

FIXED_WIDTH = {TYPE_INT64: 8, TYPE_FLOAT64: 8, TYPE_INT32: 4, TYPE_DATE32: 4, TYPE_UINT8: 1}


# ---- errors: mirror the reference's exception classes (Main.kt) -----------------------------
class QueryEngineError(RuntimeError):
    """Base class; ``status`` is the C ABI status code."""

    def __init__(self, status: int, message: str):
        super().__init__(f"[{status}] {message}")
        self.status = status


class IllegalStateException(QueryEngineError):
    """QE_ERR_UNSUPPORTED (Main.kt:195, :469, :677, :792, :799)."""


class IllegalArgumentException(QueryEngineError):
    """QE_ERR_INVALID_ARG (Main.kt:49)."""


class NumberFormatException(IllegalArgumentException):
    """CAST(utf8 AS double) of a string outside java.lang.Double.parseDouble's grammar (K:791)."""


class CapacityError(QueryEngineError):
    """QE_ERR_CAPACITY: an output buffer is too small."""


class DeviceError(QueryEngineError):
    """QE_ERR_DEVICE / QE_ERR_OOM."""


class CommError(QueryEngineError):
    """QE_ERR_COMM: RCCL missing or a collective failed."""


_ERR_CLASS = {
    QE_ERR_UNSUPPORTED: IllegalStateException,
    QE_ERR_INVALID_ARG: IllegalArgumentException,
    QE_ERR_CAPACITY: CapacityError,
    QE_ERR_COMM: CommError,
}


# ---- structs ----------------------------------------------------------------------------------
class QeColumn(C.Structure):
    _fields_ = [
        ("type", C.c_int32),
        ("max_len", C.c_int32),  # UTF8: the producer's bound on value lengths (0: unknown)
        ("length", C.c_int64),
        ("validity", C.c_void_p),
        ("values", C.c_void_p),
        ("offsets", C.c_void_p),
    ]


class QeScalar(C.Structure):
    _fields_ = [("type", C.c_int32), ("is_null", C.c_int32), ("bits", C.c_int64)]


class QeOperand(C.Structure):
    _fields_ = [("col", C.POINTER(QeColumn)), ("lit", QeScalar)]


class QeGlobalAgg(C.Structure):
    _fields_ = [
        ("rows", C.c_int64),
        ("count", C.c_int64),
        ("type", C.c_int32),
        ("valid", C.c_int32),
        ("sum", C.c_int64),
        ("min", C.c_int64),
        ("max", C.c_int64),
        ("avg", C.c_double),
    ]


class QeAggDesc(C.Structure):
    _fields_ = [("fn", C.c_int32), ("input_type", C.c_int32)]


class QePredTerm(C.Structure):
    _fields_ = [
        ("col", C.c_int32),
        ("op", C.c_int32),
        ("rhs_col", C.c_int32),
        ("reserved", C.c_int32),
        ("lit", QeScalar),
    ]


class QeToken(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32), ("lit", QeScalar)]


class QeAggProgram(C.Structure):
    _fields_ = [("ntokens", C.c_int32), ("reserved", C.c_int32), ("tokens", QeToken * MAX_TOKENS)]


class QeFusedSpec(C.Structure):
    _fields_ = [
        ("mask_col", C.c_int32),
        ("nterms", C.c_int32),
        ("terms", QePredTerm * MAX_TERMS),
        ("key_cols", C.c_int32 * MAX_KEYS),
        ("inputs", QeAggProgram * MAX_AGGS),
    ]


class QeCsvOptions(C.Structure):
    _fields_ = [("delimiter", C.c_int32), ("has_header", C.c_int32), ("nfields", C.c_int32),
                ("flags", C.c_int32), ("field_index", C.POINTER(C.c_int32))]


CSV_PARTIAL_TAIL = 1  # QE_CSV_PARTIAL_TAIL


class QeSelectSpec(C.Structure):
    _fields_ = [
        ("mask_col", C.c_int32),
        ("nterms", C.c_int32),
        ("terms", QePredTerm * MAX_TERMS),
        ("nout", C.c_int32),
        ("reserved", C.c_int32),
        ("outputs", QeAggProgram * MAX_AGGS),
    ]


# ---- library ------------------------------------------------------------------------------------
_lib = None

# (name, restype, argtypes) for every entry point declared in include/qe_hip.h
HASHAGG_DETERMINISTIC = 1  # qe_hashagg_create_ex flags
HASHAGG_FAST_FP64 = 2
_P = C.c_void_p
_PP = C.POINTER(C.c_void_p)
_I64P = C.POINTER(C.c_int64)
_COLP = C.POINTER(QeColumn)
_OPP = C.POINTER(QeOperand)
SLOT_HEADER = 64  # QE_SLOT_HEADER: bytes before a slot's records
KEYED_HEADER = 128  # QE_KEYED_HEADER: bytes before a keyed block's sections
GLOBAL_PARTIAL_BYTES = 128  # QE_GLOBAL_PARTIAL_BYTES
GLOBAL_EXACT_BYTES = 320  # QE_GLOBAL_EXACT_BYTES
QE_NEED_EXACT = 1  # qe_agg_global_merge: run the exact round (not an error)

SIGNATURES = [
    ("qe_ctx_create", C.c_int, [C.c_int, _P, _PP]),
    ("qe_ctx_create_owned", C.c_int, [C.c_int, _PP]),
    ("qe_ctx_set_jit", C.c_int, [_P, C.c_int32]),
    ("qe_ctx_destroy", C.c_int, [_P]),
    ("qe_ctx_stream", _P, [_P]),
    ("qe_ctx_synchronize", C.c_int, [_P]),
    ("qe_last_error", C.c_char_p, []),
    ("qe_abi_version", C.c_int, []),
    ("qe_device_alloc", C.c_int, [_P, C.c_size_t, _PP]),
    ("qe_device_free", C.c_int, [_P, _P]),
    ("qe_release_cached_memory", C.c_int, [C.c_int]),
    ("qe_copy_to_device", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("qe_file_to_device", C.c_int, [_P, C.c_char_p, C.c_int64, C.c_int64, _P]),
    ("qe_copy_to_host", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("qe_generate", C.c_int, [_P, _COLP, C.c_int32, C.c_int64, C.c_uint64, C.c_uint64, C.c_int64, C.c_int32]),
    ("qe_stream_read", C.c_int, [_P, _COLP, C.c_int32, C.POINTER(C.c_double)]),
    ("qe_stream_read_best", C.c_int, [_P, _COLP, C.c_int32, C.c_int32, C.POINTER(C.c_double), C.c_char_p, C.c_int32]),
    ("qe_eval_arith", C.c_int, [_P, C.c_int32, _OPP, _OPP, _COLP]),
    ("qe_eval_cmp", C.c_int, [_P, C.c_int32, _OPP, _OPP, _COLP]),
    ("qe_eval_bool", C.c_int, [_P, C.c_int32, _COLP, _COLP, _COLP]),
    ("qe_cast_utf8_to_f64", C.c_int, [_P, _COLP, _COLP, _I64P]),
    ("qe_filter_count", C.c_int, [_P, _COLP, _I64P]),
    ("qe_filter_apply", C.c_int, [_P, _COLP, _COLP, C.c_int32, _COLP, _I64P]),
    ("qe_filter_apply_async", C.c_int, [_P, _COLP, _COLP, C.c_int32, _COLP, _P]),
    ("qe_eval_arith_dlen", C.c_int, [_P, C.c_int32, _OPP, _OPP, _COLP, _P]),
    ("qe_agg_global", C.c_int, [_P, _COLP, _COLP, C.POINTER(QeGlobalAgg)]),
    ("qe_agg_global_partial", C.c_int, [_P, _COLP, _COLP, C.c_int64, _P]),
    ("qe_agg_global_merge", C.c_int, [_P, C.c_int32, _P, C.c_int32, C.POINTER(QeGlobalAgg)]),
    ("qe_agg_global_exact_partial", C.c_int, [_P, _COLP, _COLP, _P]),
    ("qe_agg_global_merge_exact", C.c_int, [_P, _P, C.c_int32, C.POINTER(QeGlobalAgg)]),
    ("qe_hashagg_create", C.c_int,
     [_P, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(QeAggDesc), C.c_int64, _PP]),
    ("qe_hashagg_create_ex", C.c_int,
     [_P, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(QeAggDesc), C.c_int64, C.c_int32, _PP]),
    ("qe_hashagg_destroy", C.c_int, [_P]),
    ("qe_hashagg_reset", C.c_int, [_P]),
    ("qe_hashagg_update", C.c_int, [_P, _COLP, _COLP, _COLP]),
    ("qe_hashagg_update_fused", C.c_int, [_P, _COLP, C.c_int32, C.POINTER(QeFusedSpec)]),
    ("qe_hashagg_num_groups", C.c_int, [_P, _I64P]),
    ("qe_hashagg_finalize", C.c_int, [_P, _COLP, _COLP, _I64P]),
    ("qe_hashagg_record_bytes", C.c_int, [_P, _I64P]),
    ("qe_hashagg_export_counts", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_hashagg_export", C.c_int, [_P, C.c_int32, _P]),
    ("qe_hashagg_import", C.c_int, [_P, _P, C.c_int64]),
    ("qe_hashagg_export_slots", C.c_int, [_P, C.c_int32, C.c_int64, _P]),
    ("qe_hashagg_import_slots", C.c_int, [_P, _P, C.c_int32, C.c_int64, _I64P, _I64P]),
    ("qe_hashagg_slot_capacity", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_hashagg_finalize_sizes", C.c_int, [_P, _I64P, _I64P]),
    ("qe_hashagg_export_keyed_sizes", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_hashagg_export_keyed", C.c_int, [_P, C.c_int32, _P]),
    ("qe_hashagg_import_keyed", C.c_int, [_P, _P, C.c_int32, _I64P]),
    ("qe_hashagg_merge", C.c_int, [_P, _P]),
    ("qe_hashagg_bind_key_dict", C.c_int, [_P, C.c_int32, _P]),
    ("qe_hashagg_key_bytes_bound", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_hashagg_key_layout", C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("qe_comm_unique_id", C.c_int, [_P]),
    ("qe_comm_create", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.POINTER(C.c_void_p)]),
    ("qe_comm_destroy", C.c_int, [_P]),
    ("qe_comm_loopback_hub_create", C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    ("qe_comm_loopback_hub_destroy", C.c_int, [_P]),
    ("qe_comm_create_loopback", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.POINTER(C.c_void_p)]),
    ("qe_hashagg_exchange", C.c_int, [_P, _P, _P, C.c_int64, _I64P]),
    ("qe_hashagg_set_row_base", C.c_int, [_P, C.c_int64]),
    ("qe_hashagg_set_async", C.c_int, [_P, C.c_int32]),
    ("qe_hashagg_last_kernel_time", C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    ("qe_hashagg_last_kernel_signature", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("qe_hashagg_last_kernel_kind", C.c_int, [_P, C.POINTER(C.c_int32), C.c_char_p, C.c_int32]),
    ("qe_strdict_create", C.c_int, [_P, C.c_int64, _PP]),
    ("qe_strdict_destroy", C.c_int, [_P]),
    ("qe_strdict_size", C.c_int, [_P, _I64P]),
    ("qe_strdict_encode", C.c_int, [_P, _COLP, _COLP]),
    ("qe_strdict_decode_bytes", C.c_int, [_P, _COLP, _I64P]),
    ("qe_strdict_decode", C.c_int, [_P, _COLP, _COLP]),
    ("qe_strdict_decode_trusted", C.c_int, [_P, _COLP, _COLP]),
    ("qe_strdict_encode_packed", C.c_int, [_P, _COLP, _COLP]),
    ("qe_strdict_decode_packed", C.c_int, [_P, _COLP, _COLP]),
    ("qe_strdict_encode_tuple", C.c_int, [_P, _COLP, C.c_int32, _COLP]),
    ("qe_strdict_decode_tuple", C.c_int, [_P, _COLP, C.c_int32, _COLP]),
    ("qe_hash_partition", C.c_int, [_P, _COLP, C.c_int32, C.c_int32, _P]),
    ("qe_select_project", C.c_int, [_P, _COLP, C.c_int32, C.POINTER(QeSelectSpec), _COLP, _I64P]),
    ("qe_select_project_async", C.c_int, [_P, _COLP, C.c_int32, C.POINTER(QeSelectSpec), _COLP, C.POINTER(_P)]),
    ("qe_select_pending_wait", C.c_int, [_P, _I64P]),
    ("qe_csv_parse", C.c_int, [_P, _P, C.c_int64, C.POINTER(QeCsvOptions), _PP]),
    ("qe_csv_rows", C.c_int, [_P, _I64P]),
    ("qe_csv_consumed", C.c_int, [_P, _I64P]),
    ("qe_csv_column", C.c_int, [_P, C.c_int32, _COLP]),
    ("qe_csv_column_bytes", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_csv_column_max_len", C.c_int, [_P, C.c_int32, _I64P]),
    ("qe_csv_column_copy", C.c_int, [_P, C.c_int32, _COLP]),
    ("qe_csv_destroy", C.c_int, [_P]),
    ("qe_csv_record_end", C.c_int, [_P, C.c_int64, C.c_int32, _I64P]),
    ("qe_batch_import", C.c_int, [_P, _P, _P, _PP]),
    ("qe_batch_import_device", C.c_int, [_P, _P, _P, _PP]),
    ("qe_batch_destroy", C.c_int, [_P]),
    ("qe_batch_num_columns", C.c_int, [_P, C.POINTER(C.c_int32), _I64P]),
    ("qe_batch_column", C.c_int, [_P, C.c_int32, _COLP, C.POINTER(C.c_char_p)]),
    ("qe_batch_export", C.c_int, [_P, _COLP, C.c_int32, C.POINTER(C.c_char_p), _P, _P]),
]


def load_library(path: os.PathLike | str | None = None) -> C.CDLL:
    """Loads libqe_hip.so and binds every entry point. Raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # QE_LIB: another build of the library (experiments: A/B of two builds on one box)
    p = pathlib.Path(path) if path else pathlib.Path(os.environ.get("QE_LIB") or LIB_PATH)
    if not p.exists():
        raise ImportError(
            f"libqe_hip.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)"
        )
    lib = C.CDLL(str(p))
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def lib() -> C.CDLL:
    return load_library()


def check(status: int) -> None:
    if status != QE_OK:
        msg = lib().qe_last_error().decode(errors="replace")
        raise _ERR_CLASS.get(status, DeviceError)(status, msg)


def scalar(value, type_id: int | None = None) -> QeScalar:
    """Literal: None -> null int64; int -> INT64; float -> FLOAT64 (IEEE bits)."""
    import struct

    if value is None:
        return QeScalar(type_id or TYPE_INT64, 1, 0)
    if type_id == TYPE_FLOAT64 or (type_id is None and isinstance(value, float)):
        return QeScalar(TYPE_FLOAT64, 0, struct.unpack("<q", struct.pack("<d", float(value)))[0])
    v = int(value)
    if not -(1 << 63) <= v < (1 << 63):
        raise IllegalArgumentException(QE_ERR_INVALID_ARG, f"int64 literal out of range: {v}")
    return QeScalar(TYPE_INT64, 0, v)
