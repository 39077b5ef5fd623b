"""kquery — host side of the MI355X columnar execution kernel for kquerydiy.

Mirrors the reference's physical layer (folkol/query-engines kquerydiy/src/Main.kt) over the
C ABI in include/qe_hip.h; all data-path work runs in the HIP kernels of libqe_hip.so.
"""
from . import native  # noqa: F401
from .columnar import (  # noqa: F401
    ArrowTypes,
    ColumnVector,
    Context,
    DeviceColumn,
    Field,
    HostColumn,
    RecordBatch,
    Schema,
)
from .native import IllegalArgumentException, IllegalStateException, QueryEngineError  # noqa: F401
