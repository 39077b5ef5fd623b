"""Data sources (Main.kt:63-66): InMemoryDataSource (Main.kt:1292-1304) and the synthetic
device-resident RecordBatches of the benchmark configs (BASELINE.json configs[1..3]).

Synthetic columns come from the counter-based generator (qe_generate, restated bit-for-bit in
oracle/gen.py): u = splitmix64(seed ^ col*phi ^ row), so every GPU shard and the CPU oracle
regenerate any row without transfer.
"""
from __future__ import annotations

from typing import Iterator, List, Sequence

from . import native as N
from .columnar import Context, DeviceColumn, Field, RecordBatch, Schema


class DataSource:
    def schema(self) -> Schema:
        raise NotImplementedError

    def scan(self, projection: Sequence[str]) -> Iterator[RecordBatch]:
        raise NotImplementedError


class InMemoryDataSource(DataSource):
    """Main.kt:1292-1304: projects by column index. Like the reference it passes the FULL schema
    to every projected batch (Main.kt:1301); harmless because operators never read it."""

    def __init__(self, schema: Schema, data: List[RecordBatch]):
        self._schema = schema
        self.data = list(data)

    def schema(self) -> Schema:
        return self._schema

    def scan(self, projection: Sequence[str]) -> Iterator[RecordBatch]:
        names = [f.name for f in self._schema.fields]
        idx = [names.index(p) if p in names else -1 for p in projection]
        for batch in self.data:
            yield RecordBatch(self._schema, [batch.field(i) for i in idx])


# ---- synthetic columns ------------------------------------------------------------------------------
SEED = 42


class ColumnSpec:
    """One generated column: name, Arrow type, distribution, param, generator column id."""

    def __init__(self, name: str, type_id: int, dist: int, param: int, col_id: int, null_permille: int = 0):
        self.name = name
        self.type = type_id
        self.dist = dist
        self.param = param
        self.col_id = col_id
        self.null_permille = null_permille

    def field(self) -> Field:
        return Field(self.name, self.type)


# BASELINE.json configs
C2_COLUMNS = [  # 10M rows: filter(a > 2^19) + project(a + b)
    ColumnSpec("a", N.TYPE_INT64, N.GEN_MOD, 1 << 20, 1),
    ColumnSpec("b", N.TYPE_INT64, N.GEN_RAW, 0, 2),
]
C3_COLUMNS = [  # 100M fp64: SUM/MIN/MAX/COUNT
    ColumnSpec("x", N.TYPE_FLOAT64, N.GEN_UNIT53, 0, 3),
]
C4_COLUMNS = [  # 1B rows: SELECT k, SUM(a+b), COUNT(*), MIN(a), MAX(b) WHERE a > 2^19 GROUP BY k
    ColumnSpec("k", N.TYPE_INT64, N.GEN_MOD, 1024, 0),
    ColumnSpec("a", N.TYPE_INT64, N.GEN_MOD, 1 << 20, 1),
    ColumnSpec("b", N.TYPE_INT64, N.GEN_MOD, 1 << 20, 2),
]
C4_THRESHOLD = 1 << 19

# 10B rows over 8 GPUs (1.25B per GPU), TPC-H-lineitem-shaped, 38 B/row
C5_COLUMNS = [
    ColumnSpec("l_quantity", N.TYPE_INT64, N.GEN_MOD, 50, 10),             # [0, 50)
    ColumnSpec("l_extendedprice", N.TYPE_FLOAT64, N.GEN_MOD_F64, 10_000_000, 11),  # [0, 100000) step 0.01
    ColumnSpec("l_discount", N.TYPE_FLOAT64, N.GEN_MOD_F64, 11, 12),        # 0.00 .. 0.10
    ColumnSpec("l_tax", N.TYPE_FLOAT64, N.GEN_MOD_F64, 9, 13),              # 0.00 .. 0.08
    ColumnSpec("l_returnflag", N.TYPE_UINT8, N.GEN_MOD, 3, 14),             # dictionary code of A/N/R
    ColumnSpec("l_linestatus", N.TYPE_UINT8, N.GEN_MOD, 2, 15),             # dictionary code of F/O
    ColumnSpec("l_shipdate", N.TYPE_DATE32, N.GEN_MOD, 2557, 16),           # days in a 7-year window
]
C5_SHIPDATE_MAX = 2400


def generate_column(spec: ColumnSpec, n: int, row0: int = 0, seed: int = SEED, ctx: Context = None) -> DeviceColumn:
    ctx = ctx or Context.get(0)
    col = DeviceColumn.empty(spec.type, n, spec.null_permille > 0, ctx=ctx)
    c = col.as_c()
    N.check(N.lib().qe_generate(ctx.handle, N.C.byref(c), spec.dist, spec.param, seed, spec.col_id, row0,
                                spec.null_permille))
    return col


class SyntheticDataSource(DataSource):
    """Device-resident synthetic table, generated once (inputs resident in HBM before timing)."""

    def __init__(self, specs: Sequence[ColumnSpec], rows: int, batch_rows: int = 1 << 30, row0: int = 0,
                 seed: int = SEED, ctx: Context = None):
        self.specs = list(specs)
        self._schema = Schema([s.field() for s in self.specs])
        self.rows = rows
        self.row0 = row0
        ctx = ctx or Context.get(0)
        self.batches: List[RecordBatch] = []
        for start in range(0, rows, batch_rows):
            n = min(batch_rows, rows - start)
            cols = [generate_column(s, n, row0 + start, seed, ctx) for s in self.specs]
            self.batches.append(RecordBatch(self._schema, cols))
        ctx.synchronize()

    def schema(self) -> Schema:
        return self._schema

    def scan(self, projection: Sequence[str]) -> Iterator[RecordBatch]:
        names = [s.name for s in self.specs]
        idx = [names.index(p) for p in projection] if projection else list(range(len(names)))
        sch = Schema([self._schema.fields[i] for i in idx])
        for b in self.batches:
            yield RecordBatch(sch, [b.field(i) for i in idx])
