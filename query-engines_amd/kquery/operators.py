"""Physical operators (Main.kt:442-446, :564-660) over device-resident RecordBatches.

``ScanExec`` / ``ProjectionExec`` / ``HashAggregateExec`` keep the reference's names, arguments
and pull-based ``execute()`` sequence; ``SelectionExec`` is the north star's filter operator
(absent from the reference). ``fuse`` is the planner hook (the reference's selection
point is createPhysicalPlan, Main.kt:680-706): it rewrites HashAggregateExec over a
Selection/Projection/Scan chain into ``FusedHashAggregateExec`` — one HIP kernel pass over HBM.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Sequence

from . import native as N
from .aggregate import HashAggregateState, dictionary_keys, output_type
from .columnar import DeviceColumn, DeviceCount, Field, RecordBatch, Schema
from .expressions import (
    AggregateExpression,
    AndExpression,
    ArithmeticExpression,
    ColumnExpression,
    ComparisonExpression,
    Expression,
    LiteralDoubleExpression,
    LiteralLongExpression,
    ScalarColumn,
)


class PhysicalPlan:
    def schema(self) -> Schema:
        raise NotImplementedError

    def execute(self) -> Iterator[RecordBatch]:
        raise NotImplementedError

    def children(self) -> List["PhysicalPlan"]:
        raise NotImplementedError


class ScanExec(PhysicalPlan):
    """Main.kt:564-580."""

    def __init__(self, ds, projection: Sequence[str]):
        self.ds = ds
        self.projection = list(projection)

    def schema(self) -> Schema:
        return self.ds.schema().select(self.projection)

    def execute(self) -> Iterator[RecordBatch]:
        return self.ds.scan(self.projection)

    def children(self) -> List[PhysicalPlan]:
        return []

    def __repr__(self) -> str:
        return f"ScanExec: schema={self.schema()}, projection={self.projection}"


class ProjectionExec(PhysicalPlan):
    """Main.kt:582-603: per batch, evaluate every expression; row count and order unchanged."""

    def __init__(self, input: PhysicalPlan, schema: Schema, expr: Sequence[Expression]):  # noqa: A002
        self.input = input
        self._schema = schema
        self.expr = list(expr)

    def schema(self) -> Schema:
        return self._schema

    def execute(self) -> Iterator[RecordBatch]:
        for batch in self.input.execute():
            yield RecordBatch(self._schema, [e.evaluate(batch) for e in self.expr])

    def children(self) -> List[PhysicalPlan]:
        return [self.input]

    def __repr__(self) -> str:
        return f"ProjectionExec: {self.expr}"


class SelectionExec(PhysicalPlan):
    """Filter (build-defined): keeps rows whose predicate is true (null -> dropped), in order.
    K3b order-preserving compaction (qe_filter_apply)."""

    def __init__(self, input: PhysicalPlan, expr: Expression):  # noqa: A002
        self.input = input
        self.expr = expr

    def schema(self) -> Schema:
        return self.input.schema()

    def execute(self) -> Iterator[RecordBatch]:
        for batch in self.input.execute():
            mask = self.expr.evaluate(batch)
            if not isinstance(mask, DeviceColumn) or mask.type != N.TYPE_BOOL:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "selection predicate must be BOOLEAN")
            yield filter_batch(batch, mask)

    def children(self) -> List[PhysicalPlan]:
        return [self.input]

    def __repr__(self) -> str:
        return f"SelectionExec: {self.expr}"


def _alloc_like(c: DeviceColumn, n: int, ctx) -> DeviceColumn:
    if c.type != N.TYPE_UTF8:
        return DeviceColumn.empty(c.type, n, c.nullable, ctx=ctx)
    import torch

    from .columnar import bitmap_bytes

    nbytes = int(c.offsets[c.length].item() - c.offsets[0].item()) if c.length else 0
    dev = ctx.torch_device
    return DeviceColumn(N.TYPE_UTF8, n, torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev),
                        torch.zeros(max(bitmap_bytes(n), 4), dtype=torch.uint8, device=dev) if c.nullable else None,
                        torch.empty(n + 1, dtype=torch.int32, device=dev), ctx)


# How SelectionExec compacts non-nullable int64 / fp64 columns: "select_project" (one pass of the
# select-project kernel with the mask as the selection, then a wait for its row count: C2 10M rows
# 0.130-0.133 ms per cmp -> compact -> arith chain) or "gather" (count, scan and gather with the
# count left in HBM and read back at the end, qe_filter_apply_async: 0.148 ms; the form every other
# fixed-width batch takes).
SELECTION_COMPACTION = "select_project"


_SELPROJ_SPECS = {}  # column count -> the compaction's select-project spec (read-only once built)


def _compact_selproj(batch: RecordBatch, cols, mask: DeviceColumn) -> Optional[RecordBatch]:
    """The compaction through the select-project kernel (qe_select_project_async with the mask
    column as the selection and the columns themselves as the outputs: one pass with a decoupled
    look-back instead of count, scan and gather), then its row count. None: the kernel cannot take
    the plan."""
    ctx = mask.ctx
    n = mask.length
    spec = _SELPROJ_SPECS.get(len(cols))
    if spec is None:  # (the spec depends only on the column count: built once)
        spec = N.QeSelectSpec()
        spec.mask_col = len(cols)
        spec.nterms = 0
        spec.nout = len(cols)
        for i in range(len(cols)):
            spec.outputs[i].ntokens = 1
            spec.outputs[i].tokens[0] = N.QeToken(N.TOK_COL, i, N.QeScalar())
        _SELPROJ_SPECS[len(cols)] = spec
    outs = [DeviceColumn.empty(c.type, n, False, ctx=ctx) for c in cols]
    cc = (N.QeColumn * (len(cols) + 1))(*([c.as_c() for c in cols] + [mask.as_c()]))
    oc = (N.QeColumn * len(outs))(*[o.as_c() for o in outs])
    pending = N.C.c_void_p()
    st = N.lib().qe_select_project_async(ctx.handle, cc, len(cols) + 1, N.C.byref(spec), oc, N.C.byref(pending))
    if st == N.QE_ERR_UNSUPPORTED:
        return None
    N.check(st)
    cnt = N.C.c_int64()
    N.check(N.lib().qe_select_pending_wait(pending, N.C.byref(cnt)))
    for o in outs:
        o.length = cnt.value
    return RecordBatch(batch.schema, outs)


def filter_batch(batch: RecordBatch, mask: DeviceColumn) -> RecordBatch:
    """SelectionExec's compaction. Fixed-width columns (at most 8) take the stream-ordered form
    (qe_filter_apply_async): outputs sized by the mask, the selected-row count left in HBM and read
    back only when a consumer needs a length (DeviceColumn.length), so cmp -> filter -> arith runs
    without a host round trip. UTF8 columns take qe_filter_apply (their byte sizes need the count)."""
    ctx = mask.ctx
    cols = batch.fields
    if (SELECTION_COMPACTION == "select_project" and 0 < len(cols) < N.MAX_COLS and len(cols) <= N.MAX_AGGS
            and all(isinstance(c, DeviceColumn) and c.type in (N.TYPE_INT64, N.TYPE_FLOAT64) and not c.nullable
                    for c in cols)):
        done = _compact_selproj(batch, cols, mask)
        if done is not None:
            return done
    if (0 < len(cols) <= N.MAX_COLS and all(isinstance(c, DeviceColumn) and c.type in N.FIXED_WIDTH for c in cols)):
        import torch

        n = mask.length
        outs = [DeviceColumn.empty(c.type, n, c.nullable, ctx=ctx) for c in cols]
        cnt = DeviceCount(torch.empty(1, dtype=torch.int64, device=ctx.torch_device), ctx)
        mc = mask.as_c()
        ins = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        os_ = (N.QeColumn * len(cols))(*[o.as_c() for o in outs])
        N.check(N.lib().qe_filter_apply_async(ctx.handle, N.C.byref(mc), ins, len(cols), os_, cnt.ptr()))
        for o in outs:
            o.pending = cnt
        return RecordBatch(batch.schema, outs)
    cnt = N.C.c_int64()
    mc = mask.as_c()
    N.check(N.lib().qe_filter_count(ctx.handle, N.C.byref(mc), N.C.byref(cnt)))
    n = cnt.value
    cols = batch.fields
    for c in cols:
        if not isinstance(c, DeviceColumn):
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "selection input must be device columns")
    outs = [_alloc_like(c, n, ctx) for c in cols]
    done: list = [None] * len(cols)
    # qe_filter_apply gathers up to 8 columns per launch
    for s in range(0, len(cols), N.MAX_COLS):
        part = cols[s:s + N.MAX_COLS]
        ins = (N.QeColumn * len(part))(*[c.as_c() for c in part])
        os_ = (N.QeColumn * len(part))(*[o.as_c() for o in outs[s:s + N.MAX_COLS]])
        got = N.C.c_int64()
        N.check(N.lib().qe_filter_apply(ctx.handle, N.C.byref(mc), ins, len(part), os_, N.C.byref(got)))
        for k, o in enumerate(outs[s:s + N.MAX_COLS]):
            o.length = got.value
            done[s + k] = o
    return RecordBatch(batch.schema, done)


class HashAggregateExec(PhysicalPlan):
    """Main.kt:605-660: consumes every input batch, emits ONE batch of group columns then
    aggregate columns. Row-at-a-time HashMap + Accumulator objects are replaced by the device
    hash-aggregate (K4b). A global aggregate over empty input yields 0 rows (Main.kt:637)."""

    def __init__(self, input: PhysicalPlan, groupExpr: Sequence[Expression],  # noqa: A002,N803
                 aggregateExpr: Sequence[AggregateExpression], schema: Schema,  # noqa: N803
                 expected_groups: int = 1024):
        self.input = input
        self.groupExpr = list(groupExpr)
        self.aggregateExpr = list(aggregateExpr)
        self._schema = schema
        self.expected_groups = expected_groups
        self.state: Optional[HashAggregateState] = None

    def schema(self) -> Schema:
        return self._schema

    def children(self) -> List[PhysicalPlan]:
        return [self.input]

    def partial_state(self) -> Optional[HashAggregateState]:
        """Runs the aggregation and returns the device state (for the two-phase exchange)."""
        state = None
        for batch in self.input.execute():
            keys = [e.evaluate(batch) for e in self.groupExpr]
            inputs = [a.inputExpression().evaluate(batch) if a.inputExpression() is not None else None
                      for a in self.aggregateExpr]
            for c in keys + [i for i in inputs if i is not None]:
                if not isinstance(c, DeviceColumn):
                    raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "aggregate inputs must be device columns")
            present = keys + [i for i in inputs if i is not None]
            if not present and batch.fields:  # COUNT(*) alone: any column gives the row count
                present = [batch.field(0)]
                inputs = [present[0] if a.fn == N.AGG_COUNT_STAR else i for a, i in zip(self.aggregateExpr, inputs)]
            if not present:
                raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "COUNT(*) over a batch without columns")
            if state is None:
                state = HashAggregateState(
                    present[0].ctx, [k.type for k in keys],
                    [(a.fn, (i.type if i is not None and a.fn != N.AGG_COUNT_STAR else N.TYPE_INT64))
                     for a, i in zip(self.aggregateExpr, inputs)],
                    self.expected_groups, async_update=True)
            state.update(keys, inputs)
        self.state = state
        return state

    def execute(self) -> Iterator[RecordBatch]:
        state = self.partial_state()
        yield finalize_batch(state, self._schema, self.groupExpr, self.aggregateExpr)

    def __repr__(self) -> str:
        return f"HashAggregateExec: groupExpr={self.groupExpr}, aggrExpr={self.aggregateExpr}"


def finalize_batch(state: Optional[HashAggregateState], schema: Schema, groupExpr, aggregateExpr) -> RecordBatch:  # noqa: N803
    if state is None:  # no input batch at all: empty output
        from .columnar import Context

        ctx = Context.get(0)
        cols = [DeviceColumn.empty(f.dataType if f.dataType in N.FIXED_WIDTH else N.TYPE_INT64, 0, True, ctx=ctx)
                for f in schema.fields]
        return RecordBatch(schema, cols)
    keys, aggs = state.finalize()
    return RecordBatch(schema, keys + aggs)


# ---------------------------------------------------------------------------------------------------
# Fusion: HashAggregateExec(Projection?(Selection?(Scan))) -> one kernel
# ---------------------------------------------------------------------------------------------------
class FusedHashAggregateExec(PhysicalPlan):
    """SelectionExec -> ProjectionExec -> HashAggregateExec in ONE pass over the scanned columns
    (qe_hashagg_update_fused). Same results as the unfused chain."""

    def __init__(self, scan: PhysicalPlan, slots: Sequence[int], spec: N.QeFusedSpec, key_types, aggs,
                 schema: Schema, groupExpr, aggregateExpr, expected_groups: int = 1024,  # noqa: N803
                 key_scan: Optional[Sequence[int]] = None):
        self.scan = scan
        self.key_scan = list(key_scan) if key_scan is not None else None  # dictionary keys: scan columns
        self.slots = list(slots)  # scan column index per slot
        self.spec = spec
        self.key_types = list(key_types)
        self.aggs = list(aggs)
        self._schema = schema
        self.groupExpr = groupExpr
        self.aggregateExpr = aggregateExpr
        self.expected_groups = expected_groups
        self.state: Optional[HashAggregateState] = None

    def schema(self) -> Schema:
        return self._schema

    def children(self) -> List[PhysicalPlan]:
        return [self.scan]

    def partial_state(self, state: Optional[HashAggregateState] = None) -> Optional[HashAggregateState]:
        for batch in self.scan.execute():
            cols = [batch.field(i) for i in self.slots]
            key_cols = [batch.field(i) for i in self.key_scan] if self.key_scan is not None else None
            if state is None:
                # stream-ordered updates: the host prepares batch i + 1 while batch i's kernel runs
                state = HashAggregateState((cols or key_cols)[0].ctx, self.key_types, self.aggs, self.expected_groups,
                                           async_update=True)
            state.update_fused(cols, self.spec, key_cols)
        self.state = state
        return state

    def execute(self) -> Iterator[RecordBatch]:
        yield finalize_batch(self.partial_state(), self._schema, self.groupExpr, self.aggregateExpr)

    def __repr__(self) -> str:
        return f"FusedHashAggregateExec: slots={self.slots}, aggrExpr={self.aggregateExpr}"


class FusedSelectProjectExec(PhysicalPlan):
    """SelectionExec -> ProjectionExec (or a bare SelectionExec) in ONE pass over the scanned
    columns (qe_select_project): order-preserving, same rows and values as the unfused chain.
    Falls back to the unfused operators when the kernel cannot take the plan."""

    def __init__(self, scan: PhysicalPlan, slots: Sequence[int], spec: N.QeSelectSpec, out_types: Sequence[int],
                 schema: Schema, unfused: PhysicalPlan):
        self.scan = scan
        self.slots = list(slots)
        self.spec = spec
        self.out_types = list(out_types)
        self._schema = schema
        self.unfused = unfused
        self.last_kernel_rows = 0

    def schema(self) -> Schema:
        return self._schema

    def children(self) -> List[PhysicalPlan]:
        return [self.scan]

    def launch_batch(self, batch: RecordBatch):
        """Queues the select-project of one batch (qe_select_project_async) and returns
        (outputs, pending), or None when the kernel cannot take the plan."""
        cols = [batch.field(i) for i in self.slots]
        ctx = cols[0].ctx
        n = cols[0].length
        outs = [DeviceColumn.empty(t, n, self._may_be_null(k, cols), ctx=ctx) for k, t in enumerate(self.out_types)]
        cc = (N.QeColumn * len(cols))(*[c.as_c() for c in cols])
        oc = (N.QeColumn * len(outs))(*[o.as_c() for o in outs])
        pending = N.C.c_void_p()
        st = N.lib().qe_select_project_async(ctx.handle, cc, len(cols), N.C.byref(self.spec), oc, N.C.byref(pending))
        if st == N.QE_ERR_UNSUPPORTED:
            return None
        N.check(st)
        return outs, pending, cols

    def finish_batch(self, launched) -> RecordBatch:
        """Waits for that batch's kernels only (not for what was queued behind them) and sets the
        output row count."""
        outs, pending, _cols = launched
        cnt = N.C.c_int64()
        N.check(N.lib().qe_select_pending_wait(pending, N.C.byref(cnt)))
        for o in outs:
            o.length = cnt.value
        return RecordBatch(self._schema, outs)

    def run_batch(self, batch: RecordBatch) -> Optional[RecordBatch]:
        launched = self.launch_batch(batch)
        return None if launched is None else self.finish_batch(launched)

    def _may_be_null(self, k: int, cols: Sequence[DeviceColumn]) -> bool:
        """Whether output k can hold a null, as compile_program decides it (qe_hashagg.hip): a
        referenced column with a validity bitmap, a null literal, or a division (int64 x / 0 ->
        null). Only such outputs get a validity bitmap: allocating and filling one for the C2
        output cost ~10 us of a ~73 us operator call (tools/selproj_op_overhead.py)."""
        pg = self.spec.outputs[k]
        for i in range(pg.ntokens):
            tk = pg.tokens[i]
            if tk.op == N.TOK_COL and cols[tk.arg].validity is not None:
                return True
            if (tk.op == N.TOK_LIT and tk.lit.is_null) or tk.op == N.TOK_DIV:
                return True
        return False

    def execute(self) -> Iterator[RecordBatch]:
        """Pipelined one batch ahead: batch i+1's kernels are queued before batch i's row count is
        read back, so the host wait for batch i overlaps batch i+1 on the device and the stream
        never drains between batches. Batches come out in input order (row order preserved)."""
        inflight = []  # launched, not yet waited on (at most two: this batch and the one ahead)
        try:
            for batch in self.scan.execute():
                launched = self.launch_batch(batch)
                if launched is not None:
                    inflight.append(launched)
                if len(inflight) > 1 or (launched is None and inflight):
                    yield self.finish_batch(inflight.pop(0))
                if launched is None:  # kernel specialisation unavailable: per-family operators
                    yield from _replay(self.unfused, batch)
            while inflight:
                yield self.finish_batch(inflight.pop(0))
        finally:
            # the consumer stopped early, or a scan / launch raised: every queued call is still
            # waited on once, which frees its pinned slot and event and runs its look-back stall
            # check (qe_select_pending_wait); an error here must not mask the one propagating
            for _outs, pending, _cols in inflight:
                N.lib().qe_select_pending_wait(pending, N.C.byref(N.C.c_int64()))

    def __repr__(self) -> str:
        return f"FusedSelectProjectExec: slots={self.slots}, outputs={self.out_types}"


class _OneBatch(PhysicalPlan):
    def __init__(self, batch: RecordBatch):
        self.batch = batch

    def execute(self) -> Iterator[RecordBatch]:
        yield self.batch


def _replay(plan: PhysicalPlan, batch: RecordBatch) -> Iterator[RecordBatch]:
    """Runs the unfused Projection/Selection chain of ``plan`` over one scanned batch."""
    if isinstance(plan, ProjectionExec):
        return ProjectionExec(_ReplayInput(plan.input, batch), plan.schema(), plan.expr).execute()
    if isinstance(plan, SelectionExec):
        return SelectionExec(_ReplayInput(plan.input, batch), plan.expr).execute()
    return iter([batch])


class _ReplayInput(PhysicalPlan):
    def __init__(self, plan: PhysicalPlan, batch: RecordBatch):
        self.plan = plan
        self.batch = batch

    def schema(self) -> Schema:
        return self.plan.schema()

    def execute(self) -> Iterator[RecordBatch]:
        return _replay(self.plan, self.batch)


class _NotFusable(Exception):
    pass


def _conjuncts(e: Expression) -> List[Expression]:
    if isinstance(e, AndExpression):
        return _conjuncts(e.l) + _conjuncts(e.r)
    return [e]


class _SlotMap:
    def __init__(self, scan_schema: Schema):
        self.schema = scan_schema
        self.slots: List[int] = []

    def slot(self, col_index: int) -> int:
        if col_index not in self.slots:
            if len(self.slots) >= N.MAX_COLS:
                raise _NotFusable("too many columns")
            self.slots.append(col_index)
        return self.slots.index(col_index)

    def type_of(self, col_index: int) -> int:
        return self.schema.fields[col_index].dataType


def _resolve(e: Expression, proj: Optional[List[Expression]]) -> Expression:
    """Substitute projection outputs (ColumnExpression over a ProjectionExec) by their definitions."""
    if proj is None:
        return e
    if isinstance(e, ColumnExpression):
        return proj[e.i]
    if isinstance(e, ArithmeticExpression):
        return type(e)(_resolve(e.l, proj), _resolve(e.r, proj))
    if isinstance(e, ComparisonExpression):
        return type(e)(_resolve(e.l, proj), _resolve(e.r, proj))
    return e


def _literal(e: Expression):
    if isinstance(e, LiteralLongExpression):
        return N.scalar(e.value, N.TYPE_INT64)
    if isinstance(e, LiteralDoubleExpression):
        return N.scalar(e.value, N.TYPE_FLOAT64)
    return None


def _program(e: Expression, sm: _SlotMap, out: list) -> bool:
    """Postfix tokens for an arithmetic tree; returns whether the result is fp64."""
    if isinstance(e, ColumnExpression):
        t = sm.type_of(e.i)
        if t not in N.FIXED_WIDTH:
            raise _NotFusable("non fixed-width input")
        out.append(N.QeToken(N.TOK_COL, sm.slot(e.i), N.QeScalar()))
        return t == N.TYPE_FLOAT64
    lit = _literal(e)
    if lit is not None:
        out.append(N.QeToken(N.TOK_LIT, 0, lit))
        return lit.type == N.TYPE_FLOAT64
    if isinstance(e, ArithmeticExpression):
        fl = _program(e.l, sm, out)
        fr = _program(e.r, sm, out)
        out.append(N.QeToken({N.OP_ADD: N.TOK_ADD, N.OP_SUB: N.TOK_SUB, N.OP_MUL: N.TOK_MUL,
                               N.OP_DIV: N.TOK_DIV}[e.op], 0, N.QeScalar()))
        return fl or fr
    raise _NotFusable(f"expression {e!r}")


def fuse(plan: PhysicalPlan) -> PhysicalPlan:
    """Rewrite HashAggregateExec over [ProjectionExec] over [SelectionExec] over ScanExec into a
    FusedHashAggregateExec when every expression is expressible in the fused kernel; otherwise
    return ``plan`` unchanged (the per-family operators then run)."""
    if isinstance(plan, (ProjectionExec, SelectionExec)):
        return _fuse_select_project(plan)
    if not isinstance(plan, HashAggregateExec):
        return plan
    try:
        node = plan.input
        proj = None
        if isinstance(node, ProjectionExec):
            proj = node.expr
            node = node.input
        pred = None
        if isinstance(node, SelectionExec):
            pred = node.expr
            node = node.input
        if not isinstance(node, ScanExec):
            raise _NotFusable("input is not a scan")
        sm = _SlotMap(node.schema())
        spec = N.QeFusedSpec()
        spec.mask_col = -1
        terms = _conjuncts(pred) if pred is not None else []
        if len(terms) > N.MAX_TERMS:
            raise _NotFusable("too many predicate terms")
        for i, t in enumerate(terms):
            if not isinstance(t, ComparisonExpression) or not isinstance(t.l, ColumnExpression):
                raise _NotFusable("predicate term")
            if sm.type_of(t.l.i) not in N.FIXED_WIDTH:
                raise _NotFusable("predicate on non fixed-width column")
            pt = spec.terms[i]
            pt.col = sm.slot(t.l.i)
            pt.op = t.op
            if isinstance(t.r, ColumnExpression):
                if sm.type_of(t.r.i) not in N.FIXED_WIDTH:
                    raise _NotFusable("predicate on non fixed-width column")
                pt.rhs_col = sm.slot(t.r.i)
            else:
                lit = _literal(t.r)
                if lit is None:
                    raise _NotFusable("predicate rhs")
                pt.rhs_col = -1
                pt.lit = lit
        spec.nterms = len(terms)
        key_types, key_scan = [], []
        for g in plan.groupExpr:
            g = _resolve(g, proj)
            if not isinstance(g, ColumnExpression):
                raise _NotFusable("group key must be a column")
            if sm.type_of(g.i) not in N.FIXED_WIDTH and sm.type_of(g.i) != N.TYPE_UTF8:
                raise _NotFusable("group key type")
            key_scan.append(g.i)
            key_types.append(sm.type_of(g.i))
        # UTF-8 keys / key sets wider than 63 bits: encoded to dictionary codes per batch, which
        # join the launch as extra slots (HashAggregateState.update_fused)
        ndict = dictionary_keys(key_types)
        if ndict is None:
            for k, i in enumerate(key_scan):
                spec.key_cols[k] = sm.slot(i)
        aggs = []
        for j, a in enumerate(plan.aggregateExpr):
            if a.fn == N.AGG_COUNT_STAR:
                aggs.append((a.fn, N.TYPE_INT64))
                continue
            toks: list = []
            is_f = _program(_resolve(a.inputExpression(), proj), sm, toks)
            if len(toks) > N.MAX_TOKENS:
                raise _NotFusable("expression too long")
            spec.inputs[j].ntokens = len(toks)
            for t, tok in enumerate(toks):
                spec.inputs[j].tokens[t] = tok
            aggs.append((a.fn, N.TYPE_FLOAT64 if is_f else N.TYPE_INT64))
        if ndict is not None and len(sm.slots) + ndict > N.MAX_COLS:
            raise _NotFusable("too many columns with the key codes")
        if not sm.slots and ndict is None:
            raise _NotFusable("no input columns")
        return FusedHashAggregateExec(node, sm.slots, spec, key_types, aggs, plan.schema(), plan.groupExpr,
                                      plan.aggregateExpr, plan.expected_groups,
                                      key_scan if ndict is not None else None)
    except _NotFusable:
        return plan


def _terms_into(pred: Optional[Expression], sm: "_SlotMap", terms, max_terms: int) -> int:
    conj = _conjuncts(pred) if pred is not None else []
    if len(conj) > max_terms:
        raise _NotFusable("too many predicate terms")
    for i, t in enumerate(conj):
        if not isinstance(t, ComparisonExpression) or not isinstance(t.l, ColumnExpression):
            raise _NotFusable("predicate term")
        if sm.type_of(t.l.i) not in N.FIXED_WIDTH:
            raise _NotFusable("predicate on non fixed-width column")
        pt = terms[i]
        pt.col = sm.slot(t.l.i)
        pt.op = t.op
        if isinstance(t.r, ColumnExpression):
            if sm.type_of(t.r.i) not in N.FIXED_WIDTH:
                raise _NotFusable("predicate on non fixed-width column")
            pt.rhs_col = sm.slot(t.r.i)
        else:
            lit = _literal(t.r)
            if lit is None:
                raise _NotFusable("predicate rhs")
            pt.rhs_col = -1
            pt.lit = lit
    return len(conj)


def _fuse_select_project(plan: PhysicalPlan) -> PhysicalPlan:
    """ProjectionExec(SelectionExec(ScanExec)), SelectionExec(ScanExec) or
    ProjectionExec(ScanExec) -> FusedSelectProjectExec; anything else unchanged."""
    try:
        node = plan
        proj = None
        if isinstance(node, ProjectionExec):
            proj = node.expr
            node = node.input
        pred = None
        if isinstance(node, SelectionExec):
            pred = node.expr
            node = node.input
        if not isinstance(node, ScanExec) or (proj is None and pred is None):
            raise _NotFusable("not a selection/projection over a scan")
        sm = _SlotMap(node.schema())
        spec = N.QeSelectSpec()
        spec.mask_col = -1
        spec.nterms = _terms_into(pred, sm, spec.terms, N.MAX_TERMS)
        exprs = proj if proj is not None else [ColumnExpression(i) for i in range(len(node.schema().fields))]
        if len(exprs) > N.MAX_AGGS:
            raise _NotFusable("too many outputs")
        out_types = []
        for k, e in enumerate(exprs):
            toks: list = []
            is_f = _program(e, sm, toks)
            if len(toks) > N.MAX_TOKENS:
                raise _NotFusable("expression too long")
            spec.outputs[k].ntokens = len(toks)
            for t, tok in enumerate(toks):
                spec.outputs[k].tokens[t] = tok
            if isinstance(e, ColumnExpression):
                if sm.type_of(e.i) == N.TYPE_BOOL:
                    raise _NotFusable("BOOL pass-through")
                out_types.append(sm.type_of(e.i))
            else:
                out_types.append(N.TYPE_FLOAT64 if is_f else N.TYPE_INT64)
        spec.nout = len(exprs)
        if not sm.slots:
            raise _NotFusable("no input columns")
        return FusedSelectProjectExec(node, sm.slots, spec, out_types, plan.schema(), plan)
    except _NotFusable:
        return plan


def aggregate_schema(input_schema: Schema, group_cols: Sequence[int], aggs: Sequence[AggregateExpression],
                     agg_input_types: Sequence[int]) -> Schema:
    """Output schema helper: group fields then one field per aggregate named by the function
    (the reference names every aggregate field after its function, Main.kt:91/:99)."""
    fields = [input_schema.fields[i] for i in group_cols]
    for a, t in zip(aggs, agg_input_types):
        fields.append(Field(a.name, output_type(a.fn, t)))
    return Schema(fields)
