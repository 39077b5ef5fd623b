"""Physical expressions: ``Expression.evaluate(RecordBatch): ColumnVector`` (Main.kt:448-450).

* ``ColumnExpression`` (Main.kt:452-460) is a zero-copy column reference, as in the reference.
* Literal / arithmetic / comparison / boolean expressions do not exist in the reference
  (absence evidenced by Main.kt:662-678 and :807-816); they are build-defined here
  with the semantics listed in include/qe_hip.h and evaluated by the HIP kernel families
  K1/K2/K3a through the C ABI. There is no CPU path.
* Aggregate expressions follow ``AggregateExpression`` (Main.kt:514-517): ``inputExpression()``
  plus the aggregate function; ``MaxExpression`` is the reference's (Main.kt:524-536), the
  others are build-defined siblings with the same null/order rules.
"""
from __future__ import annotations

from typing import Optional, Union

import numpy as np

from . import native as N
from .columnar import ColumnVector, DeviceColumn, RecordBatch


class ScalarColumn(ColumnVector):
    """A literal broadcast to ``n`` rows (never materialised; passed to kernels as qe_scalar)."""

    def __init__(self, value, n: int, type_id: int):
        self.value = value
        self.n = n
        self.type = type_id

    def getValue(self, i: int):  # noqa: N802
        return self.value

    def size(self) -> int:
        return self.n

    def as_scalar(self) -> N.QeScalar:
        return N.scalar(self.value, self.type)


class Expression:
    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002 (reference name)
        raise NotImplementedError


class ColumnExpression(Expression):
    """Main.kt:452-460."""

    def __init__(self, i: int):
        self.i = i

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        return input.field(self.i)

    def __repr__(self) -> str:
        return f"#{self.i}"


class LiteralLongExpression(Expression):
    def __init__(self, value: int):
        self.value = int(value)

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        return ScalarColumn(self.value, input.rowCount(), N.TYPE_INT64)

    def __repr__(self) -> str:
        return str(self.value)


class LiteralDoubleExpression(Expression):
    def __init__(self, value: float):
        self.value = float(value)

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        return ScalarColumn(self.value, input.rowCount(), N.TYPE_FLOAT64)

    def __repr__(self) -> str:
        return repr(self.value)


class LiteralStringExpression(Expression):
    def __init__(self, value: str):
        self.value = value

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        ctx = _ctx_of(input)
        return DeviceColumn.from_strings([self.value], ctx=ctx)

    def __repr__(self) -> str:
        return f"'{self.value}'"


def _ctx_of(batch: RecordBatch):
    for f in batch.fields:
        if isinstance(f, DeviceColumn):
            return f.ctx
    from .columnar import Context

    return Context.get(0)


def _operand(cv: ColumnVector, keep: list, pending_ok: bool = False) -> N.QeOperand:
    if isinstance(cv, ScalarColumn):
        return N.QeOperand(None, cv.as_scalar())
    if isinstance(cv, DeviceColumn):
        c = cv.as_c(pending_ok)
        keep.append(c)
        return N.QeOperand(N.C.pointer(c), N.QeScalar())
    raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"operand {type(cv).__name__} is not device-resident")


def _is_f64(cv: ColumnVector) -> bool:
    return getattr(cv, "type", None) == N.TYPE_FLOAT64


def _nullable(cv: ColumnVector) -> bool:
    if isinstance(cv, ScalarColumn):
        return cv.value is None
    return cv.validity is not None


def _pending(*cvs):
    """The one DeviceCount the device columns among cvs share, or None (then every length is
    resolved first: columns of different selections never mix unresolved)."""
    cols = [cv for cv in cvs if isinstance(cv, DeviceColumn)]
    ps = {id(c.pending): c.pending for c in cols}
    if len(ps) == 1 and None not in ps.values():
        return next(iter(ps.values()))
    for c in cols:
        _ = c.length
    return None


def _ref_column(*cvs) -> DeviceColumn:
    for cv in cvs:
        if isinstance(cv, DeviceColumn):
            return cv
    raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "at least one operand must be a column")


class BinaryExpression(Expression):
    op: int = 0
    symbol: str = "?"

    def __init__(self, l: Expression, r: Expression):  # noqa: E741
        self.l = l
        self.r = r

    def __repr__(self) -> str:
        return f"({self.l} {self.symbol} {self.r})"


class ArithmeticExpression(BinaryExpression):
    """K1: int64 + - * wrap, / truncates (x/0 -> null); fp64 promotion (IEEE)."""

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        lv, rv = self.l.evaluate(input), self.r.evaluate(input)
        ref = _ref_column(lv, rv)
        out_t = N.TYPE_FLOAT64 if (_is_f64(lv) or _is_f64(rv)) else N.TYPE_INT64
        nullable = _nullable(lv) or _nullable(rv) or (out_t == N.TYPE_INT64 and self.op == N.OP_DIV)
        pend = _pending(lv, rv)
        keep: list = []
        if pend is not None:  # rows of a stream-ordered selection: compute below its device count
            out = DeviceColumn.empty(out_t, ref.capacity, nullable, ctx=ref.ctx)
            a, b = _operand(lv, keep, True), _operand(rv, keep, True)
            oc = out.as_c()
            N.check(N.lib().qe_eval_arith_dlen(ref.ctx.handle, self.op, N.C.byref(a), N.C.byref(b), N.C.byref(oc),
                                               pend.ptr()))
            out.pending = pend
            return out
        out = DeviceColumn.empty(out_t, ref.length, nullable, ctx=ref.ctx)
        a, b = _operand(lv, keep), _operand(rv, keep)
        oc = out.as_c()
        N.check(N.lib().qe_eval_arith(ref.ctx.handle, self.op, N.C.byref(a), N.C.byref(b), N.C.byref(oc)))
        return out


class AddExpression(ArithmeticExpression):
    op, symbol = N.OP_ADD, "+"


class SubtractExpression(ArithmeticExpression):
    op, symbol = N.OP_SUB, "-"


class MultiplyExpression(ArithmeticExpression):
    op, symbol = N.OP_MUL, "*"


class DivideExpression(ArithmeticExpression):
    op, symbol = N.OP_DIV, "/"


class ComparisonExpression(BinaryExpression):
    """K2: signed int64 / IEEE fp64 (NaN: only != is true) / UTF8 byte equality -> BOOL."""

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        lv, rv = self.l.evaluate(input), self.r.evaluate(input)
        ref = _ref_column(lv, rv)
        nullable = _nullable(lv) or _nullable(rv)
        out = DeviceColumn.empty(N.TYPE_BOOL, ref.length, nullable, ctx=ref.ctx)
        keep: list = []
        a, b = _operand(lv, keep), _operand(rv, keep)
        oc = out.as_c()
        N.check(N.lib().qe_eval_cmp(ref.ctx.handle, self.op, N.C.byref(a), N.C.byref(b), N.C.byref(oc)))
        return out


class EqExpression(ComparisonExpression):
    op, symbol = N.OP_EQ, "="


class NeqExpression(ComparisonExpression):
    op, symbol = N.OP_NE, "!="


class LtExpression(ComparisonExpression):
    op, symbol = N.OP_LT, "<"


class LtEqExpression(ComparisonExpression):
    op, symbol = N.OP_LE, "<="


class GtExpression(ComparisonExpression):
    op, symbol = N.OP_GT, ">"


class GtEqExpression(ComparisonExpression):
    op, symbol = N.OP_GE, ">="


class BooleanExpression(BinaryExpression):
    """K3a: SQL three-valued AND / OR on BOOL columns."""

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        lv, rv = self.l.evaluate(input), self.r.evaluate(input)
        if not (isinstance(lv, DeviceColumn) and isinstance(rv, DeviceColumn)):
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "boolean operands must be BOOL columns")
        out = DeviceColumn.empty(N.TYPE_BOOL, lv.length, lv.nullable or rv.nullable, ctx=lv.ctx)
        a, b, oc = lv.as_c(), rv.as_c(), out.as_c()
        N.check(N.lib().qe_eval_bool(lv.ctx.handle, self.op, N.C.byref(a), N.C.byref(b), N.C.byref(oc)))
        return out


class AndExpression(BooleanExpression):
    op, symbol = N.OP_AND, "AND"


class OrExpression(BooleanExpression):
    op, symbol = N.OP_OR, "OR"


class UnaryBooleanExpression(Expression):
    op: int = 0
    name: str = "?"

    def __init__(self, expr: Expression):
        self.expr = expr

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        v = self.expr.evaluate(input)
        if not isinstance(v, DeviceColumn):
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, "operand must be a column")
        nullable = self.op == N.OP_NOT and v.nullable
        out = DeviceColumn.empty(N.TYPE_BOOL, v.length, nullable, ctx=v.ctx)
        a, oc = v.as_c(), out.as_c()
        N.check(N.lib().qe_eval_bool(v.ctx.handle, self.op, N.C.byref(a), None, N.C.byref(oc)))
        return out

    def __repr__(self) -> str:
        return f"{self.name}({self.expr})"


class NotExpression(UnaryBooleanExpression):
    op, name = N.OP_NOT, "NOT"


class IsNullExpression(UnaryBooleanExpression):
    op, name = N.OP_IS_NULL, "IS_NULL"


class IsNotNullExpression(UnaryBooleanExpression):
    op, name = N.OP_IS_NOT_NULL, "IS_NOT_NULL"


class CastExpression(Expression):
    """Main.kt:772-805. Only String values cast (K:791 ``vv.toDouble()``, i.e.
    java.lang.Double.parseDouble): a UTF8 column runs qe_cast_utf8_to_f64 on the device. Any other
    input type throws on its first non-null value, as the reference does (K:792); an all-null
    column casts to all-null. Targets other than double throw (K:799)."""

    def __init__(self, expr: Expression, dataType: int):  # noqa: N803
        self.expr = expr
        self.dataType = dataType

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        v = self.expr.evaluate(input)
        if self.dataType != N.TYPE_FLOAT64:
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"Cast to {self.dataType} is not supported")
        n = v.size()
        if isinstance(v, DeviceColumn) and v.type == N.TYPE_UTF8:
            out = DeviceColumn.empty(N.TYPE_FLOAT64, n, v.nullable, ctx=v.ctx)
            oc, ic = out.as_c(), v.as_c()
            row = N.C.c_int64(-1)
            st = N.lib().qe_cast_utf8_to_f64(v.ctx.handle, N.C.byref(ic), N.C.byref(oc), N.C.byref(row))
            if st == N.QE_ERR_INVALID_ARG and row.value >= 0:
                raise N.NumberFormatException(st, N.lib().qe_last_error().decode(errors="replace"))
            N.check(st)
            return out
        # K:790-792: the first non-null non-String value throws; nulls stay null
        first = (int(np.argmax(v.valid_mask())) if v.valid_mask().any() else -1) if isinstance(v, DeviceColumn) \
            else next((i for i in range(n) if v.getValue(i) is not None), -1)
        if first >= 0:
            raise N.IllegalStateException(N.QE_ERR_UNSUPPORTED, f"Cannot cast value to Double: {v.getValue(first)}")
        ctx = v.ctx if isinstance(v, DeviceColumn) else None
        return DeviceColumn.empty(N.TYPE_FLOAT64, n, True, ctx=ctx)

    def __repr__(self) -> str:
        return f"CAST({self.expr} AS {self.dataType})"


class _Given(Expression):
    def __init__(self, cv: ColumnVector):
        self.cv = cv

    def evaluate(self, input: RecordBatch) -> ColumnVector:  # noqa: A002
        return self.cv


# ---- aggregate expressions (Main.kt:514-536) -----------------------------------------------------
class AggregateExpression:
    fn: int = 0
    name: str = "?"

    def __init__(self, expr: Optional[Expression]):
        self.expr = expr

    def inputExpression(self) -> Optional[Expression]:  # noqa: N802
        return self.expr

    def __repr__(self) -> str:
        return f"{self.name}({self.expr if self.expr is not None else '*'})"


class MaxExpression(AggregateExpression):
    """Main.kt:524-536 / MaxAccumulator :538-561."""

    fn, name = N.AGG_MAX, "MAX"


class MinExpression(AggregateExpression):
    fn, name = N.AGG_MIN, "MIN"


class SumExpression(AggregateExpression):
    fn, name = N.AGG_SUM, "SUM"


class CountExpression(AggregateExpression):
    fn, name = N.AGG_COUNT, "COUNT"


class CountStarExpression(AggregateExpression):
    fn, name = N.AGG_COUNT_STAR, "COUNT"

    def __init__(self):
        super().__init__(None)


class AvgExpression(AggregateExpression):
    fn, name = N.AGG_AVG, "AVG"


Operand = Union[DeviceColumn, ScalarColumn]
