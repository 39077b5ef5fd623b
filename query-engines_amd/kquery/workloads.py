"""Fused plans of the BASELINE.json configurations, as qe_fused_spec programs.

C4: SELECT k, SUM(a+b), COUNT(*), MIN(a), MAX(b) WHERE a > 2^19 GROUP BY k
C5: SELECT l_returnflag, l_linestatus, SUM(l_quantity), SUM(l_extendedprice),
           SUM(l_extendedprice * (1 - l_discount)), SUM(l_extendedprice * (1 - l_discount) * (1 + l_tax)),
           AVG(l_extendedprice), COUNT(*)
    WHERE l_shipdate <= 2400 AND l_discount >= 0.05 AND l_discount <= 0.07 AND l_quantity < 24
    GROUP BY l_returnflag, l_linestatus                      (TPC-H Q1-like, three predicates)
"""
from __future__ import annotations

from . import native as N


def _tok(op, arg=0, lit=None):
    return N.QeToken(op, arg, N.scalar(lit) if lit is not None else N.QeScalar())


def _prog(spec, j, toks):
    p = spec.inputs[j]
    p.ntokens = len(toks)
    for i, t in enumerate(toks):
        p.tokens[i] = t


def c4_spec(threshold: int = 1 << 19) -> N.QeFusedSpec:
    """Slots: 0 k, 1 a, 2 b."""
    spec = N.QeFusedSpec()
    spec.mask_col = -1
    spec.nterms = 1
    spec.terms[0] = N.QePredTerm(1, N.OP_GT, -1, 0, N.scalar(threshold))
    spec.key_cols[0] = 0
    _prog(spec, 0, [_tok(N.TOK_COL, 1), _tok(N.TOK_COL, 2), _tok(N.TOK_ADD)])
    _prog(spec, 2, [_tok(N.TOK_COL, 1)])
    _prog(spec, 3, [_tok(N.TOK_COL, 2)])
    return spec


C4_AGGS = [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_COUNT_STAR, N.TYPE_INT64), (N.AGG_MIN, N.TYPE_INT64),
           (N.AGG_MAX, N.TYPE_INT64)]

C5_AGGS = [(N.AGG_SUM, N.TYPE_INT64), (N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_SUM, N.TYPE_FLOAT64),
           (N.AGG_SUM, N.TYPE_FLOAT64), (N.AGG_AVG, N.TYPE_FLOAT64), (N.AGG_COUNT_STAR, N.TYPE_INT64)]
C5_KEY_TYPES = [N.TYPE_UINT8, N.TYPE_UINT8]


def c5_spec(shipdate_max: int = 2400) -> N.QeFusedSpec:
    """Slots = C5_COLUMNS order: 0 quantity, 1 extendedprice, 2 discount, 3 tax, 4 returnflag,
    5 linestatus, 6 shipdate."""
    spec = N.QeFusedSpec()
    spec.mask_col = -1
    spec.nterms = 4
    spec.terms[0] = N.QePredTerm(6, N.OP_LE, -1, 0, N.scalar(shipdate_max))
    spec.terms[1] = N.QePredTerm(2, N.OP_GE, -1, 0, N.scalar(0.05))
    spec.terms[2] = N.QePredTerm(2, N.OP_LE, -1, 0, N.scalar(0.07))
    spec.terms[3] = N.QePredTerm(0, N.OP_LT, -1, 0, N.scalar(24))
    spec.key_cols[0] = 4
    spec.key_cols[1] = 5
    disc_price = [_tok(N.TOK_COL, 1), _tok(N.TOK_LIT, lit=1.0), _tok(N.TOK_COL, 2), _tok(N.TOK_SUB), _tok(N.TOK_MUL)]
    _prog(spec, 0, [_tok(N.TOK_COL, 0)])
    _prog(spec, 1, [_tok(N.TOK_COL, 1)])
    _prog(spec, 2, disc_price)
    _prog(spec, 3, disc_price + [_tok(N.TOK_LIT, lit=1.0), _tok(N.TOK_COL, 3), _tok(N.TOK_ADD), _tok(N.TOK_MUL)])
    _prog(spec, 4, [_tok(N.TOK_COL, 1)])
    return spec
