#!/usr/bin/env python3
"""Experiment: C2 select-project kernel vs the stream-read ceiling at the same size (10M rows,
2 int64 columns). Run under rocprofv3 --kernel-trace --stats and compare qe_selproj with
k_stream_read (results of the variants tried are noted in qe_jit.hip and DESIGN.md)."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "query-engines_amd")]

from kquery import native as N  # noqa: E402
from kquery.columnar import Context, DeviceColumn  # noqa: E402
from kquery.datasource import C2_COLUMNS, generate_column  # noqa: E402


def main():
    ctx = Context.get(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    cols = [generate_column(s, n, 0, 42, ctx) for s in C2_COLUMNS]
    cc = (N.QeColumn * 2)(*[c.as_c() for c in cols])
    ms = N.C.c_double()
    for _ in range(20):
        N.check(N.lib().qe_stream_read(ctx.handle, cc, 2, N.C.byref(ms)))
    print("stream_read ms", ms.value, "GB/s", n * 16 / ms.value / 1e6)
    spec = N.QeSelectSpec()
    spec.mask_col = -1
    spec.nterms = 1
    spec.terms[0].col, spec.terms[0].op, spec.terms[0].rhs_col = 0, N.OP_GT, -1
    spec.terms[0].lit = N.scalar(1 << 19)
    spec.nout = 1
    spec.outputs[0].ntokens = 3
    spec.outputs[0].tokens[0] = N.QeToken(N.TOK_COL, 0, N.QeScalar())
    spec.outputs[0].tokens[1] = N.QeToken(N.TOK_COL, 1, N.QeScalar())
    spec.outputs[0].tokens[2] = N.QeToken(N.TOK_ADD, 0, N.QeScalar())
    out = DeviceColumn.empty(N.TYPE_INT64, n, False, ctx=ctx)
    oc = (N.QeColumn * 1)(out.as_c())
    cnt = N.C.c_int64()
    for _ in range(30):
        oc[0].length = n
        N.check(N.lib().qe_select_project(ctx.handle, cc, 2, N.C.byref(spec), oc, N.C.byref(cnt)))
    print("selected", cnt.value)


if __name__ == "__main__":
    main()
