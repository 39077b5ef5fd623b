"""CPU tests of the drop-in boundary: libqe_hip.so loads, exports every entry point that
include/qe_hip.h declares, and the ctypes mirror matches the header's struct layouts.
No compute calls (no GPU here)."""
import ctypes as C
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "qe_hip.h"


def _declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qe_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from kquery import native as N

    lib = N.load_library()
    names = _declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    bound = {s[0] for s in N.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_abi_version_and_error_string():
    from kquery import native as N

    lib = N.load_library()
    assert lib.qe_abi_version() == 1
    assert isinstance(lib.qe_last_error(), bytes)


def test_struct_layouts_match_header():
    """Compile a tiny C program against the header and compare sizeof/offsetof with ctypes."""
    import subprocess
    import tempfile

    from kquery import native as N

    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "qe_hip.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(qe_column), sizeof(qe_scalar), sizeof(qe_operand),
   sizeof(qe_global_agg), sizeof(qe_agg_desc), sizeof(qe_pred_term), sizeof(qe_token), sizeof(qe_agg_program),
   sizeof(qe_fused_spec));
 printf("%zu %zu %zu %zu\n", offsetof(qe_fused_spec, terms), offsetof(qe_fused_spec, key_cols),
   offsetof(qe_fused_spec, inputs), offsetof(qe_global_agg, avg));
 printf("%zu %zu\n", sizeof(qe_select_spec), offsetof(qe_select_spec, outputs));
 printf("%zu %zu %zu %zu %zu\n", sizeof(struct ArrowSchema), sizeof(struct ArrowArray),
   sizeof(struct ArrowDeviceArray), offsetof(struct ArrowDeviceArray, device_type),
   offsetof(struct ArrowDeviceArray, sync_event));
 return 0; }
"""
    with tempfile.TemporaryDirectory() as d:
        c = pathlib.Path(d) / "t.c"
        c.write_text(src)
        exe = pathlib.Path(d) / "t"
        subprocess.run(["gcc", "-I", str(ROOT / "include"), str(c), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    sizes = [int(x) for x in out[0].split()]
    offs = [int(x) for x in out[1].split()]
    assert sizes == [C.sizeof(t) for t in (N.QeColumn, N.QeScalar, N.QeOperand, N.QeGlobalAgg, N.QeAggDesc,
                                           N.QePredTerm, N.QeToken, N.QeAggProgram, N.QeFusedSpec)]
    assert offs == [N.QeFusedSpec.terms.offset, N.QeFusedSpec.key_cols.offset, N.QeFusedSpec.inputs.offset,
                    N.QeGlobalAgg.avg.offset]
    from kquery import arrow_io as A

    sel = [int(x) for x in out[2].split()]
    assert sel == [C.sizeof(N.QeSelectSpec), N.QeSelectSpec.outputs.offset]
    arrow = [int(x) for x in out[3].split()]
    assert arrow == [C.sizeof(A.ArrowSchemaC), C.sizeof(A.ArrowArrayC), C.sizeof(A.ArrowDeviceArrayC),
                     A.ArrowDeviceArrayC.device_type.offset, A.ArrowDeviceArrayC.sync_event.offset]
    assert arrow[:3] == [72, 80, 128]  # the Arrow C (device) data interface ABI


def test_missing_library_fails_loudly(tmp_path):
    from kquery import native as N

    with pytest.raises(ImportError):
        N.load_library(tmp_path / "nope.so")


def test_product_path_never_imports_oracle():
    """The product package must not reference the oracle (no CPU fallback)."""
    pkg = ROOT / "query-engines_amd"
    for p in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.hpp")):
        assert "oracle" not in p.read_text().replace("oracle/", "").lower() or "import oracle" not in p.read_text(), p
        assert "from oracle" not in p.read_text() and "import oracle" not in p.read_text(), p
