"""Generated kernel sources compile for gfx950 (CPU suite, no GPU): the select-project generator's
every tile-order mode (qe_jit.hip gen_selproj_source) for a C2 plan
and a nullable two-output plan, and the two-bucket GROUP BY kernels (fused pass, spilling pass,
record aggregation, and the radix-partitioned scatters and aggregation passes with 32-bit records) for the C4 plan, a nullable fp64 MAX plan and a deterministic (fixed-point) fp64 SUM/AVG plan (single-pass: through the per-wave fx queue), emitted by tests/native/gen_sources.cpp through the library's own
plan compiler and compiled with hipcc as hipRTC would (same options, device code only)."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def sources(tmp_path_factory):
    if not pathlib.Path(HIPCC).exists():
        pytest.skip("hipcc not present")
    if not (ROOT / "query-engines_amd" / "lib" / "libqe_hip.so").exists():
        pytest.skip("libqe_hip.so not built")
    out = tmp_path_factory.mktemp("jitsrc")  # per xdist worker: no shared build output
    csrc, lib = ROOT / "query-engines_amd" / "csrc", ROOT / "query-engines_amd" / "lib"
    exe = out / "gen_sources"
    subprocess.run([HIPCC, "-O1", "-std=c++17", f"-I{csrc}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "native" / "gen_sources.cpp"), f"-L{lib}", "-lqe_hip",
                    f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True, capture_output=True)
    r = subprocess.run([str(exe), str(out)], check=True, capture_output=True, text=True)
    return [pathlib.Path(p) for p in r.stdout.split()]


def test_all_modes_emitted(sources):
    names = sorted(p.name for p in sources)
    assert names == sorted([f"{s}_m{m}.hip" for s in ("c2", "nullable") for m in range(5)] + ["c2_m5.hip", "c2_m6.hip"] +
                           [f"{s}_{k}.hip" for s in ("c4", "f64max", "det")
                            for k in ("fused", "spill", "pagg", "pscatter", "pscatter_soa", "pagg_rows",
                                      "pscatter_n32", "pdirect_n32", "pagg_n32", "pagg_unchunked_n32", "spill_n32",
                                      "pagg_soa_n32", "pagg_big_n32", "fused1")] + ["c4_fused_compact.hip", "c4_spill_compact.hip", "c4_spill_compact_sb4.hip",
                                                                             "c5_fused1.hip"])


@pytest.mark.parametrize("name", ["c2_m0", "c2_m1", "c2_m2", "c2_m3", "c2_m4", "c2_m5", "c2_m6", "nullable_m1", "nullable_m3",
                                  "nullable_m4", "c4_fused", "c4_spill", "c4_pagg", "f64max_spill",
                                  "f64max_pagg", "det_fused", "det_spill", "det_pagg", "c4_pscatter",
                                  "c4_pscatter_soa", "c4_pagg_rows", "det_pscatter_soa", "f64max_pscatter_soa",
                                  "c4_pscatter_n32", "c4_pdirect_n32", "c4_pagg_n32", "c4_pagg_unchunked_n32",
                                  "f64max_pagg_n32", "c4_spill_n32", "c4_pagg_soa_n32", "c4_fused_compact",
                                  "c4_pagg_big_n32", "c4_spill_compact", "c4_spill_compact_sb4", "c4_fused1", "det_fused1", "c5_fused1"])
def test_compiles_for_gfx950(sources, name, tmp_path):
    if name in ("det_fused1", "c5_fused1"):  # exact fp64 SUMs of a single-pass plan go through the per-wave queue
        assert "q_slot" in next(p for p in sources if p.stem == name).read_text()
    src = next(p for p in sources if p.stem == name)
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-munsafe-fp-atomics", "--cuda-device-only", "-include", "hip/hip_runtime.h", "-c",
                        str(src), "-o", str(tmp_path / (name + ".o"))], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
