"""Sanitizers (SURVEY §5 "Race detection / sanitizers"): host code under AddressSanitizer +
UndefinedBehaviorSanitizer, on the CPU.

* the device CAST parser (query-engines_amd/csrc/qe_cast_parse.hpp, shared by k_cast_utf8_f64
  and k_cast_slow) built for the host with -fsanitize=address,undefined: every input is an
  exact-size heap copy, so a read past a string's end is a report; the results must equal the
  oracle (Double.parseDouble) bit for bit;
* the oracle's C restatement (oracle/cpu_baseline.c, the bench's CPU baseline) multi-threaded
  under the same sanitizers, checked against the Python oracle;
* the JNI shim (query-engines_amd/jni/qe_jni.c) driven through its argument-checking and
  exception paths by tests/native/jni_harness.c (test-double JNIEnv; leak detection off: the
  harness keeps its fake Java objects for the process lifetime, as a JVM's GC would own them).

A sanitizer report makes the driver exit non-zero (-fno-sanitize-recover for UBSan), which fails
the test. GPU code is not sanitized (no GPU ASan on this pool); the device paths get the
run-to-run determinism check in test_determinism.py instead."""
import fcntl
import os
import pathlib
import random
import struct
import subprocess

import pytest

from oracle import cast_ref as R
from oracle import gen
from oracle import semantics as S

NATIVE = pathlib.Path(__file__).resolve().parent / "native"
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")


@pytest.fixture(scope="module")
def drivers():
    # one build at a time: under pytest-xdist another worker may be running the binaries that a
    # concurrent make would relink ("Text file busy")
    (NATIVE / "_build").mkdir(exist_ok=True)
    with open(NATIVE / "_build" / ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", str(NATIVE), "san"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-400:])
    return NATIVE / "_build" / "san_cast", NATIVE / "_build" / "san_oracle"


def _run(cmd, stdin=None):
    r = subprocess.run([str(c) for c in cmd], input=stdin, capture_output=True, text=True, env=ENV, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    return r.stdout


def _cast_inputs():
    from test_cast import KAT, corpus

    strings = corpus(seed=11, n_random=1500) + [e["in"] for e in KAT]
    rng = random.Random(5)
    # malformed and edge inputs: truncations of valid numbers, stray bytes, huge exponents
    for s in list(strings[:600]):
        cut = rng.randrange(len(s) + 1)
        strings.append(s[:cut])
        strings.append(s[:cut] + rng.choice(["x", "e", ".", "+", "-", "p", "0x", " ", "e+", "E-9999999999"]))
    strings += ["", " ", ".", "e5", "-", "+.e1", "0x", "0x.p1", "0x1p", "1e" + "9" * 40, "1e-" + "9" * 40,
                "0." + "0" * 400 + "1", "9" * 800, "NaN", "-Infinity", "Infinityx", "0x1.fffffffffffff8p1023"]
    return [s for s in strings if "\n" not in s and "\r" not in s and "\x00" not in s]


def _java(s):
    try:
        return R.parse_java_double(s)
    except R.NumberFormatException:
        return None


def test_cast_parser_asan_ubsan(drivers):
    san_cast, _ = drivers
    strings = _cast_inputs()
    out = _run([san_cast], "\n".join(strings) + "\n").splitlines()
    assert len(out) == len(strings)
    bad = []
    for s, got in zip(strings, out):
        want = _java(s)
        g = None if got == "NFE" else struct.unpack("<d", int(got, 16).to_bytes(8, "little"))[0]
        if (g is None) != (want is None) or (g is not None and not R.same_f64(g, want)):
            bad.append((s[:60], got, want))
    assert not bad, (len(bad), bad[:10])


@pytest.mark.parametrize("threads,row0,rows", [(1, 0, 20_000), (4, 987_654, 50_001)])
def test_cpu_baseline_asan_ubsan(drivers, threads, row0, rows):
    _, san_oracle = drivers
    out = _run([san_oracle, row0, rows, threads])
    got = {}
    for line in out.splitlines():
        k, s, c, mn, mx = map(int, line.split())
        got[(k,)] = [s, c, mn, mx]
    k, _ = gen.generate(gen.GEN_MOD, 1024, 42, 0, row0, rows)
    a, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 1, row0, rows)
    b, _ = gen.generate(gen.GEN_MOD, 1 << 20, 42, 2, row0, rows)
    want = S.group_aggregate([k], [None], [S.arith(S.OP_ADD, a, None, b, None)[0], None, a, b], [None] * 4,
                             [S.AGG_SUM, S.AGG_COUNT_STAR, S.AGG_MIN, S.AGG_MAX], a > (1 << 19))
    assert got == want


def test_jni_shim_host_paths_under_asan_ubsan():
    (NATIVE / "_build").mkdir(exist_ok=True)
    with open(NATIVE / "_build" / ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", str(NATIVE), "_build/san_jni_harness"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-400:])
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23")
    p = subprocess.run([str(NATIVE / "_build" / "san_jni_harness"), "cpu"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert p.returncode == 0 and "ALL OK" in p.stdout, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
