"""ORACLE (test infrastructure only — never imported by the product path).

CPU restatement of CastExpression UTF-8 -> double (folkol/query-engines kquerydiy/src/Main.kt,
K:772-805). The reference converts each non-null String with Kotlin ``String.toDouble()``
(K:791), which is ``java.lang.Double.parseDouble``: a JDK library routine, not in
/root/reference. Its behaviour is restated from its published specification:

* grammar: the regular expression the ``java.lang.Double.valueOf(String)`` javadoc gives as the
  exact set of accepted strings (JDK 8-21 unchanged), transcribed below as ``_JAVA_FP``;
  leading/trailing characters <= U+0020 are ignored (``String.trim``);
* value: "rounded to type double by the usual round-to-nearest rule of IEEE 754" — the exact
  decimal or hexadecimal value rounded half-even. Python's ``float()`` (decimal) and
  ``float.fromhex()`` (hex) are correctly rounded the same way, so once the Java grammar has
  accepted a string they give Java's result;
* null in -> null out (K:787-788); an unaccepted string raises NumberFormatException.

Parity: pinned to the JDK specification (no JVM exists in this container — SURVEY §8c), with a
known-answer table in tests/golden/cast_kat.json whose entries are the JDK-documented results.
"""
from __future__ import annotations

import math
import re
from typing import List, Optional, Sequence, Tuple

import numpy as np

_DIGITS = r"(\d+)"  # Java \p{Digit} = ASCII [0-9] (no UNICODE_CHARACTER_CLASS)
_HEX = r"([0-9a-fA-F]+)"
_EXP = r"[eE][+-]?" + _DIGITS
_JAVA_FP = re.compile(
    r"[+-]?("
    r"NaN|"
    r"Infinity|"
    r"((("
    + _DIGITS + r"(\.)?(" + _DIGITS + r"?)(" + _EXP + r")?)|"
    r"(\.(" + _DIGITS + r")(" + _EXP + r")?)|"
    r"(("
    r"(0[xX]" + _HEX + r"(\.)?)|"
    r"(0[xX]" + _HEX + r"?(\.)" + _HEX + r")"
    r")[pP][+-]?" + _DIGITS + r"))"
    r"[fFdD]?))",
    re.ASCII,
)
_TRIM = "".join(chr(c) for c in range(0x21))


class NumberFormatException(ValueError):
    pass


def parse_java_double(s: str) -> float:
    """java.lang.Double.parseDouble(s) (via K:791 String.toDouble)."""
    t = s.strip(_TRIM)
    if not _JAVA_FP.fullmatch(t):
        raise NumberFormatException(f'For input string: "{s}"')
    neg = t.startswith("-")
    body = t[1:] if t[:1] in "+-" else t
    if body == "NaN":
        return math.nan
    if body == "Infinity":
        return -math.inf if neg else math.inf
    if body[-1] in "fFdD":
        body = body[:-1]
    if body[:2] in ("0x", "0X"):
        try:
            v = float.fromhex(body)
        except OverflowError:  # rounds beyond Double.MAX_VALUE: Java returns Infinity
            v = math.inf
    else:
        v = float(body)
    return -v if neg else v


def cast_utf8_to_f64(strings: Sequence[Optional[str]]) -> Tuple[np.ndarray, np.ndarray]:
    """CastExpression.evaluate for a Utf8 column (K:778-804): (values, valid). Raises
    NumberFormatException naming the first offending row (the reference throws on it)."""
    n = len(strings)
    vals = np.zeros(n, dtype=np.float64)
    valid = np.zeros(n, dtype=bool)
    for i, s in enumerate(strings):
        if s is None:
            continue
        try:
            vals[i] = parse_java_double(s)
        except NumberFormatException as e:
            raise NumberFormatException(f"{e} (row {i})") from None
        valid[i] = True
    return vals, valid


def f64_bits(x: float) -> int:
    return int(np.array([x], dtype=np.float64).view(np.int64)[0])


def same_f64(a: float, b: float) -> bool:
    """Bit-exact equality, any NaN equal to any NaN (Java's parseDouble NaN is canonical)."""
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return f64_bits(a) == f64_bits(b)


def bad_rows(strings: Sequence[Optional[str]]) -> List[int]:
    out = []
    for i, s in enumerate(strings):
        if s is None:
            continue
        try:
            parse_java_double(s)
        except NumberFormatException:
            out.append(i)
    return out
