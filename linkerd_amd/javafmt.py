"""Java number formatting used by the exporters: Long.toString, Float.toString,
Double.toString (JLS / java.lang.Double#toString rules: plain notation for
1e-3 <= |x| < 1e7 with at least one fractional digit, otherwise d.dddE<n>).
Digits are the shortest round-trip digits (what JDK 19+ prints; JDK 8's
FloatingDecimal prints one extra digit in rare cases -- unpinned here)."""
from __future__ import annotations

import math

import numpy as np


def _format(sign: str, digits: str, e10: int, plain: bool) -> str:
    if plain:
        if e10 >= 0:
            ip = digits[: e10 + 1].ljust(e10 + 1, "0")
            fp = digits[e10 + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e10 - 1) + digits
        return f"{sign}{ip}.{fp}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{e10}"


def _java_str(x: float, sci: str) -> str:
    mant, exp = sci.split("e")
    sign = ""
    if mant.startswith("-"):
        sign, mant = "-", mant[1:]
    digits = mant.replace(".", "").rstrip("0") or "0"
    e10 = int(exp)
    ax = abs(x)
    return _format(sign, digits, e10, 1e-3 <= ax < 1e7)


def double_to_string(x: float) -> str:
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    return _java_str(x, np.format_float_scientific(np.float64(x), unique=True, trim="0"))


def float_to_string(x: float) -> str:
    f = np.float32(x)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if math.copysign(1.0, float(f)) < 0 else "0.0"
    return _java_str(float(f), np.format_float_scientific(f, unique=True, trim="0"))


def long_to_string(x: int) -> str:
    return str(int(x))
