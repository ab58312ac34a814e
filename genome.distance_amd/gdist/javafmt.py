"""Java text emission for the hot-path writers.

Double.toString (JDK 19+ algorithm; the reference targets JDK 21, pom.xml:17)
is what `"..." + distance` and TextStringBuilder.append(double) print at
FastaDistanceProcessor.java:189-190, GenomeProcessor.java:144,
DistanceRepsProcessor.java:250-251: the shortest decimal that rounds to the
double (the closest such; a one-digit result is widened to the closest
two-digit decimal), laid out plain for 1e-3 <= |d| < 1e7 and as d.dddE±n
otherwise.
"""
from __future__ import annotations

import math

import numpy as np


def _shortest(d: float) -> tuple[str, int]:
    """Significant digits and decimal exponent (d = D.DDD × 10^e)."""
    r = repr(abs(d))
    mant, e = r, 0
    if "e" in r:
        mant, ex = r.split("e")
        e = int(ex)
    ip, _, fp = mant.partition(".")
    digits = ip + fp
    e += len(ip) - 1
    stripped = digits.lstrip("0")
    e -= len(digits) - len(stripped)
    digits = stripped.rstrip("0") or "0"
    if len(digits) == 1:  # widen to the closest two-digit decimal
        m2, _, ex2 = ("%.1e" % abs(d)).partition("e")
        digits = m2.replace(".", "").rstrip("0") or "0"
        e = int(ex2)
    return digits, e


def java_double(d: float) -> str:
    d = float(d)
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    digits, e = _shortest(d)
    a = abs(d)
    if 1e-3 <= a < 1e7:
        if e >= 0:
            ip = (digits + "0" * (e + 1))[: e + 1]
            s = ip + "." + (digits[e + 1:] or "0")
        else:
            s = "0." + "0" * (-e - 1) + digits
    else:
        s = digits[0] + "." + (digits[1:] or "0") + "E" + str(e)
    return ("-" if d < 0 else "") + s


def java_doubles(a: np.ndarray) -> list[str]:
    return [java_double(x) for x in np.asarray(a, dtype=np.float64).ravel()]


def java_format_f(x: float, width: int, prec: int) -> str:
    """java.util.Formatter "%<width>.<prec>f" (WidthProcessor.java:193).
    Java's Formatter (FormattedFloatingDecimal) rounds HALF_UP the decimal
    digits FloatingDecimal produces for the double, i.e. the shortest
    round-trip digits, not the exact binary value: "%.3f" of 1.0005 is
    "1.001" and "%.4f" of 0.03125 is "0.0313" (Python's "%.4f" gives
    "0.0312"). FloatingDecimal's digit generator is occasionally one digit
    longer than shortest; that corner is unpinned (no JVM here)."""
    from decimal import ROUND_HALF_UP, Decimal
    if math.isnan(x):
        s = "NaN"
    elif math.isinf(x):
        s = "Infinity" if x > 0 else "-Infinity"
    else:
        q = Decimal(repr(float(x))).quantize(Decimal(1).scaleb(-prec), rounding=ROUND_HALF_UP)
        s = f"{q:.{prec}f}"
    return s.rjust(width)
