"""Java number formatting used by the exporters: Long.toString, Float.toString,
Double.toString as printed by the JVM linkerd 1.x runs on (JDK 8).

JDK 8's Double.toString / Float.toString are sun.misc.FloatingDecimal
(BinaryToASCIIBuffer.dtoa + getChars), which is NOT the shortest round-trip
algorithm of JDK 19+: it generates digits with Steele & White's free-format loop
and a symmetric half-ULP stopping test, and prints integral values below 2^63
exactly with long arithmetic (e.g. 2.82879384806159E17 prints as
"2.82879384806159008E17", JDK-4511638).  This module restates that algorithm
(public OpenJDK 8 behaviour, not reference code; the reference only calls
Double.toString through Jackson / string concatenation, e.g.
PrometheusTelemeter.scala:100-127, InfluxDbTelemeter.scala:87-104).  Pinned by
the 142 raw JDK-8 ``stat.avg`` texts of the reference's metrics.js fixture
(tests/test_javafmt.py).
"""
from __future__ import annotations

import math
import struct

EXP_SHIFT = 52
FRACT_HOB = 1 << EXP_SHIFT
EXP_BIAS = 1023
MAX_SMALL_BIN_EXP = 62
MIN_SMALL_BIN_EXP = -(63 // 3)
N_5_BITS = [(5 ** i).bit_length() for i in range(27)]  # FloatingDecimal.N_5_BITS (27 entries)
INSIGNIFICANT_DIGITS = [
    0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3,
    4, 4, 4, 5, 5, 5, 6, 6, 6, 6, 7, 7, 7,
    8, 8, 8, 9, 9, 9, 9, 10, 10, 10, 11, 11, 11,
    12, 12, 12, 12, 13, 13, 13, 14, 14, 14,
    15, 15, 15, 15, 16, 16, 16, 17, 17, 17,
    18, 18, 18, 19,
]


def _wrap(v: int, bits: int) -> int:
    m = 1 << bits
    v &= m - 1
    return v - m if v >= m >> 1 else v


def _estimate_dec_exp(fract_bits: int, bin_exp: int) -> int:
    """floor((d2 - 1.5)*0.289529654 + 0.176091259 + binExp*log10(2)), d2 in [1,2)."""
    d2 = struct.unpack("<d", struct.pack("<Q", (EXP_BIAS << EXP_SHIFT) | (fract_bits & (FRACT_HOB - 1))))[0]
    d = (d2 - 1.5) * 0.289529654 + 0.176091259 + float(bin_exp) * 0.301029995663981
    return math.floor(d)


class _Digits:
    def __init__(self):
        self.digits = []
        self.dec_exponent = 0

    def roundup(self):
        d = self.digits
        i = len(d) - 1
        q = d[i]
        if q == 9:
            while q == 9 and i > 0:
                d[i] = 0
                i -= 1
                q = d[i]
            if q == 9:  # carry out: high-order 1, rest 0s, larger exponent
                self.dec_exponent += 1
                d[0] = 1
                return
        d[i] = q + 1


def _develop_long_digits(dec_exponent: int, lvalue: int, insignificant: int) -> _Digits:
    if insignificant:
        pow10 = 10 ** insignificant
        residue = lvalue % pow10
        lvalue //= pow10
        dec_exponent += insignificant
        if residue >= (pow10 >> 1):
            lvalue += 1
    s = str(lvalue)
    stripped = s.rstrip("0")
    out = _Digits()
    out.digits = [int(c) for c in stripped]
    out.dec_exponent = dec_exponent + len(s)
    return out


def _dtoa(bin_exp: int, fract_bits: int, n_significant_bits: int) -> _Digits:
    """FloatingDecimal.BinaryToASCIIBuffer.dtoa with isCompatibleFormat = true."""
    tail_zeros = (fract_bits & -fract_bits).bit_length() - 1
    n_fract_bits = EXP_SHIFT + 1 - tail_zeros
    n_tiny_bits = max(0, n_fract_bits - bin_exp - 1)
    if MIN_SMALL_BIN_EXP <= bin_exp <= MAX_SMALL_BIN_EXP:
        if n_tiny_bits < 27 and n_fract_bits + N_5_BITS[n_tiny_bits] < 64 and n_tiny_bits == 0:
            # integral value that fits a long: print its digits exactly
            insignificant = 0
            if bin_exp > n_significant_bits:
                p2 = bin_exp - n_significant_bits - 1
                insignificant = INSIGNIFICANT_DIGITS[p2] if 1 < p2 < len(INSIGNIFICANT_DIGITS) else 0
            lv = fract_bits << (bin_exp - EXP_SHIFT) if bin_exp >= EXP_SHIFT else fract_bits >> (EXP_SHIFT - bin_exp)
            return _develop_long_digits(0, lv, insignificant)
    dec_exp = _estimate_dec_exp(fract_bits, bin_exp)
    B5 = max(0, -dec_exp)
    B2 = B5 + n_tiny_bits + bin_exp
    S5 = max(0, dec_exp)
    S2 = S5 + n_tiny_bits
    M5 = B5
    M2 = B2 - n_significant_bits
    fract_bits >>= tail_zeros
    B2 -= n_fract_bits - 1
    common2 = min(B2, S2)
    B2 -= common2
    S2 -= common2
    M2 -= common2
    if n_fract_bits == 1:  # exact power of two: the next smaller number is half as far
        M2 -= 1
    if M2 < 0:
        B2 -= M2
        S2 -= M2
        M2 = 0
    Bbits = n_fract_bits + B2 + (N_5_BITS[B5] if B5 < len(N_5_BITS) else B5 * 3)
    tenSbits = S2 + 1 + (N_5_BITS[S5 + 1] if S5 + 1 < len(N_5_BITS) else (S5 + 1) * 3)
    out = _Digits()
    digits = out.digits
    if Bbits < 64 and tenSbits < 64:
        # int (32-bit) or long (64-bit) arithmetic; m may overflow, which the JDK
        # catches with `m > 0` (then both stopping tests hold)
        bits = 32 if (Bbits < 32 and tenSbits < 32) else 64
        b = _wrap((fract_bits * 5 ** B5) << B2, bits)
        s = _wrap(5 ** S5 << S2, bits)
        m = _wrap(5 ** M5 << M2, bits)
        tens = _wrap(s * 10, bits)
        q = b // s
        b = _wrap(10 * (b % s), bits)
        m = _wrap(m * 10, bits)
        low = b < m
        high = _wrap(b + m, bits) > tens
        if q == 0 and not high:
            dec_exp -= 1  # the estimate was one too high: drop the leading zero
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:  # E-form: at least two digits
            high = low = False
        while not low and not high:
            q = b // s
            b = _wrap(10 * (b % s), bits)
            m = _wrap(m * 10, bits)
            if m > 0:
                low = b < m
                high = _wrap(b + m, bits) > tens
            else:
                low = high = True
            digits.append(q)
        low_digit_difference = _wrap((b << 1) - tens, bits)
    else:
        # FDBigInteger arithmetic (exact); note the `>=` in the high test
        Sval = 5 ** S5 << S2
        Bval = fract_bits * 5 ** B5 << B2
        Mval = 5 ** (M5 + 1) << (M2 + 1)  # 10 * M
        tenSval = 5 ** (S5 + 1) << (S2 + 1)
        q, Bval = divmod(Bval, Sval)
        Bval *= 10
        low = Bval < Mval
        high = Bval + Mval >= tenSval
        if q == 0 and not high:
            dec_exp -= 1
        else:
            digits.append(q)
        if dec_exp < -3 or dec_exp >= 8:
            high = low = False
        while not low and not high:
            q, Bval = divmod(Bval, Sval)
            Bval *= 10
            Mval *= 10
            low = Bval < Mval
            high = Bval + Mval >= tenSval
            digits.append(q)
        low_digit_difference = ((Bval << 1) - tenSval) if (high and low) else 0
    out.dec_exponent = dec_exp + 1
    if high:
        if low:
            if low_digit_difference == 0:
                if digits[-1] & 1:  # tie: round to an even last digit
                    out.roundup()
            elif low_digit_difference > 0:
                out.roundup()
        else:
            out.roundup()
    return out


def _get_chars(neg: bool, d: _Digits) -> str:
    """BinaryToASCIIBuffer.getChars (plain form for 1e-3 <= |x| < 1e7)."""
    digits = "".join(map(str, d.digits))
    n = len(digits)
    e = d.dec_exponent
    sign = "-" if neg else ""
    if 0 < e < 8:
        k = min(n, e)
        ip = digits[:k] + "0" * (e - k)
        fp = digits[k:] if k < n else "0"
        if k < e:
            fp = "0"
        return f"{sign}{ip}.{fp}"
    if -3 < e <= 0:
        return f"{sign}0.{'0' * (-e)}{digits}"
    exp = e - 1
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{exp}"


def _to_string(bits: int, exp_bits: int, frac_bits: int) -> str:
    neg = bits >> (exp_bits + frac_bits) & 1 == 1
    bin_exp = bits >> frac_bits & ((1 << exp_bits) - 1)
    fract = bits & ((1 << frac_bits) - 1)
    if bin_exp == (1 << exp_bits) - 1:
        return "NaN" if fract else ("-Infinity" if neg else "Infinity")
    bias = (1 << (exp_bits - 1)) - 1
    # widen to the double layout: fraction bits left-aligned to bit 52
    fract <<= EXP_SHIFT - frac_bits
    if bin_exp == 0:
        if fract == 0:
            return "-0.0" if neg else "0.0"
        lead = 64 - fract.bit_length()  # Long.numberOfLeadingZeros
        shift = lead - (63 - EXP_SHIFT)
        fract <<= shift
        bin_exp = 1 - shift
        n_sig = 64 - lead - (EXP_SHIFT - frac_bits)
    else:
        fract |= FRACT_HOB
        n_sig = frac_bits + 1
    bin_exp -= bias
    return _get_chars(neg, _dtoa(bin_exp, fract, n_sig))


def double_to_string(x: float) -> str:
    """java.lang.Double.toString(double) on JDK 8."""
    return _to_string(struct.unpack("<Q", struct.pack("<d", float(x)))[0], 11, 52)


def float_to_string(x: float) -> str:
    """java.lang.Float.toString(float) on JDK 8 (FloatingDecimal's float path:
    the same digit loop with the float's 24 significant bits)."""
    return _to_string(struct.unpack("<I", struct.pack("<f", float(x)))[0], 8, 23)


def long_to_string(x: int) -> str:
    return str(int(x))
