#!/usr/bin/env python3
"""Constant tables of csrc/farms_libm.h (double-double splits of exact values),
computed with the decimal module at 60 digits.  Re-run to regenerate:
    python3 tools/gen_libm_tables.py > /tmp/tables.inc
"""
from decimal import Decimal as D, getcontext
from fractions import Fraction as F

getcontext().prec = 80


def pi():
    # Machin: pi = 16 atan(1/5) - 4 atan(1/239)
    return 16 * atan_small(D(1) / 5) - 4 * atan_small(D(1) / 239)


def atan_small(x):
    s, term, n, x2 = D(0), x, 1, x * x
    while True:
        t = term / n
        if abs(t) < D(10) ** -75:
            break
        s += t if (n // 2) % 2 == 0 else -t
        term *= x2
        n += 2
    return s


def atan(x):
    # halve the argument until small: atan(x) = 2 atan(x / (1 + sqrt(1 + x^2)))
    k = 0
    while abs(x) > D("0.1"):
        x = x / (1 + (1 + x * x).sqrt())
        k += 1
    return atan_small(x) * (2 ** k)


def split(v, parts=2):
    out = []
    for _ in range(parts):
        h = float(v)
        out.append(h)
        v -= D(h)
    return out


def fmt(x):
    return float.hex(x)


P = pi()
print("// pi/2 as three doubles, pi and pi/2 and pi/4 as double-doubles")
print("constexpr double kPio2_1 = %s, kPio2_2 = %s, kPio2_3 = %s;" % tuple(fmt(v) for v in split(P / 2, 3)))
print("constexpr double kPi_hi = %s, kPi_lo = %s;" % tuple(fmt(v) for v in split(P)))
print("constexpr double kPio2_hi = %s, kPio2_lo = %s;" % tuple(fmt(v) for v in split(P / 2)))
print("constexpr double kPio4_hi = %s, kPio4_lo = %s;" % tuple(fmt(v) for v in split(P / 4)))
print("constexpr double k3Pio4_hi = %s, k3Pio4_lo = %s;" % tuple(fmt(v) for v in split(3 * P / 4)))
print("constexpr double k2oPi = %s;" % fmt(float(2 / P)))
print("// atan(j/64), j = 0..64, {hi, lo}")
print("__device__ __host__ constexpr double kAtanTab[65][2] = {")
for j in range(65):
    h, l = split(atan(D(j) / 64))
    print("    {%s, %s}," % (fmt(h), fmt(l)))
print("};")
# Taylor coefficients as double-doubles
def coef(fr):
    h = float(fr)
    l = float(fr - F(h))
    return h, l
import math
print("// sin: (-1)^n / (2n+1)!, n = 0..14; cos: (-1)^n / (2n)!, n = 0..14")
print("__device__ __host__ constexpr double kSinC[15][2] = {")
for n in range(15):
    print("    {%s, %s}," % tuple(fmt(v) for v in coef(F((-1) ** n, math.factorial(2 * n + 1)))))
print("};")
print("__device__ __host__ constexpr double kCosC[15][2] = {")
for n in range(15):
    print("    {%s, %s}," % tuple(fmt(v) for v in coef(F((-1) ** n, math.factorial(2 * n)))))
print("};")
print("// atan: (-1)^n / (2n+1), n = 0..9")
print("__device__ __host__ constexpr double kAtanC[10][2] = {")
for n in range(10):
    print("    {%s, %s}," % tuple(fmt(v) for v in coef(F((-1) ** n, 2 * n + 1))))
print("};")
