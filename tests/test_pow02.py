"""The device step control's x^0.2 (pft_kernels.hip pow02_fix, used by gate_decide for the gated
steps of f4): given a candidate within one ulp of x^0.2 -- ocml's pow on the device -- it returns
x^0.2 rounded to nearest, by comparing x with the 5th powers of the midpoints in double-double
arithmetic.  The host build of the same code is checked here against a 60-digit reference, with
candidates one ulp below, at and above glibc's pow; and glibc's own pow (the host solver's,
rk_solver.c: pow((delta/eps), 0.2), hybrid2.c:580) is measured against the same reference, which
is what bounds the gated steps a host would have to discard.  CPU only: no GPU call.
"""
import math
import random
from decimal import Decimal, getcontext

import porousfreezethaw_amd as P

import ctypes as C


def _lib():
    L = P.lib()
    L.pft_pow02_fix.restype = C.c_double
    L.pft_pow02_fix.argtypes = [C.c_double, C.c_double]
    return L


def _cr(x):
    getcontext().prec = 60
    return float(str((Decimal(x).ln() * Decimal(0.2)).exp()))


def _args():
    rng = random.Random(7)
    xs = [10 ** rng.uniform(-6, 8) for _ in range(6000)] + [rng.uniform(0.5, 2.0) for _ in range(3000)]
    return xs + [2.0 ** k for k in range(-40, 41)] + [1.0, 0.8 ** 5, 2.0 ** 899, 2.0 ** -899]


def test_pow02_fix_correctly_rounded():
    L = _lib()
    bad, glibc_bad = [], 0
    for x in _args():
        ref = _cr(x)
        c = math.pow(x, 0.2)
        glibc_bad += c != ref
        # every candidate within one ulp of the correctly rounded value must come back as it
        for cand in (math.nextafter(ref, 0.0), ref, math.nextafter(ref, math.inf)):
            got = L.pft_pow02_fix(x, cand)
            if got != ref:
                bad.append((x.hex(), cand.hex(), got.hex(), ref.hex()))
    assert not bad, bad[:5]
    # glibc's pow rounds all but a small fraction correctly: the device and the host agree there
    assert glibc_bad <= len(_args()) // 200, glibc_bad


def test_pow02_fix_outside_the_safe_range_keeps_the_candidate():
    L = _lib()
    # (beyond 2^+-900 the candidate stays: the host's bitwise check of the decision catches it)
    for x, c in ((0.0, 0.0), (math.inf, math.inf), (1e-310, 1e-62), (2.0 ** 950, 2.0 ** 190), (1e300, 1e60)):
        assert L.pft_pow02_fix(x, c) == c
    nan = L.pft_pow02_fix(math.nan, math.nan)
    assert nan != nan
