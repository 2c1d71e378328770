"""Host model of the integer-digit evaluation contraction (kl_eval_int.h),
checked against exact arithmetic -- the error bounds DESIGN.md states for it.

The kernel computes, per (slot, pixel), the phase in 32-bit fixed-point turns
R = combine(P_4 .. P_9), P_k = sum over digit pairs (i, j), i + j = k, of
sum_d a_i[d] b_j[d] (int32, wrapping), where a / b are the 6 balanced
base-256 digits of Cq = rint(Cpix 2^36) and cq = rint(coef / 2 pi 2^44).
This module restates that in Python integers (int32 wrap emulated) and
compares R 2^-32 with:
  * the exact value sum_d Cq cq 2^-80 modulo 1 turn (only the dropped
    diagonals k <= 3 and the two arithmetic shifts separate them:
    <= ~1.3 units of 2^-32 turn);
  * the fp64 phase sum_d Cpix coef / 2 pi (adds the operand rounding:
    sum |coef / 2 pi| 2^-37 + sum |Cpix| 2^-45; over the allowed ranges --
    D <= 60, |coef / 2 pi| <= 8.031 turns (the digit range), |Cpix| < 1904.6
    (sf_set_grid) -- at most 3.51e-9 + 3.25e-9 + 0.30e-9 = 7.06e-9 turn
    < 2^-27, which the adversarial case below approaches).
CPU only (no GPU): pins the algorithm the GPU tests exercise through cos/sin.
"""

from fractions import Fraction

import numpy as np
import pytest

SIGMA, TAU, NDIG = 36, 44, 6


def digits(v):
    """balanced base-256 digits (kl_eval_int.h dig_split); remainder 0 iff
    v fits 6 digits"""
    out = []
    for _ in range(NDIG):
        lo = v & 0xFF
        b = lo - 256 if lo >= 128 else lo
        out.append(b)
        v = (v - b) >> 8
    return out, v


def wrap32(x):
    return ((x + 2 ** 31) % 2 ** 32) - 2 ** 31


def combine(p):
    """dig_combine: p = [P4 .. P9] (int32), arithmetic shifts, wrap mod 2^32"""
    t = wrap32(p[1] + (p[0] >> 8))
    t = wrap32(p[2] + (t >> 8))
    return wrap32(t + (p[3] << 8) + (p[4] << 16) + (p[5] << 24))


def int_phase(cpix_row, coef):
    """R (units of 2^-32 turn, in [-2^31, 2^31)) for one (slot, pixel)"""
    return int_phase_turns(cpix_row, [x / (2 * np.pi) for x in coef])


def int_phase_turns(cpix_row, turns):
    """int_phase with the coefficients already in turns (coef / 2 pi)"""
    a = []
    for c in cpix_row:
        dg, rem = digits(int(np.rint(np.ldexp(c, SIGMA))))
        assert rem == 0, "Cpix out of the digit range"
        a.append(dg)
    b = []
    for x in turns:
        dg, rem = digits(int(np.rint(np.ldexp(x, TAU))))
        assert rem == 0, "coefficient out of the digit range"
        b.append(dg)
    p = []
    for k in range(4, 10):
        s = 0
        for i in range(NDIG):
            j = k - i
            if 0 <= j < NDIG:
                s += sum(a[d][i] * b[d][j] for d in range(len(turns)))
        assert abs(s) < 2 ** 31  # exact in int32 (the MFMA accumulators)
        p.append(wrap32(s))
    return combine(p)


def frac_turn(x):
    """x modulo 1 turn into [-1/2, 1/2)"""
    return x - np.floor(x + 0.5)


@pytest.mark.parametrize("seed,D,cscale,coef_scale", [
    (1, 50, 600.0, 0.02),    # config-5-like magnitudes
    (2, 64, 2000.0, 1.0),    # the largest K, near the Cpix limit, big phases
    (3, 45, 1.0, 7.0),       # coefficients near the digit range (7 turns)
    (4, 20, 300.0, 0.3),
])
def test_int_contraction_error_bounds(seed, D, cscale, coef_scale):
    rng = np.random.default_rng(seed)
    for _ in range(6):
        cpix = -np.abs(rng.normal(0, cscale, D))           # Cpix <= 0
        cpix = np.clip(cpix, -1900.0, 0.0)
        coef = rng.normal(0, coef_scale, D) * 2 * np.pi     # coef in radians
        coef = np.clip(coef, -7.5 * 2 * np.pi, 7.5 * 2 * np.pi)
        R = int_phase(cpix, coef)
        # exact value of the quantized operands modulo 1 turn
        cq = [int(np.rint(np.ldexp(c, SIGMA))) for c in cpix]
        kq = [int(np.rint(np.ldexp(x / (2 * np.pi), TAU))) for x in coef]
        exact = Fraction(sum(c * k for c, k in zip(cq, kq)), 2 ** (SIGMA + TAU))
        exact_frac = exact - round(exact)
        units = abs(Fraction(R, 2 ** 32) - exact_frac) * 2 ** 32
        units = min(units, 2 ** 32 - units)
        assert units <= 1.3, float(units)
        # against the fp64 phase (what the fp64 contraction computes)
        rev = float(np.dot(cpix, coef / (2 * np.pi)))
        err = abs(frac_turn(R * 2.0 ** -32 - rev))
        bound = (np.abs(coef / (2 * np.pi)).sum() * 2.0 ** -37
                 + np.abs(cpix).sum() * 2.0 ** -45 + 1.3 * 2.0 ** -32
                 + abs(rev) * 2.0 ** -50)            # fp64 rounding of rev
        assert err <= bound, (err, bound)
        assert err <= 2.0 ** -28


def test_digit_split_range():
    """6 balanced digits hold [-128 (256^6 - 1) / 255, 127 (256^6 - 1) / 255]"""
    m = (256 ** 6 - 1) // 255
    for v in (0, 1, -1, 127 * m, -128 * m, 2 ** 46, -(2 ** 46), 12345678901234):
        dg, rem = digits(v)
        assert rem == 0 and sum(d * 256 ** i for i, d in enumerate(dg)) == v
        assert all(-128 <= d <= 127 for d in dg)
    for v in (127 * m + 1, -128 * m - 1, 2 ** 47):
        assert digits(v)[1] != 0


# the allowed ranges (kl_eval_int.h): D <= SF_MAX_DIR = 60; coefficients
# whose rint(coef / 2 pi 2^44) fits 6 balanced digits ([-128 m, 127 m],
# m = (256^6 - 1) / 255: -8.031 .. 7.969 turns); |Cpix| 2^36 < 1.86 2^46
# (sf_set_grid's cmax check, which carries a 1 % margin itself)
M6 = (256 ** 6 - 1) // 255
K_POS, K_NEG = 127 * M6 / 2.0 ** TAU, -128 * M6 / 2.0 ** TAU
CPIX_MAX = 1.86 * 2.0 ** 10
BOUND_TURNS = 2.0 ** -27   # kl_eval_int.h / include/screenfit.h


def test_stated_bound_covers_the_range_limits():
    """The per-term accounting at the range limits stays below 2^-27."""
    worst = (60 * max(K_POS, -K_NEG) * 2.0 ** -37 + 60 * CPIX_MAX * 2.0 ** -45
             + 1.3 * 2.0 ** -32)
    assert 2.0 ** -28 < worst < BOUND_TURNS, worst


def test_int_contraction_adversarial_worst_case():
    """D = 60 at the range limits with every rounding error of the same
    sign: Cq and cq both round by ~1/2 unit, signed so that every term
    delta_C k + Cpix delta_k adds.  The error against the exact product of
    the fp64 operands exceeds the old 2^-28 claim and stays below 2^-27."""
    D = 60
    cpix, turns = [], []
    for d in range(D):
        sign = 1.0 if d % 2 == 0 else -1.0
        # k 2^44 = integer + 15/32 (k ~ 8 has 2^-5 resolution there): rint
        # rounds it down, delta_k < 0, and with Cpix < 0 Cpix delta_k > 0
        base = (127.0 * M6 - 1.0 if sign > 0 else -128.0 * M6 + 1.0) + 15.0 / 32.0
        k = np.ldexp(base, -TAU)
        assert np.ldexp(k, TAU) == base
        # Cpix 2^36 = integer +- 31/64 so that rint moves it toward sign(k):
        # delta_C k > 0
        cb = np.floor(-(CPIX_MAX - 20.0 - d) * 2.0 ** SIGMA)
        cb = cb + (1.0 - 31.0 / 64.0 if sign > 0 else 31.0 / 64.0)
        c = np.ldexp(cb, -SIGMA)
        assert np.ldexp(c, SIGMA) == cb
        cpix.append(float(c))
        turns.append(float(k))
    R = int_phase_turns(cpix, turns)
    exact = sum(Fraction(c) * Fraction(k) for c, k in zip(cpix, turns))
    exact_frac = exact - round(exact)
    err = abs(Fraction(R, 2 ** 32) - exact_frac)
    err = float(min(err, 1 - err))
    assert 2.0 ** -28 < err <= BOUND_TURNS, (err, np.log2(err))
