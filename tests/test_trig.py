"""Accuracy of the kernel's own fp64 tan/sincos (diplomjourney_amd/csrc/mpc_trig.h),
host build: faithful (< 1 ulp) against mpmath, and how often they agree bit
for bit with glibc, which the reference calls (math.tan, numpy cos/sin)."""
import ctypes
import math

import mpmath as mp
import numpy as np
import pytest

from harness import tan_small, trig_eval

_m = ctypes.CDLL("libm.so.6")
for _f in ("tan", "sin", "cos"):
    getattr(_m, _f).restype = ctypes.c_double
    getattr(_m, _f).argtypes = [ctypes.c_double]


def _ulp_err(got, x, fn):
    exact = fn(mp.mpf(float(x)))
    u = np.spacing(abs(float(exact))) if float(exact) != 0 else 5e-324
    return abs(float((mp.mpf(float(got)) - exact) / u))


@pytest.mark.parametrize("lo,hi", [(-1.06, 1.06), (-7.0, 7.0), (-2e3, 2e3)])
def test_faithful_against_mpmath(lo, hi):
    mp.mp.prec = 120
    x = np.random.default_rng(7).uniform(lo, hi, 3000)
    t, s, c = trig_eval(x)
    worst = [max(_ulp_err(g, xi, fn) for g, xi in zip(out, x))
             for out, fn in ((t, mp.tan), (s, mp.sin), (c, mp.cos))]
    assert max(worst) < 1.0, worst


def test_agreement_with_glibc():
    x = np.random.default_rng(8).uniform(-1.06, 1.06, 100_000)
    t, s, c = trig_eval(x)
    agree = [np.mean(out == np.array([f(v) for v in x]))
             for out, f in ((t, _m.tan), (s, _m.sin), (c, _m.cos))]
    assert min(agree) > 0.90, agree        # ~0.94-0.96 measured; the rest differ by 1 ulp
    for out, f in ((t, _m.tan), (s, _m.sin), (c, _m.cos)):
        g = np.array([f(v) for v in x])
        assert np.all(np.abs(out - g) <= np.spacing(np.abs(g)))


def test_payne_hanek_faithful_against_mpmath():
    """Arguments beyond the Cody-Waite range (|x| > 2^19*pi/2) take the
    kernel's own Payne-Hanek reduction (reduce_pio2_large): faithful against
    mpmath from 1e6 to DBL_MAX, incl. the double closest to a multiple of
    pi/2 (6381956970095103 * 2^797, remainder ~4.7e-19) and arguments just
    beyond the switch-over."""
    mp.mp.prec = 2200                    # exact reduction of arguments up to 2^1024
    rng = np.random.default_rng(9)
    x = np.concatenate([
        rng.uniform(1, 2, 1500) * 2.0 ** rng.integers(20, 1024, 1500),
        [math.ldexp(6381956970095103, 797), 2.0 ** 19 * math.pi / 2 * (1 + 2 ** -52),
         823550.0, 1e22, 2.0 ** 1023 * (2 - 2 ** -52), 3.0 * 2 ** 60]])
    x = np.concatenate([x, -x])
    t, s, c = trig_eval(x)
    worst = [max(_ulp_err(g, xi, fn) for g, xi in zip(out, x))
             for out, fn in ((t, mp.tan), (s, mp.sin), (c, mp.cos))]
    assert max(worst) < 1.0, worst
    agree = [np.mean(out == np.array([f(v) for v in x]))
             for out, f in ((t, _m.tan), (s, _m.sin), (c, _m.cos))]
    assert min(agree) > 0.85, agree


def test_special_values():
    x = np.array([0.0, -0.0, 5e-324, -5e-324, 1e-300, math.pi / 2, 1e6, -1e6, 1e7, 3e9,
                  math.inf, -math.inf, math.nan])
    t, s, c = trig_eval(x)
    assert math.copysign(1, t[1]) == -1 and math.copysign(1, s[1]) == -1 and c[1] == 1.0
    assert t[2] == 5e-324 and s[3] == -5e-324
    for i in range(4, 10):                  # incl. beyond the Cody-Waite range (fallback)
        for out, f in ((t, math.tan), (s, math.sin), (c, math.cos)):
            assert abs(out[i] - f(x[i])) <= 2 * np.spacing(abs(f(x[i])))
    assert np.all(np.isnan(t[10:])) and np.all(np.isnan(s[10:])) and np.all(np.isnan(c[10:]))


def test_tan_small_accuracy():
    """The rollout loop's steering tangent (rational, no reduction, |x| <=
    kTanMax = 1.1): within 2 ulp of the exact value (1.87 measured, 1.3 %
    of arguments at or above 1 ulp), odd, exact at 0."""
    mp.mp.prec = 120
    rng = np.random.default_rng(9)
    x = np.concatenate([rng.uniform(-1.1, 1.1, 4000), np.linspace(1.0, 1.1, 500),
                        rng.uniform(-1e-3, 1e-3, 200)])
    t = tan_small(x)
    worst = max(_ulp_err(g, xi, mp.tan) for g, xi in zip(t, x))
    assert worst < 2.0, worst
    assert np.array_equal(tan_small(-x), -t)
    z = tan_small(np.array([0.0, -0.0, 5e-324, 1e-300]))
    assert z[0] == 0.0 and math.copysign(1, z[1]) == -1 and z[2] == 5e-324 and z[3] == 1e-300
    g = np.array([_m.tan(v) for v in x])
    assert np.mean(t == g) > 0.8            # ~0.87 measured
