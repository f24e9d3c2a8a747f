"""The exact attitude rules of the HIP kernels (gpd_device.h attitude_decide) against glibc.

The reference truncates on ``abs(roll) > .4 or abs(pitch) > .4`` (HoverAviary.py:111,
MultiHoverAviary.py:124) and gates the ground effect on ``abs(rpy) < np.pi/2``
(BaseAviary.py:742), on pybullet's getEulerZYX outputs: libm ``atan2`` / ``asin`` (glibc here and
on the GPU box; Python's ``math`` calls the same functions).  The kernel decides the lanes near a
threshold without atan2 / asin, by comparisons against constants derived at 400 bits
(AttK in gpd_device.h).  These CPU tests:
* re-derive those constants with mpmath and compare them with the literals in the source;
* run the kernel's double-double comparison, emulated operation by operation in Python floats
  (the FMA's exact error term via Fraction), on every near-threshold case the GPU tests use and
  on random samples around each threshold, and require glibc's decision every time.
"""
import math
import pathlib
import re
from fractions import Fraction

import numpy as np
import pytest

from tests.attitude_cases import literal_args, oracle_rpy, tilt_cases, upright_edge_cases

SRC = pathlib.Path(__file__).resolve().parents[1] / "gym_pybullet_drones_routing_amd" / "csrc" / "gpd_device.h"


def _attk():
    text = SRC.read_text()
    body = text[text.index("struct AttK {"):]
    body = body[:body.index("};")]
    vals = {}
    for name, lit in re.findall(r"(\w+) = (-?0x[0-9a-fp.+-]+)", body):
        vals[name] = float.fromhex(lit)
    return vals


K = _attk()


def test_constants_match_a_400_bit_derivation():
    mp = pytest.importorskip("mpmath")
    mp.mp.prec = 400
    m = mp.mpf(0.4) + mp.mpf(2) ** -55                 # rounding midpoint above 0.4
    s = mp.sin(m)
    sin_lim = float(s)
    if mp.mpf(sin_lim) <= s:
        sin_lim = math.nextafter(sin_lim, 2.0)
    assert K["sin_lim"] == sin_lim
    t = mp.tan(m)
    assert K["tan_hi"] == float(t) and K["tan_lo"] == float(t - mp.mpf(float(t)))
    mg = mp.mpf(math.pi / 2) - mp.mpf(2) ** -53         # rounding midpoint below RN(pi/2)
    c = mp.cot(mg)
    assert K["cot_hi"] == float(c) and K["cot_lo"] == float(c - mp.mpf(float(c)))


def dd_above(u, hi, lo, v):
    """gpd_device.h dd_above in Python floats: p = hi*v rounded, e = fma(hi, v, -p) (exact)."""
    p = hi * v
    e = float(Fraction(hi) * Fraction(v) - Fraction(p))   # representable: the exact FMA result
    return ((u - p) - e) - lo * v > 0.0


def kernel_tilt(sarg, a, b):
    gimbal = sarg <= -0.99999 or sarg >= 0.99999
    zero_roll = a == 0.0 and b == 0.0 and math.copysign(1.0, b) > 0
    roll_out = dd_above(abs(a), K["tan_hi"], K["tan_lo"], b) if b > 0.0 else not zero_roll
    return gimbal or abs(sarg) >= K["sin_lim"] or roll_out


def kernel_up(sarg, a, b):
    gimbal = sarg <= -0.99999 or sarg >= 0.99999
    zero_roll = a == 0.0 and b == 0.0 and math.copysign(1.0, b) > 0
    roll_in = dd_above(b, K["cot_hi"], K["cot_lo"], abs(a)) if b > 0.0 else zero_roll
    return not gimbal and roll_in


def glibc_tilt(sarg, a, b):
    if sarg <= -0.99999 or sarg >= 0.99999:
        return True
    return abs(math.atan2(a, b)) > .4 or abs(math.asin(min(1.0, max(-1.0, sarg)))) > .4


def glibc_up(sarg, a, b):
    if sarg <= -0.99999 or sarg >= 0.99999:
        return False                                    # pitch = +-pi/2 -> not < pi/2
    return bool(np.abs(math.atan2(a, b)) < np.pi / 2)


def test_rules_equal_glibc_on_the_gpu_cases():
    q, _ = tilt_cases()
    for x in q:
        args = literal_args(x)
        assert kernel_tilt(*args) == glibc_tilt(*args)
        r = oracle_rpy(x)
        assert glibc_tilt(*args) == (abs(r[0]) > .4 or abs(r[1]) > .4)
    for x in upright_edge_cases():
        args = literal_args(x)
        assert kernel_up(*args) == glibc_up(*args)
        r = oracle_rpy(x)
        assert glibc_up(*args) == bool(np.abs(r[0]) < np.pi / 2 and np.abs(r[1]) < np.pi / 2)


def _misrounded(a, b, mid):
    """glibc's atan2(a, b) (a, b > 0 region) rounded to the wrong side of the midpoint `mid`
    (an mpmath value): then the true value lies within 1e-2 ulp of it."""
    mp = pytest.importorskip("mpmath")
    mp.mp.prec = 300
    t = mp.atan2(mp.mpf(abs(a)), mp.mpf(b))
    return abs(t - mid) < mp.mpf(1e-2) * mp.mpf(math.ulp(0.4 if mid < 1 else 1.5))


def test_rules_equal_glibc_on_random_near_threshold_samples():
    """Equal to glibc everywhere except where glibc's atan2 is not correctly rounded: within
    ~2e-3 ulp of a rounding midpoint glibc 2.35 can return the neighbour (e.g. atan2 at
    0.49992 ulp above 0.4 returns 0.4 + ulp).  There the kernel keeps the correctly rounded
    decision; such samples are counted and must stay rare (<= 1e-3 of the samples)."""
    mp = pytest.importorskip("mpmath")
    mp.mp.prec = 300
    m_tilt = mp.mpf(0.4) + mp.mpf(2) ** -55
    m_up = mp.mpf(math.pi / 2) - mp.mpf(2) ** -53
    rng = np.random.default_rng(3)
    n_flip, n_mis = [0, 0, 0], [0, 0]
    N = 20000
    # roll: a = tan(0.4) b (1 + k 2^-52), b in (0.2, 1]
    for _ in range(N):
        b = float(rng.uniform(0.2, 1.0))
        a = math.tan(0.4) * b * (1 + int(rng.integers(-8, 9)) * 2.0 ** -52) * (1 if rng.random() < .5 else -1)
        g = glibc_tilt(0.0, a, b)
        if kernel_tilt(0.0, a, b) != g:
            assert _misrounded(a, b, m_tilt), (a, b)
            assert kernel_tilt(0.0, a, b) == (mp.atan2(abs(a), b) > m_tilt)
            n_mis[0] += 1
        n_flip[0] += g
    # pitch: sarg within a few ulp of sin(0.4) (one threshold on sarg: exact, glibc asin is monotonic)
    s0 = math.sin(0.4)
    for k in range(-64, 65):
        s = s0 + k * math.ulp(s0)
        for sg in (1.0, -1.0):
            assert kernel_tilt(sg * s, 0.0, 1.0) == glibc_tilt(sg * s, 0.0, 1.0)
            n_flip[1] += glibc_tilt(sg * s, 0.0, 1.0)
    # ground-effect gate: b ~ 1.7e-16 |a|
    for _ in range(N):
        a = float(rng.uniform(0.3, 1.0)) * (1 if rng.random() < .5 else -1)
        b = abs(a) * float(rng.uniform(0.5e-16, 3e-16))
        g = glibc_up(0.0, a, b)
        if kernel_up(0.0, a, b) != g:
            assert _misrounded(a, b, m_up), (a, b)
            assert kernel_up(0.0, a, b) == (mp.atan2(abs(a), b) < m_up)
            n_mis[1] += 1
        n_flip[2] += g
    # every threshold was crossed (both decisions occur); glibc misroundings are rare
    assert 0 < n_flip[0] < N and 0 < n_flip[1] < 258 and 0 < n_flip[2] < N
    assert max(n_mis) <= N // 1000, n_mis


def test_previous_rounded_limits_were_wrong_near_the_threshold():
    """The round-2 predicates (|a| > RN(tan 0.4) b; upright = b > 0) disagree with the reference
    on some of the GPU cases even on the literal arguments: the tests have power."""
    wrong_tilt = sum((abs(s) > 0.38941834230865049 or (abs(a) > 0.42279321873816178 * b if b > 0 else True))
                     != glibc_tilt(s, a, b) for s, a, b in map(literal_args, tilt_cases()[0]))
    wrong_up = sum(((not (s <= -0.99999 or s >= 0.99999)) and b > 0) != glibc_up(s, a, b)
                   for s, a, b in map(literal_args, upright_edge_cases()))
    assert wrong_tilt > 0 and wrong_up > 0
