"""The exact jump-ahead walk (common/gss_phase.h) against the brute-force reference recurrences
(one IEEE double add per sample, gpssim.c:2212-2250): bit-identical, including forced
round-half-even ties, zero phase, both Doppler signs and tiny steps."""
import math
import random

import pytest

import gpssim_amd as G
import oracle

DELT = 1.0 / 2600000.0


def cases(seed, n):
    rng = random.Random(seed)
    for i in range(n):
        f = rng.uniform(-6000, 6000) if i % 5 else rng.uniform(-60, 60)
        s = f * DELT
        if i % 7 == 0:                       # tie w.r.t. the top-binade lattice 2^-53
            u = 2.0 ** -53
            s = math.copysign((math.floor(abs(s) / u) + 0.5) * u, s)
        x = rng.random()
        if i % 11 == 0:
            x = 0.0
        if i % 13 == 0:
            x = 1.0 - 2.0 ** -53
        yield x, s, rng.randint(1, 300000)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_carrier_walk_exact(seed):
    for x, s, n in cases(seed, 150):
        assert G.carr_advance(x, s, n) == oracle.carr_brute(x, s, n), (x, s, n)


@pytest.mark.parametrize("seed", [4, 5])
def test_code_walk_exact(seed):
    rng = random.Random(seed)
    for i in range(150):
        f = rng.uniform(-6000, 6000)
        cs = (1.023e6 + f / 1540.0) * DELT
        if i % 6 == 0:                       # tie w.r.t. the [512,1024) lattice 2^-43
            u = 2.0 ** -43
            cs = (math.floor(cs / u) + 0.5) * u
        c0 = rng.random() * 1023.0 if i % 9 else 0.0
        st = (rng.randrange(20), rng.randrange(30), rng.randrange(3))
        n = rng.randint(1, 600000)
        assert G.code_advance(c0, cs, n, *st) == oracle.code_brute(c0, cs, n, *st), (c0, cs, n)


def test_stationary_and_single_steps():
    for x, s in [(0.25, 1e-20), (0.75, -1e-19), (0.5, 2.0 ** -55)]:
        for n in (1, 2, 3, 1000):
            assert G.carr_advance(x, s, n) == oracle.carr_brute(x, s, n)
