"""The exact phase arithmetic (common/gss_phase.h) against the brute-force reference recurrences
(one IEEE double add per sample, gpssim.c:2212-2250): the plain binade walk (Stage-B lanes), the
cycle-cached walk (Stage A and the host planner) and the anchors Stage A emits are all
bit-identical to brute force, including forced round-half-even ties, zero phase, both Doppler
signs, tiny and LEO-sized Dopplers, 2.6 and 20 MS/s."""
import ctypes as C
import math
import random

import numpy as np
import pytest

from conftest import walk_lib

import gpssim_amd as G
import oracle


def cases(seed, n):
    rng = random.Random(seed)
    for i in range(n):
        fs = 2.6e6 if i % 3 else 2.0e7
        f = rng.uniform(-6000, 6000)
        if i % 5 == 0:
            f = rng.uniform(-60, 60)
        if i % 17 == 0:
            f = rng.uniform(-40000, 40000)
        s = f / fs
        if i % 7 == 0:                       # tie w.r.t. the top-binade lattice 2^-53
            u = 2.0 ** -53
            s = math.copysign((math.floor(abs(s) / u) + 0.5) * u, s)
        if i % 19 == 0:                      # exact multiple of 2^-53
            u = 2.0 ** -53
            s = math.copysign(math.floor(abs(s) / u) * u, s)
        x = rng.random()
        if i % 11 == 0:
            x = 0.0
        if i % 13 == 0:
            x = 1.0 - 2.0 ** -53
        yield x, s, rng.randint(1, int(fs / 10))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_carrier_walks_exact(seed):
    W = walk_lib()
    for x, s, n in cases(seed, 120):
        want = oracle.carr_brute(x, s, n)
        assert W.wc_carr_plain(x, s, n) == want, ("plain", x, s, n)
        assert W.wc_carr_cached(x, s, n) == want, ("cached", x, s, n)
        nw = C.c_int32(0)
        assert W.wc_carr_f(x, s, n, C.byref(nw)) == want, ("f64", x, s, n)
        assert W.wc_carr_bf(x, s, n, C.byref(nw)) == want, ("branch-free", x, s, n)
        assert W.wc_carr_trip(x, s, n) == want, ("specialised trip", x, s, n)
        assert G.carr_advance(x, s, n) == want
        if n < 1 << 31 and seed == 1:
            end, ck = G.carr_advance_ck(x, s, n)
            assert end == want
            at = [j * n // G.NCK for j in range(G.NCK)]
            assert np.array_equal(ck, oracle.carr_brute_trace(x, s, at)), ("ck", x, s, n)


@pytest.mark.parametrize("seed", [4, 5])
def test_code_walks_exact(seed):
    W = walk_lib()
    rng = random.Random(seed)
    for i in range(120):
        fs = 2.6e6 if i % 4 else 2.0e7
        f = rng.uniform(-6000, 6000)
        cs = (1.023e6 + f / 1540.0) / fs
        if i % 6 == 0:                       # tie w.r.t. the [512,1024) lattice 2^-43
            u = 2.0 ** -43
            cs = (math.floor(cs / u) + 0.5) * u
        c0 = rng.random() * 1023.0 if i % 9 else 0.0
        st = (rng.randrange(20), rng.randrange(30), rng.randrange(3))
        n = rng.randint(1, int(fs / 10))
        want = oracle.code_brute(c0, cs, n, *st)
        for cached in (0, 1):
            a, b, d = C.c_int32(st[0]), C.c_int32(st[1]), C.c_int32(st[2])
            ph = W.wc_code(cached, c0, cs, n, C.byref(a), C.byref(b), C.byref(d))
            assert (ph, a.value, b.value, d.value) == want, (cached, c0, cs, n)
        a, b, d = C.c_int32(st[0]), C.c_int32(st[1]), C.c_int32(st[2])
        ph = W.wc_code_f(c0, cs, n, C.byref(a), C.byref(b), C.byref(d))
        assert (ph, a.value, b.value, d.value) == want, ("f64", c0, cs, n)
        a, b, d = C.c_int32(st[0]), C.c_int32(st[1]), C.c_int32(st[2])
        ph = W.wc_code_bf(c0, cs, n, C.byref(a), C.byref(b), C.byref(d))
        assert (ph, a.value, b.value, d.value) == want, ("branch-free", c0, cs, n)
        assert G.code_advance(c0, cs, n, *st) == want


def test_anchors_are_exact_states():
    """Every anchor Stage A emits is a state of the brute-force chain at its sample index, lies
    at or before its segment start, and is the last wrap before it."""
    W = walk_lib()
    rng = random.Random(9)
    R, N = 1024, 260000
    nseg = (N + R - 1) // R
    for _ in range(12):
        s = rng.uniform(-5000, 5000) / 2.6e6
        x0 = rng.random()
        an = np.zeros(nseg, np.int32)
        ax = np.zeros(nseg)
        assert W.wc_carr_anchors(x0, s, N, R, nseg, an.ctypes.data, ax.ctypes.data) == nseg
        x, pos = x0, 0
        wraps = {0: x0}
        for seg in range(nseg):
            tgt = int(an[seg])
            assert tgt <= seg * R
            while pos < tgt:
                x = oracle.carr_brute(x, s, 1)
                pos += 1
            assert x == ax[seg], (seg, tgt)


@pytest.mark.parametrize("seed", [10, 11])
def test_segment_start_states_f64(seed):
    """GPU form of Stage A + Stage-B lane start (f64 jump walk): the carrier value at every
    segment start equals the brute-force chain, and no lane-start walk crosses a wrap."""
    W = walk_lib()
    rng = random.Random(seed)
    R, N = 1024, 260000
    nseg = (N + R - 1) // R
    for i in range(6):
        s = rng.uniform(-5000, 5000) / 2.6e6
        if i == 0:
            s = (math.floor(abs(s) / 2.0 ** -53) + 0.5) * 2.0 ** -53     # tie at the wrap step
        x0 = rng.random() if i != 1 else 0.0
        out = np.zeros(nseg)
        assert W.wc_carr_seg_starts_f(x0, s, N, R, nseg, out.ctypes.data) == 0
        want = oracle.carr_brute_trace(x0, s, [seg * R for seg in range(nseg)])
        assert np.array_equal(out, want), i


@pytest.mark.parametrize("seed", [20, 21, 22])
def test_stage_a_segment_states(seed):
    """gss_seg_states (the GPU Stage A core): the exact carrier / code state at every segment
    start, straight from the walk (lattice jumps interpolated exactly), equals brute force;
    includes Dopplers so small that one trip spans many segments, forced ties, zero phase, and
    the block-end value."""
    W = walk_lib()
    rng = random.Random(seed)
    R, N = 1024, 260000
    nseg = (N + R - 1) // R
    at = [j * R for j in range(nseg)]
    for i in range(8):
        f = rng.uniform(-5000, 5000)
        if i == 1:
            f = rng.uniform(-0.5, 0.5)                     # jumps across many segments
        if i == 2:
            f = 0.0
        s = f / 2.6e6
        if i == 3:
            s = (math.floor(abs(s) / 2.0 ** -53) + 0.5) * 2.0 ** -53     # tie at the wrap step
        x0 = rng.random() if i != 4 else 0.0
        ox = np.zeros(nseg)
        oc = np.zeros(nseg, np.uint32)
        end = W.wc_seg_states(x0, s, 0, 0, 0, N, R, nseg, 1, ox.ctypes.data, oc.ctypes.data)
        want = oracle.carr_brute_trace(x0, s, at)
        assert np.array_equal(ox, want), i
        assert end == oracle.carr_brute(x0, s, N), i
        # the same as 8 sub-chains started from the planner's checkpoints (GPU Stage A with
        # host checkpoints): segment states and block-end value identical
        nck = W.wc_nck()
        ck = np.zeros(nck)
        assert W.wc_carr_walk_ck(x0, s, N, ck.ctypes.data) == end
        pos = [j * N // nck for j in range(nck)] + [N]
        assert np.array_equal(ck, oracle.carr_brute_trace(x0, s, pos[:-1])), i
        ox2 = np.full(nseg, np.nan)
        for j in range(nck):
            e2 = W.wc_seg_states(ck[j], s, 0, 0, pos[j], pos[j + 1], R, nseg, int(j == nck - 1),
                                 ox2.ctypes.data, oc.ctypes.data)
        assert np.array_equal(ox2, want), i
        assert e2 == end, i
        # code chain with counters
        cs = (1.023e6 + f / 1540.0) / 2.6e6
        if i == 5:
            cs = (math.floor(cs / 2.0 ** -43) + 0.5) * 2.0 ** -43
        c0 = rng.random() * 1023.0 if i != 6 else 0.0
        st = (rng.randrange(20), rng.randrange(30), rng.randrange(3))
        cnt0 = st[0] | (st[1] << 8) | (st[2] << 16)
        W.wc_seg_states(c0, cs, 1, cnt0, 0, N, R, nseg, 0, ox.ctypes.data, oc.ctypes.data)
        c, (a, b, d) = c0, st
        for j in range(nseg):
            if j:
                c, a, b, d = oracle.code_brute(c, cs, R, a, b, d)
            assert ox[j] == c and oc[j] == (a | (b << 8) | (d << 16)), (i, j)


@pytest.mark.parametrize("seed", [30, 31])
def test_code_chain_branch_free(seed):
    """gss_code_seg_states_bf (the GPU Stage A code waves) equals gss_seg_states' code chain and
    brute force at every segment start: 1, 2.6 and 20 MS/s (top-binade jumps spanning several
    segments), forced ties on the 2^-43 lattice, zero phase, a phase just below 1023, counter
    roll-overs, no motion; the dummy slot past nseg absorbs the trips without a start."""
    W = walk_lib()
    rng = random.Random(seed)
    R = 1024
    for i in range(9):
        fs = [2.6e6, 2.0e7, 1.0e6][i % 3] if i != 7 else 2.0e4     # 2e4: code step ~51 chips
        N = int(fs / 10)
        nseg = (N + R - 1) // R
        f = rng.uniform(-6000, 6000)
        cs = (1.023e6 + f / 1540.0) / fs
        if i == 4:
            cs = (math.floor(cs / 2.0 ** -43) + 0.5) * 2.0 ** -43
        if i == 8:
            cs = 0.0
        c0 = [rng.random() * 1023.0, 0.0, 1022.9999999][i % 3 if i < 6 else 0]
        st = (rng.randrange(20), rng.randrange(30), rng.randrange(40))
        cnt0 = st[0] | (st[1] << 8) | (st[2] << 16)
        want_x = np.zeros(nseg)
        want_c = np.zeros(nseg, np.uint32)
        W.wc_seg_states(c0, cs, 1, cnt0, 0, N, R, nseg, 0, want_x.ctypes.data, want_c.ctypes.data)
        got_x = np.full(nseg + 1, np.nan)
        got_c = np.zeros(nseg + 1, np.uint32)
        W.wc_code_seg_bf(c0, cs, cnt0, N, R, nseg, nseg, got_x.ctypes.data, got_c.ctypes.data)
        assert np.array_equal(got_x[:nseg], want_x), i
        assert np.array_equal(got_c[:nseg], want_c), i
        if i < 3:
            c, (a, b, d) = c0, st
            for j in range(nseg):
                if j:
                    c, a, b, d = oracle.code_brute(c, cs, R, a, b, d)
                assert got_x[j] == c and got_c[j] == (a | (b << 8) | (d << 16)), (i, j)


def test_stationary_and_single_steps():
    """Stationary values, and steps so small that K < 2^26 in the upper binades (the
    branch-free walk's exact-division fallback)."""
    W = walk_lib()
    for x, s in [(0.25, 1e-20), (0.75, -1e-19), (0.5, 2.0 ** -55), (0.3, 3e-9), (0.9, -5e-9),
                 (0.999, 7.3e-10), (1e-9, 2.5e-9)]:
        for n in (1, 2, 3, 1000, 400000):
            want = oracle.carr_brute(x, s, n)
            assert W.wc_carr_plain(x, s, n) == want
            assert W.wc_carr_cached(x, s, n) == want
            nw = C.c_int32(0)
            assert W.wc_carr_f(x, s, n, C.byref(nw)) == want
            assert W.wc_carr_bf(x, s, n, C.byref(nw)) == want
            assert W.wc_carr_trip(x, s, n) == want


@pytest.mark.parametrize("seed", [40, 41])
def test_long_walks_multi_cycle(seed):
    """Long walks (a 20 MS/s block and 10^8 samples): the cycle-cached walk takes many cached
    cycles at once (gss_carr_next_wrap with `multi`), stopping at every checkpoint; the end value
    and all checkpoints equal brute force, including steps whose cycle drifts across a cache
    entry's [lo, hi] (near-integer 1/s), ties and zero phase."""
    W = walk_lib()
    rng = random.Random(seed)
    for i in range(10):
        n = [2_000_000, 100_000_000][i % 2] if i < 8 else rng.randint(1, 5_000_000)
        f = rng.uniform(-6000, 6000)
        s = f / 2.6e6
        if i == 2:                            # 1/s within 1e-9 of an integer: slow drift
            L = rng.randint(300, 3000)
            s = 1.0 / L + rng.choice([-1, 1]) * 1e-12
        if i == 3:
            s = (math.floor(abs(s) / 2.0 ** -53) + 0.5) * 2.0 ** -53
        x0 = rng.random() if i != 4 else 0.0
        want = oracle.carr_brute(x0, s, n)
        assert W.wc_carr_cached(x0, s, n) == want, (i, x0, s, n)
        if n < 1 << 31:
            nck = W.wc_nck()
            ck = np.zeros(nck)
            assert W.wc_carr_walk_ck(x0, s, n, ck.ctypes.data) == want, i
            at = [j * n // nck for j in range(nck)]
            assert np.array_equal(ck, oracle.carr_brute_trace(x0, s, at)), i


@pytest.mark.parametrize("seed", [50, 51])
def test_block_chains_successor_fast_path(seed):
    """The planner's chain as it runs: 0.1 s blocks at 2.6 MS/s chained end to start, with the
    step drifting a little per block, for Dopplers across +-5 kHz and near zero: every block end
    and every checkpoint of the cycle-cached walks equals brute force."""
    W = walk_lib()
    rng = random.Random(seed)
    n = 260_000
    nck = W.wc_nck()
    at = [j * n // nck for j in range(nck)]
    for i in range(8):
        f = rng.uniform(-5000, 5000) if i % 4 else rng.uniform(-80, 80)
        s = f / 2.6e6
        x = rng.random()
        for b in range(3):
            want = oracle.carr_brute(x, s, n)
            assert W.wc_carr_cached(x, s, n) == want, (seed, i, b, x, s)
            ck = np.zeros(nck)
            assert W.wc_carr_walk_ck(x, s, n, ck.ctypes.data) == want, (seed, i, b, x, s)
            assert np.array_equal(ck, oracle.carr_brute_trace(x, s, at)), (seed, i, b, x, s)
            x, s = want, s * (1.0 + rng.uniform(-2e-7, 2e-7))


@pytest.mark.parametrize("seed", [4, 5])
def test_margin_walk_cycle_cache(seed):
    """The speculative walks' cycle-cached margins (gss_walk_margins_cc, -DGSS_SPEC_CC=1 builds:
    2.3x faster on the host, slower on the GPU, so off by default): from a post-wrap start the
    same end and wrap as the plain margin walk, an interval inside the plain one, and every
    lattice translation d inside it moves the brute-force end by exactly d."""
    W = walk_lib()
    rng = random.Random(seed)
    D = C.c_double
    checked = 0
    for x, s, n in cases(seed, 60):
        if s == 0.0 or abs(s) > 0.01:
            continue
        unit = 2.0 ** -52 if s > 0 else 2.0 ** -53
        w = math.floor(rng.random() * abs(s) / unit) * unit      # a post-wrap lattice value
        n = min(n, 200000)
        lo0, hi0, lo1, hi1 = D(), D(), D(), D()
        we0, we1 = C.c_int32(0), C.c_int32(0)
        e0 = W.wc_margins(w, s, n, 0, C.byref(lo0), C.byref(hi0), C.byref(we0))
        e1 = W.wc_margins(w, s, n, 1, C.byref(lo1), C.byref(hi1), C.byref(we1))
        assert e0 == e1 == oracle.carr_brute(w, s, n), (w, s, n)
        assert we0.value == we1.value
        assert lo0.value <= lo1.value <= 0.0 <= hi1.value <= hi0.value, (w, s, n)
        for k in (math.ceil(lo1.value / unit), math.floor(hi1.value / unit), 1, -1):
            d = k * unit
            if lo1.value <= d <= hi1.value and 0.0 <= w + d < 1.0:
                assert oracle.carr_brute(w + d, s, n) == e1 + d, (w, s, n, d)
                checked += 1
    assert checked > 20
