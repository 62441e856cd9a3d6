"""The certified integer linearisation (gps-sdr-sim_amd/csrc/host/linearize.c) on the CPU.

* gss_minmax_mod (the certificate's core) against brute force;
* blocks rendered from the certified lines by tests/helpers/lin_check.c (the GPU fast path's
  arithmetic in scalar C) against the scalar oracle of the reference loop (gpssim.c:2190-2288)
  on synthetic parameter sweeps, and against the reference's own golden block hashes on the real
  static scenario;
* samples where the line comes within the proof's Delta of a cell or chip boundary (code wraps
  that start a new data bit included): decided exactly, patched where the line is wrong;
* how many blocks the proof certifies on the BASELINE scenarios (the rest take the exact path).
"""
import ctypes as C
import hashlib
import math
import os
import subprocess
import zlib

import numpy as np
import pytest

from conftest import LOC, NAV, PKG, REPO

import gpssim_amd as G
import oracle

HELP = os.path.join(REPO, "tests", "helpers")
_lc = None


def lc():
    global _lc
    if _lc is None:
        src = os.path.join(HELP, "lin_check.c")
        so = os.path.join(HELP, "_lin_check.so")
        hdrs = [os.path.join(REPO, "include", "gpssim_amd.h"),
                os.path.join(PKG, "csrc", "common", "gss_lin.h")]
        if not os.path.exists(so) or os.path.getmtime(so) < max(
                [os.path.getmtime(src)] + [os.path.getmtime(h) for h in hdrs]):
            subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", so, src])
        L = C.CDLL(so)
        L.lc_render.restype = C.c_int
        L.lc_render.argtypes = [C.c_void_p] * 7 + [C.c_int, C.c_int, C.c_int, C.c_void_p]
        _lc = L
    return _lc


def _p(a):
    return C.c_void_p(a.ctypes.data)


def render_lin(blk, nch, lin, fast, ca, n, fmt):
    s, c = G.lut()
    out = np.zeros(len(nch) * G.block_bytes(n, fmt), np.uint8)
    nr = lc().lc_render(_p(np.ascontiguousarray(blk)), _p(nch), _p(lin), _p(fast), _p(ca), _p(s),
                        _p(c), len(nch), n, fmt, _p(out))
    return out, nr


# ---------------------------------------------------------------------------------------------
def brute_minmax(n, m, a, s):
    v = [(a + p * s) % m for p in range(n)]
    return min(v), max(v)


def test_minmax_mod_small_vs_brute():
    rng = np.random.default_rng(1)
    for _ in range(3000):
        m = int(rng.integers(1, 5000))
        n = int(rng.integers(1, 3000))
        a, s = int(rng.integers(0, m)), int(rng.integers(0, m))
        assert G.minmax_mod(n, m, a, s) == brute_minmax(n, m, a, s), (n, m, a, s)


def test_minmax_mod_edges():
    for (n, m, a, s) in [(1, 7, 3, 5), (10, 7, 0, 0), (100, 2, 1, 1), (5, 1 << 55, 0, 1 << 54),
                         (1000, 1 << 55, (1 << 55) - 1, 1), (300000, 1 << 50, 12345, 3),
                         (7, 1 << 63, (1 << 63) - 5, (1 << 63) - 1)]:
        if n <= 400000 and m < (1 << 64):
            assert G.minmax_mod(n, m, a, s) == brute_minmax(n, m, a, s), (n, m, a, s)


@pytest.mark.parametrize("lgm", [50, 55])
def test_minmax_mod_pow2_vs_numpy(lgm):
    """The certificate's actual moduli (2^50 chips, 2^55 LUT cells), long runs, vs numpy."""
    rng = np.random.default_rng(lgm)
    m = 1 << lgm
    for _ in range(60):
        n = int(rng.integers(1, 300000))
        a = int(rng.integers(0, m, dtype=np.uint64))
        s = int(rng.integers(0, m, dtype=np.uint64))
        if rng.random() < 0.3:       # steps near a rational p/q of small q: long clustered runs
            q = int(rng.integers(1, 40))
            s = (m * int(rng.integers(0, q)) // q + int(rng.integers(-1000, 1000))) % m
        p = np.arange(n, dtype=np.uint64)
        v = (np.uint64(a) + p * np.uint64(s)) & np.uint64(m - 1)    # m | 2^64: wrapping is exact
        assert G.minmax_mod(n, m, a, s) == (int(v.min()), int(v.max())), (n, a, s)


def brute_first_below(n, m, a, s, w):
    for p in range(n):
        if (a + p * s) % m < w:
            return p
    return n


def test_first_below_small_vs_brute():
    """The proof's ambiguous-sample search (first_below) against a scan."""
    rng = np.random.default_rng(7)
    for _ in range(4000):
        m = int(rng.integers(1, 3000))
        n = int(rng.integers(0, 2000))
        a, s = int(rng.integers(0, m)), int(rng.integers(0, m))
        w = int(rng.integers(1, m + 1)) if rng.random() < 0.3 else int(rng.integers(1, max(2, m // 50)))
        assert G.first_below(n, m, a, s, w) == brute_first_below(n, m, a, s, w), (n, m, a, s, w)


def _first_below_ref(n, m, a, s, w):
    """smallest p in [0, n) with (a + p s) mod m < w, or n: an independent Python restatement by
    the classic reduction of the modular inequality (exact integers, any size)"""
    a, s = a % m, s % m
    if n <= 0:
        return 0
    if a < w:
        return 0

    def first_in(s, m, lo, hi):              # least x >= 0 with (s x) mod m in [lo, hi], lo > 0
        if s == 0:
            return None
        x = -(-lo // s)
        if s * x <= hi:
            return x
        y = first_in(m % s, s, (-hi) % s, (-lo) % s)   # least y: (m y) mod s in [s - hi%s, ..]
        if y is None:
            return None
        return -(-(lo + m * y) // s)

    x = first_in(s, m, m - a, m - a + w - 1)
    return n if x is None or x >= n else x


def test_first_below_any_n():
    """first_below with run lengths and moduli far beyond a block's (up to 2^62): it ends at
    once, agrees with an independent restatement, and the sample it returns lies in the window
    with no earlier one (checked against the restatement's minimality).  The division on its way
    back up (gss_pf_udiv) then meets quotients of up to ~2^62; it must stay exact there."""
    rng = np.random.default_rng(11)
    for _ in range(300):
        lgm = int(rng.integers(20, 62))
        m = int(rng.integers(1 << (lgm - 1), 1 << lgm))
        n = int(rng.integers(1, 1 << 62)) if rng.random() < 0.7 else int(rng.integers(1, 10**6))
        a, s = int(rng.integers(0, m)), int(rng.integers(1, m))
        w = int(rng.integers(1, max(2, m >> int(rng.integers(1, lgm)))))
        got = G.first_below(n, m, a, s, w)
        want = _first_below_ref(n, m, a, s, w)
        if got == (1 << 64) - 2:             # GSS_PF_GIVE_UP: a descent deeper than 64 levels
            continue
        assert got == want, (n, m, a, s, w)
        if got < n:
            assert (a + got * s) % m < w


@pytest.mark.parametrize("lgm", [50, 55])
def test_first_below_pow2_vs_numpy(lgm):
    """The proof's moduli and window widths (2 D of 2^-34 cycle / 2^-25 chip and wider), runs of a
    whole block, steps near small rationals, vs numpy; and the hits enumerated one after another."""
    rng = np.random.default_rng(100 + lgm)
    m = 1 << lgm
    for _ in range(60):
        n = int(rng.integers(1, 300000))
        a = int(rng.integers(0, m, dtype=np.uint64))
        s = int(rng.integers(0, m, dtype=np.uint64))
        if rng.random() < 0.5:
            q = int(rng.integers(1, 40))
            s = (m * int(rng.integers(0, q)) // q + int(rng.integers(-1000, 1000))) % m
        w = 1 << int(rng.integers(lgm - 40, lgm - 8))
        p = np.arange(n, dtype=np.uint64)
        v = (np.uint64(a) + p * np.uint64(s)) & np.uint64(m - 1)
        hits = np.flatnonzero(v < np.uint64(w))[:8]
        got, p0 = [], 0
        while len(got) < len(hits) + 1 and p0 < n:
            i = G.first_below(n - p0, m, (a + p0 * s) % m, s, w)
            if i >= n - p0:
                break
            got.append(p0 + i)
            p0 += i + 1
        assert got[:len(hits)] == [int(h) for h in hits], (n, a, s, w)
        if len(hits) < 8:
            assert len(got) == len(hits), (n, a, s, w)


def test_hits_mod_three_gaps_vs_brute():
    """The proof's hit enumeration (gss_proof.h hits_mod: first hit by a descent, the rest by the
    three-gap stepping) equals a scan and the one-descent-per-hit loop, over small moduli where
    every gap case, caps and empty ranges occur."""
    rng = np.random.default_rng(77)
    for _ in range(3000):
        lgb = int(rng.choice([4, 6, 8, 10, 12]))
        b = 1 << lgb
        w = int(rng.integers(1, b // 2)) if rng.random() < 0.5 else int(rng.integers(1, b // 32 + 2))
        w = min(w, b // 2 - 1)
        n = int(rng.integers(1, 2000))
        st = int(rng.integers(0, b)) if rng.random() > 0.05 else int(rng.choice([0, 1, b - 1, b // 2]))
        a0 = int(rng.integers(0, b))
        cap = int(rng.choice([1, 3, 8, 64, 400]))
        v = (a0 + np.arange(1, n, dtype=np.int64) * st) % b
        want = (np.flatnonzero(v < w) + 1).tolist()
        want = want if len(want) <= cap else None
        case = (n, lgb, a0, st, w, cap)
        assert G.hits_mod(n, lgb, a0, st, w, cap=cap) == want, case
        assert G.hits_mod(n, lgb, a0, st, w, cap=cap, scan=True) == want, case


@pytest.mark.parametrize("lgb", [40, 55])
def test_hits_mod_pow2_vs_numpy(lgb):
    """hits_mod at the proof's moduli and window widths over runs of a whole block, vs numpy."""
    rng = np.random.default_rng(200 + lgb)
    b = 1 << lgb
    for _ in range(40):
        n = int(rng.integers(1, 600000))
        w = int(rng.integers(1, b >> int(rng.integers(8, 24))))
        st = int(rng.integers(0, b, dtype=np.uint64))
        if rng.random() < 0.5:
            q = int(rng.integers(1, 40))
            st = (b * int(rng.integers(0, q)) // q + int(rng.integers(-1000, 1000))) % b
        a0 = int(rng.integers(0, b, dtype=np.uint64))
        p = np.arange(1, n, dtype=np.uint64)
        v = (np.uint64(a0) + p * np.uint64(st)) & np.uint64(b - 1)
        want = (np.flatnonzero(v < np.uint64(w)) + 1).tolist()
        want = want if len(want) <= 2048 else None
        assert G.hits_mod(n, lgb, a0, st, w, cap=2048) == want, (n, a0, st, w)


# ---------------------------------------------------------------------------------------------
def synth_params(rng, nblk, nch_list, n_per_blk, ties=False, tiny=False, fs=None):
    """random blocks of n_per_blk samples at sample rate fs (realistic Doppler and code rate);
    fs defaults to the reference's 10 n_per_blk (gpssim.c:1877-1881), whose nominal chip rate the
    fast kernel's window table assumes (gss_lin.h, gss_lin_win16_ok)"""
    blk = np.zeros((nblk, G.MAXCH), G.CHAN_DTYPE)
    nch = np.array(nch_list, np.int32)
    delt = 1.0 / (fs if fs is not None else 10.0 * n_per_blk)
    nav = rng.integers(0, 1 << 30, size=(8, 60), dtype=np.uint32)
    for b in range(nblk):
        for k in range(nch[b]):
            f = rng.uniform(-5500, 5500) if (k % 4 or not tiny) else rng.uniform(-40, 40)
            s = f * delt
            if ties and k % 3 == 0:
                u = 2.0 ** -53
                s = math.copysign((math.floor(abs(s) / u) + 0.5) * u, s)
            p = blk[b, k]
            p["carr0"] = [0.0, 1.0 - 2.0 ** -53, rng.random()][k % 3] if b == 0 else rng.random()
            p["carr_step"] = s
            p["code0"] = rng.random() * 1023.0 if k % 5 else 1022.9999999
            p["code_step"] = (1.023e6 + f / 1540.0) * delt
            p["icode"] = rng.integers(0, 20)
            p["ibit"] = rng.integers(0, 30)
            p["iword"] = rng.integers(0, 54)
            p["gain"] = rng.integers(30, 130)
            p["ca_tbl"] = rng.integers(0, 32)
            p["nav_tbl"] = rng.integers(0, 8)
    return blk, nch, nav


@pytest.mark.parametrize("fmt", [16, 8, 1])
@pytest.mark.parametrize("case", ["mixed", "ties_tiny"])
def test_lines_render_like_oracle(fmt, case):
    seed = zlib.crc32(f"{fmt}:{case}".encode())      # stable across processes (no hash())
    rng = np.random.default_rng(seed)
    n = 260000
    nch = [12, 0, 1, 7, 12, 3, 16, 11]
    blk, nchv, nav = synth_params(rng, len(nch), nch, n, ties=case == "ties_tiny",
                                  tiny=case == "ties_tiny")
    ca = G.ca_table()
    lin, fast = G.linearize(blk, nchv, nav, n)
    assert fast.sum() >= len(nch) - 2, (seed, fast)  # the proof rarely fails
    want, rc = oracle.synth(blk, nchv, ca, nav, n, fmt)
    got, nr = render_lin(blk, nchv, lin, fast, ca, n, fmt)
    assert nr == fast.sum()
    bb = G.block_bytes(n, fmt)
    for b in np.nonzero(fast)[0]:
        assert np.array_equal(got[b * bb:(b + 1) * bb], want[b * bb:(b + 1) * bb]), \
            f"seed {seed}: block {b}"


def test_lines_full_blocks_like_oracle():
    """260000-sample blocks (the BASELINE block size): the lines are proven over the whole block."""
    rng = np.random.default_rng(5)
    n = 260000
    blk, nch, nav = synth_params(rng, 3, [12, 12, 9], n)
    ca = G.ca_table()
    lin, fast = G.linearize(blk, nch, nav, n)
    assert fast.all(), fast
    want, _ = oracle.synth(blk, nch, ca, nav, n, 16)
    got, _ = render_lin(blk, nch, lin, fast, ca, n, 16)
    assert np.array_equal(got, want)


def test_lines_real_scenario_vs_reference_golden(golden):
    """The static BASELINE scenario: every block the proof certifies, rendered from its lines,
    has the reference's own block hash."""
    s = G.Scenario(NAV, llh=LOC, duration=10.0, data_format=16)
    blk, nch = s.next(100)
    lin, fast = G.linearize(blk, nch, s.nav_table(), s.n_per_blk)
    assert fast.mean() >= 0.99
    got, _ = render_lin(blk, nch, lin, fast, G.ca_table(), s.n_per_blk, 16)
    bb = G.block_bytes(s.n_per_blk, 16)
    gold = golden["static_d30_b16"]["block_sha16"]
    for i in np.nonzero(fast)[0]:
        assert hashlib.sha256(got[i * bb:(i + 1) * bb].tobytes()).hexdigest()[:16] == gold[i], i


@pytest.mark.parametrize("kw,min_frac", [
    (dict(llh=LOC, duration=300.0, data_format=16), 0.99),
    (dict(llh=LOC, duration=30.0, samp_freq=2.0e7, data_format=16), 0.97),
])
def test_certified_fraction(kw, min_frac):
    s = G.Scenario(NAV, **kw)
    blk, nch = s.all_blocks(batch=1000)
    lin, fast = G.linearize(blk, nch, s.nav_table(), s.n_per_blk)
    frac = fast.mean()
    print(f"certified {fast.sum()}/{len(fast)} blocks ({frac:.4f})")
    assert frac >= min_frac


# ---------------------------------------------------------------------------------------------
def boundary_params(nb=36, n=260000, fs=2.6e6, seed=11):
    """One-channel blocks whose code reaches 1023 (a wrap that starts a new data bit) and whose
    carrier reaches a LUT cell boundary at one sample each, within about 1e-11 of the real line:
    there the exact values may fall on either side of the line's."""
    rng = np.random.default_rng(seed)
    blk = np.zeros((nb, G.MAXCH), G.CHAN_DTYPE)
    nch = np.ones(nb, np.int32)
    nav = rng.integers(0, 1 << 30, size=(2, 60), dtype=np.uint32)
    eps = [0.0, 1e-12, -1e-12, 1e-11, -1e-11, 3e-13]
    for b in range(nb):
        p = blk[b, 0]
        f = rng.uniform(-4000, 4000)
        cs, s = (1.023e6 + f / 1540.0) / fs, f / fs
        q = int(rng.integers(100, 2500))
        p["code0"], p["code_step"] = 1023.0 - q * cs + eps[b % 6], cs
        qc = int(rng.integers(1, n))
        c = (int(rng.integers(0, 512)) / 512.0 - qc * s + eps[(b // 6) % 6]) % 1.0
        p["carr0"], p["carr_step"] = (c if c < 1.0 else 0.0), s
        p["icode"], p["ibit"], p["iword"] = 19, int(rng.integers(0, 30)), int(rng.integers(0, 50))
        p["gain"], p["ca_tbl"], p["nav_tbl"] = 100, int(rng.integers(0, 32)), b % 2
    return blk, nch, nav, n


def test_boundary_samples_like_oracle():
    blk, nch, nav, n = boundary_params()
    lin, fast = G.linearize(blk, nch, nav, n)
    unused = np.iinfo(np.int32).max
    npatched = int((lin["ppos"][:, 0, 0] != unused).sum())
    print(f"certified {int(fast.sum())}/{len(fast)}, {npatched} channels patched")
    assert fast.sum() >= len(fast) - 2
    assert npatched > 0
    ca = G.ca_table()
    want, _ = oracle.synth(blk, nch, ca, nav, n, 16)
    got, _ = render_lin(blk, nch, lin, fast, ca, n, 16)
    bb = G.block_bytes(n, 16)
    for b in np.nonzero(fast)[0]:
        assert np.array_equal(got[b * bb:(b + 1) * bb], want[b * bb:(b + 1) * bb]), f"block {b}"


def test_patched_real_blocks_vs_reference_golden(golden):
    """20 MS/s blocks of the static scenario that carry patches, rendered with them, have the
    reference's own block hashes."""
    s = G.Scenario(NAV, llh=LOC, duration=30.0, samp_freq=2.0e7, data_format=16)
    blk, nch = s.all_blocks(batch=1000)
    lin, fast = G.linearize(blk, nch, s.nav_table(), s.n_per_blk)
    unused = np.iinfo(np.int32).max
    patched = [int(b) for b in np.nonzero(fast)[0] if (lin[b]["ppos"] != unused).any()]
    print(f"{len(patched)} of {int(fast.sum())} certified blocks carry patches")
    assert patched
    sel = np.array(patched[:3])
    got, _ = render_lin(blk[sel], nch[sel], lin[sel], fast[sel], G.ca_table(), s.n_per_blk, 16)
    bb = G.block_bytes(s.n_per_blk, 16)
    gold = golden["static_d30_s20M_b16"]["block_sha16"]
    for i, b in enumerate(sel):
        assert hashlib.sha256(got[i * bb:(i + 1) * bb].tobytes()).hexdigest()[:16] == gold[b], b


# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,fs,nb", [("intcarr_static_d30_b16", 2.6e6, 40),
                                        ("intcarr_static_d30_s20M_b1", 2.0e7, 6)])
def test_integer_carrier_lines_vs_reference_golden(golden, name, fs, nb):
    """--carrier=int: the chain is exact (multiples of 2^-25 cycle), so the proof certifies every
    block with no ambiguous carrier sample, and the render model reproduces the reference built
    with FLOAT_CARR_PHASE off (gpssim.h:4), block for block."""
    g = golden[name]
    s = G.Scenario(NAV, llh=LOC, duration=30.0, samp_freq=fs, data_format=g["fmt"],
                   carrier="int")
    blk, nch = s.next(nb)
    lin, fast = G.linearize(blk, nch, s.nav_table(), s.n_per_blk)
    assert fast.all(), fast
    got, _ = render_lin(blk, nch, lin, fast, G.ca_table(), s.n_per_blk, g["fmt"])
    bb = G.block_bytes(s.n_per_blk, g["fmt"])
    for i in range(nb):
        assert hashlib.sha256(got[i * bb:(i + 1) * bb].tobytes()).hexdigest()[:16] == \
            g["block_sha16"][i], i


def test_integer_carrier_on_cell_boundaries_like_oracle():
    """Exact integer chains that sit exactly on LUT cell boundaries at many samples (steps with
    large powers of two, starts on a boundary): every block certified, bytes equal the oracle's
    (patches come only from the code chain here)."""
    rng = np.random.default_rng(17)
    n = 260000
    blk, nch, nav = synth_params(rng, 4, [12, 12, 12, 12], n)
    one = float(1 << 25)
    for b in range(4):
        for k in range(12):
            p = blk[b, k]
            step = int(rng.integers(-20000, 20000)) & ~((1 << (4 * (k % 4))) - 1)
            p["carr_step"] = step / one
            p["carr0"] = (int(rng.integers(0, 512)) << 16) / one if k % 2 else \
                int(rng.integers(0, 1 << 25)) / one
    lin, fast = G.linearize(blk, nch, nav, n)
    assert fast.all(), fast
    ca = G.ca_table()
    want, _ = oracle.synth(blk, nch, ca, nav, n, 16)
    got, _ = render_lin(blk, nch, lin, fast, ca, n, 16)
    assert np.array_equal(got, want)


def test_gain_bound_of_the_mfma_operand():
    """The fast kernel's gains are f16 MFMA operands (gss_synth.hip, LIN_MFMA): the proof
    certifies a block only when every |gain| <= 1024, so that the gain and its doubled
    data-bit difference are exact f16 integers; larger gains go to the exact path."""
    rng = np.random.default_rng(7)
    n = 260000
    blk, nch, nav = synth_params(rng, 4, [7, 7, 7, 3], n)
    blk[0, :7]["gain"] = 1024                          # sum 7168 <= 8000: certified
    blk[1, :7]["gain"] = -1024
    blk[2, 2]["gain"] = 1025                           # one channel above the bound
    blk[3, 0]["gain"] = -1025
    _, fast = G.linearize(blk, nch, nav, n)
    assert list(fast) == [1, 1, 0, 0]
