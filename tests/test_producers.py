"""The 30 s producers of SURVEY §8 row f3 as the GPU runs them (csrc/common/gss_nav.h): the C/A
table from the two shift registers, and every nav-table row rebuilt from its compact source
(subframe data words, TOW count, week, and the previous frame's row or its given words), against
the host plane's own table, word for word: static 300 s (nine 30 s updates), circle.csv (channel
re-allocation), and a seek into the run (the first rows after a seek carry their head words).
The device kernels are compared with the same host results in tests/test_gpu_parity.py."""
import os

import numpy as np
import pytest

import gpssim_amd as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAV = os.path.join(REPO, "tests", "golden", "data", "brdc3540.14n")
CIRCLE = os.path.join(REPO, "tests", "golden", "data", "circle.csv")
LOC = (30.286502, 120.032669, 100.0)


def _rows_from_sources(s):
    src = s.nav_sources()
    want = s.nav_table()
    assert len(src) == len(want)
    return src, want


@pytest.mark.parametrize("kw", [
    dict(llh=LOC, duration=300.0),
    dict(motion_file=CIRCLE, duration=300.0, data_format=8),
])
def test_nav_rows_from_sources(kw):
    s = G.Scenario(NAV, **kw)
    s.all_blocks(batch=500, threads=2)
    src, want = _rows_from_sources(s)
    assert (src["prev"] == G.NAV_HEAD_INIT).any() and (src["prev"] >= 0).any()
    # chains: next is the inverse of prev
    for r, (p, nx) in enumerate(zip(src["prev"], src["next"])):
        if p >= 0:
            assert p < r and src["next"][p] == r
        if nx >= 0:
            assert src["prev"][nx] == r
    got = G.nav_rows_host(src)
    assert np.array_equal(got, want)
    # in pieces, as gss_run builds them slot by slot
    cut = len(src) // 3
    part = G.nav_rows_host(src[:cut])
    got2 = G.nav_rows_host(src[cut:], first=cut, rows=part)
    assert np.array_equal(got2, want)


def test_nav_rows_after_seek():
    s = G.Scenario(NAV, llh=LOC, duration=120.0)
    s.seek(650, threads=2)                       # past two 30 s updates
    s.next_deferred(400, threads=2)
    src, want = _rows_from_sources(s)
    assert (src["prev"] == G.NAV_HEAD_GIVEN).any()
    assert np.array_equal(G.nav_rows_host(src), want)


def test_ca_table_from_registers():
    """the shared register code (gss_nav.h) gives the host table (itself pinned to the IS-GPS-200
    first-10-chip octal heads in test_oracle.py)"""
    ca = G.ca_table()
    assert ca.shape == (32, G.CA_WORDS)
    # chip 1023 (padding) is zero in every row
    assert not (ca[:, -1] >> 31).any()
