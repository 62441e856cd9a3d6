"""GPU parity of the certified fast path (gss_lin_kernel via gss_synth_host / gss_synth_lin_device)
against the scalar oracle of the reference loop and the reference's golden hashes.

gss_synth_host takes the fast path by default (test_gpu_parity.py therefore covers it on every
scenario); these cases pin it on realistic sample rates, ragged block lengths, all formats and
the mixed batches where some blocks are certified and others go through the exact path in the
same call, and check that the fast kernel really ran.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import LOC, NAV
from test_linearize import boundary_params, synth_params

import gpssim_amd as G
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    d = G.Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("fmt", [16, 8, 1])
@pytest.mark.parametrize("n", [260000, 260004, 2000000])
def test_lin_synthetic_vs_oracle(dev, fmt, n):
    rng = np.random.default_rng(n * 31 + fmt)
    nch = [12, 0, 1, 7, 12, 16] if n < 1000000 else [12, 11]
    blk, nchv, nav = synth_params(rng, len(nch), nch, n)
    ca = G.ca_table()
    lin, fast = G.linearize(blk, nchv, nav, n)
    assert fast.sum() >= len(nch) - 1
    want, rc = oracle.synth(blk, nchv, ca, nav, n, fmt)
    assert rc == 0
    dev.timing_reset()
    got = dev.synth_host(blk, nchv, ca, nav, n, fmt)
    n_lin, _ = dev.timing_lin()
    assert n_lin == 1                                  # the fast kernel ran
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"


def test_lin_mixed_batch_with_exact_leftovers(dev):
    """Blocks the proof rejects (here: a code step too large for the fast kernel's chip window,
    and a start phase on a cell boundary forced uncertifiable) take the exact path inside the
    same call; all bytes equal the oracle's."""
    rng = np.random.default_rng(11)
    n = 260000
    blk, nch, nav = synth_params(rng, 6, [12, 12, 5, 12, 3, 9], n)
    blk[1, 3]["code_step"] = 0.9                      # 127 * 0.9 chips > the 64-chip window
    blk[4, 0]["gain"] = 9000                          # > packed accumulator range
    ca = G.ca_table()
    lin, fast = G.linearize(blk, nch, nav, n)
    assert fast[1] == 0 and fast[4] == 0 and fast.sum() >= 3
    want, _ = oracle.synth(blk, nch, ca, nav, n, 16)
    got = dev.synth_host(blk, nch, ca, nav, n, 16)
    assert np.array_equal(got, want)


def test_walk_path_env_still_exact(dev, monkeypatch):
    rng = np.random.default_rng(3)
    n = 26000
    blk, nch, nav = synth_params(rng, 3, [12, 7, 12], n)
    ca = G.ca_table()
    want, _ = oracle.synth(blk, nch, ca, nav, n, 8)
    monkeypatch.setenv("GSS_PATH", "walk")
    dev.timing_reset()
    got = dev.synth_host(blk, nch, ca, nav, n, 8)
    assert dev.timing_lin()[0] == 0
    assert np.array_equal(got, want)


def test_lin_device_entry_scenario(dev, golden):
    """gss_synth_lin_device with device-resident inputs as bench.py drives it, on 10 s of the
    static BASELINE scenario, against the reference's golden block hashes."""
    import torch
    dev_t = torch.device("cuda", 0)
    s = G.Scenario(NAV, llh=LOC, duration=10.0, data_format=16)
    blk, nch, ck = s.next(200, with_ck=True)
    nav = s.nav_table()
    ca = G.ca_table()
    npb = s.n_per_blk
    lin, fast = G.linearize(blk, nch, nav, npb)
    fb = np.nonzero(fast == 0)[0].astype(np.int32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev_t)   # noqa: E731
    d_blk, d_nch, d_ck = t(blk.view(np.uint8).reshape(-1)), t(nch), t(ck)
    d_lin, d_fast = t(lin.view(np.uint8).reshape(-1)), t(fast)
    d_fb = t(fb if len(fb) else np.zeros(1, np.int32))
    d_ca, d_nav = t(ca.view(np.int32)), t(nav.view(np.int32))
    bb = G.block_bytes(npb, 16)
    out = torch.empty(len(nch) * bb, dtype=torch.uint8, device=dev_t)
    dev.synth_lin_device(d_blk.data_ptr(), d_nch.data_ptr(), int(nch.max()), d_lin.data_ptr(),
                         d_fast.data_ptr(), d_fb.data_ptr(), len(fb), d_ca.data_ptr(), len(ca),
                         d_nav.data_ptr(), len(nav), len(nch), npb, 16, out.data_ptr(),
                         stream=torch.cuda.current_stream(dev_t).cuda_stream,
                         ck_ptr=d_ck.data_ptr())
    torch.cuda.synchronize(dev_t)
    o = out.cpu().numpy()
    hs = [hashlib.sha256(o[i * bb:(i + 1) * bb].tobytes()).hexdigest()[:16]
          for i in range(len(nch))]
    assert hs == golden["static_d30_b16"]["block_sha16"][:len(nch)]


def test_lin_patched_samples_vs_oracle(dev):
    """Code wraps (starting new data bits) and carrier cells placed within about 1e-11 of the
    line: the kernel applies the exact values the proof found (patches); bytes equal the
    oracle's."""
    blk, nch, nav, n = boundary_params()
    lin, fast = G.linearize(blk, nch, nav, n)
    assert (lin["ppos"][fast.astype(bool)] != np.iinfo(np.int32).max).any()
    ca = G.ca_table()
    want, _ = oracle.synth(blk, nch, ca, nav, n, 16)
    dev.timing_reset()
    got = dev.synth_host(blk, nch, ca, nav, n, 16)
    assert dev.timing_lin()[0] == 1
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"


@pytest.mark.parametrize("fmt", [16, 8, 1])
def test_lin_mfma_sum_extremes_vs_oracle(dev, fmt):
    """The largest certified sums: 7 channels at |gain| 1024 (sum 7168, |sum I| up to 1.8 M),
    mixed signs and data-bit flips, against the oracle's integer loop: the matrix cores' f32
    sums from 1.5 2^23 + 64 stay exact integers and the packing from the f32 bits is the
    reference's (sum + 64) >> 7 (gpssim.c:2257-2287)."""
    rng = np.random.default_rng(1024 + fmt)
    n = 260004
    blk, nch, nav = synth_params(rng, 4, [7, 7, 7, 12], n)
    blk[0, :7]["gain"] = 1024
    blk[1, :7]["gain"] = [1024, -1024, 1024, -1024, 1000, -999, 1]
    blk[2, :7]["gain"] = -1024
    ca = G.ca_table()
    _, fast = G.linearize(blk, nch, nav, n)
    assert fast.sum() >= 3
    want, rc = oracle.synth(blk, nch, ca, nav, n, fmt)
    assert rc == 0
    got = dev.synth_host(blk, nch, ca, nav, n, fmt)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:5]}"
