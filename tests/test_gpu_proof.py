"""The fast path's proofs on the GPU (gss_linearize_device, csrc/hip/gss_proof.hip) against the
host's gss_linearize, byte for byte: the same per-channel proof (csrc/common/gss_proof.h) compiled
for both sides must give the same lines, gain schedules, patches and fast flags -- on the
reference scenarios, on synthetic rows that exercise the boundary cases (ambiguous samples,
patches, gain changes, ragged block lengths) and on rows the proof must reject (the rows after
a block's first failing channel keep the host's initial state)."""
import numpy as np
import pytest

from conftest import CIRCLE, LOC, NAV
from test_linearize import boundary_params, synth_params

import gpssim_amd as G

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    d = G.Device(0)
    yield d
    d.close()


def device_proof(dev, blk, nch, nav, n, anch=None):
    t = torch.device("cuda", 0)
    ca = G.ca_table()

    def up(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(t)
    d_blk, d_nch = up(np.ascontiguousarray(blk, G.CHAN_DTYPE)), up(np.asarray(nch, np.int32))
    d_ca, d_nav = up(ca), up(np.ascontiguousarray(nav, np.uint32))
    nb = len(nch)
    d_lin = torch.full((nb * G.MAXCH * G.LIN_DTYPE.itemsize,), 0xA5, dtype=torch.uint8, device=t)
    d_fast = torch.full((nb * 4,), 0x5A, dtype=torch.uint8, device=t)
    d_anch = up(np.ascontiguousarray(anch, G.ANCHOR_DTYPE)) if anch is not None else None
    dev.linearize_device(d_blk.data_ptr(), d_nch.data_ptr(), nb, n, d_ca.data_ptr(), len(ca),
                         d_nav.data_ptr(), len(nav), d_lin.data_ptr(), d_fast.data_ptr(),
                         torch.cuda.current_stream(t).cuda_stream,
                         anch_ptr=d_anch.data_ptr() if d_anch is not None else None)
    torch.cuda.synchronize(t)
    lin = d_lin.cpu().numpy().view(G.LIN_DTYPE).reshape(nb, G.MAXCH)
    fast = d_fast.cpu().numpy().view(np.int32)
    return lin, fast


def check_same(dev, blk, nch, nav, n, anch=None):
    want_lin, want_fast = G.linearize(blk, nch, nav, n)
    got_lin, got_fast = device_proof(dev, blk, nch, nav, n, anch)
    assert np.array_equal(got_fast, want_fast), np.nonzero(got_fast != want_fast)[0][:10]
    a, b = want_lin.view(np.uint8).reshape(len(nch), -1), got_lin.view(np.uint8).reshape(len(nch), -1)
    bad = np.nonzero((a != b).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} blocks' rows differ, first {bad[:5]}"
    return want_fast


@pytest.mark.parametrize("case", ["static", "circle", "fs20", "b1_late", "carrier_int"])
def test_proof_device_equals_host_scenarios(dev, case):
    kw = {"llh": LOC}
    dur, fs, fmt, seek = 120.0, 2.6e6, 16, 0
    if case == "circle":
        kw = {"motion_file": CIRCLE}
    elif case == "fs20":
        dur, fs = 20.0, 2.0e7
    elif case == "b1_late":
        dur, fmt, seek = 7200.0, 1, 71000           # blocks past two hours into the run
    elif case == "carrier_int":
        kw["carrier"] = "int"
    s = G.Scenario(NAV, duration=dur, samp_freq=fs, data_format=fmt, **kw)
    if seek:
        s.seek(seek)
        s.set_carrier(np.linspace(0.05, 0.95, G.MAXCH))  # any start phases: a proof input
        blk, nch = s.next(600, 8)[:2]
    else:
        blk, nch = s.all_blocks(batch=2000, threads=8)
    fast = check_same(dev, blk, nch, s.nav_table(), s.n_per_blk)
    assert fast.sum() >= len(nch) * 0.95


@pytest.mark.parametrize("fs,dur", [(2.6e6, 300.0), (2.0e7, 30.0)])
def test_proof_device_with_anchors_equals_host(dev, fs, dur):
    """gss_linearize_device_ex: the proofs' carrier walks start at the chain's anchors
    (gss_carr_chain_anchored, exact values at the segment starts), on the device as on the host:
    the same rows, byte for byte, as the host's proofs without them."""
    s = G.Scenario(NAV, llh=LOC, duration=dur, samp_freq=fs)
    n = s.n_per_blk
    c0 = s.carrier()
    blk, nch, chain = s.next_deferred(int(dur * 10), threads=8)
    gi = G.carr_chain_guess(c0, blk, nch, chain, n, starts_only=True)
    spec = G.spec_host(gi, n, threads=8)
    _, _, anch = G.carr_chain_anchored(c0, blk, nch, chain, n, gi, spec)
    nav = s.nav_table()
    host_lin, host_fast = G.linearize(blk, nch, nav, n, anch=anch)
    want_lin, want_fast = G.linearize(blk, nch, nav, n)
    assert host_lin.tobytes() == want_lin.tobytes() and host_fast.tobytes() == want_fast.tobytes()
    fast = check_same(dev, blk, nch, nav, n, anch)
    assert fast.sum() >= len(nch) * 0.95


@pytest.mark.parametrize("n", [260000, 260004, 2000000])
def test_proof_device_equals_host_synthetic(dev, n):
    rng = np.random.default_rng(n + 5)
    nchs = [12, 0, 1, 7, 12, 16, 16, 3] if n < 1000000 else [12, 11, 9]
    blk, nch, nav = synth_params(rng, len(nchs), nchs, n)
    check_same(dev, blk, nch, nav, n)


def test_proof_device_equals_host_boundaries(dev):
    """rows placed on cell and chip boundaries: ambiguous samples, exact walks and patches"""
    blk, nch, nav, n = boundary_params(24, 260000)
    check_same(dev, blk, nch, nav, n)


def test_proof_device_rejects_like_host(dev):
    """rejections at every position of the channel loop: the block's fast flag and all its rows
    (proven, failing, and never reached) as the host leaves them"""
    rng = np.random.default_rng(3)
    n = 260000
    blk, nch, nav = synth_params(rng, 6, [12, 12, 5, 12, 3, 9], n)
    blk[0, 3]["code_step"] = 0.9                      # beyond the kernel's chip window
    blk[1, 0]["gain"] = 1500                          # not an exact f16 operand (|g| > 1024)
    blk[2, 4]["nav_tbl"] = 10 ** 6                    # no such nav row
    blk[3, 11]["ca_tbl"] = -1                         # no such C/A row
    for k in range(9):
        blk[5, k]["gain"] = 1000                      # sum |gain| > 8000
    fast = check_same(dev, blk, nch, nav, n)
    assert not fast[[0, 1, 2, 3, 5]].any()


@pytest.mark.parametrize("stride", ["4", "16", "32"])
def test_proof_device_every_lane_stride(dev, stride, monkeypatch):
    """every launch shape of the proof kernel (threads per channel slot, proof_stride; forced
    here by GSS_PROOF_STRIDE, read per launch) gives the host's rows: rejections, ragged channel
    counts, boundary rows and 20 MS/s blocks with anchors"""
    monkeypatch.setenv("GSS_PROOF_STRIDE", stride)
    rng = np.random.default_rng(3)
    n = 260000
    blk, nch, nav = synth_params(rng, 6, [12, 12, 5, 12, 3, 9], n)
    blk[0, 3]["code_step"] = 0.9
    blk[1, 0]["gain"] = 1500
    blk[2, 4]["nav_tbl"] = 10 ** 6
    blk[3, 11]["ca_tbl"] = -1
    for k in range(9):
        blk[5, k]["gain"] = 1000
    fast = check_same(dev, blk, nch, nav, n)
    assert not fast[[0, 1, 2, 3, 5]].any()
    blk, nch, nav, n = boundary_params(24, 260000)
    check_same(dev, blk, nch, nav, n)
    s = G.Scenario(NAV, llh=LOC, duration=6.0, samp_freq=2.0e7)
    n = s.n_per_blk
    c0 = s.carrier()
    blk, nch, chain = s.next_deferred(60, threads=8)
    gi = G.carr_chain_guess(c0, blk, nch, chain, n, starts_only=True)
    spec = G.spec_host(gi, n, threads=8)
    _, _, anch = G.carr_chain_anchored(c0, blk, nch, chain, n, gi, spec)
    fast = check_same(dev, blk, nch, s.nav_table(), n, anch)
    assert fast.sum() >= len(nch) * 0.95
