"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference's golden
outputs.  Bit-exact everywhere (integer/byte output of exact double recurrences).

* synthetic parameter sweeps vs the scalar oracle (gpssim.c:2190-2288 restated), including the
  edge cases the reference can reach: 0 and 16 channels, both Doppler signs, tiny Doppler,
  round-half-even ties, large gains, ragged blocks, carrier phase 0 and just below 1;
* real scenarios (BASELINE.json configs) vs the golden sha256 of the reference binary;
* checkpoint-stage carrier end phases vs the host planner's next-block start phases;
* the CLI end to end.
"""
import hashlib
import math
import os
import subprocess
import tempfile
import zlib

import numpy as np
import pytest

from conftest import CIRCLE, LOC, NAV

import gpssim_amd as G
import oracle

pytestmark = pytest.mark.gpu

DELT = 1.0 / 2600000.0


@pytest.fixture(scope="module")
def dev():
    d = G.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="module")
def ca():
    return G.ca_table()


def synth_params(rng, nblk, nch_list, n_per_blk, big_gain=False, ties=False):
    blk = np.zeros((nblk, G.MAXCH), G.CHAN_DTYPE)
    nch = np.array(nch_list, np.int32)
    delt = 1.0 / (n_per_blk * 10)
    nav = rng.integers(0, 1 << 30, size=(8, 60), dtype=np.uint32)
    for b in range(nblk):
        for k in range(nch[b]):
            f = rng.uniform(-5500, 5500) if k % 4 else rng.uniform(-40, 40)
            cs = (1.023e6 + f / 1540.0) * delt
            s = f * delt
            if ties and k % 3 == 0:
                u = 2.0 ** -53
                s = math.copysign((math.floor(abs(s) / u) + 0.5) * u, s)
            p = blk[b, k]
            p["carr0"] = [0.0, 1.0 - 2.0 ** -53, rng.random()][k % 3] if b == 0 else rng.random()
            p["carr_step"] = s
            p["code0"] = rng.random() * 1023.0 if k % 5 else 1022.9999999
            p["code_step"] = cs
            p["icode"] = rng.integers(0, 20)
            p["ibit"] = rng.integers(0, 30)
            p["iword"] = rng.integers(0, 54)
            p["gain"] = rng.integers(2000, 9000) if big_gain else rng.integers(30, 130)
            p["ca_tbl"] = rng.integers(0, 32)
            p["nav_tbl"] = rng.integers(0, 8)
    return blk, nch, nav


@pytest.mark.parametrize("fmt", [16, 8, 1])
@pytest.mark.parametrize("case", ["mixed", "full16", "ties_biggain", "ragged"])
def test_synthetic_vs_oracle(dev, ca, fmt, case):
    seed = zlib.crc32(f"{fmt}:{case}".encode())      # stable across processes (no hash())
    rng = np.random.default_rng(seed)
    n = 26000
    if case == "mixed":
        nch = [12, 0, 1, 7, 12, 3]
        kw = {}
    elif case == "full16":
        nch = [16, 16, 16]
        kw = {}
    elif case == "ties_biggain":
        nch = [12, 12, 5]
        kw = dict(big_gain=True, ties=True)
    else:
        n = 26004 if fmt == 1 else 26003          # last segment is ragged
        nch = [11, 4, 11]
        kw = {}
    blk, nchv, nav = synth_params(rng, len(nch), nch, n, **kw)
    want, rc = oracle.synth(blk, nchv, ca, nav, n, fmt)
    assert rc == 0, f"oracle rc {rc} (seed {seed})"
    got = dev.synth_host(blk, nchv, ca, nav, n, fmt)
    assert got.shape == want.shape, f"seed {seed}"
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"seed {seed}: {bad.size} bytes differ, first at {bad[:5]}"


def test_carr_end_matches_oracle(dev, ca):
    rng = np.random.default_rng(7)
    blk, nch, nav = synth_params(rng, 4, [12, 9, 16, 2], 260000, ties=True)
    want, cend_o, rc = oracle.synth(blk, nch, ca, nav, 260000, 16, want_carr_end=True)
    got, cend_g = dev.synth_host(blk, nch, ca, nav, 260000, 16, want_carr_end=True)
    assert np.array_equal(got, want)
    for b in range(4):
        assert np.array_equal(cend_g[b, :nch[b]], cend_o[b, :nch[b]])


def run_scenario(dev, batch=300, use_ck=True, **kw):
    """The product path: host plane -> (planner carrier checkpoints) -> GPU, block hashes."""
    s = G.Scenario(NAV, **kw)
    ca = G.ca_table()
    h = hashlib.sha256()
    blocks = []
    bb = G.block_bytes(s.n_per_blk, s.data_format)
    total = 0
    while True:
        if use_ck:
            blk, nch, ck = s.next(batch, with_ck=True)
        else:
            (blk, nch), ck = s.next(batch), None
        if len(nch) == 0:
            break
        out = dev.synth_host(blk, nch, ca, s.nav_table(), s.n_per_blk, s.data_format, ck=ck)
        h.update(out.tobytes())
        total += out.size
        for i in range(len(nch)):
            blocks.append(hashlib.sha256(out[i * bb:(i + 1) * bb].tobytes()).hexdigest()[:16])
    return h.hexdigest(), total, blocks


@pytest.mark.parametrize("name,kw", [
    ("static_d30_b16", dict(llh=LOC, duration=30.0, data_format=16)),
    ("static_d30_b8", dict(llh=LOC, duration=30.0, data_format=8)),
    ("static_d30_b1", dict(llh=LOC, duration=30.0, data_format=1)),
    ("static_d65_b8_noiono", dict(llh=(-33.8688, 151.2093, 58), duration=65.0, data_format=8,
                                  iono=False)),
    ("ecef_d35_s3M_b16", dict(xyz=(-2700000.0, -4290000.0, 3860000.0), duration=35.0,
                              samp_freq=3.0e6, data_format=16)),
])
def test_scenario_bit_exact(dev, golden, name, kw):
    sha, total, blocks = run_scenario(dev, **kw)
    g = golden[name]
    if blocks != g["block_sha16"]:
        first = next(i for i, (a, b) in enumerate(zip(blocks, g["block_sha16"])) if a != b)
        raise AssertionError(f"{name}: first differing block {first}")
    assert total == g["bytes"] and sha == g["sha256"]


def test_scenario_without_checkpoints(dev, golden):
    """Callers that pass no planner checkpoints (e.g. INTEGRATION.md's gpssim.c patch): the GPU
    walks whole blocks and gets the same bytes."""
    sha, total, blocks = run_scenario(dev, use_ck=False, llh=LOC, duration=30.0, data_format=16)
    g = golden["static_d30_b16"]
    assert blocks == g["block_sha16"]
    assert total == g["bytes"] and sha == g["sha256"]


@pytest.mark.parametrize("name,kw", [
    ("circle_b8", dict(motion_file=CIRCLE, data_format=8)),
    ("static_d300_b16", dict(llh=LOC, duration=300.0, data_format=16)),
    ("static_d30_s20M_b16", dict(llh=LOC, duration=30.0, samp_freq=2.0e7, data_format=16)),
])
def test_baseline_configs_bit_exact(dev, golden, name, kw):
    sha, total, blocks = run_scenario(dev, batch=100, **kw)
    g = golden[name]
    assert blocks == g["block_sha16"]
    assert total == g["bytes"] and sha == g["sha256"]


@pytest.mark.parametrize("name,kw", [
    ("intcarr_static_d30_b16", dict(llh=LOC, duration=30.0, data_format=16)),
    ("intcarr_static_d65_b8", dict(llh=LOC, duration=65.0, data_format=8)),
    ("intcarr_circle_b8", dict(motion_file=CIRCLE, data_format=8)),
    ("intcarr_static_d30_s20M_b1", dict(llh=LOC, duration=30.0, samp_freq=2.0e7, data_format=1)),
])
def test_integer_carrier_bit_exact(dev, golden, name, kw):
    """--carrier=int against the reference built with FLOAT_CARR_PHASE off (gpssim.h:4): the
    integer chain travels as exact doubles, so the same kernels render it"""
    sha, total, blocks = run_scenario(dev, batch=100, carrier="int", **kw)
    g = golden[name]
    if blocks != g["block_sha16"]:
        first = next(i for i, (a, b) in enumerate(zip(blocks, g["block_sha16"])) if a != b)
        raise AssertionError(f"{name}: first differing block {first}")
    assert total == g["bytes"] and sha == g["sha256"]


def test_cli_end_to_end(golden):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "gpssim.bin")
        r = subprocess.run([G.CLI_PATH, "-e", NAV, "-l", ",".join(map(str, LOC)), "-d", "30",
                            "-b", "16", "-o", out], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "Done!" in r.stderr
        h = hashlib.sha256(open(out, "rb").read()).hexdigest()
    assert h == golden["static_d30_b16"]["sha256"]


def test_pipelined_stages_bit_exact(golden):
    """The split ABI as bench.py drives it: Stage A of batch k+1 (anchor set (k+1)%2) on one
    stream while Stage B renders batch k on another, device-resident inputs; every block equals
    the reference's golden hash."""
    import torch
    dev_t = torch.device("cuda", 0)
    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=16)
    batches = [s.next(100, with_ck=True) for _ in range(3)]
    nav = s.nav_table()
    ca = G.ca_table()
    npb = s.n_per_blk
    bb = G.block_bytes(npb, 16)
    d = G.Device(0)
    try:
        d_ca = torch.from_numpy(ca.view(np.int32)).to(dev_t)
        d_nav = torch.from_numpy(nav.view(np.int32)).to(dev_t)
        ins = [(torch.from_numpy(b.view(np.uint8).reshape(-1)).to(dev_t),
                torch.from_numpy(n).to(dev_t), torch.from_numpy(c).to(dev_t), len(n),
                int(n.max())) for b, n, c in batches]
        outs = [torch.empty(x[3] * bb, dtype=torch.uint8, device=dev_t) for x in ins]
        s_a = torch.cuda.Stream(dev_t, priority=-1)
        s_b = torch.cuda.Stream(dev_t)
        ev_a = [torch.cuda.Event() for _ in range(2)]
        ev_b = [torch.cuda.Event() for _ in range(2)]

        def anchor(k):
            b, n, c, nb, nm = ins[k]
            if k >= 2:
                s_a.wait_event(ev_b[k % 2])
            d.anchor_device(k % 2, b.data_ptr(), n.data_ptr(), nm, nb, npb, ck_ptr=c.data_ptr(),
                            stream=s_a.cuda_stream)
            ev_a[k % 2].record(s_a)

        anchor(0)
        for k in range(3):
            b, n, c, nb, nm = ins[k]
            s_b.wait_event(ev_a[k % 2])
            d.render_device(k % 2, b.data_ptr(), n.data_ptr(), nm, d_ca.data_ptr(), len(ca),
                            d_nav.data_ptr(), len(nav), nb, npb, 16, outs[k].data_ptr(),
                            stream=s_b.cuda_stream)
            ev_b[k % 2].record(s_b)
            if k + 1 < 3:
                anchor(k + 1)
        torch.cuda.synchronize(dev_t)
        whole = b"".join(o.cpu().numpy().tobytes() for o in outs)
    finally:
        d.close()
    hashes = [hashlib.sha256(whole[i * bb:(i + 1) * bb]).hexdigest()[:16]
              for i in range(len(whole) // bb)]
    assert hashes == golden["static_d30_b16"]["block_sha16"][:len(hashes)]
    assert len(hashes) == 299


def test_streaming_run_bit_exact(dev, golden):
    """gss_run (planner thread, async copies, pinned sinks): a whole 30 s run in small batches,
    and a block range starting mid-run, against the reference's golden hashes."""
    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=8)
    bb = G.block_bytes(s.n_per_blk, 8)
    h = hashlib.sha256()
    seen = []

    def sink(buf, first, nb):
        assert first == (seen[-1][0] + seen[-1][1] if seen else 0)
        seen.append((first, nb))
        h.update(buf)

    dev.run(s, sink, batch=37, threads=4)
    g = golden["static_d30_b8"]
    assert sum(nb for _, nb in seen) == 299
    assert h.hexdigest() == g["sha256"]

    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=8)
    blocks = []

    def sink2(buf, first, nb):
        for i in range(nb):
            blocks.append((first + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))

    dev.run(s, sink2, first_block=123, n_blocks=61, batch=25)
    assert [b for b, _ in blocks] == list(range(123, 184))
    assert [x for _, x in blocks] == g["block_sha16"][123:184]


@pytest.mark.parametrize("proof", ["gpu", "host", "split", "gpu_late"])
@pytest.mark.parametrize("fmt,every", [(16, 5), (8, 7)])
def test_streaming_run_mixed_exact(dev, golden, monkeypatch, fmt, every, proof):
    """gss_run with every k-th block sent to the exact path (GSS_RUN_FORCE_EXACT, a test hook):
    the planner walks the chain without checkpoints and computes them afterwards for those
    blocks only (fill_fb_ck); with the proofs on the GPU a rejected block renders on the exact
    path in the same launch when its slot's proof is done at submission, else drain renders
    them again (redo_rejected).  The proofs usually finish first, so "gpu_late"
    (GSS_RUN_LATE_VERDICTS=1) forces the redo path on every slot.  Whole run and a mid-run
    range against the golden hashes."""
    monkeypatch.setenv("GSS_RUN_FORCE_EXACT", str(every))
    monkeypatch.setenv("GSS_RUN_PROOF", "gpu" if proof == "gpu_late" else proof)
    monkeypatch.setenv("GSS_RUN_LATE_VERDICTS", "1" if proof == "gpu_late" else "0")
    g = golden[f"static_d30_b{fmt}"]
    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=fmt)
    bb = G.block_bytes(s.n_per_blk, fmt)
    blocks = []

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append((first + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))

    dev.run(s, sink, batch=40, threads=4)
    assert [x for _, x in blocks] == g["block_sha16"]
    blocks.clear()
    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=fmt)
    dev.run(s, sink, first_block=101, n_blocks=77, batch=30)
    assert [b for b, _ in blocks] == list(range(101, 178))
    assert [x for _, x in blocks] == g["block_sha16"][101:178]


@pytest.mark.parametrize("proof", ["host", "gpu", "split"])
def test_streaming_run_rows_ahead_midrun_exact_path(dev, golden, monkeypatch, proof):
    """The rows thread's nav sources are copied when each row is new, before the next frame of
    its channel exists, so a slot that takes many rows at once (a range starting past a 30 s
    update) must rebuild their chains' next links (take_nav_sources) or the device nav table
    misses rows.  The fast path never reads that table; every block on the exact path does."""
    monkeypatch.setenv("GSS_RUN_SPEC", "1")
    monkeypatch.setenv("GSS_RUN_ROWS_AHEAD", "1")
    monkeypatch.setenv("GSS_RUN_FORCE_EXACT", "1")
    monkeypatch.setenv("GSS_RUN_PROOF", proof)
    g = golden["static_d65_b8_noiono"]
    blocks = []
    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    bb = G.block_bytes(s.n_per_blk, 8)

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append((first + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))

    dev.run(s, sink, first_block=333, n_blocks=150, batch=64)
    assert [b for b, _ in blocks] == list(range(333, 483))
    assert [x for _, x in blocks] == g["block_sha16"][333:483]


@pytest.mark.parametrize("world,handoff,gold,args", [
    # every rank plans the blocks before its range itself (no run id)
    (2, False, "static_d30_b16", ["-l", ",".join(map(str, LOC)), "-d", "30", "-b", "16"]),
    # planned once per node: rank 1 seeks to block 324, past the 30 s update after block 299,
    # and takes the slot carriers there from rank 0's hand-off file (gss_run_ex)
    (2, True, "static_d65_b8_noiono", ["-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8", "-i"]),
    # three ranks: rank 1 both receives (block 216) and hands on (block 432)
    (3, True, "static_d65_b8_noiono", ["-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8", "-i"]),
    # the same without the chain speculated across the ranks (GSS_HANDOFF_SPEC=0)
    (3, "nospec", "static_d65_b8_noiono",
     ["-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8", "-i"]),
    # four ranks over 30 s -b 16 (a map composed of three)
    (4, True, "static_d30_b16", ["-l", ",".join(map(str, LOC)), "-d", "30", "-b", "16"]),
])
def test_cli_two_ranks_one_file(golden, world, handoff, gold, args):
    """The CLI as several ranks (RANK/WORLD_SIZE, all on GPU 0 here): each pwrite()s its block
    range into the same file, which equals the single-process reference output.  With a run id
    the ranks hand the slot carriers on through files and, by default, speculate the chain across
    the ranks first (two rounds of map files, gss_run_opts_t.carr_predict); every file is consumed
    or removed by the end."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "gpssim.bin")
        procs = []
        for r in range(world):
            env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK="0")
            env.pop("TORCHELASTIC_RUN_ID", None)
            env.pop("GSS_RUN_ID", None)
            env.pop("GSS_HANDOFF_SPEC", None)
            if handoff:
                env["GSS_RUN_ID"] = "t%d" % os.getpid()
                env["GSS_RUN_FORCE_EXACT"] = "9"     # + the hand-off path's lazy checkpoints
            if handoff == "nospec":
                env["GSS_HANDOFF_SPEC"] = "0"
            procs.append(subprocess.Popen(
                [G.CLI_PATH, "-e", NAV] + args + ["-o", out], env=env,
                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
        for p in procs:
            _, err = p.communicate(timeout=300)
            assert p.returncode == 0, err[-2000:]
        h = hashlib.sha256(open(out, "rb").read()).hexdigest()
        left = [f for f in os.listdir(td) if f != "gpssim.bin"]
    assert h == golden[gold]["sha256"]
    assert left == [], left                      # the hand-off and map files are gone


def test_cli_handoff_ignores_a_stale_file(golden):
    """torchrun's default run id is "none" for every launch: a hand-off file (and speculation map
    files) an interrupted earlier run left at the same path (here: junk carriers, another
    scenario's fingerprint) is not consumed; rank 1 waits for rank 0's own files and the output
    is the reference's."""
    import struct
    args = ["-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8", "-i"]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "gpssim.bin")
        first = (int(round(65 * 10)) - 1) // 2          # rank 1's first block
        stale = f"{out}.gss-carr-none-{first}"
        with open(stale, "wb") as f:
            f.write(struct.pack("<IQ", 0x67737364, 0x0123456789ABCDEF) +
                    struct.pack("<16d", *([0.25] * 16)))
        for rnd in (0, 1):                      # and rank 0's speculation maps, both rounds
            with open(f"{out}.gss-map-none-{rnd}-0", "wb") as f:
                f.write(struct.pack("<IQ", 0x6773736d, 0x0123456789ABCDEF) +
                        struct.pack("<48d", *([0.5] * 48)))
        procs = []
        for r in range(2):
            env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0",
                       TORCHELASTIC_RUN_ID="none")
            env.pop("GSS_RUN_ID", None)
            procs.append(subprocess.Popen(
                [G.CLI_PATH, "-e", NAV] + args + ["-o", out], env=env,
                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
        for p in procs:
            _, err = p.communicate(timeout=300)
            assert p.returncode == 0, err[-2000:]
        h = hashlib.sha256(open(out, "rb").read()).hexdigest()
        left = [f for f in os.listdir(td) if f != "gpssim.bin"]
    assert h == golden["static_d65_b8_noiono"]["sha256"]
    assert left == [], left


def test_cli_handoff_speculation_mismatch_fails_fast():
    """Ranks that disagree on speculating the carrier chain: rank 0 runs with GSS_RUN_SPEC=0
    (so the library rules speculation out and publishes no maps), rank 1 with the default.  Rank
    0 writes no-speculation markers in place of its maps (carr_predict round -1) and rank 1 stops
    at once with a message naming the settings, instead of polling for maps until the hand-off
    timeout."""
    import time
    args = ["-l", "-33.8688,151.2093,58", "-d", "20", "-b", "8", "-i"]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "gpssim.bin")
        procs = []
        t0 = time.perf_counter()
        for r in range(2):
            env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0",
                       GSS_RUN_ID="m%d" % os.getpid(), GSS_HANDOFF_TIMEOUT="600")
            env.pop("TORCHELASTIC_RUN_ID", None)
            env.pop("GSS_HANDOFF_SPEC", None)
            env.pop("GSS_RUN_SPEC", None)
            if r == 0:
                env["GSS_RUN_SPEC"] = "0"
            procs.append(subprocess.Popen(
                [G.CLI_PATH, "-e", NAV] + args + ["-o", out], env=env,
                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE))
        errs = [p.communicate(timeout=300)[1].decode(errors="replace") for p in procs]
        dt = time.perf_counter() - t0
    assert procs[0].returncode == 0, errs[0][-2000:]
    assert procs[1].returncode != 0
    assert "does not speculate" in errs[1], errs[1][-2000:]
    assert dt < 120


def test_streaming_run_walk_path(dev, golden, monkeypatch):
    """gss_run with GSS_PATH=walk (the exact path for every block): the same bytes."""
    monkeypatch.setenv("GSS_PATH", "walk")
    s = G.Scenario(NAV, llh=LOC, duration=30.0, data_format=8)
    bb = G.block_bytes(s.n_per_blk, 8)
    blocks = []

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append(hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16])

    dev.run(s, sink, first_block=200, n_blocks=40, batch=16)
    assert blocks == golden["static_d30_b8"]["block_sha16"][200:240]


INTEG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                     "_ref", "gps-sdr-sim-integ")


@pytest.mark.parametrize("exe,name,args", [
    ("", "static_d30_b16", ["-l", ",".join(map(str, LOC)), "-d", "30", "-b", "16"]),
    ("", "circle_b8", ["-u", CIRCLE, "-b", "8"]),
    # the reference built without FLOAT_CARR_PHASE (gpssim.h:4): gss_integ.c's integer branch
    ("-intcarr", "intcarr_static_d30_b16", ["-l", ",".join(map(str, LOC)), "-d", "30", "-b", "16"]),
    ("-intcarr", "intcarr_static_d65_b8", ["-l", ",".join(map(str, LOC)), "-d", "65", "-b", "8"]),
])
def test_integration_patch_bit_exact(golden, exe, name, args):
    """INTEGRATION.md applied to the reference's own gpssim.c (tools/integration/build_integ.py:
    its sample loop replaced by gss_integ_block, batches flushed at every 30 s update) writes the
    reference's bytes; circle.csv crosses nine nav/allocation updates, the 65 s integer-carrier
    run two."""
    if not os.path.exists(INTEG + exe):
        pytest.skip(f"oracle/_ref/gps-sdr-sim-integ{exe} not built (needs the reference sources)")
    p = subprocess.run([INTEG + exe, "-e", NAV] + args + ["-o", "-"], capture_output=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert hashlib.sha256(p.stdout).hexdigest() == golden[name]["sha256"]


def test_producers_on_device(dev, golden):
    """The 30 s producers on the GPU: the C/A table and a whole run's nav rows, in
    two launches as gss_run builds them, equal the host plane's table word for word."""
    import torch
    ca = torch.zeros((32, G.CA_WORDS), dtype=torch.int32, device="cuda")
    dev.ca_table_device(ca.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(ca.cpu().numpy().view(np.uint32), G.ca_table())
    for kw in (dict(llh=LOC, duration=300.0), dict(motion_file=CIRCLE, data_format=8)):
        s = G.Scenario(NAV, **kw)
        s.all_blocks(batch=500, threads=4)
        src, want = s.nav_sources(), s.nav_table()
        d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
        rows = torch.zeros(want.shape, dtype=torch.int32, device="cuda")
        cut = len(src) // 2
        dev.nav_rows_device(d_src.data_ptr(), 0, cut, rows.data_ptr())
        dev.nav_rows_device(d_src.data_ptr() + cut * G.NAV_SRC_DTYPE.itemsize, cut,
                            len(src) - cut, rows.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(rows.cpu().numpy().view(np.uint32), want), kw


def _spec_walks_agree(got, want, gi, kw):
    """The device's walks against the host's (gss_spec_host): the same ends, wraps and first wraps
    bit for bit, and each segment's interval of exact start translations inside the host's (the
    device walks cycles from a cache its row's lanes share, whose entries' intervals are narrower:
    gss_producers.hip, sc_seg_walk); padding rows are not walked."""
    live = gi.reshape(-1)["s"] != 0
    assert np.array_equal(got["p1"][live], want["p1"][live]), kw
    assert np.array_equal(got["w1"][live], want["w1"][live]), kw
    narrower = 0
    for r in np.flatnonzero(live):
        k = gi.reshape(-1)["k"][r]
        g, w = got["seg"][r][:k], want["seg"][r][:k]
        assert g["end"].tobytes() == w["end"].tobytes(), (kw, r)
        assert np.array_equal(g["wrap_end"], w["wrap_end"]), (kw, r)
        empty = w["dlo"] > w["dhi"]                      # not walked: the same empty interval
        assert g[empty].tobytes() == w[empty].tobytes(), (kw, r)
        assert np.all(g["dlo"][~empty] >= w["dlo"][~empty]), (kw, r)
        assert np.all(g["dhi"][~empty] <= w["dhi"][~empty]), (kw, r)
        assert np.all(g["dlo"][~empty] <= 0) and np.all(g["dhi"][~empty] >= 0), (kw, r)
        narrower += int(np.sum((g["dlo"] != w["dlo"]) | (g["dhi"] != w["dhi"])))
    return narrower


def test_spec_walks_on_device(dev):
    """The carrier chain run ahead: the GPU's speculative block walks
    (gss_spec_device, a lane per segment, rows channel-major) agree with the host's
    (gss_spec_host: _spec_walks_agree), and
    the chain from them equals the exact chain (gss_carr_chain), for a static run across 30 s
    updates and the circle.csv run; nearly every block takes the translation."""
    import torch
    for kw in (dict(llh=LOC, duration=400.0), dict(motion_file=CIRCLE, data_format=8)):
        s = G.Scenario(NAV, **kw)
        carr = s.carrier()
        n = s.n_per_blk
        blk, nch, chain = s.next_deferred(300, threads=8)
        gi = G.carr_chain_guess(carr, blk, nch, chain, n)
        want = G.spec_host(gi, n, threads=8)
        d_in = torch.from_numpy(gi.reshape(-1).view(np.uint8).copy()).cuda()
        d_spec = torch.zeros(want.nbytes, dtype=torch.uint8, device="cuda")
        dev.spec_device(d_in.data_ptr(), len(want), n, d_spec.data_ptr())
        torch.cuda.synchronize()
        got = d_spec.cpu().numpy().view(G.SPEC_DTYPE)
        live = gi.reshape(-1)["s"] != 0                   # padding rows are not walked
        _spec_walks_agree(got, want, gi, kw)
        ref = blk.copy()
        end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
        end, hit = G.carr_chain_spec(carr, blk, nch, chain, n, gi, got)
        assert np.array_equal(blk["carr0"], ref["carr0"]) and np.array_equal(end, end_ref), kw
        assert hit >= 0.95 * int(nch.sum()), (kw, hit)
        # the starts alone (gss_run's path): the lanes guess the segment starts, write them back
        # bit-equal to the host's guesses, and walk the same segments
        g0 = G.carr_chain_guess(carr, blk, nch, chain, n, starts_only=True)
        d_in = torch.from_numpy(g0.reshape(-1).view(np.uint8).copy()).cuda()
        d_spec.zero_()
        dev.spec_device(d_in.data_ptr(), len(want), n, d_spec.data_ptr())
        torch.cuda.synchronize()
        assert d_in.cpu().numpy().tobytes() == gi.reshape(-1).tobytes(), kw
        got2 = d_spec.cpu().numpy().view(G.SPEC_DTYPE)
        assert np.array_equal(got2["p1"][live], got["p1"][live]), kw
        for r in np.flatnonzero(live):
            k = gi.reshape(-1)["k"][r]
            assert got2["seg"][r][:k].tobytes() == got["seg"][r][:k].tobytes(), (kw, r)
    # the kernel stages rows and walks through LDS in 8- and 16-byte words: misaligned buffers
    # are refused, not read or written across their ends
    with pytest.raises(G.GssError, match="aligned"):
        dev.spec_device(d_in.data_ptr() + 4, 16, n, d_spec.data_ptr())
    with pytest.raises(G.GssError, match="aligned"):
        dev.spec_device(d_in.data_ptr(), 16, n, d_spec.data_ptr() + 8)


def test_spec_records_on_device(dev):
    """gss_spec_records_device (gss_run's default): the walks stay on the device and only each
    row's 72-byte record comes back; the walks agree with the host's (_spec_walks_agree), the
    records equal the host's over the device's walks (gss_spec_records) byte for byte, and the
    chain from them (gss_carr_chain_records) equals the exact chain, for a static run across 30 s
    updates and the circle.csv run."""
    import torch
    for kw in (dict(llh=LOC, duration=400.0), dict(motion_file=CIRCLE, data_format=8)):
        s = G.Scenario(NAV, **kw)
        carr = s.carrier()
        n = s.n_per_blk
        b0, n0, c0 = s.next_deferred(50, threads=8)     # past the slots' first rows (resets)
        carr, _ = G.carr_chain(carr, b0, n0, c0, n, with_ck=False)
        blk, nch, chain = s.next_deferred(400, threads=8)
        g0 = G.carr_chain_guess(carr, blk, nch, chain, n, starts_only=True)
        gi = g0.copy()
        host = G.spec_host(gi, n, threads=8)
        nrow = g0.size
        h_in = torch.from_numpy(g0.reshape(-1).view(np.uint8).copy()).pin_memory()
        d_in = torch.zeros(nrow * G.SPEC_IN_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        d_spec = torch.zeros(nrow * G.SPEC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        h_rec = torch.zeros(nrow * G.SPEC_REC_DTYPE.itemsize, dtype=torch.uint8).pin_memory()
        dev.spec_records_device(h_in.data_ptr(), nrow, n, d_in.data_ptr(), d_spec.data_ptr(),
                                h_rec.data_ptr())
        torch.cuda.synchronize()
        got = h_rec.numpy().view(G.SPEC_REC_DTYPE).reshape(g0.shape)
        walks = d_spec.cpu().numpy().view(G.SPEC_DTYPE)
        gi = d_in.cpu().numpy().view(G.SPEC_IN_DTYPE).reshape(g0.shape)    # with the guesses
        _spec_walks_agree(walks, host, gi, kw)
        want = G.spec_records(gi, walks.reshape(gi.shape), n)
        live = g0["s"] != 0
        assert got[live].tobytes() == want[live].tobytes(), kw
        assert (got["ok"][live] & 2).sum() >= 0.9 * 2 * live.sum(), kw     # linked rows
        ref = blk.copy()
        end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
        end, hit = G.carr_chain_records(carr, blk, nch, chain, n, got)
        assert np.array_equal(blk["carr0"], ref["carr0"]) and np.array_equal(end, end_ref), kw
        assert hit >= 0.95 * int(nch.sum()), (kw, hit)
    with pytest.raises(G.GssError, match="aligned"):
        dev.spec_records_device(h_in.data_ptr(), 16, n, d_in.data_ptr(), d_spec.data_ptr() + 8,
                                h_rec.data_ptr())


def test_streaming_run_sink_error_stops_cleanly(dev, golden):
    """A sink that raises mid-run stops gss_run (planner, rows thread and GPU streams wound down),
    the exception reaches the caller, and the next run on the same device is exact again."""
    g = golden["static_d65_b8_noiono"]
    args = ["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8", "-i"]
    calls = []

    def bad(buf, first, nb):
        calls.append(first)
        if len(calls) == 3:
            raise KeyError("stop")

    s, _ = G.Scenario.from_cli(args)
    with pytest.raises(KeyError):
        dev.run(s, bad, batch=16, threads=4)
    assert calls == [0, 16, 32]
    blocks = []
    bb = G.block_bytes(s.n_per_blk, 8)

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append(hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16])

    s, _ = G.Scenario.from_cli(args)
    dev.run(s, sink, batch=40, threads=4)
    assert blocks == g["block_sha16"]


@pytest.mark.parametrize("spec,ahead,prover,proof,batch", [
    ("0", "1", "1", "host", 57), ("1", "0", "1", "host", 57), ("1", "1", "0", "host", 57),
    ("1", "1", "1", "host", 57), ("1", "1", "1", "host", 1),
    ("0", "1", "1", "gpu", 57), ("1", "0", "1", "gpu", 57), ("1", "1", "1", "gpu", 57),
    ("1", "1", "1", "gpu", 1), ("1", "1", "1", "split", 57), ("1", "0", "1", "split", 1),
    ("1", "1", "1", "host-dma", 57), ("0", "0", "1", "gpu-dma", 57),
    ("1", "1", "1", "host-walks", 57), ("1", "0", "1", "gpu-walks", 57),
    ("1", "1", "1", "host-walks", 1), ("1", "1", "1", "gpu-devanch", 57),
    ("1", "1", "1", "gpu-devanch", 1)])
def test_streaming_run_chain_modes(dev, golden, monkeypatch, spec, ahead, prover, proof, batch):
    """gss_run with the carrier chain walked on the host (GSS_RUN_SPEC=0) and run ahead on the
    GPU (the default), with the rows produced on the planner thread (GSS_RUN_ROWS_AHEAD=0) or
    ahead on their own (the default; one-block batches too), and the proofs on the planner thread
    (GSS_RUN_PROVER=0) or their own, or on the GPU (GSS_RUN_PROOF=gpu; split: every other slot),
    the slots' inputs uploaded by kernel (the default) or by the copy engine (-dma), and the
    walks' records back from the GPU (the default) or the walks themselves (-walks,
    GSS_RUN_REC=0, with the chain's anchors for the proofs): a 65 s run across two 30 s updates,
    whole and from a mid-run block, against the reference's golden hashes."""
    monkeypatch.setenv("GSS_RUN_SPEC", spec)
    if proof.endswith("-walks"):
        proof = proof[:-6]
        monkeypatch.setenv("GSS_RUN_REC", "0")
    if proof.endswith("-devanch"):            # GPU proofs anchored on the batch's device walks
        proof = proof[:-8]
        monkeypatch.setenv("GSS_RUN_DEV_ANCHORS", "1")
    if proof.endswith("-dma"):                # the slots' uploads by the copy engine
        proof = proof[:-4]
        monkeypatch.setenv("GSS_RUN_UPLOAD", "dma")
    monkeypatch.setenv("GSS_RUN_PROOF", proof)
    monkeypatch.setenv("GSS_RUN_ROWS_AHEAD", ahead)
    monkeypatch.setenv("GSS_RUN_PROVER", prover)
    g = golden["static_d65_b8_noiono"]
    bb = None
    blocks = []

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append((first + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))

    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    bb = G.block_bytes(s.n_per_blk, 8)
    dev.run(s, sink, batch=batch, threads=4)
    assert [x for _, x in blocks] == g["block_sha16"]
    blocks.clear()
    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    dev.run(s, sink, first_block=333, n_blocks=150, batch=64 if batch > 1 else 1)
    assert [b for b, _ in blocks] == list(range(333, 483))
    assert [x for _, x in blocks] == g["block_sha16"][333:483]


@pytest.mark.gpu
@pytest.mark.parametrize("proof", ["gpu", "split"])
def test_streaming_run_twice_on_one_handle_gpu_proofs(dev, golden, monkeypatch, proof):
    """Two gss_run calls on one scenario handle with the proofs on the GPU: the second run starts
    where the first stopped, after the first run's nav rows (and its 30 s updates) are already in
    the handle's table, so the second run's device nav table must be sized from the rows the
    handle holds, not from the run length alone (nav_rows_bound).  65 s across two 30 s updates
    against the reference's golden hashes."""
    monkeypatch.setenv("GSS_RUN_PROOF", proof)
    g = golden["static_d65_b8_noiono"]
    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    bb = G.block_bytes(s.n_per_blk, 8)
    blocks = []

    def sink(buf, first, nb):
        for i in range(nb):
            blocks.append((first + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))

    dev.run(s, sink, first_block=0, n_blocks=310, batch=64, threads=4)
    dev.run(s, sink, first_block=310, n_blocks=-1, batch=64, threads=4)
    assert [b for b, _ in blocks] == list(range(len(g["block_sha16"])))
    assert [x for _, x in blocks] == g["block_sha16"]
    # a run cannot start before the handle's position
    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    blocks.clear()
    dev.run(s, sink, first_block=0, n_blocks=100, batch=64, threads=4)
    with pytest.raises(Exception):
        dev.run(s, sink, first_block=50, n_blocks=10, batch=64, threads=4)
    # ... and a later start skips ahead (planned, dropped), as from a fresh handle
    dev.run(s, sink, first_block=400, n_blocks=60, batch=64, threads=4)
    assert [b for b, _ in blocks] == list(range(100)) + list(range(400, 460))
    assert [x for _, x in blocks] == g["block_sha16"][:100] + g["block_sha16"][400:460]

