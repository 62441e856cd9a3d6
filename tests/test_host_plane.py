"""Host control plane (gss_scn_*): block count/size, per-block parameters, error behaviour,
and the exact carrier planner checked against the brute-force recurrence across blocks."""
import numpy as np
import pytest

from conftest import CIRCLE, LOC, NAV

import gpssim_amd as G
import oracle


def test_static_geometry():
    s = G.Scenario(NAV, llh=LOC, duration=30.0)
    assert (s.n_per_blk, s.n_blocks, s.data_format) == (260000, 299, 16)
    assert s.samp_freq == 2600000.0 and s.delt == 1.0 / 2600000.0
    assert (s.start_week, s.start_sec) == (1823, 518400.0)
    blk, nch = s.all_blocks(batch=64)
    assert len(nch) == 299 and set(nch.tolist()) == {11}
    act = blk[0, :11]
    assert set(act["ca_tbl"] + 1) == {1, 2, 3, 6, 9, 10, 12, 17, 20, 23, 28}
    assert np.all((act["carr0"] >= 0) & (act["carr0"] < 1))
    assert np.all((act["code0"] >= 0) & (act["code0"] < 1023))
    assert np.all(act["gain"] > 0) and np.all(act["gain"] < 200)
    assert np.all(np.abs(act["carr_step"]) < 5000 / 2.6e6)


def test_sample_rate_rounding():
    s = G.Scenario(NAV, llh=LOC, duration=1.0, samp_freq=2600047.0)
    assert s.n_per_blk == 260004 and s.samp_freq == 2600040.0


@pytest.mark.parametrize("kw,msg", [
    (dict(samp_freq=5e5), "Invalid sampling frequency"),
    (dict(data_format=4), "Invalid I/Q data format"),
    (dict(duration=90000.0), "Invalid duration"),
    (dict(samp_freq=2600020.0, data_format=1), "divisible by 4"),
])
def test_errors(kw, msg):
    with pytest.raises(G.GssError) as e:
        G.Scenario(NAV, llh=LOC, **kw)
    assert msg in str(e.value)


def test_missing_files():
    with pytest.raises(G.GssError, match="ephemeris file not found"):
        G.Scenario("/nonexistent.14n", llh=LOC, duration=1.0)
    with pytest.raises(G.GssError, match="Failed to open user motion"):
        G.Scenario(NAV, motion_file="/nonexistent.csv", duration=1.0)


def test_start_time_out_of_range():
    with pytest.raises(G.GssError, match="Invalid start time"):
        G.Scenario(NAV, llh=LOC, duration=1.0, start=(2014, 12, 25, 0, 0, 0))


def test_dynamic_block_count():
    s = G.Scenario(NAV, motion_file=CIRCLE)
    assert s.n_blocks == 2999
    with pytest.raises(G.GssError, match="Invalid duration"):
        G.Scenario(NAV, motion_file=CIRCLE, duration=301.0)


def test_planner_chain_matches_brute_force():
    """carr0 of block b+1 == brute-force advance of block b's carr0 by N samples, for every
    channel that stays allocated (same PRN); crosses a 30 s re-allocation boundary."""
    s = G.Scenario(NAV, llh=LOC, duration=31.0, samp_freq=1.0e6)
    blk, nch = s.all_blocks(batch=100)
    n = s.n_per_blk
    checked = 0
    for b in range(0, len(nch) - 1, 37):
        for k in range(nch[b]):
            prn = blk[b, k]["ca_tbl"]
            nxt = [j for j in range(nch[b + 1]) if blk[b + 1, j]["ca_tbl"] == prn]
            if not nxt:
                continue
            want = oracle.carr_brute(blk[b, k]["carr0"], blk[b, k]["carr_step"], n)
            assert blk[b + 1, nxt[0]]["carr0"] == want
            checked += 1
    assert checked > 50


def test_planner_checkpoints_match_brute_force():
    """The carrier checkpoints the planner records on its walk (gss_scn_next carr_ck) are the
    brute-force carrier at samples j*N/NCK of every block; padding rows are zero."""
    s = G.Scenario(NAV, llh=LOC, duration=3.0)
    blk, nch, ck = s.all_blocks(batch=10, with_ck=True)
    n = s.n_per_blk
    pos = [j * n // G.NCK for j in range(G.NCK)]
    for b in range(0, len(nch), 7):
        for k in range(nch[b]):
            want = oracle.carr_brute_trace(blk[b, k]["carr0"], blk[b, k]["carr_step"], pos)
            assert np.array_equal(ck[b, k], want), (b, k)
        assert not ck[b, nch[b]:].any()


def test_nav_table_rows():
    s = G.Scenario(NAV, llh=LOC, duration=31.0)
    blk, nch = s.all_blocks()
    nav = s.nav_table()
    assert nav.shape[1] == 60 and np.all(nav < (1 << 30))
    # every 30 s frame gets new rows: 11 initial + 11 at t=30 s
    assert len(nav) == 22
    assert blk[-1, :nch[-1]]["nav_tbl"].min() >= 11
    # TLM preamble 0x8B in every subframe's first word (bits 29..22, possibly inverted by D30*)
    for row in nav:
        for sf in range(6):
            w = int(row[sf * 10])
            pre = (w >> 22) & 0xFF
            assert pre in (0x8B, 0x74)


@pytest.mark.parametrize("kind,threads,starts_only", [("static", 8, False), ("circle", 3, False),
                                                     ("intcarr", 4, False), ("static", 8, True),
                                                     ("circle", 3, True)])
def test_speculative_chain_equals_exact_chain(kind, threads, starts_only):
    """The planner's carrier chain with every block's walk run ahead from a guessed start
    (gss_carr_chain_guess -> gss_spec_host -> gss_carr_chain_spec, the path gss_run takes with
    the walks on the GPU) gives the same carr0 of every row and the same end carriers as the
    exact chain (gss_carr_chain), over several batches across 30 s updates and re-allocations,
    and nearly every block takes the translation (one partial cycle on the serial path).
    starts_only: the starts alone (gss_carr_chain_starts, as gss_run), the walker guessing each
    row's segment starts and writing back exactly the host's guesses."""
    if kind == "static":
        s = G.Scenario(NAV, llh=LOC, duration=400.0)
    elif kind == "circle":
        s = G.Scenario(NAV, motion_file=CIRCLE, duration=300.0)
    else:
        s = G.Scenario(NAV, llh=LOC, duration=70.0, carrier="int")
    carr = s.carrier()
    n = s.n_per_blk
    total = hit = 0
    for _ in range(4):
        blk, nch, chain = s.next_deferred(350, threads=threads)
        if len(nch) == 0:
            break
        ref = blk.copy()
        end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, carrier_int=s.carrier_int,
                                  with_ck=False, threads=threads)
        gi = G.carr_chain_guess(carr, blk, nch, chain, n, starts_only=starts_only)
        full = G.carr_chain_guess(carr, blk, nch, chain, n)
        assert np.array_equal(gi["g"], full["g"]) and np.array_equal(gi["s"], full["s"])
        if starts_only:
            assert (gi["k"][gi["s"] != 0] == 0).all()
        spec = G.spec_host(gi, n, threads=threads)
        assert gi.tobytes() == full.tobytes(), kind          # the walker's guesses = the host's
        end, h = G.carr_chain_spec(carr, blk, nch, chain, n, gi, spec, threads=threads)
        assert np.array_equal(blk["carr0"], ref["carr0"]), kind
        assert np.array_equal(end, end_ref), kind
        total += int(nch.sum())
        hit += h
        carr = end
    assert total > 0
    if kind != "intcarr":
        assert hit >= 0.95 * total, (hit, total)


def test_line_end_prediction_two_batches_ahead():
    """gss_carr_line_end: the slots' carriers after a batch by the lines (what gss_run starts the
    next batch's guesses from while this batch's chain is pending) equal a Python restatement
    bit for bit, lie within 1e-8 cycle of the exact chain's end, and guesses started from them
    keep nearly every block of the next batch on the translation; that chain stays exact."""
    s = G.Scenario(NAV, llh=LOC, duration=90.0)
    carr = s.carrier()
    n = s.n_per_blk
    b1, n1, c1 = s.next_deferred(300, threads=8)
    b2, n2, c2 = s.next_deferred(300, threads=8)
    pred = G.carr_line_end(carr, b1, n1, c1, n)
    run = carr.copy()
    for b in range(len(n1)):
        for k in range(n1[b]):
            sl = c1[b, k]["slot"]
            if c1[b, k]["reset"]:
                run[sl] = c1[b, k]["init"]
            v = run[sl] + n * b1[b, k]["carr_step"]
            run[sl] = v - np.floor(v)
    assert pred.tobytes() == run.tobytes()
    r1 = b1.copy()
    end1, _ = G.carr_chain(carr, r1, n1, c1, n, with_ck=False)
    live = sorted({int(c1[b, k]["slot"]) for b in range(len(n1)) for k in range(n1[b])})
    d = np.abs(((pred[live] - end1[live]) + 0.5) % 1.0 - 0.5)
    assert d.max() < 1e-8, d.max()
    gi = G.carr_chain_guess(pred, b2, n2, c2, n)
    spec = G.spec_host(gi, n, threads=8)
    got, ref = b2.copy(), b2.copy()
    end2_ref, _ = G.carr_chain(end1, ref, n2, c2, n, with_ck=False)
    end2, hit = G.carr_chain_spec(end1, got, n2, c2, n, gi, spec, threads=8)
    assert np.array_equal(got["carr0"], ref["carr0"]) and np.array_equal(end2, end2_ref)
    assert hit >= 0.95 * int(n2.sum()), (hit, int(n2.sum()))


def test_speculative_chain_exact_with_wrong_guesses():
    """gss_carr_chain_spec is exact whatever the guesses: starts moved far outside every
    translation interval, segment starts moved off their wraps or to wrong values, and segment
    counts cut: the chain still equals the exact one, with (almost) no block taking the
    translation."""
    s = G.Scenario(NAV, llh=LOC, duration=120.0)
    carr = s.carrier()
    n = s.n_per_blk
    blk, nch, chain = s.next_deferred(600, threads=8)
    ref = blk.copy()
    end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
    gi = G.carr_chain_guess(carr, blk, nch, chain, n)
    rng = np.random.default_rng(7)
    for mode in ("start", "segments", "counts"):
        g = gi.copy().reshape(-1)
        live = g["s"] != 0
        if mode == "start":                   # the start guess 1e-4 cycle off: another p1/w1
            g["g"][live] = np.mod(g["g"][live] + 1e-4, 1.0)
        elif mode == "segments":              # segment starts one sample late, values shifted
            g["P"][:, 1:] += (g["P"][:, 1:] > 0)
            g["W"][:, 1:] = np.where(g["P"][:, 1:] > 0, np.mod(g["W"][:, 1:] + 3e-7, 1.0), 0.0)
        else:                                 # fewer segments than walked, random cut
            g["k"] = np.minimum(g["k"], rng.integers(1, 4, size=len(g)))
        spec = G.spec_host(g.reshape(gi.shape), n, threads=8)
        b = blk.copy()
        end, hit = G.carr_chain_spec(carr, b, nch, chain, n, g.reshape(gi.shape), spec)
        assert np.array_equal(b["carr0"], ref["carr0"]), mode
        assert np.array_equal(end, end_ref), mode
        if mode != "counts":
            assert hit < 0.05 * int(nch.sum()), (mode, hit)


@pytest.mark.parametrize("kind,pert", [("static", 0.0), ("static", 3e-10), ("circle", 1e-9),
                                       ("static", 1e-4)])
def test_linked_chain_equals_exact_chain(kind, pert):
    """gss_spec_links + gss_carr_chain_linked (the multi-rank planner's chain after the baton,
    shard.chain_speculated): each row's walk folded with its predecessor's into one record ahead
    of time, the chain then a compare and two adds per row where the translation holds.  Bit
    for bit the exact chain's carr0 and end carriers, over a whole window guessed from a start
    off by `pert` (1e-4: no translation holds, every row walked exactly), with the same blocks
    translated as gss_carr_chain_spec."""
    if kind == "static":
        s = G.Scenario(NAV, llh=LOC, duration=300.0)
    else:
        s = G.Scenario(NAV, motion_file=CIRCLE, duration=300.0)
    n = s.n_per_blk
    b0, n0, c0 = s.next_deferred(100, threads=8)        # the slots' first rows are resets:
    carr, _ = G.carr_chain(s.carrier(), b0, n0, c0, n, with_ck=False)   # start after them
    blk, nch, chain = s.next_deferred(2900, threads=8)
    ref = blk.copy()
    end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
    gi = G.carr_chain_guess(np.mod(carr + pert, 1.0), blk, nch, chain, n, starts_only=True)
    spec = G.spec_host(gi, n, threads=8)
    link = G.spec_links(nch, chain, n, gi, spec, threads=8)
    b1, b2 = blk.copy(), blk.copy()
    end1, hit1 = G.carr_chain_spec(carr, b1, nch, chain, n, gi, spec)
    end2, hit2 = G.carr_chain_linked(carr, b2, nch, chain, n, gi, spec, link)
    assert b2["carr0"].tobytes() == ref["carr0"].tobytes()
    assert end2.tobytes() == end_ref.tobytes()
    assert hit2 == hit1
    rows = int(nch.sum())
    if pert < 1e-6:
        assert hit2 >= 0.97 * rows and (link["lo"] <= link["hi"]).sum() >= 0.95 * rows
    else:
        assert hit2 < 0.05 * rows, (hit2, rows)


@pytest.mark.parametrize("kind,pert", [("static", 0.0), ("static", 3e-10), ("circle", 1e-9),
                                       ("static", 1e-4)])
def test_records_chain_equals_exact_chain(kind, pert):
    """gss_spec_records + gss_carr_chain_records (gss_run's default chain: the walks folded into
    72-byte records, on the GPU there, only the records back): the exact chain's carr0 and end
    carriers bit for bit from a start off by `pert`, the same rows translated as
    gss_carr_chain_spec, and the links (gi["pad"]: the previous row of the slot) on nearly every
    row."""
    if kind == "static":
        s = G.Scenario(NAV, llh=LOC, duration=290.0)
    else:
        s = G.Scenario(NAV, motion_file=CIRCLE, duration=290.0)
    n = s.n_per_blk
    b0, n0, c0 = s.next_deferred(100, threads=8)
    carr, _ = G.carr_chain(s.carrier(), b0, n0, c0, n, with_ck=False)
    blk, nch, chain = s.next_deferred(2790, threads=8)
    ref = blk.copy()
    end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
    gi = G.carr_chain_guess(np.mod(carr + pert, 1.0), blk, nch, chain, n, starts_only=True)
    spec = G.spec_host(gi, n, threads=8).reshape(gi.shape)
    rec = G.spec_records(gi, spec, n)
    b1, b2 = blk.copy(), blk.copy()
    _, hit1 = G.carr_chain_spec(carr, b1, nch, chain, n, gi, spec)
    end2, hit2 = G.carr_chain_records(carr, b2, nch, chain, n, rec)
    assert b2["carr0"].tobytes() == ref["carr0"].tobytes()
    assert end2.tobytes() == end_ref.tobytes()
    assert hit2 == hit1
    rows = int(nch.sum())
    assert ((rec["ok"] & 2) != 0).sum() >= 0.95 * rows
    if pert < 1e-6:
        assert hit2 >= 0.97 * rows


@pytest.mark.parametrize("bad", ["zero", "shift", "distance"])
def test_records_chain_exact_with_wrong_links(bad):
    """Records whose link does not belong to the slot's previous row: rows with wrong in[].pad
    (zero-filled, or every pad one slot row too far back), and correct records whose stored row
    distance (ok bits 2..) is altered.  The chain applies a link only when its distance names
    the slot's actual previous row, so it stays exact; with the distances altered no link
    holds and the rows fall back to their own records and walks."""
    s = G.Scenario(NAV, llh=LOC, duration=120.0)
    n = s.n_per_blk
    b0, n0, c0 = s.next_deferred(60, threads=8)
    carr, _ = G.carr_chain(s.carrier(), b0, n0, c0, n, with_ck=False)
    blk, nch, chain = s.next_deferred(600, threads=8)
    ref = blk.copy()
    end_ref, _ = G.carr_chain(carr, ref, nch, chain, n, with_ck=False)
    gi = G.carr_chain_guess(carr, blk, nch, chain, n, starts_only=True)
    flat = gi.reshape(-1)
    if bad == "zero":
        flat["pad"] = 0
    elif bad == "shift":
        pads = flat["pad"].copy()
        flat["pad"] = np.where(pads >= 0, pads[np.maximum(pads, 0)], -1)   # the row before last
    spec = G.spec_host(gi, n, threads=8).reshape(gi.shape)
    rec = G.spec_records(gi, spec, n)
    if bad == "distance":
        # poisoned links: any translation passes their interval and they move the carrier by a
        # quarter cycle; with their true row distance the chain takes them (control), with an
        # altered one it must refuse them
        linked = (rec["ok"] & 2) != 0
        assert linked.sum() >= 0.9 * int(nch.sum())
        d = rec["ok"] >> 2
        assert (d[linked] >= 1).all()
        rec["llo"] = np.where(linked, -1.0, rec["llo"])
        rec["lhi"] = np.where(linked, 1.0, rec["lhi"])
        rec["ldd"] = np.where(linked, rec["ldd"] + 0.25, rec["ldd"])
        b1 = blk.copy()
        G.carr_chain_records(carr, b1, nch, chain, n, rec)
        assert b1["carr0"].tobytes() != ref["carr0"].tobytes()       # the links are in use
        rec["ok"] = np.where(linked, (rec["ok"] & 3) | ((d + G.MAXCH) << 2), rec["ok"])
    b2 = blk.copy()
    end2, _ = G.carr_chain_records(carr, b2, nch, chain, n, rec)
    assert b2["carr0"].tobytes() == ref["carr0"].tobytes()
    assert end2.tobytes() == end_ref.tobytes()


def test_worker_pool_after_fork():
    """The host plane's persistent worker threads do not survive fork(): a child that plans
    (gss_pool_run on 8 threads) after the parent has grown its pools must still finish, with the
    parent's rows (pool.c's pthread_atfork reset)."""
    import os
    import signal
    import time
    s = G.Scenario(NAV, llh=LOC, duration=10.0)
    want_blk, want_nch = s.next(40, threads=8)          # grows the default pool in the parent
    s2 = G.Scenario(NAV, llh=LOC, duration=10.0)
    pid = os.fork()
    if pid == 0:                                         # child: plan again, exit 0 if equal
        try:
            blk, nch = s2.next(40, threads=8)
            ok = np.array_equal(nch, want_nch) and \
                np.array_equal(blk.view(np.uint8), want_blk.view(np.uint8))
            os._exit(0 if ok else 3)
        except BaseException:
            os._exit(4)
    t0 = time.time()
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() - t0 > 60:
            os.kill(pid, signal.SIGKILL)
            os.waitpid(pid, 0)
            pytest.fail("the child's planning hung (worker pool after fork)")
        time.sleep(0.05)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0, status


@pytest.mark.parametrize("fmt,fs,dur,first,count", [(1, 2.6e6, 1200.0, 4000, 5000),
                                                    (16, 2.0e7, 60.0, 200, 150)])
def test_plan_window_chain_run_ahead(fmt, fs, dur, first, count):
    """shard.plan_window with the chain run ahead (speculative walks, here on the host:
    gss_spec_host; bench.py and node.py use the GPU's) gives the host chain's rows bit for bit,
    across 30 s updates and in more than one 4,096-block chunk for the first case."""
    from gpssim_amd.shard import host_walker, plan_window
    s1 = G.Scenario(NAV, llh=LOC, duration=dur, samp_freq=fs, data_format=fmt)
    b1, n1, ck1, _ = plan_window(s1, first, count, threads=8)
    s2 = G.Scenario(NAV, llh=LOC, duration=dur, samp_freq=fs, data_format=fmt)
    b2, n2, ck2, t2 = plan_window(s2, first, count, threads=8, walker=host_walker(8))
    assert np.array_equal(n1, n2)
    assert np.array_equal(b1.view(np.uint8), b2.view(np.uint8))
    assert ck2 is None and t2["spec_hits"] > 0.9 * int(n2.sum())


def test_host_threads_under_sanitizers(tmp_path):
    """gss_run itself on the CPU fake of the HIP runtime (tests/helpers/run_fake.cpp, every run
    mode) and the host plane's threads (tests/helpers/run_harness.c), built with ThreadSanitizer
    and with AddressSanitizer + UBSan (tools/sanitize.sh, shortened here to every third run mode;
    the committed logs under profiles/round5/sanitize are the full runs): no report, every byte
    as expected."""
    import os
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(repo, "tools", "sanitize.sh")],
                       env=dict(os.environ, SECS="20", FAKE_ARGS="20 16 8",
                                HARNESS_ARGS="20 64 16", RUN_FAKE_QUICK="1", OUT=str(tmp_path)),
                       capture_output=True, text=True, timeout=900)
    logs = "".join(open(os.path.join(tmp_path, f)).read() for f in sorted(os.listdir(tmp_path)))
    assert r.returncode == 0, logs[-3000:]
    assert "sanitizer reports: 0" in logs and "sanitizer reports: 1" not in logs


@pytest.mark.parametrize("kind", ["static", "circle"])
def test_rows_independent_of_threads_and_batches(kind):
    """The per-block refreshes of a range pass run in parallel (scenario.c refresh_part) and the
    channel state is then set as the serial loop of gpssim.c:2156-2188 leaves it: rows, chains
    and the scenario's state after them must not depend on the thread count or on where batches
    end (across 30 s updates, channel allocations and a seek)."""
    kw = {"motion_file": CIRCLE} if kind == "circle" else {"llh": LOC}

    def rows(threads, sizes, seek=0):
        s = G.Scenario(NAV, duration=95.0, samp_freq=2.6e6, data_format=8, **kw)
        if seek:
            s.seek(seek)
        out = []
        for n in sizes:
            b, c, ch = s.next_deferred(n, threads)
            out.append((b.copy(), c.copy(), ch.copy()))
        blk = np.concatenate([o[0] for o in out])
        nch = np.concatenate([o[1] for o in out])
        chain = np.concatenate([o[2] for o in out])
        return blk.tobytes(), nch.tobytes(), chain.tobytes(), s.carrier().tobytes()

    want = rows(1, [950])
    assert rows(8, [950]) == want
    assert rows(8, [1, 299, 300, 7, 343]) == want
    assert rows(3, [17] * 55 + [15]) == want
    # a seek to a mid-run block, then the same rows as the whole run's tail
    full = rows(8, [950])
    b0 = np.frombuffer(full[0], G.CHAN_DTYPE).reshape(-1, G.MAXCH)[412:]
    got = rows(8, [538], seek=412)
    gb = np.frombuffer(got[0], G.CHAN_DTYPE).reshape(-1, G.MAXCH)
    fields = [f for f in G.CHAN_DTYPE.names if f != "carr0"]  # carriers: unknown after a seek
    assert all(np.array_equal(gb[f], b0[f]) for f in fields)
