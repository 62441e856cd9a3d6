"""The oracle is pinned before it is trusted: its LUT against the reference's table, the C/A
generator against IS-GPS-200 Table 3-Ia, and the all-CPU restatement (product host plane +
scalar oracle loop) against the reference binary's golden outputs."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import CIRCLE, LOC, NAV, REPO

import gpssim_amd as G
import oracle

LUT_FIX = os.path.join(REPO, "tests", "golden", "lut512.json")


def test_lut_matches_reference_table():
    fix = json.load(open(LUT_FIX))
    s, c = oracle.lut()
    assert s.tolist() == fix["sinTable512"]
    assert c.tolist() == fix["cosTable512"]
    ps, pc = G.lut()
    assert ps.tolist() == fix["sinTable512"] and pc.tolist() == fix["cosTable512"]


def _chips(row, n=10):
    return [(int(row[i >> 5]) >> (i & 31)) & 1 for i in range(n)]


def test_ca_known_answer():
    # IS-GPS-200 Table 3-Ia: first 10 chips in octal (1 = chip '1')
    ca = G.ca_table()
    expect = {1: 0o1440, 2: 0o1620, 3: 0o1710, 4: 0o1744, 5: 0o1133, 10: 0o1504, 32: 0o1712}
    for prn, octal in expect.items():
        bits = _chips(ca[prn - 1])
        assert int("".join(map(str, bits)), 2) == octal, prn
    # balanced Gold codes: 512 ones per period
    for prn in range(1, 33):
        assert sum(_chips(ca[prn - 1], 1023)) == 512


def run_cpu_restatement(args):
    p = subprocess.run([oracle.CLI, "-e", NAV] + args + ["-o", "-"], capture_output=True,
                       check=True)
    return p.stdout


def block_hashes(buf, bb):
    return [hashlib.sha256(buf[i:i + bb]).hexdigest()[:16] for i in range(0, len(buf), bb)]


@pytest.mark.parametrize("fmt", [16, 8, 1])
def test_cpu_restatement_prefix_matches_reference(golden, fmt):
    g = golden[f"static_d30_b{fmt}"]
    out = run_cpu_restatement(["-l", ",".join(map(str, LOC)), "-d", "3", "-b", str(fmt)])
    bb = G.block_bytes(260000, fmt)
    assert len(out) == 29 * bb
    assert block_hashes(out, bb) == g["block_sha16"][:29]
    assert out[: len(g["head_hex"]) // 2].hex() == g["head_hex"]


def test_cpu_restatement_full_30s_b1(golden):
    out = run_cpu_restatement(["-l", ",".join(map(str, LOC)), "-d", "30", "-b", "1"])
    assert hashlib.sha256(out).hexdigest() == golden["static_d30_b1"]["sha256"]


def test_cpu_restatement_dynamic_prefix(golden):
    g = golden["circle_b8"]
    out = run_cpu_restatement(["-u", CIRCLE, "-d", "2", "-b", "8"])
    assert block_hashes(out, 520000) == g["block_sha16"][:19]


@pytest.mark.parametrize("name,args,nblk", [
    ("static_d300_b16", ["-l", ",".join(map(str, LOC)), "-d", "31", "-b", "16"], 309),
    ("circle_b8", ["-u", CIRCLE, "-d", "31", "-b", "8"], 309),
])
def test_cpu_restatement_across_first_nav_update(golden, name, args, nblk):
    """Past the first 30 s boundary: the nav-message regeneration and channel re-allocation that
    run after block 299 (gpssim.c:2294-2332) feed blocks 300..308, byte for byte."""
    g = golden[name]
    out = run_cpu_restatement(args)
    bb = g["bytes"] // g["blocks"]
    assert len(out) == nblk * bb
    assert block_hashes(out, bb) == g["block_sha16"][:nblk]


# the rest of the CLI surface (tests/golden/make_golden.py): NMEA input, valid -t, -T, a
# USER_MOTION_SIZE=4000 build for rocket.csv, the LEO satellite.csv run with -i
DATA = os.path.join(REPO, "tests", "golden", "data")
CLI_CASES = ["nmea_triumph_b8", "static_t0200_d30_b8", "static_T1221_d30_b8",
             "rocket_um4000_b8", "satellite_i_b8"]


def fixture_argv(g):
    """the fixture's command line with the reference's data files mapped to tests/golden/data"""
    return [os.path.join(DATA, a) if os.path.exists(os.path.join(DATA, a)) else a
            for a in g["argv"]]


def limit_duration(argv, seconds):
    a = list(argv)
    if "-d" in a:
        a[a.index("-d") + 1] = str(seconds)
    else:
        a += ["-d", str(seconds)]
    return a


@pytest.mark.parametrize("name", CLI_CASES)
def test_cpu_restatement_cli_surface_prefix(golden, name, monkeypatch):
    """The first 2.9 s of each run, byte for byte (the GPU tests check whole runs)."""
    g = golden[name]
    monkeypatch.setenv("GSS_USER_MOTION_SIZE", str(g["user_motion_size"]))
    out = run_cpu_restatement(limit_duration(fixture_argv(g), 3))
    bb = G.block_bytes(g["n_per_blk"], g["fmt"])
    assert len(out) == 29 * bb
    assert block_hashes(out, bb) == g["block_sha16"][:29]


@pytest.mark.parametrize("name", ["static_d31_v", "circle_d31"])
def test_cpu_restatement_stderr_matches_reference(name):
    """Banner, ephemeris/iono/UTC lines (-v), the channel table, its 30 s reprint (-v) and the
    progress lines, as the reference prints them (gpssim.c:1939-1948, 2037-2039, 2131-2136,
    2335-2352), minus the CPU-time line."""
    e = json.load(open(os.path.join(REPO, "tests", "golden", "stderr.json")))[name]
    argv = [os.path.join(DATA, a) if os.path.exists(os.path.join(DATA, a)) else a
            for a in e["argv"]]
    p = subprocess.run([oracle.CLI, "-e", NAV] + argv + ["-o", "/dev/null"],
                       capture_output=True, check=True)
    got = "".join(l for l in p.stderr.decode().splitlines(True)
                  if not l.startswith("Process time"))
    assert got == e["stderr"]


# the integer-carrier variant: the reference built with FLOAT_CARR_PHASE off (gpssim.h:4,
# oracle/Makefile _ref/gps-sdr-sim-intcarr), rendered by the product with --carrier=int
INT_CASES = [
    ("intcarr_static_d30_b16", ["-d", "3"], 29),
    ("intcarr_static_d65_b8", ["-d", "31"], 309),      # across the first nav/allocation update
    ("intcarr_circle_b8", ["-d", "2"], 19),
    ("intcarr_static_d30_s20M_b1", ["-d", "1"], 9),
]


@pytest.mark.parametrize("name,dur,nblk", INT_CASES)
def test_cpu_restatement_integer_carrier_prefix(golden, name, dur, nblk):
    g = golden[name]
    assert g["carrier"] == "int"
    argv = fixture_argv(g)
    out = run_cpu_restatement(["--carrier=int"] + limit_duration(argv, dur[1]))
    bb = G.block_bytes(g["n_per_blk"], g["fmt"])
    assert len(out) == nblk * bb
    assert block_hashes(out, bb) == g["block_sha16"][:nblk]


def test_integer_carrier_differs_from_float(golden):
    """the two reference builds give different streams, so the flag is honoured"""
    assert golden["intcarr_static_d30_b16"]["sha256"] != golden["static_d30_b16"]["sha256"]
    out = run_cpu_restatement(["-l", ",".join(map(str, LOC)), "-d", "1", "-b", "16",
                               "--carrier=float"])
    assert block_hashes(out, 1040000) == golden["static_d30_b16"]["block_sha16"][:9]


def test_carrier_flag_rejects_unknown_mode():
    p = subprocess.run([oracle.CLI, "-e", NAV, "-l", "30,120,100", "-d", "1", "--carrier=fixed",
                        "-o", "/dev/null"], capture_output=True)
    assert p.returncode == 1 and b"Invalid carrier mode" in p.stderr
