"""The product CLI (bin/gps-sdr-sim: host plane + gss_run + GPU kernels) on the rest of the
reference's option surface, whole runs against the reference's own outputs
(tests/golden/make_golden.py): NMEA input (-g triumphv3.txt, 1560 blocks), a valid -t start, -T
(TOC/TOE overwrite, the fall-through into -t's parser, gpssim.c:1804-1835), rocket.csv with the
reference built for USER_MOTION_SIZE=4000 (our GSS_USER_MOTION_SIZE=4000), the LEO satellite.csv
scenario with -i; and the stderr text (-v details, channel tables, progress) byte for byte."""
import hashlib
import json
import os
import subprocess

import pytest

from conftest import NAV, REPO

import gpssim_amd as G

pytestmark = pytest.mark.gpu

DATA = os.path.join(REPO, "tests", "golden", "data")
CASES = ["nmea_triumph_b8", "static_t0200_d30_b8", "static_T1221_d30_b8", "rocket_um4000_b8",
         "satellite_i_b8",
         # --carrier=int vs the reference built with FLOAT_CARR_PHASE off (gpssim.h:4)
         "intcarr_static_d30_b16", "intcarr_static_d65_b8", "intcarr_circle_b8",
         "intcarr_static_d30_s20M_b1"]


def _argv(args):
    return [os.path.join(DATA, a) if os.path.exists(os.path.join(DATA, a)) else a for a in args]


@pytest.mark.parametrize("name", CASES)
def test_cli_surface_whole_run(golden, name, tmp_path):
    g = golden[name]
    bb = G.block_bytes(g["n_per_blk"], g["fmt"])
    env = dict(os.environ, GSS_USER_MOTION_SIZE=str(g["user_motion_size"]))
    errf = open(tmp_path / "stderr.txt", "w+b")      # a file: a pipe would fill and stall it
    mode = ["--carrier=int"] if g.get("carrier") == "int" else []
    p = subprocess.Popen([G.CLI_PATH, "-e", NAV] + _argv(g["argv"]) + mode + ["-o", "-"], env=env,
                         stdout=subprocess.PIPE, stderr=errf)
    h, blocks, total = hashlib.sha256(), [], 0
    while True:
        buf = p.stdout.read(bb)
        if not buf:
            break
        h.update(buf)
        total += len(buf)
        blocks.append(hashlib.sha256(buf).hexdigest()[:16])
    rc = p.wait()
    errf.seek(0)
    assert rc == 0, errf.read()[-2000:]
    if blocks != g["block_sha16"]:
        bad = [i for i, (a, b) in enumerate(zip(blocks, g["block_sha16"])) if a != b]
        raise AssertionError(f"{name}: {len(bad)} blocks differ, first {bad[:1]}; "
                             f"{len(blocks)} vs {len(g['block_sha16'])} blocks")
    assert total == g["bytes"] and h.hexdigest() == g["sha256"]


@pytest.mark.parametrize("name", ["static_d31_v", "circle_d31"])
def test_cli_stderr_matches_reference(name, tmp_path):
    e = json.load(open(os.path.join(REPO, "tests", "golden", "stderr.json")))[name]
    p = subprocess.run([G.CLI_PATH, "-e", NAV] + _argv(e["argv"]) +
                       ["-o", str(tmp_path / "x.bin")], capture_output=True)
    assert p.returncode == 0, p.stderr[-2000:]
    got = "".join(l for l in p.stderr.decode().splitlines(True)
                  if not l.startswith("Process time"))
    assert got == e["stderr"]
