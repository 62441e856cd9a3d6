"""Shared test setup.  `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box.

Input data (tests/golden/data/): brdc3540.14n (RINEX nav, 2014-12-20) and circle.csv (10 Hz
motion) — the reference's own sample inputs, copied as data so the GPU box (which has no
/root/reference) can run the BASELINE configs.  Expected outputs (tests/golden/golden.json,
lut512.json) come from the reference binary via tests/golden/make_golden.py.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gps-sdr-sim_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(REPO, "oracle"))

DATA = os.path.join(REPO, "tests", "golden", "data")
NAV = os.path.join(DATA, "brdc3540.14n")
CIRCLE = os.path.join(DATA, "circle.csv")
LOC = (30.286502, 120.032669, 100.0)
GOLDEN = os.path.join(REPO, "tests", "golden", "golden.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "libgpssim_amd.so")
    ora = os.path.join(REPO, "oracle", "_ref", "libgss_oracle.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-C", PKG, "-j8"])
    if not os.path.exists(ora):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "oracle"])


@pytest.fixture(scope="session", autouse=True)
def built():
    _ensure_built()


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)
