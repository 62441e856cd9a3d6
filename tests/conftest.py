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


def pytest_collection_modifyitems(config, items):
    """The long full-stream digests (test_gpu_long.py, 344 GB hashed) run last, so that with -x
    every BASELINE-config and CLI parity test has reported before them."""
    items.sort(key=lambda it: "test_gpu_long" in it.nodeid)


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
    import gpssim_amd
    # measurement builds (tools/ablate.sh) may be parity-checked only when asked for explicitly
    assert gpssim_amd.IN_TREE or os.environ.get("GSS_TEST_VARIANT") == "1", \
        f"tests must run on the in-tree build, not {gpssim_amd.LIB_PATH}"


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


_walk = None


def walk_lib():
    """ctypes handle on tests/helpers/walk_check.c (built on first use with gcc)."""
    global _walk
    if _walk is None:
        import ctypes as C
        src = os.path.join(REPO, "tests", "helpers", "walk_check.c")
        so = os.path.join(REPO, "tests", "helpers", "_walk_check.so")
        if not os.path.exists(so) or os.path.getmtime(so) < max(
                os.path.getmtime(src),
                os.path.getmtime(os.path.join(PKG, "csrc", "common", "gss_phase.h"))):
            subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-o",
                                   so, src, "-lm"])
        L = C.CDLL(so)
        D, I64, P = C.c_double, C.c_int64, C.POINTER(C.c_int32)
        for f in ("wc_carr_plain", "wc_carr_cached"):
            getattr(L, f).restype = D
            getattr(L, f).argtypes = [D, D, I64]
        L.wc_code.restype = D
        L.wc_code.argtypes = [C.c_int, D, D, I64, P, P, P]
        L.wc_carr_f.restype = D
        L.wc_carr_f.argtypes = [D, D, I64, P]
        L.wc_carr_bf.restype = D
        L.wc_carr_bf.argtypes = [D, D, I64, P]
        L.wc_code_bf.restype = D
        L.wc_code_bf.argtypes = [D, D, I64, P, P, P]
        L.wc_code_f.restype = D
        L.wc_code_f.argtypes = [D, D, I64, P, P, P]
        L.wc_carr_seg_starts_f.restype = C.c_int
        L.wc_carr_seg_starts_f.argtypes = [D, D, I64, C.c_int, C.c_int, C.c_void_p]
        L.wc_carr_trip.restype = D
        L.wc_carr_trip.argtypes = [D, D, I64]
        L.wc_seg_states.restype = D
        L.wc_seg_states.argtypes = [D, D, C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.wc_code_seg_bf.restype = None
        L.wc_code_seg_bf.argtypes = [D, D, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_void_p, C.c_void_p]
        L.wc_carr_walk_ck.restype = D
        L.wc_carr_walk_ck.argtypes = [D, D, C.c_int, C.c_void_p]
        L.wc_margins.restype = D
        L.wc_margins.argtypes = [D, D, I64, C.c_int, C.POINTER(D), C.POINTER(D), P]
        L.wc_carr_anchors.restype = C.c_int
        L.wc_carr_anchors.argtypes = [D, D, I64, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        _walk = L
    return _walk
