"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU oracle (oracle/_ref/libgss_oracle.so)
and the reference binary (oracle/_ref/gps-sdr-sim).  Imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by the product (gps-sdr-sim_amd/)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
LIB = os.path.join(REF_DIR, "libgss_oracle.so")
CLI = os.path.join(REF_DIR, "gss_oracle_cli")
REF_BIN = os.path.join(REF_DIR, "gps-sdr-sim")

_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.oracle_synth.restype = C.c_int
        L.oracle_synth.argtypes = [P, P, P, P, C.c_int, C.c_int, C.c_int, P, P]
        L.oracle_block_bytes.restype = C.c_size_t
        L.oracle_block_bytes.argtypes = [C.c_int, C.c_int]
        L.oracle_carr_brute.restype = C.c_double
        L.oracle_carr_brute.argtypes = [C.c_double, C.c_double, C.c_int64]
        L.oracle_carr_trace.restype = None
        L.oracle_carr_trace.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_int, C.c_void_p]
        L.oracle_code_brute.restype = C.c_double
        L.oracle_code_brute.argtypes = [C.c_double, C.c_double, C.c_int64,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32)]
        L.oracle_lut.restype = None
        L.oracle_lut.argtypes = [P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def synth(blk, nch, ca, nav, n_per_blk, fmt, want_carr_end=False):
    """Reference sample loop on the CPU (gpssim.c:2190-2288) for the given block parameters."""
    blk = np.ascontiguousarray(blk)
    nch = np.ascontiguousarray(nch, np.int32)
    ca = np.ascontiguousarray(ca, np.uint32)
    nav = np.ascontiguousarray(nav, np.uint32)
    nblk = len(nch)
    out = np.empty(nblk * lib().oracle_block_bytes(n_per_blk, fmt), np.uint8)
    cend = np.zeros((nblk, 16)) if want_carr_end else None
    rc = lib().oracle_synth(_p(blk), _p(nch), _p(ca), _p(nav), nblk, n_per_blk, fmt, _p(out),
                            _p(cend))
    return (out, cend, rc) if want_carr_end else (out, rc)


def carr_brute(x, s, n):
    return lib().oracle_carr_brute(x, s, n)


def carr_brute_trace(x, s, at):
    """Brute-force carrier chain from x sampled at the ascending sample indices `at`."""
    at = np.ascontiguousarray(at, np.int64)
    out = np.zeros(len(at))
    lib().oracle_carr_trace(x, s, at.ctypes.data, len(at), out.ctypes.data)
    return out


def code_brute(c, s, n, icode, ibit, iword):
    a, b, d = C.c_int32(icode), C.c_int32(ibit), C.c_int32(iword)
    ph = lib().oracle_code_brute(c, s, n, C.byref(a), C.byref(b), C.byref(d))
    return ph, a.value, b.value, d.value


def lut():
    s = np.zeros(512, np.int32)
    c = np.zeros(512, np.int32)
    lib().oracle_lut(_p(s), _p(c))
    return s, c
