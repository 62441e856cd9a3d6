"""Python binding of libgpssim_amd.so (C ABI declared in include/gpssim_amd.h).

The product is the C library: a host control plane (gss_scn_*) mirroring gpssim.c's main() and a
gfx950 HIP hot path (gss_synth_*) replacing its per-sample loop (gpssim.c:2190-2288).  This module
is plumbing for the tests and bench: ctypes prototypes, numpy views of the parameter rows, and
thin wrappers.  There is no Python or CPU implementation of the synthesis here: when the shared
library or a GPU is missing, the calls raise.
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
# The in-tree build (make -C gps-sdr-sim_amd).  Measurement builds of kernel variants
# (tools/ablate.sh) load only with both GSS_LIB_PATH and GSS_ALLOW_LIB_OVERRIDE=1 set; bench.py
# records the path it measured and the tests refuse to run on anything but the in-tree build.
_INTREE = os.path.join(PKG_DIR, "lib", "libgpssim_amd.so")
if os.environ.get("GSS_LIB_PATH") and os.environ.get("GSS_ALLOW_LIB_OVERRIDE") != "1":
    raise ImportError("GSS_LIB_PATH is set without GSS_ALLOW_LIB_OVERRIDE=1: refusing to load a "
                      "library other than the in-tree build " + _INTREE)
LIB_PATH = os.environ.get("GSS_LIB_PATH") or _INTREE
IN_TREE = os.path.abspath(LIB_PATH) == os.path.abspath(_INTREE)
CLI_PATH = os.path.join(PKG_DIR, "bin", "gps-sdr-sim")

MAXCH = 16
CA_WORDS = 32
NAV_WORDS = 60
NCK = 8                       # GSS_NCK: carrier checkpoints per block (gss_scn_next)
FMT_SC01, FMT_SC08, FMT_SC16 = 1, 8, 16

# gss_chan_blk_t (56 bytes), gpssim_amd.h
CHAN_DTYPE = np.dtype([
    ("carr0", "<f8"), ("carr_step", "<f8"), ("code0", "<f8"), ("code_step", "<f8"),
    ("icode", "<i4"), ("ibit", "<i4"), ("iword", "<i4"), ("gain", "<i4"),
    ("ca_tbl", "<i4"), ("nav_tbl", "<i4"),
])
assert CHAN_DTYPE.itemsize == 56

NGC = 8                       # GSS_NGC: signed-gain schedule entries
NPATCH = 8                    # GSS_NPATCH: patched samples per block and channel
# gss_lin_t (192 bytes): certified integer lines of one block and channel, gpssim_amd.h
LIN_DTYPE = np.dtype([
    ("x0", "<u8"), ("xs", "<u8"), ("z0", "<u8"), ("zs", "<u8"),
    ("pdelta", "<i8", (NPATCH,)),
    ("gpos", "<i4", (NGC,)), ("gval", "<i4", (NGC,)), ("ppos", "<i4", (NPATCH,)),
])
assert LIN_DTYPE.itemsize == 192

# gss_chain_t (16 bytes): the carrier chain a (block, channel) row continues, gpssim_amd.h
CHAIN_DTYPE = np.dtype([("slot", "i1"), ("reset", "u1"), ("pad", "u1", (6,)), ("init", "<f8")])
assert CHAIN_DTYPE.itemsize == 16
# the carrier chain run ahead (gss_carr_chain_guess / gss_spec_* / gss_carr_chain_spec)
# speculative segments per block (GSS_SPEC_K: 32 in the product build; a measurement build of
# another value is loaded with GSS_SPEC_K set to it as well -- lib() checks that the library
# agrees, without loading it at import: torch must load its HIP runtime first)
SPEC_K = int(os.environ.get("GSS_SPEC_K", "32"))
SPEC_IN_DTYPE = np.dtype([("g", "<f8"), ("s", "<f8"), ("k", "<i4"), ("pad", "<i4"),
                          ("P", "<i8", (SPEC_K,)), ("W", "<f8", (SPEC_K,))])
assert SPEC_IN_DTYPE.itemsize == 24 + 16 * SPEC_K
SPEC_SEG_DTYPE = np.dtype([("end", "<f8"), ("dlo", "<f8"), ("dhi", "<f8"), ("wrap_end", "<i8")])
SPEC_DTYPE = np.dtype([("p1", "<i8"), ("w1", "<f8"), ("seg", SPEC_SEG_DTYPE, (SPEC_K,))])
assert SPEC_DTYPE.itemsize == 16 + 32 * SPEC_K
SPEC_LINK_DTYPE = np.dtype([("lo", "<f8"), ("hi", "<f8"), ("dd", "<f8"), ("end", "<f8")])
assert SPEC_LINK_DTYPE.itemsize == 32
# gss_spec_rec_t: a row's speculative walk folded into one record (gss_spec_records*)
SPEC_REC_DTYPE = np.dtype([("w1", "<f8"), ("slo", "<f8"), ("shi", "<f8"), ("sdd", "<f8"),
                           ("end", "<f8"), ("llo", "<f8"), ("lhi", "<f8"), ("ldd", "<f8"),
                           ("p1", "<i4"), ("ok", "<i4")])
assert SPEC_REC_DTYPE.itemsize == 72
# gss_carr_anchor_t: the chain's exact carrier values inside a block (the proofs' walk starts)
ANCHOR_DTYPE = np.dtype([("pos", "<i4", (SPEC_K,)), ("val", "<f8", (SPEC_K,))])
assert ANCHOR_DTYPE.itemsize == 12 * SPEC_K
# gss_nav_src_t: one nav-table row's source for the GPU producer (include/gpssim_amd.h)
NAV_SRC_DTYPE = np.dtype([("sbf", "<u4", (5, 10)), ("tow", "<u4"), ("wn", "<u4"), ("prev", "<i4"),
                          ("next", "<i4"), ("head", "<u4", (10,))])
assert NAV_SRC_DTYPE.itemsize == 256
NAV_HEAD_INIT, NAV_HEAD_GIVEN = -1, -2


class GssError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gpssim_amd error {code}: {msg}")
        self.code = code


class _Opts(C.Structure):
    _fields_ = [
        ("nav_file", C.c_char_p), ("motion_file", C.c_char_p), ("nmea", C.c_int),
        ("has_xyz", C.c_int), ("xyz", C.c_double * 3), ("has_llh", C.c_int),
        ("llh", C.c_double * 3), ("samp_freq", C.c_double), ("data_format", C.c_int),
        ("duration", C.c_double), ("has_start", C.c_int), ("time_overwrite", C.c_int),
        ("start", C.c_int * 6), ("start_sec", C.c_double), ("iono_disable", C.c_int),
        ("verbose", C.c_int), ("user_motion_size", C.c_int), ("quiet", C.c_int),
        ("carrier_int", C.c_int),
    ]


class _Cli(C.Structure):
    _fields_ = [("opt", _Opts), ("nav_file", C.c_char * 256), ("motion_file", C.c_char * 256),
                ("out_file", C.c_char * 256)]


class _Info(C.Structure):
    _fields_ = [("n_per_blk", C.c_int), ("n_blocks", C.c_int), ("data_format", C.c_int),
                ("samp_freq", C.c_double), ("delt", C.c_double), ("week", C.c_int),
                ("sec", C.c_double), ("next_block", C.c_int64), ("rows_out", C.c_int64),
                ("carrier_int", C.c_int)]


_lib = None

# name -> (restype, argtypes); every symbol include/gpssim_amd.h declares
_P = C.c_void_p
# gss_sink_fn(user, bytes, n, first_block, nblocks)
SINK_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int64, C.c_int)
_SIGS = {
    "gss_run": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int, C.c_int, SINK_FN, _P]),
    "gss_run_ex": (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int, C.c_int, SINK_FN, _P, _P]),
    "gss_dev_open": (C.c_int, [C.POINTER(_P), C.c_int]),
    "gss_dev_close": (C.c_int, [_P]),
    "gss_dev_reserve": (C.c_int, [_P, C.c_int, C.c_int]),
    "gss_block_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "gss_anchor_device": (C.c_int, [_P, C.c_int, _P, _P, C.c_int, _P, C.c_int, C.c_int, _P,
                                    _P]),
    "gss_render_device": (C.c_int, [_P, C.c_int, _P, _P, C.c_int, _P, C.c_int, _P, C.c_int,
                                    C.c_int, C.c_int, C.c_int, _P, _P, _P]),
    "gss_synth_device": (C.c_int, [_P, _P, _P, C.c_int, _P, _P, C.c_int, _P, C.c_int,
                                   C.c_int, C.c_int, C.c_int, _P, _P, _P, _P]),
    "gss_synth_host": (C.c_int, [_P, _P, _P, _P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int,
                                 C.c_int, _P, _P]),
    "gss_linearize": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, _P, C.c_int, _P, _P,
                                C.c_int]),
    "gss_linearize_device": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, _P, C.c_int, _P, C.c_int, _P,
                                       _P, _P]),
    "gss_synth_lin_device": (C.c_int, [_P, _P, _P, C.c_int, _P, _P, _P, C.c_int, _P, _P,
                                       C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P,
                                       _P]),
    "gss_minmax_mod": (None, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                              C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "gss_first_below": (C.c_uint64, [C.c_uint64] * 5),
    "gss_hits_mod": (C.c_int, [C.c_uint64] * 5 + [_P, C.c_int, C.c_int]),
    "gss_dev_timing": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_float),
                                 C.POINTER(C.c_float)]),
    "gss_dev_timing_lin": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_float)]),
    "gss_scn_open": (C.c_int, [C.POINTER(_P), C.POINTER(_Opts)]),
    "gss_scn_info": (C.c_int, [_P, C.POINTER(_Info)]),
    "gss_scn_next": (C.c_int, [_P, C.c_int, _P, _P, _P, C.POINTER(C.c_int), C.c_int]),
    "gss_scn_next_deferred": (C.c_int, [_P, C.c_int, _P, _P, _P, C.POINTER(C.c_int), C.c_int]),
    "gss_carr_chain": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int]),
    "gss_carr_chain_guess": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P]),
    "gss_carr_chain_starts": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P]),
    "gss_carr_line_end": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P]),
    "gss_spec_host": (C.c_int, [_P, C.c_int, C.c_int, _P, C.c_int]),
    "gss_spec_device": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P]),
    "gss_carr_chain_spec": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, _P, C.c_int,
                                      C.POINTER(C.c_int)]),
    "gss_spec_links": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P, _P, C.c_int]),
    "gss_carr_chain_anchored": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, _P, C.c_int,
                                          C.POINTER(C.c_int), _P]),
    "gss_carr_anchors": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P, _P, C.c_int]),
    "gss_spec_records": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int]),
    "gss_spec_records_device": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P, _P, _P]),
    "gss_carr_chain_records": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, C.c_int,
                                         C.POINTER(C.c_int)]),
    "gss_linearize_ex": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, _P, C.c_int, _P, _P, _P,
                                   C.c_int]),
    "gss_linearize_device_ex": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, _P, C.c_int, _P, C.c_int,
                                          _P, _P, _P, _P]),
    "gss_carr_chain_linked": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_int, _P, _P, _P, C.c_int,
                                        C.POINTER(C.c_int)]),
    "gss_scn_seek": (C.c_int, [_P, C.c_int64, C.c_int]),
    "gss_scn_carrier": (C.c_int, [_P, _P]),
    "gss_scn_set_carrier": (C.c_int, [_P, _P]),
    "gss_scn_nav_table": (C.c_int, [_P, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_int)]),
    "gss_ca_table": (C.c_int, [_P]),
    "gss_scn_nav_sources": (C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_int)]),
    "gss_nav_rows_host": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "gss_nav_rows_device": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, _P]),
    "gss_ca_table_device": (C.c_int, [_P, _P, _P]),
    "gss_scn_plan_seconds": (C.c_double, [_P]),
    "gss_scn_close": (C.c_int, [_P]),
    "gss_carr_advance": (C.c_double, [C.c_double, C.c_double, C.c_int64]),
    "gss_carr_advance_ck": (C.c_double, [C.c_double, C.c_double, C.c_int, C.c_void_p]),
    "gss_code_advance": (C.c_double, [C.c_double, C.c_double, C.c_int64,
                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                      C.POINTER(C.c_int32)]),
    "gss_lut": (C.c_int, [_P, _P]),
    "gss_cli_parse": (C.c_int, [C.c_int, C.POINTER(C.c_char_p), C.POINTER(_Cli)]),
    "gss_cli_usage": (None, []),
    "gss_last_error": (C.c_char_p, []),
    "gss_version": (C.c_char_p, []),
    "gss_build_info": (C.c_char_p, []),
}
EXPORTED = tuple(_SIGS)


def lib():
    """Load the in-tree shared library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: run `make -C gps-sdr-sim_amd` "
                          "(or __graft_entry__.build())")
        try:
            # A process that also uses PyTorch-ROCm must resolve libamdhip64 to torch's copy:
            # load torch first so the library binds to the already-loaded runtime (two HIP
            # runtimes in one process leave torch seeing no GPU).
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        kv = dict(x.split("=", 1) for x in L.gss_build_info().decode().split())
        if int(kv.get("spec_k", "8")) != SPEC_K:          # (builds before round 6: 8)
            raise ImportError(f"{LIB_PATH} was built with GSS_SPEC_K={kv.get('spec_k')}: set "
                              f"GSS_SPEC_K to match (Python's walk dtypes use {SPEC_K})")
        _lib = L
    return _lib


def build_info():
    """The kernels' build configuration as a dict, e.g. {"lin_mfma": "1", "lin_ch": "16", ...}."""
    return dict(kv.split("=", 1) for kv in lib().gss_build_info().decode().split())


def lib_mfma():
    """True when the fast path accumulates on the matrix cores (LIN_MFMA build)."""
    return build_info().get("lin_mfma", "0") != "0"


def _check(rc):
    if rc != 0:
        raise GssError(rc, lib().gss_last_error().decode(errors="replace"))


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def block_bytes(n_per_blk, fmt):
    return int(lib().gss_block_bytes(n_per_blk, fmt))


def ca_table():
    out = np.zeros((32, CA_WORDS), np.uint32)
    _check(lib().gss_ca_table(_ptr(out)))
    return out


def nav_rows_host(src, first=0, rows=None):
    """rows [first, first + len(src)) from their sources (gss_nav_rows_host); rows: the table so
    far (>= first rows), extended and returned"""
    src = np.ascontiguousarray(src, NAV_SRC_DTYPE)
    out = np.zeros((first + len(src), NAV_WORDS), np.uint32)
    if first:
        out[:first] = rows[:first]
    _check(lib().gss_nav_rows_host(_ptr(src), first, len(src), _ptr(out)))
    return out


def lut():
    s = np.zeros(512, np.int32)
    c = np.zeros(512, np.int32)
    _check(lib().gss_lut(_ptr(s), _ptr(c)))
    return s, c


def linearize(blk, nch, nav, n_per_blk, threads=8, ca=None, anch=None):
    """(lin[nblk, 16] LIN_DTYPE, fast[nblk] int32): the certified integer lines of every block
    (gss_linearize); fast[b] == 1 where the fast path renders block b exactly.  ca: the C/A
    table the blocks' ca_tbl index (default: ca_table(), PRN 1..32).  anch: the chain's anchors
    (ANCHOR_DTYPE [nblk, 16], gss_linearize_ex): the same rows, shorter carrier walks."""
    blk = np.ascontiguousarray(blk, CHAN_DTYPE)
    nch = np.ascontiguousarray(nch, np.int32)
    nav = np.ascontiguousarray(nav, np.uint32)
    ca = np.ascontiguousarray(ca_table() if ca is None else ca, np.uint32)
    lin = np.zeros((len(nch), MAXCH), LIN_DTYPE)
    fast = np.zeros(len(nch), np.int32)
    if anch is None:
        _check(lib().gss_linearize(_ptr(blk), _ptr(nch), len(nch), n_per_blk, _ptr(ca), len(ca),
                                   _ptr(nav), len(nav), _ptr(lin), _ptr(fast), threads))
    else:
        anch = np.ascontiguousarray(anch, ANCHOR_DTYPE)
        assert anch.size == len(nch) * MAXCH
        _check(lib().gss_linearize_ex(_ptr(blk), _ptr(nch), len(nch), n_per_blk, _ptr(ca),
                                      len(ca), _ptr(nav), len(nav), _ptr(anch), _ptr(lin),
                                      _ptr(fast), threads))
    return lin, fast


def minmax_mod(n, m, a, s):
    """exact (min, max) of (a + p s) mod m over 0 <= p < n (the certificate's core)"""
    mn, mx = C.c_uint64(), C.c_uint64()
    lib().gss_minmax_mod(n, m, a, s, C.byref(mn), C.byref(mx))
    return mn.value, mx.value


def hits_mod(n, lgB, a0, st, w, cap=64, scan=False):
    """the proof's ambiguous samples (gss_hits_mod): list of p, or None if more than cap"""
    out = np.zeros(max(cap, 1), np.int64)
    k = lib().gss_hits_mod(n, lgB, a0, st, w, _ptr(out), cap, int(bool(scan)))
    if k == -2:
        raise ValueError("invalid hits_mod arguments")
    return None if k < 0 else [int(v) for v in out[:k]]


def first_below(n, m, a, s, w):
    """least p in [0, n) with (a + p s) mod m < w, or n (the proof's ambiguous-sample search)"""
    return lib().gss_first_below(n, m, a, s, w)


def carr_advance(carr, step, n):
    return lib().gss_carr_advance(carr, step, n)


def carr_advance_ck(carr, step, n):
    """(phase after n samples, the NCK checkpoints of the block)"""
    ck = np.zeros(NCK)
    end = lib().gss_carr_advance_ck(carr, step, n, _ptr(ck))
    return end, ck


def code_advance(code, step, n, icode, ibit, iword):
    a, b, c = C.c_int32(icode), C.c_int32(ibit), C.c_int32(iword)
    ph = lib().gss_code_advance(code, step, n, C.byref(a), C.byref(b), C.byref(c))
    return ph, a.value, b.value, c.value


class Scenario:
    """Host control plane: gpssim.c's main() around the sample loop (gss_scn_*)."""

    def __init__(self, nav_file, *, llh=None, xyz=None, motion_file=None, nmea=False,
                 samp_freq=2.6e6, data_format=16, duration=None, start=None,
                 time_overwrite=False, iono=True, verbose=False, quiet=True,
                 user_motion_size=3000, carrier="float"):
        if carrier not in ("float", "int"):
            raise ValueError(f"carrier must be 'float' or 'int', not {carrier!r}")
        self._keep = []
        o = _Opts()
        o.nav_file = self._s(nav_file)
        o.motion_file = self._s(motion_file) if motion_file else None
        o.nmea = int(bool(nmea))
        if xyz is not None:
            o.has_xyz = 1
            o.xyz[:] = list(map(float, xyz))
        if llh is not None:
            o.has_llh = 1
            o.llh[:] = list(map(float, llh))
        o.samp_freq = float(samp_freq)
        o.data_format = int(data_format)
        o.duration = -1.0 if duration is None else float(duration)
        if start is not None:
            o.has_start = 1
            o.start[:] = [int(v) for v in start[:5]] + [int(start[5])]
            o.start_sec = float(start[5])
            o.time_overwrite = int(bool(time_overwrite))
        o.iono_disable = 0 if iono else 1
        o.verbose = int(bool(verbose))
        o.user_motion_size = int(user_motion_size)
        o.quiet = int(bool(quiet))
        o.carrier_int = int(carrier == "int")      # FLOAT_CARR_PHASE off (gpssim.h:4)
        self._carrier_int = o.carrier_int
        self._h = C.c_void_p()
        _check(lib().gss_scn_open(C.byref(self._h), C.byref(o)))
        self._init_info()

    @classmethod
    def from_cli(cls, argv):
        """(Scenario, output path) from the reference's command line (gss_cli_parse: same
        options, defaults and error messages, gpssim.c:1650-1852).  Raises SystemExit(1) where
        the reference exits 1."""
        cli = _Cli()
        args = [b"gps-sdr-sim"] + [str(a).encode() for a in argv]
        arr = (C.c_char_p * len(args))(*args)
        if lib().gss_cli_parse(len(args), arr, C.byref(cli)):
            raise SystemExit(1)
        self = cls.__new__(cls)
        self._keep = [cli]
        self._carrier_int = cli.opt.carrier_int
        self._h = C.c_void_p()
        _check(lib().gss_scn_open(C.byref(self._h), C.byref(cli.opt)))
        self._init_info()
        return self, cli.out_file.decode()

    def _init_info(self):
        inf = _Info()
        _check(lib().gss_scn_info(self._h, C.byref(inf)))
        self.n_per_blk, self.n_blocks = inf.n_per_blk, inf.n_blocks
        self.data_format, self.samp_freq, self.delt = inf.data_format, inf.samp_freq, inf.delt
        self.start_week, self.start_sec = inf.week, inf.sec

    def position(self):
        """(next run block this handle produces, blocks whose rows it has produced)"""
        inf = _Info()
        _check(lib().gss_scn_info(self._h, C.byref(inf)))
        return inf.next_block, inf.rows_out

    def seek(self, block, threads=8):
        """Skip to run block `block` without producing the blocks before it (gss_scn_seek): only
        the 30 s updates are replayed.  The slot carriers are unknown until set_carrier()."""
        _check(lib().gss_scn_seek(self._h, int(block), threads))

    def carrier(self):
        """The planner's carrier phase per channel slot at the next block ([16] float64)."""
        c = np.zeros(MAXCH, np.float64)
        _check(lib().gss_scn_carrier(self._h, _ptr(c)))
        return c

    def set_carrier(self, carr):
        c = np.ascontiguousarray(carr, np.float64)
        assert c.shape == (MAXCH,)
        _check(lib().gss_scn_set_carrier(self._h, _ptr(c)))

    def next_deferred(self, max_blocks, threads=8):
        """Next batch without its carrier phases: (blk, nch, chain[nb, 16] CHAIN_DTYPE);
        carr_chain() fills blk["carr0"] once the slot carriers at the first block are known."""
        blk = np.zeros((max_blocks, MAXCH), CHAN_DTYPE)
        nch = np.zeros(max_blocks, np.int32)
        chain = np.zeros((max_blocks, MAXCH), CHAIN_DTYPE)
        nb = C.c_int(0)
        _check(lib().gss_scn_next_deferred(self._h, max_blocks, _ptr(blk), _ptr(nch),
                                           _ptr(chain), C.byref(nb), threads))
        n = nb.value
        return blk[:n].copy(), nch[:n].copy(), chain[:n].copy()

    @property
    def carrier_int(self):
        return bool(self._carrier_int)

    def _s(self, v):
        b = str(v).encode()
        self._keep.append(b)
        return b

    def next(self, max_blocks, threads=8, with_ck=False):
        """Next batch: (blk[nb, 16] CHAN_DTYPE, nch[nb] int32), plus the carrier checkpoints
        ck[nb, 16, NCK] float64 when with_ck (recorded by the planner's own carrier walk)."""
        blk = np.zeros((max_blocks, MAXCH), CHAN_DTYPE)
        nch = np.zeros(max_blocks, np.int32)
        ck = np.zeros((max_blocks, MAXCH, NCK), np.float64) if with_ck else None
        nb = C.c_int(0)
        _check(lib().gss_scn_next(self._h, max_blocks, _ptr(blk), _ptr(nch), _ptr(ck),
                                  C.byref(nb), threads))
        n = nb.value
        if with_ck:
            return blk[:n].copy(), nch[:n].copy(), ck[:n].copy()
        return blk[:n].copy(), nch[:n].copy()

    def all_blocks(self, batch=500, threads=8, with_ck=False):
        parts = []
        while True:
            r = self.next(batch, threads, with_ck)
            if len(r[1]) == 0:
                break
            parts.append(r)
        if not parts:
            empty = (np.zeros((0, MAXCH), CHAN_DTYPE), np.zeros(0, np.int32))
            return empty + ((np.zeros((0, MAXCH, NCK)),) if with_ck else ())
        return tuple(np.concatenate([p[i] for p in parts]) for i in range(len(parts[0])))

    def nav_table(self):
        rows = C.POINTER(C.c_uint32)()
        n = C.c_int(0)
        _check(lib().gss_scn_nav_table(self._h, C.byref(rows), C.byref(n)))
        if n.value == 0:
            return np.zeros((1, NAV_WORDS), np.uint32)
        return np.ctypeslib.as_array(rows, shape=(n.value, NAV_WORDS)).copy()

    def nav_sources(self):
        """the rows' GPU-producer sources (NAV_SRC_DTYPE [n]), same order as nav_table()"""
        src = _P()
        n = C.c_int(0)
        _check(lib().gss_scn_nav_sources(self._h, C.byref(src), C.byref(n)))
        if n.value == 0:
            return np.zeros(0, NAV_SRC_DTYPE)
        buf = (C.c_uint8 * (n.value * NAV_SRC_DTYPE.itemsize)).from_address(src.value)
        return np.frombuffer(buf, NAV_SRC_DTYPE).copy()

    def plan_seconds(self):
        return lib().gss_scn_plan_seconds(self._h)

    def close(self):
        if self._h:
            lib().gss_scn_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def carr_chain(carr, blk, nch, chain, n_per_blk, carrier_int=False, with_ck=True, threads=8):
    """The carrier chain over deferred rows (gss_carr_chain): fills blk["carr0"] in place from
    carr[16] = the slot carriers at the first block; returns (carrier after the last block,
    checkpoints [nb, 16, NCK] or None)."""
    c = np.array(carr, np.float64, copy=True)
    assert c.shape == (MAXCH,) and blk.flags.c_contiguous and blk.dtype == CHAN_DTYPE
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    nb = len(nch)
    ck = np.zeros((nb, MAXCH, NCK), np.float64) if with_ck else None
    _check(lib().gss_carr_chain(_ptr(c), _ptr(blk), _ptr(nch), _ptr(chain), nb, int(n_per_blk),
                                int(bool(carrier_int)), _ptr(ck), threads))
    return c, ck


def carr_chain_guess(carr, blk, nch, chain, n_per_blk, starts_only=False):
    """Each row's guesses (gss_carr_chain_guess): SPEC_IN_DTYPE [nb, 16].  starts_only: the
    starts alone (gss_carr_chain_starts), live rows with k = 0 for the walkers to complete."""
    c = np.ascontiguousarray(carr, np.float64)
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    gi = np.zeros((len(nch), MAXCH), SPEC_IN_DTYPE)
    fn = lib().gss_carr_chain_starts if starts_only else lib().gss_carr_chain_guess
    _check(fn(_ptr(c), _ptr(np.ascontiguousarray(blk)), _ptr(nch), _ptr(chain), len(nch),
              int(n_per_blk), _ptr(gi)))
    return gi


def carr_line_end(carr, blk, nch, chain, n_per_blk):
    """The slots' carriers after the batch by the lines of gss_carr_chain_starts (a prediction)."""
    c = np.ascontiguousarray(carr, np.float64)
    out = np.zeros(MAXCH, np.float64)
    nch = np.ascontiguousarray(nch, np.int32)
    _check(lib().gss_carr_line_end(_ptr(c), _ptr(np.ascontiguousarray(blk)), _ptr(nch),
                                   _ptr(np.ascontiguousarray(chain, CHAIN_DTYPE)), len(nch),
                                   int(n_per_blk), _ptr(out)))
    return out


def spec_host(gi, n_per_blk, threads=8):
    """The speculative walk of every row's segments (gss_spec_host): SPEC_DTYPE rows.  Rows with
    k = 0 get their segment guesses first, written back into gi (a contiguous array)."""
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE).reshape(-1)
    spec = np.zeros(len(gi), SPEC_DTYPE)
    _check(lib().gss_spec_host(_ptr(gi), len(gi), int(n_per_blk), _ptr(spec), threads))
    return spec


def carr_chain_spec(carr, blk, nch, chain, n_per_blk, gi, spec, threads=8):
    """The carrier chain from the rows' speculative walks (gss_carr_chain_spec): fills
    blk["carr0"] in place; returns (carrier after the last block, blocks where the translation
    carried through)."""
    c = np.array(carr, np.float64, copy=True)
    assert c.shape == (MAXCH,) and blk.flags.c_contiguous and blk.dtype == CHAN_DTYPE
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    assert spec.size == gi.size == len(nch) * MAXCH
    hit = C.c_int(0)
    _check(lib().gss_carr_chain_spec(_ptr(c), _ptr(blk), _ptr(nch), _ptr(chain), len(nch),
                                     int(n_per_blk), _ptr(gi), _ptr(spec), threads,
                                     C.byref(hit)))
    return c, hit.value


def carr_chain_anchored(carr, blk, nch, chain, n_per_blk, gi, spec, threads=8):
    """carr_chain_spec, also returning the chain's anchors (gss_carr_chain_anchored):
    (end carriers, hits, ANCHOR_DTYPE [nb, 16])."""
    c = np.array(carr, np.float64, copy=True)
    assert c.shape == (MAXCH,) and blk.flags.c_contiguous and blk.dtype == CHAN_DTYPE
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    assert spec.size == gi.size == len(nch) * MAXCH
    anch = np.zeros((len(nch), MAXCH), ANCHOR_DTYPE)
    hit = C.c_int(0)
    _check(lib().gss_carr_chain_anchored(_ptr(c), _ptr(blk), _ptr(nch), _ptr(chain), len(nch),
                                         int(n_per_blk), _ptr(gi), _ptr(spec), threads,
                                         C.byref(hit), _ptr(anch)))
    return c, hit.value, anch


def carr_anchors(blk, nch, n_per_blk, gi, spec, threads=8):
    """The anchors of rows whose carr0 a chain has set (gss_carr_anchors): ANCHOR_DTYPE [nb, 16]."""
    blk = np.ascontiguousarray(blk, CHAN_DTYPE)
    nch = np.ascontiguousarray(nch, np.int32)
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    assert spec.size == gi.size == len(nch) * MAXCH
    anch = np.zeros((len(nch), MAXCH), ANCHOR_DTYPE)
    _check(lib().gss_carr_anchors(_ptr(blk), _ptr(nch), len(nch), int(n_per_blk), _ptr(gi),
                                  _ptr(spec), _ptr(anch), threads))
    return anch


def spec_records(gi, spec, n_per_blk, threads=8):
    """Each row's record (gss_spec_records; the previous row of its slot from gi["pad"]):
    SPEC_REC_DTYPE rows shaped like gi."""
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    assert spec.size == gi.size
    rec = np.zeros(gi.shape, SPEC_REC_DTYPE)
    _check(lib().gss_spec_records(_ptr(gi), _ptr(spec), gi.size, int(n_per_blk), _ptr(rec),
                                  threads))
    return rec


def carr_chain_records(carr, blk, nch, chain, n_per_blk, rec, threads=8):
    """The chain from the rows' records (gss_carr_chain_records): fills blk["carr0"] in place;
    returns (carrier after the last block, rows whose record held)."""
    c = np.array(carr, np.float64, copy=True)
    assert c.shape == (MAXCH,) and blk.flags.c_contiguous and blk.dtype == CHAN_DTYPE
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    rec = np.ascontiguousarray(rec, SPEC_REC_DTYPE)
    assert rec.size == len(nch) * MAXCH
    hit = C.c_int(0)
    _check(lib().gss_carr_chain_records(_ptr(c), _ptr(blk), _ptr(nch), _ptr(chain), len(nch),
                                        int(n_per_blk), _ptr(rec), threads, C.byref(hit)))
    return c, hit.value


def spec_links(nch, chain, n_per_blk, gi, spec, threads=8):
    """Each row's link from its slot's previous row (gss_spec_links): SPEC_LINK_DTYPE [nb, 16]."""
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    assert spec.size == gi.size == len(nch) * MAXCH
    link = np.zeros((len(nch), MAXCH), SPEC_LINK_DTYPE)
    _check(lib().gss_spec_links(_ptr(nch), _ptr(chain), len(nch), int(n_per_blk), _ptr(gi),
                                _ptr(spec), _ptr(link), threads))
    return link


def carr_chain_linked(carr, blk, nch, chain, n_per_blk, gi, spec, link, threads=8):
    """carr_chain_spec's result with the rows' links (gss_carr_chain_linked): fills blk["carr0"]
    in place; returns (carrier after the last block, blocks where the translation held)."""
    c = np.array(carr, np.float64, copy=True)
    assert c.shape == (MAXCH,) and blk.flags.c_contiguous and blk.dtype == CHAN_DTYPE
    nch = np.ascontiguousarray(nch, np.int32)
    chain = np.ascontiguousarray(chain, CHAIN_DTYPE)
    gi = np.ascontiguousarray(gi, SPEC_IN_DTYPE)
    spec = np.ascontiguousarray(spec, SPEC_DTYPE)
    link = np.ascontiguousarray(link, SPEC_LINK_DTYPE)
    assert spec.size == gi.size == link.size == len(nch) * MAXCH
    hit = C.c_int(0)
    _check(lib().gss_carr_chain_linked(_ptr(c), _ptr(blk), _ptr(nch), _ptr(chain), len(nch),
                                       int(n_per_blk), _ptr(gi), _ptr(spec), _ptr(link), threads,
                                       C.byref(hit)))
    return c, hit.value


class Device:
    """One GPU (gss_dev_*).  synth_host() moves host arrays; synth_device() takes raw device
    pointers (e.g. torch tensors' data_ptr()) and is stream-ordered."""

    def __init__(self, ordinal=0):
        self._h = C.c_void_p()
        _check(lib().gss_dev_open(C.byref(self._h), int(ordinal)))

    def reserve(self, max_blocks, n_per_blk):
        _check(lib().gss_dev_reserve(self._h, max_blocks, n_per_blk))

    def synth_host(self, blk, nch, ca, nav, n_per_blk, fmt, want_carr_end=False, ck=None):
        """ck: optional carrier checkpoints [nblk, 16, NCK] (Scenario.next(with_ck=True))."""
        blk = np.ascontiguousarray(blk, CHAN_DTYPE)
        if ck is not None:
            ck = np.ascontiguousarray(ck, np.float64)
            assert ck.shape == (len(nch), MAXCH, NCK), ck.shape
        nch = np.ascontiguousarray(nch, np.int32)
        ca = np.ascontiguousarray(ca, np.uint32)
        nav = np.ascontiguousarray(nav, np.uint32)
        nblk = len(nch)
        out = np.empty(nblk * block_bytes(n_per_blk, fmt), np.uint8)
        cend = np.zeros((nblk, MAXCH), np.float64) if want_carr_end else None
        _check(lib().gss_synth_host(self._h, _ptr(blk), _ptr(nch), _ptr(ck), _ptr(ca), len(ca),
                                    _ptr(nav), len(nav), nblk, n_per_blk, fmt, _ptr(out),
                                    _ptr(cend)))
        return (out, cend) if want_carr_end else out

    def synth_device(self, blk_ptr, nch_ptr, nch_max, ca_ptr, n_ca, nav_ptr, n_nav, nblk,
                     n_per_blk, fmt, out_ptr, carr_end_ptr=0, status_ptr=0, stream=0, ck_ptr=0):
        _check(lib().gss_synth_device(self._h, blk_ptr, nch_ptr, nch_max, ck_ptr or None, ca_ptr,
                                      n_ca, nav_ptr,
                                      n_nav, nblk, n_per_blk, fmt, out_ptr,
                                      carr_end_ptr or None, status_ptr or None, stream or None))

    def ca_table_device(self, out_ptr, stream=0):
        """the C/A table built on the device (gss_ca_table_device) into out_ptr [32][CA_WORDS]"""
        _check(lib().gss_ca_table_device(self._h, out_ptr, stream or None))

    def nav_rows_device(self, src_ptr, first, n, rows_ptr, stream=0):
        """nav rows [first, first + n) from device sources (gss_nav_rows_device)"""
        _check(lib().gss_nav_rows_device(self._h, src_ptr, first, n, rows_ptr, stream or None))

    def synth_lin_device(self, blk_ptr, nch_ptr, nch_max, lin_ptr, fast_ptr, fb_ptr, n_fb, ca_ptr,
                         n_ca, nav_ptr, n_nav, nblk, n_per_blk, fmt, out_ptr, status_ptr=0,
                         stream=0, ck_ptr=0):
        """gss_synth_lin_device: the certified fast path for blocks with fast[b] == 1 and the
        exact path for the n_fb blocks listed at fb_ptr; device pointers, stream-ordered."""
        _check(lib().gss_synth_lin_device(self._h, blk_ptr, nch_ptr, nch_max, lin_ptr, fast_ptr,
                                          fb_ptr or None, n_fb, ck_ptr or None, ca_ptr, n_ca,
                                          nav_ptr, n_nav, nblk, n_per_blk, fmt, out_ptr,
                                          status_ptr or None, stream or None))

    def timing_lin(self):
        """(fast-path launches, their average ms) since the last timing_reset()"""
        n, t = C.c_int(), C.c_float()
        _check(lib().gss_dev_timing_lin(self._h, C.byref(n), C.byref(t)))
        return n.value, t.value

    def anchor_device(self, set_, blk_ptr, nch_ptr, nch_max, nblk, n_per_blk, ck_ptr=0,
                      carr_end_ptr=0, stream=0):
        """Stage A of a batch into anchor set set_ (0/1), asynchronous on stream."""
        _check(lib().gss_anchor_device(self._h, set_, blk_ptr, nch_ptr, nch_max, ck_ptr or None,
                                       nblk, n_per_blk, carr_end_ptr or None, stream or None))

    def render_device(self, set_, blk_ptr, nch_ptr, nch_max, ca_ptr, n_ca, nav_ptr, n_nav, nblk,
                      n_per_blk, fmt, out_ptr, status_ptr=0, stream=0):
        """Stage B of a batch from anchor set set_, asynchronous on stream."""
        _check(lib().gss_render_device(self._h, set_, blk_ptr, nch_ptr, nch_max, ca_ptr, n_ca,
                                       nav_ptr, n_nav, nblk, n_per_blk, fmt, out_ptr,
                                       status_ptr or None, stream or None))

    def run(self, scn, sink, first_block=0, n_blocks=-1, batch=100, threads=8):
        """Stream blocks [first_block, first_block + n_blocks) of Scenario scn through gss_run;
        sink(memoryview, first_block, nblocks) gets each batch's bytes in run order (the view
        is valid only during the call).  An exception in sink stops the run and is re-raised."""
        err = []

        def _sink(user, ptr, n, first, nb):
            try:
                sink(memoryview((C.c_char * n).from_address(ptr)).cast("B"), first, nb)
                return 0
            except BaseException as e:          # noqa: BLE001 — re-raised below
                err.append(e)
                return 1

        cb = SINK_FN(_sink)
        rc = lib().gss_run(self._h, scn._h, first_block, n_blocks, batch, threads, cb, None)
        if err:
            raise err[0]
        _check(rc)

    def timing_reset(self):
        _check(lib().gss_dev_timing(self._h, 1, None, None, None))

    def timing(self):
        """(Stage B launches, avg Stage A ms, avg Stage B ms) since the last reset."""
        n, a, b = C.c_int(), C.c_float(), C.c_float()
        _check(lib().gss_dev_timing(self._h, 0, C.byref(n), C.byref(a), C.byref(b)))
        return n.value, a.value, b.value

    def linearize_device(self, blk_ptr, nch_ptr, nblk, n_per_blk, ca_ptr, n_ca, nav_ptr, n_nav,
                         lin_ptr, fast_ptr, stream=0, anch_ptr=None):
        """gss_linearize_device: the fast path's proofs on the GPU (device pointers, rows as
        gss_linearize's, async on stream); anch_ptr: the chain's anchors on the device
        (gss_linearize_device_ex)."""
        if anch_ptr is None:
            _check(lib().gss_linearize_device(self._h, C.c_void_p(blk_ptr), C.c_void_p(nch_ptr),
                                              nblk, n_per_blk, C.c_void_p(ca_ptr), n_ca,
                                              C.c_void_p(nav_ptr), n_nav, C.c_void_p(lin_ptr),
                                              C.c_void_p(fast_ptr), C.c_void_p(stream)))
        else:
            _check(lib().gss_linearize_device_ex(self._h, C.c_void_p(blk_ptr),
                                                 C.c_void_p(nch_ptr), nblk, n_per_blk,
                                                 C.c_void_p(ca_ptr), n_ca, C.c_void_p(nav_ptr),
                                                 n_nav, C.c_void_p(anch_ptr), C.c_void_p(lin_ptr),
                                                 C.c_void_p(fast_ptr), C.c_void_p(stream)))

    def spec_records_device(self, in_ptr, nrow, n_per_blk, d_in_ptr, d_spec_ptr, rec_ptr,
                            stream=0):
        """gss_spec_records_device: walks and records on the GPU (in / rec host-visible, d_in /
        d_spec device scratch of nrow rows), async on stream."""
        _check(lib().gss_spec_records_device(self._h, C.c_void_p(in_ptr), nrow, n_per_blk,
                                             C.c_void_p(d_in_ptr), C.c_void_p(d_spec_ptr),
                                             C.c_void_p(rec_ptr), C.c_void_p(stream)))

    def spec_device(self, in_ptr, nrow, n_per_blk, spec_ptr, stream=0):
        """gss_spec_device on raw device pointers (nrow SPEC_IN_DTYPE rows in, SPEC_DTYPE rows
        out), async on stream."""
        _check(lib().gss_spec_device(self._h, C.c_void_p(in_ptr), nrow, n_per_blk,
                                     C.c_void_p(spec_ptr), C.c_void_p(stream)))

    def close(self):
        if self._h:
            lib().gss_dev_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
