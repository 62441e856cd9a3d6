#!/usr/bin/env python3
"""In-kernel clock of gss_lin_kernel (MI355X_MICROARCH.md, "DVFS give-back" item 6).

Runs the bench workload (BASELINE configs[1]: static 300 s, 2.6 MS/s, -b 16) through a
diagnostic build of the library (a stamp variant of gss_synth.hip built by tools/ablate.sh with
SYNTH_SRC: the product source carries no stamps; the LIN_STAMP=1 build of commit 898e226 is
one), first
back to back for --hold seconds so that the clock has settled, then --steps timed launches.  Each
wave stamps s_memtime (shader cycles) and s_memrealtime (100 MHz) around its chunk loop; the
stamps of the last launch give, per wave, the cycles it took and the clock it ran at
(cycles / ticks x 100 MHz).  Prints one JSON line: kernel ms (HIP events over the timed
launches), median wave cycles, median and quartile clocks, and the launch's wall span from the
stamps.

usage: GSS_ALLOW_LIB_OVERRIDE=1 GSS_LIB_PATH=_var/<stamp build>/libgpssim_amd.so \
           python tools/clock_stamp.py [--label NAME] [--fmt 16] [--hold 2.5] [--steps 20]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="")
    ap.add_argument("--fmt", type=int, default=16)
    ap.add_argument("--window", type=float, default=300.0)
    ap.add_argument("--hold", type=float, default=2.5, help="seconds of back-to-back launches")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()

    import torch
    import gpssim_amd as G
    from gpssim_amd.render import DeviceWindow
    from gpssim_amd.shard import plan_rank
    import bench

    blk, nch, ck, nav, npb, _ = plan_rank(bench.NAV, 0, 1, args.window, llh=bench.LOC,
                                          samp_freq=bench.FS, data_format=args.fmt,
                                          threads=args.threads)
    dev_t = torch.device("cuda", 0)
    dev = G.Device(0)
    stream = torch.cuda.current_stream(dev_t).cuda_stream
    res = DeviceWindow(torch, dev, dev_t, blk, nch, nav, npb, args.fmt, ck=ck,
                       threads=args.threads, batch=len(nch))
    t0 = time.perf_counter()
    n_hold = 0
    while time.perf_counter() - t0 < args.hold:
        for _ in range(10):
            res.step(stream)
        torch.cuda.synchronize(dev_t)
        n_hold += 10
    dev.timing_reset()
    for _ in range(args.steps):
        res.step(stream)
    torch.cuda.synchronize(dev_t)
    n_lin, lin_ms = dev.timing_lin()

    lib = G.lib()
    out = {"label": args.label, "lib": os.path.relpath(G.LIB_PATH, REPO),
           "kernel_ms": round(lin_ms, 4), "launches_held": n_hold, "steps": args.steps}
    fn = getattr(lib, "gss_diag_lin_stamps", None)
    if fn is None:
        out["error"] = "not a LIN_STAMP build (no gss_diag_lin_stamps)"
        print(json.dumps(out), flush=True)
        return
    nseg = (npb + 4095) // 4096
    wg_per_blk = (nseg + 3) // 4
    n_waves = res.nblk * wg_per_blk * 4
    buf = np.zeros((n_waves, 4), np.uint64)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    fn.restype = ctypes.c_int
    if fn(buf.ctypes.data, n_waves) != 0:
        raise RuntimeError("gss_diag_lin_stamps failed")
    ok = (buf[:, 1] > buf[:, 0]) & (buf[:, 3] > buf[:, 2])
    st = buf[ok].astype(np.float64)
    cyc = st[:, 1] - st[:, 0]
    ticks = st[:, 3] - st[:, 2]
    clk = cyc / ticks * 100.0                       # MHz
    span_ms = (st[:, 3].max() - st[:, 2].min()) / 1e5   # 100 MHz ticks -> ms
    q = np.percentile(clk, [25, 50, 75])
    out.update({"waves": int(ok.sum()), "wave_cycles_median": float(np.median(cyc)),
                "wave_cycles_sum": float(cyc.sum()),
                "clock_mhz_median": round(float(q[1]), 1),
                "clock_mhz_q25": round(float(q[0]), 1), "clock_mhz_q75": round(float(q[2]), 1),
                "wave_us_median": round(float(np.median(ticks)) / 100.0, 2),
                "launch_span_ms_from_stamps": round(float(span_ms), 4)})
    print(json.dumps(out), flush=True)
    res.free()
    dev.close()


if __name__ == "__main__":
    main()
