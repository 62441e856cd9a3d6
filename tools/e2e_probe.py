"""gss_run wall time against run length (static -b 16): the slope is the steady-state rate, the
intercept the fixed start-up (device/pinned allocations, the first planned batch).  GPU box only."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gps-sdr-sim_amd"))
import torch  # noqa: F401  (the HIP runtime the library shares)
import gpssim_amd as G

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
NAV = os.path.join(REPO, "tests", "golden", "data", "brdc3540.14n")
dev = G.Device(0)
rows = []
for window in [float(w) for w in (sys.argv[1:] or ["60", "600", "1800", "3600"])]:
    s = G.Scenario(NAV, llh=(30.286502, 120.032669, 100), duration=window, samp_freq=2.6e6,
                   data_format=16)
    t = {"first": None, "blocks": 0}
    t0 = time.perf_counter()

    def sink(mv, first, nb):
        if t["first"] is None:
            t["first"] = time.perf_counter() - t0
        t["blocks"] += nb

    dev.run(s, sink, batch=int(os.environ.get("GSS_PROBE_BATCH", "256")), threads=16)
    wall = time.perf_counter() - t0
    rows.append((window, wall, t["first"], t["blocks"]))
    print(f"window {window:7.0f} s  wall {wall:.3f} s  first sink {t['first']:.3f} s  "
          f"blocks {t['blocks']}  {t['blocks'] * 260000 / wall / 1e6:.0f} MS/s", flush=True)
(w0, t0_, _, b0), (w1, t1, _, b1) = rows[-2], rows[-1]
print(f"steady {(b1 - b0) * 260000 / (t1 - t0_) / 1e6:.0f} MS/s "
      f"({(b1 - b0) * 1040000 / (t1 - t0_) / 1e9:.1f} GB/s of -b 16 output)")
