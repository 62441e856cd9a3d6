"""gss_run over a sequence of bench.py's end-to-end workloads in one process (as bench.py runs
them: the headline's 1800 s -b 16, then configs[2..4]), each run wall-clocked: whether a run's
rate depends on the runs before it (pooled buffers, streams).  Usage: python
tools/e2e_seq_probe.py <item> [<item> ...], item = h (the headline's run) or c2/c3/c4, with
an optional :batch suffix.  GPU box only."""
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import torch  # noqa: F401  (the HIP runtime the library shares)
import gpssim_amd as G  # noqa: E402
import bench as B  # noqa: E402

dev = G.Device(0)
for item in sys.argv[1:]:
    name, _, b = item.partition(":")
    if name == "h":
        c = {"name": "headline", "fs": B.FS, "fmt": 16, "window": 1800.0, "kw": {"llh": B.LOC}}
    else:
        c = B.CONFIGS[int(name[1:]) - 2]
    bb = G.block_bytes(int(round(c["fs"] / 10)), c["fmt"])
    batch = int(b) if b else max(1, B.E2E_SLOT_BYTES // bb)
    s = G.Scenario(B.NAV, duration=c["window"], samp_freq=c["fs"], data_format=c["fmt"],
                   **c["kw"])
    got = {"bytes": 0}

    def sink(mv, first, nb):
        got["bytes"] += len(mv)

    t0 = time.perf_counter()
    dev.run(s, sink, batch=batch, threads=16)
    wall = time.perf_counter() - t0
    print(f"{c['name']} batch {batch}: {wall * 1e3:.1f} ms, {got['bytes'] / wall / 1e9:.2f} GB/s",
          flush=True)
