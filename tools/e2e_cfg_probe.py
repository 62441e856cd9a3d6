"""gss_run over one of bench.py's per-config workloads (configs[2..4]) with the run's own trace
(GSS_RUN_TRACE=1 on stderr, summarised by tools/e2e_trace_summary.py): where the end-to-end time of a
non-headline config goes.  Usage: python tools/e2e_cfg_probe.py <config index 2-4> [window s]
[threads] [batch blocks].  GPU box only."""
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import torch  # noqa: F401  (the HIP runtime the library shares)
import gpssim_amd as G
import bench as B

c = B.CONFIGS[int(sys.argv[1]) - 2]
window = float(sys.argv[2]) if len(sys.argv) > 2 else c["window"]
threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
dev = G.Device(0)
bb = G.block_bytes(int(round(c["fs"] / 10)), c["fmt"])
batch = int(sys.argv[4]) if len(sys.argv) > 4 else max(1, B.E2E_SLOT_BYTES // bb)
s = G.Scenario(B.NAV, duration=window, samp_freq=c["fs"], data_format=c["fmt"], **c["kw"])
got = {"blocks": 0, "bytes": 0}


def sink(mv, first, nb):
    got["blocks"] += nb
    got["bytes"] += len(mv)


for rep in range(int(os.environ.get("E2E_REPEAT", "1"))):   # later runs: warm (pooled buffers)
    if rep:
        s = G.Scenario(B.NAV, duration=window, samp_freq=c["fs"], data_format=c["fmt"], **c["kw"])
        got = {"blocks": 0, "bytes": 0}
    t0 = time.perf_counter()
    dev.run(s, sink, batch=batch, threads=threads)
    wall = time.perf_counter() - t0
    print(f"{c['name']} run {rep} window {window:g} s batch {batch} threads {threads}: "
          f"{got['blocks']} blocks in {wall:.3f} s = {got['blocks'] / wall:.0f} blocks/s, "
          f"{got['bytes'] / wall / 1e9:.2f} GB/s, {wall / got['blocks'] * 1e6:.1f} us/block",
          flush=True)
