"""Two gss_run legs in one process, each with its own GSS_RUN_ROWS_AHEAD: configs[4]'s whole day,
then the headline's static -b 16 1800 s (bench.py's order), to see whether a run's threads slow a
later run's downloads.  Usage: python tools/e2e_order_probe.py <ahead first> <ahead second>.
GPU box only."""
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import torch  # noqa: F401
import gpssim_amd as G
import bench as B

dev = G.Device(0)
c = B.CONFIGS[2]
os.environ["GSS_RUN_ROWS_AHEAD"] = sys.argv[1]
r4 = B.e2e_run(G, dev, 16, window=c["window"], fs=c["fs"], fmt=c["fmt"], kw=c["kw"], slope=False)
os.environ["GSS_RUN_ROWS_AHEAD"] = sys.argv[2]
r16 = B.e2e_run(G, dev, 16, batch=128)
print(f"ahead {sys.argv[1]} -> {sys.argv[2]}: configs[4] {r4['value']} ({r4['wall_s']} s); "
      f"static -b 16 {r16['value']} frac {r16['frac_of_d2h_ceiling']} steady {r16['steady_d2h_GBps']}",
      flush=True)
