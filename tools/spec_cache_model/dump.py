"""The headline window's speculative-walk rows (static 300 s, 2.6 MS/s), planned on the host with
the host walker, written to heads.bin for model.c (tools/spec_cache_model)."""
import sys, numpy as np
import os
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
sys.path.insert(0, REPO)
import gpssim_amd as G
from gpssim_amd.shard import plan_rank, host_walker
from bench import NAV, LOC
blk, nch, ck, nav, npb, t = plan_rank(NAV, 0, 1, 300.0, llh=LOC, threads=8, walker=host_walker(8), anchors=True)
h = t["spec_heads"]
print(h.shape, h.dtype, npb)
h.reshape(-1).view(np.uint8).tofile("heads.bin")       # model.c reads it
