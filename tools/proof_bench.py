"""Time gss_linearize_device against gss_linearize on one slot's rows (GPU box only).

usage: python tools/proof_bench.py [fmt] [blocks] [repeats] [sample rate]
Prints one JSON line: device ms per call (HIP events), host ms (1 and 16 threads), rows equal."""
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpssim_amd as G  # noqa: E402
import bench as B  # noqa: E402


def main():
    fmt = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    fs = float(sys.argv[4]) if len(sys.argv) > 4 else 2.6e6
    s = G.Scenario(B.NAV, llh=B.LOC, duration=nb / 10 + 1, samp_freq=fs, data_format=fmt)
    blk, nch = s.next(nb, 16)[:2]
    nav = s.nav_table()
    n = s.n_per_blk
    t = torch.device("cuda", 0)
    dev = G.Device(0)
    ca = G.ca_table()

    def up(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(t)
    d_blk, d_nch, d_ca, d_nav = up(blk), up(np.asarray(nch, np.int32)), up(ca), up(nav)
    d_lin = torch.empty(nb * G.MAXCH * G.LIN_DTYPE.itemsize, dtype=torch.uint8, device=t)
    d_fast = torch.empty(nb, dtype=torch.int32, device=t)
    st = torch.cuda.current_stream(t)
    times = []
    for r in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dev.linearize_device(d_blk.data_ptr(), d_nch.data_ptr(), nb, n, d_ca.data_ptr(), len(ca),
                             d_nav.data_ptr(), len(nav), d_lin.data_ptr(), d_fast.data_ptr(),
                             st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize(t)
        if r:
            times.append(e0.elapsed_time(e1))
    host = {}
    for th in (1, 16):
        t0 = time.perf_counter()
        lin, fast = G.linearize(blk, nch, nav, n, threads=th)
        host[th] = (time.perf_counter() - t0) * 1e3
    same = bool(np.array_equal(d_lin.cpu().numpy(), lin.view(np.uint8).reshape(-1)) and
                np.array_equal(d_fast.cpu().numpy(), fast))
    print(json.dumps({"lib": os.path.relpath(G.LIB_PATH, REPO), "fs": fs, "fmt": fmt, "blocks": nb, "channels": int(np.sum(nch)),
                      "device_ms": [round(x, 3) for x in times],
                      "host_ms_1": round(host[1], 2), "host_ms_16": round(host[16], 2),
                      "same": same, "build": G.build_info()}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
