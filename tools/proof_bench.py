"""Time gss_linearize_device against gss_linearize on one slot's rows (GPU box only).

usage: python tools/proof_bench.py [fmt] [blocks] [repeats] [sample rate]
Prints one JSON line: device ms per call (HIP events), host ms (1 and 16 threads), rows equal,
without and with the chain's anchors (gss_linearize_device_ex; the rows are planned by the
speculative chain, gss_carr_chain_anchored, so the anchors are its by-products)."""
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
    n = s.n_per_blk
    c0 = s.carrier()
    blk, nch, chain = s.next_deferred(nb, 16)
    gi = G.carr_chain_guess(c0, blk, nch, chain, n, starts_only=True)
    spec = G.spec_host(gi, n, threads=16)
    _, _, anch = G.carr_chain_anchored(c0, blk, nch, chain, n, gi, spec, threads=16)
    nav = s.nav_table()
    t = torch.device("cuda", 0)
    dev = G.Device(0)
    ca = G.ca_table()

    def up(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(t)
    d_blk, d_nch, d_ca, d_nav = up(blk), up(np.asarray(nch, np.int32)), up(ca), up(nav)
    d_anch = up(anch)
    d_lin = torch.empty(nb * G.MAXCH * G.LIN_DTYPE.itemsize, dtype=torch.uint8, device=t)
    d_fast = torch.empty(nb, dtype=torch.int32, device=t)
    st = torch.cuda.current_stream(t)
    out = {"lib": os.path.relpath(G.LIB_PATH, REPO), "fs": fs, "fmt": fmt, "blocks": nb,
           "channels": int(np.sum(nch)), "build": G.build_info()}
    for tag, a_dev, a_host in (("", None, None), ("anch_", d_anch, anch)):
        times = []
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            dev.linearize_device(d_blk.data_ptr(), d_nch.data_ptr(), nb, n, d_ca.data_ptr(),
                                 len(ca), d_nav.data_ptr(), len(nav), d_lin.data_ptr(),
                                 d_fast.data_ptr(), st.cuda_stream,
                                 anch_ptr=a_dev.data_ptr() if a_dev is not None else None)
            e1.record(st)
            torch.cuda.synchronize(t)
            if r:
                times.append(e0.elapsed_time(e1))
        host = {}
        for th in (1, 16):
            t0 = time.perf_counter()
            lin, fast = G.linearize(blk, nch, nav, n, threads=th, anch=a_host)
            host[th] = (time.perf_counter() - t0) * 1e3
        same = bool(np.array_equal(d_lin.cpu().numpy(), lin.view(np.uint8).reshape(-1)) and
                    np.array_equal(d_fast.cpu().numpy(), fast))
        out.update({tag + "device_ms": [round(x, 3) for x in times],
                    tag + "host_ms_1": round(host[1], 2), tag + "host_ms_16": round(host[16], 2),
                    tag + "same": same})
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
