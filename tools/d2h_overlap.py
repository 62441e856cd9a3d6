"""Does a device-to-host copy, or the fast-path kernel beside it, slow down when the two overlap?
(GPU box only.)  A configs[4] slot: 2048 blocks of -b 1 at 2.6 MS/s (133 MB out).

Times, with HIP events: the D2H of 133 MB from HBM into pinned memory alone; the fast-path
kernels of one 2048-block batch alone (DeviceWindow.step_batch); both at once on two streams;
the D2H beside compute-bound GEMMs; the D2H while host threads plan rows (the planner's CPU
load in gss_run); a 10 MB upload (a slot's inputs) alone and during the D2H ("_kern_ms" of the
"up" modes is the upload's time); the D2H while 8 host threads copy 64 MB arrays (copy_mem); 16 back-to-back downloads into one
buffer and cycling over four (gss_run's slots); a slot's carrier walks (gss_spec_device on pinned
rows, high-priority stream) alone, beside the download, and beside download and render.  Prints one JSON line.   usage: python tools/d2h_overlap.py [reps]"""
import json
import os
import sys
import threading
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import torch  # noqa: E402
import gpssim_amd as G  # noqa: E402
import bench as B  # noqa: E402
from gpssim_amd.render import DeviceWindow  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev_t = torch.device("cuda", 0)
    dev = G.Device(0)
    s = G.Scenario(B.NAV, llh=B.LOC, duration=205.0, samp_freq=2.6e6, data_format=1)
    blk, nch = s.all_blocks(batch=2048, threads=16)
    res = DeviceWindow(torch, dev, dev_t, blk, nch, s.nav_table(), s.n_per_blk, 1, threads=16,
                       batch=2048)
    src = torch.empty(133 << 20, dtype=torch.uint8, device=dev_t).fill_(7)
    dst = torch.empty(133 << 20, dtype=torch.uint8, pin_memory=True)
    dsts = [torch.empty(133 << 20, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    srcs = [torch.empty(133 << 20, dtype=torch.uint8, device=dev_t).fill_(5) for _ in range(4)]
    cp, cs = torch.cuda.Stream(dev_t), torch.cuda.Stream(dev_t)
    a = torch.randn(8192, 8192, device=dev_t, dtype=torch.bfloat16)
    up_src = torch.empty(10 << 20, dtype=torch.uint8, pin_memory=True).fill_(3)
    up_dst = torch.empty(10 << 20, dtype=torch.uint8, device=dev_t)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def copy_on(st):
        e0, e1 = ev(), ev()
        e0.record(st)
        with torch.cuda.stream(st):
            dst.copy_(src, non_blocking=True)
        e1.record(st)
        return e0, e1

    def kern_on(st):
        e0, e1 = ev(), ev()
        e0.record(st)
        res.step_batch(0, st.cuda_stream)
        e1.record(st)
        return e0, e1

    def up_on(st):
        e0, e1 = ev(), ev()
        e0.record(st)
        with torch.cuda.stream(st):
            up_dst.copy_(up_src, non_blocking=True)
        e1.record(st)
        return e0, e1

    # a slot's carrier walks (gss_spec_device on pinned host rows, as gss_run launches them)
    import numpy as np
    sc = G.Scenario(B.NAV, llh=B.LOC, duration=410.0, samp_freq=2.6e6, data_format=1)
    sb, sn, sch = sc.next_deferred(2048, 16)
    gi = G.carr_chain_guess(sc.carrier(), sb, sn, sch, sc.n_per_blk, starts_only=True).reshape(-1)
    nrow = gi.size
    sp_in = torch.empty(nrow * G.SPEC_IN_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
    sp_out = torch.empty(nrow * G.SPEC_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
    h_in = sp_in.numpy().view(G.SPEC_IN_DTYPE)

    def spec_on(st):
        h_in[:] = gi                                   # fresh guesses (k = 0 rows) each time
        e0, e1 = ev(), ev()
        e0.record(st)
        dev.spec_device(sp_in.data_ptr(), nrow, sc.n_per_blk, sp_out.data_ptr(),
                        stream=st.cuda_stream)
        e1.record(st)
        return e0, e1

    ss = torch.cuda.Stream(dev_t, priority=-1)
    busy = [False]

    import numpy as np
    big = [np.ones(64 << 20, np.uint8) for _ in range(16)]

    def hostmem(i):
        while busy[0]:
            np.copyto(big[2 * i + 1], big[2 * i])

    def planner():
        while busy[0]:
            sc = G.Scenario(B.NAV, llh=B.LOC, duration=300.0, samp_freq=2.6e6, data_format=1)
            sc.next_deferred(2048, 16)

    out = {"slot_MB": 133}
    for nbuf in (1, 4):                   # back-to-back downloads cycling over nbuf buffers
        torch.cuda.synchronize(dev_t)
        e0, e1 = ev(), ev()
        e0.record(cp)
        with torch.cuda.stream(cp):
            for i in range(16):
                dsts[i % nbuf].copy_(srcs[i % nbuf], non_blocking=True)
        e1.record(cp)
        torch.cuda.synchronize(dev_t)
        out["cycle%d_ms_per_copy" % nbuf] = round(e0.elapsed_time(e1) / 16, 3)
    for mode in ("copy", "kern", "both", "copy_gemm", "copy_host", "both_host", "up", "copy_up", "copy_mem",
                 "spec", "copy_spec", "both_spec"):
        tc, tk, tw = [], [], []
        for r in range(reps + 1):
            torch.cuda.synchronize(dev_t)
            th = None
            ths = []
            if mode == "copy_mem":
                busy[0] = True
                ths = [threading.Thread(target=hostmem, args=(i,)) for i in range(8)]
                for t in ths:
                    t.start()
                time.sleep(0.05)
            if mode.endswith("_host"):
                busy[0] = True
                th = threading.Thread(target=planner)
                th.start()
                time.sleep(0.05)
            if mode == "copy_gemm":
                with torch.cuda.stream(cs):
                    for _ in range(20):
                        torch.mm(a, a)
            w = spec_on(ss) if mode.endswith("spec") else None
            k = kern_on(cs) if mode in ("kern", "both", "both_host", "both_spec") else None
            c = copy_on(cp) if mode not in ("kern", "up", "spec") else None
            if mode in ("up", "copy_up", "copy_mem",
                 "spec", "copy_spec", "both_spec"):
                time.sleep(0.0005)
                k = up_on(cs)
            torch.cuda.synchronize(dev_t)
            if th or ths:
                busy[0] = False
            if th:
                th.join()
            for t in ths:
                t.join()
            if r:
                if w:
                    tw.append(w[0].elapsed_time(w[1]))
                if c:
                    tc.append(c[0].elapsed_time(c[1]))
                if k:
                    tk.append(k[0].elapsed_time(k[1]))
        if tc:
            out[mode + "_copy_ms"] = round(sorted(tc)[len(tc) // 2], 3)
        if tk:
            out[mode + "_kern_ms"] = round(sorted(tk)[len(tk) // 2], 3)
        if tw:
            out[mode + "_walks_ms"] = round(sorted(tw)[len(tw) // 2], 3)
    print(json.dumps(out), flush=True)
    res.free()
    dev.close()


if __name__ == "__main__":
    main()
