"""Why the e2e legs run slower inside bench.py than in a fresh process: one
configuration's gss_run leg first in a fresh process, then after a part of that configuration's
kernel leg (the DeviceWindow the bench times before it), then once more; each leg with the host's
CPU accounting, the run's per-batch steady rate (bench.e2e_run) and its CLOCK_MONOTONIC span (to
cut a GSS_RUN_TRACE=1 log into legs).  GPU box only.

usage: python tools/e2e_bench_probe.py <config index 2|3|4> [pre] [repeats]
  pre: all (default; plan + window + steps), plan (Scenario.all_blocks only), window (plan and
       the DeviceWindow built and freed, no launch), alloc / alloc_keep / alloc_sleepN (only
       the window's output buffer, released to the driver / kept cached / released and N s
       waited), none"""
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO]
import torch  # noqa: E402
import gpssim_amd as G  # noqa: E402
import bench as B  # noqa: E402


def kernel_leg(dev, dev_t, stream, c, pre, threads=16):
    from gpssim_amd.render import DeviceWindow
    t0 = time.perf_counter()
    if pre == "none":
        return 0.0
    if pre.startswith("alloc"):
        # only the window's output buffer: allocated, touched, released to the driver (alloc) or
        # kept in torch's cache (alloc_keep); alloc_sleepN waits N s after the release
        n = int(round(c["fs"] / 10)) * int(c["window"] * 10)
        bb = G.block_bytes(int(round(c["fs"] / 10)), c["fmt"])
        out = torch.empty(n // int(round(c["fs"] / 10)) * bb, dtype=torch.uint8, device=dev_t)
        out.fill_(1)
        torch.cuda.synchronize(dev_t)
        del out
        if pre != "alloc_keep":
            torch.cuda.empty_cache()
        if pre.startswith("alloc_sleep"):
            time.sleep(float(pre[len("alloc_sleep"):]))
        return round(time.perf_counter() - t0, 2)
    s = G.Scenario(B.NAV, duration=c["window"], samp_freq=c["fs"], data_format=c["fmt"], **c["kw"])
    blk, nch = s.all_blocks(batch=2000, threads=threads)
    if pre in ("all", "window"):
        res = DeviceWindow(torch, dev, dev_t, blk, nch, s.nav_table(), s.n_per_blk, c["fmt"],
                           threads=threads, batch=3000)
        if pre == "all":
            for _ in range(3):
                res.step(stream)
        torch.cuda.synchronize(dev_t)
        res.free()
    del blk, nch, s
    return round(time.perf_counter() - t0, 2)


def main():
    idx = int(sys.argv[1])
    pre = sys.argv[2] if len(sys.argv) > 2 else "all"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    c = B.CONFIGS[idx - 2]
    dev_t = torch.device("cuda", 0)
    dev = G.Device(0)
    stream = torch.cuda.current_stream(dev_t).cuda_stream

    def leg(tag):
        m0 = time.monotonic()
        r = B.e2e_run(G, dev, 16, c["window"], fs=c["fs"], fmt=c["fmt"], kw=c["kw"], slope=True,
                      desc=c["desc"])
        out = {"leg": tag, "pre": pre, "value": r["value"], "wall_s": r["wall_s"],
               "frac": r["frac_of_d2h_ceiling"], "steady_frac": r.get("steady_frac_of_d2h_ceiling"),
               "ceiling": r["d2h_ceiling_GBps"], "startup_s": r.get("startup_s"), "host": r["host"],
               "mono": [round(m0, 6), round(time.monotonic(), 6)]}
        print(json.dumps(out), flush=True)

    leg("fresh")
    for i in range(reps):
        print(json.dumps({"pre": pre, "kernel_leg_s": kernel_leg(dev, dev_t, stream, c, pre)}),
              flush=True)
        leg(f"after {pre} {i + 1}")
    leg("again")
    dev.close()


if __name__ == "__main__":
    main()
