#!/usr/bin/env python3
"""Benchmark: IQ MSamples/s of the GPU hot path on BASELINE.json's headline configuration.

Workload (BASELINE.json configs[1]): static receiver -l 30.286502,120.032669,100, 2.6 MS/s,
-b 16, 300 s per GPU = 2999 blocks x 260000 samples (11-12 satellites; ephemeris
brdc3540.14n).  The scenario is deterministic; there is no dataset.

One step = one pass of the hot path over the rank's whole 300 s window: checkpoint stage +
synthesis stage (gss_synth_device) from per-block parameters already resident in HBM, writing
the exact -b 16 byte stream (3.12 GB) to HBM.  Multi-GPU (torchrun, one process per GPU):
rank r owns the time window [300 r, 300 (r+1)) s of one longer static run — a weak-scaling
time-window shard with no data-path collective; RCCL is used only for the
barrier and the max-over-ranks timing.  The host control plane (ephemeris, ranges, nav words,
exact carrier planner) runs before the timed region; its wall time is reported as host_plan_s
and folded into e2e_msps.

Extra JSON fields besides the driver contract: x_realtime, stages_ms, host_plan_s, e2e_msps,
roofline (synthesis kernel: algorithmic output bytes per launch / its average HIP-event
duration over the timed steps), cpu_baseline (the reference binary itself, oracle/_ref/
gps-sdr-sim, on a bounded 60 s sample, rank 0 only, before the GPU is initialised).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))

NAV = os.path.join(REPO, "tests", "golden", "data", "brdc3540.14n")
LOC = (30.286502, 120.032669, 100.0)
FS = 2.6e6
WINDOW_S = 300.0
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters
METRIC = "IQ MSamples/s (and × real-time) at 2.6 MS/s, 12 sats, -b 16; 1/2/4/8 GPU"


def cpu_baseline(seconds=60):
    """The reference program (compiled from its own sources by oracle/Makefile) timed on one
    host core over a bounded sample; falls back to the repo's CPU restatement ("port")."""
    ref = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim")
    port = os.path.join(REPO, "oracle", "_ref", "gss_oracle_cli")
    kind, exe = ("reference", ref) if os.path.exists(ref) else ("port", port)
    if not os.path.exists(exe):
        return None
    args = [exe, "-e", NAV, "-l", ",".join(map(str, LOC)), "-d", str(seconds), "-s",
            str(int(FS)), "-b", "16", "-o", "/dev/null"]
    env = dict(os.environ, GSS_THREADS="1")
    t0 = time.perf_counter()
    r = subprocess.run(["taskset", "-c", "0"] + args, capture_output=True, env=env)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        return None
    blocks = int(seconds * 10) - 1
    msps = blocks * FS / 10 / wall / 1e6
    return {"value": round(msps, 3), "unit": "MS/s", "cores": 1, "kind": kind,
            "sample": f"static -d {seconds} -b 16 -o /dev/null ({blocks} blocks x 260000 "
                      f"samples), wall {wall:.2f} s, x_realtime {msps / 2.6:.2f}"}


def load_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the PMC passes (profiles/pmc_traffic.json), when
    they were taken on this workload"""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        if d.get("workload") == workload and str(d.get("kernel", "")).startswith(kernel):
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--window", type=float, default=WINDOW_S, help="seconds per GPU")
    ap.add_argument("--fmt", type=int, default=16, choices=[1, 8, 16])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact", action="store_true",
                    help="lin path: skip the exact-path run on the same batch (exact_path)")
    ap.add_argument("--no-ck", action="store_true",
                    help="do not pass the planner's carrier checkpoints (GPU walks whole blocks)")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 8))
    ap.add_argument("--path", choices=["lin", "walk"], default="lin",
                    help="lin: certified integer fast path (gss_linearize + gss_synth_lin_device; "
                         "uncertified blocks take the exact path inside the same call); walk: "
                         "the exact walking path only (Stage A + Stage B, gss_synth_device)")
    ap.add_argument("--pipeline", action="store_true",
                    help="run Stage A of batch k+1 on a second stream beside Stage B of batch k "
                         "(gss_anchor_device/gss_render_device) instead of one gss_synth_device "
                         "call per step; slower on MI355X today (Stage A waves displace Stage B "
                         "workgroups), kept for measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # CPU baseline first: a child process, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()

    import numpy as np
    import torch                      # loads the HIP runtime our library then shares
    import gpssim_amd as G

    dist = world > 1
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("nccl")
    dev_t = torch.device("cuda", local)

    # ---- host control plane for this rank's window (untimed setup) ----
    from gpssim_amd.shard import plan_rank
    t_plan0 = time.perf_counter()
    blk, nch, ck, nav, npb = plan_rank(NAV, rank, world, args.window, llh=LOC, samp_freq=FS,
                                       data_format=args.fmt, threads=args.threads)
    host_plan_s = time.perf_counter() - t_plan0
    nblk = len(nch)
    lin_s, n_fast = 0.0, 0
    if args.path == "lin":
        t_lin0 = time.perf_counter()
        lin, fast = G.linearize(blk, nch, nav, npb, threads=args.threads)
        lin_s = time.perf_counter() - t_lin0
        host_plan_s += lin_s
        n_fast = int(fast.sum())
        fb = np.nonzero(fast == 0)[0].astype(np.int32)

    # ---- inputs resident in HBM ----
    dev = G.Device(local)
    ca = G.ca_table()
    d_blk = torch.from_numpy(blk.view(np.uint8).reshape(-1)).to(dev_t)
    d_nch = torch.from_numpy(nch).to(dev_t)
    d_ck = torch.from_numpy(ck).to(dev_t)        # planner carrier checkpoints (host-computed)
    d_ca = torch.from_numpy(ca.view(np.int32)).to(dev_t)
    d_nav = torch.from_numpy(nav.view(np.int32)).to(dev_t)
    bb = G.block_bytes(npb, args.fmt)
    out = torch.empty(nblk * bb, dtype=torch.uint8, device=dev_t)
    dev.reserve(nblk, npb)
    nch_max = int(nch.max())
    stream = torch.cuda.current_stream(dev_t).cuda_stream

    ck_ptr = 0 if args.no_ck else d_ck.data_ptr()
    if args.path == "lin":
        d_lin = torch.from_numpy(lin.view(np.uint8).reshape(-1)).to(dev_t)
        d_fast = torch.from_numpy(fast).to(dev_t)
        d_fb = torch.from_numpy(fb if len(fb) else np.zeros(1, np.int32)).to(dev_t)

    def step_lin():
        dev.synth_lin_device(d_blk.data_ptr(), d_nch.data_ptr(), nch_max, d_lin.data_ptr(),
                             d_fast.data_ptr(), d_fb.data_ptr(), len(fb), d_ca.data_ptr(),
                             len(ca), d_nav.data_ptr(), len(nav), nblk, npb, args.fmt,
                             out.data_ptr(), stream=stream, ck_ptr=ck_ptr)

    def step_serial():
        dev.synth_device(d_blk.data_ptr(), d_nch.data_ptr(), nch_max, d_ca.data_ptr(), len(ca),
                         d_nav.data_ptr(), len(nav), nblk, npb, args.fmt, out.data_ptr(),
                         0, 0, stream, ck_ptr=ck_ptr)

    # --pipeline: batch k is rendered (Stage B) on the main stream while Stage A of batch k+1
    # runs on a second, higher-priority stream into the other anchor set.  Every step still runs
    # one full Stage A and one full Stage B; events order the ping-pong sets.
    s_b = torch.cuda.current_stream(dev_t)
    s_a = torch.cuda.Stream(dev_t, priority=-1)
    ev_a = [torch.cuda.Event() for _ in range(2)]
    ev_b = [torch.cuda.Event() for _ in range(2)]
    pipe = {"k": 0}

    def anchor(k):
        st = k % 2
        if k >= 2:                    # set st was last read by render(k-2)
            s_a.wait_event(ev_b[st])
        dev.anchor_device(st, d_blk.data_ptr(), d_nch.data_ptr(), nch_max, nblk, npb,
                          ck_ptr=ck_ptr, stream=s_a.cuda_stream)
        ev_a[st].record(s_a)

    def render(k):
        st = k % 2
        s_b.wait_event(ev_a[st])
        dev.render_device(st, d_blk.data_ptr(), d_nch.data_ptr(), nch_max, d_ca.data_ptr(),
                          len(ca), d_nav.data_ptr(), len(nav), nblk, npb, args.fmt,
                          out.data_ptr(), stream=s_b.cuda_stream)
        ev_b[st].record(s_b)

    def step_pipelined():
        k = pipe["k"]
        render(k)
        anchor(k + 1)
        pipe["k"] = k + 1

    step = step_lin if args.path == "lin" else (step_pipelined if args.pipeline else step_serial)
    if args.pipeline:
        anchor(0)                     # pipeline prologue (untimed)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev_t)
    dev.timing_reset()
    if dist:
        td.barrier()
    torch.cuda.synchronize(dev_t)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev_t)
    if dist:
        td.barrier()
    elapsed = time.perf_counter() - t0
    n_launch, ck_ms, syn_ms = dev.timing()
    n_lin, lin_ms = dev.timing_lin()
    if dist:
        t = torch.tensor([elapsed, ck_ms, syn_ms, host_plan_s, lin_ms], dtype=torch.float64,
                         device=dev_t)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed, ck_ms, syn_ms, host_plan_s, lin_ms = t.tolist()

    samples_rank = nblk * npb
    exact = None
    if args.path == "lin" and not dist and not args.no_exact:
        # the same resident batch through the exact path alone (Stage A + Stage B for every
        # block, no host-side line proofs), timed the same way
        for _ in range(args.warmup):
            step_serial()
        torch.cuda.synchronize(dev_t)
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step_serial()
        torch.cuda.synchronize(dev_t)
        el = time.perf_counter() - t1
        exact = {"value": round(samples_rank * args.steps / el / 1e6, 2),
                 "ms_per_step": round(el / args.steps * 1e3, 3)}
    ms_per_step = elapsed / args.steps * 1e3
    value = world * samples_rank * args.steps / elapsed / 1e6          # MS/s, whole job
    if args.path == "lin":
        # the dominant kernel is gss_lin_kernel; its algorithmic bytes are the certified blocks'
        kern_ms, bytes_launch = lin_ms, n_fast * bb
    else:
        kern_ms, bytes_launch = syn_ms, nblk * bb                       # algorithmic bytes
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    e2e = world * samples_rank / (host_plan_s + ms_per_step * 1e-3) / 1e6
    workload = (f"static -l {LOC[0]},{LOC[1]},{LOC[2]:g} -s 2600000 -b {args.fmt}, "
                f"{args.window:g} s per GPU ({nblk} blocks x {npb} samples)")
    traffic = load_traffic(workload, "gss_lin_kernel" if args.path == "lin" else "gss_synth_kernel")
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MS/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: deterministic static-receiver scenario (brdc3540.14n), no dataset",
        "config": {"workload": workload, "samples_per_gpu": samples_rank,
                   "path": args.path,
                   "carrier_checkpoints": 0 if args.no_ck else 8,
                   "channels_max": nch_max, "parallelism": f"time-window shards x{world}",
                   "stages": "pipelined (A of batch k+1 beside B of k)" if args.pipeline
                   else "serial (A then B, one stream)"},
        "x_realtime": round(value / (FS / 1e6), 1),
        "stages_ms": {"fast_path": round(lin_ms, 3), "checkpoint": round(ck_ms, 3),
                      "synthesis": round(syn_ms, 3), "launches_timed": max(n_launch, n_lin)},
        "blocks_fast_path": n_fast if args.path == "lin" else 0, "blocks_total": nblk,
        "host_linearize_s": round(lin_s, 3),
        "host_plan_s": round(host_plan_s, 3),
        "e2e_msps": round(e2e, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic},
        "cpu_baseline": cpu,
        "exact_path": exact,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    dev.close()
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
