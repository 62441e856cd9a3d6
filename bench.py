#!/usr/bin/env python3
"""Benchmark: IQ MSamples/s of the GPU hot path on BASELINE.json's headline configuration.

Workload (BASELINE.json configs[1]): static receiver -l 30.286502,120.032669,100, 2.6 MS/s,
-b 16, 300 s per GPU = 2999 blocks x 260000 samples (11-12 satellites; ephemeris
brdc3540.14n).  The scenario is deterministic; there is no dataset.

One step = one pass of the hot path over the rank's whole 300 s window from per-block parameters
already resident in HBM: gss_synth_lin_device (the certified fast path, gss_lin_kernel; blocks the
host proof does not certify take the exact path inside the same call), writing the exact -b 16
byte stream (3.12 GB) to HBM.  Multi-GPU (torchrun, one process per GPU): rank r owns the time
window [300 r, 300 (r+1)) s of one longer static run -- a weak-scaling time-window shard with no
data-path collective; RCCL carries only the planner's 128-byte carrier hand-off,
the barrier and the max-over-ranks timing.  The host control plane (ephemeris, ranges, nav
words, exact carrier planner) and the proofs (on the GPU: gss_linearize_device) run before the
timed region (host_plan_s, host_linearize_s), each rank planning only its own window
(gpssim_amd/shard.py).

Extra JSON fields besides the driver contract:
  x_realtime, stages_ms, host_plan_s, host_linearize_s (max over ranks), lib (the library that
  was measured);
  host_plan_per_rank  each rank's planning: seek (30 s updates only), its own rows, the wait for
                the slot carriers from rank r-1, its carrier walk, its proofs, and the rows it
                produced (= its window: no rank plans another rank's blocks);
  roofline      fast-path kernel: algorithmic output bytes per launch / its average HIP-event
                duration over the timed steps; traffic = HBM bytes per launch from live
                rocprofv3 PMC passes of this bench (same steps and warm-up), attached when the
                profiled kernel time is within 10 % of this run's un-profiled event time (both
                reported in roofline.profile); fallback profiles/pmc_traffic.json under the same
                rule for the same library build;
  per_config    rank 0 at N=1: the other BASELINE configurations on the same path, each timed
                the same way (configs[2] circle -b 8, configs[3] 20 MS/s -b 16 per-GPU share of
                3600 s over 8 GPUs, configs[4] 24 h -b 1), with their own algorithmic bytes and
                roofline fraction;
  e2e           rank 0 at N=1: gss_run (planner thread + proofs + H2D + kernels + D2H into
                pinned host buffers + a discarding sink, all overlapped) over the 300 s run,
                wall-clocked: the PCIe-inclusive rate (a 1800 s run, so that the pinned
                buffers' setup is amortised as in a real run);
  cpu_baseline  the reference program built from its own sources (oracle/_ref/gps-sdr-sim) on a
                bounded sample, on 1 core and as C concurrent processes on C host cores, rank 0
                only, before the GPU is initialised;
  exact_path    the same resident batch through the exact walking path alone;
  window        the fast path including its proofs on the device, per step: gss_linearize_device
                over the window's resident rows (the proof kernel) and then the render
                (gss_synth_lin_device: window tables, segment rows, gss_lin_kernel) -- the cost of
                a window that is proven once and rendered once, beside the kernel-only headline;
                window.device_window adds the carrier chain's speculative walks and records
                (gss_spec_records_device) in front: the whole per-window GPU pipeline;
                window.device_pipeline runs those three stages as gss_run's streams do (the next
                window's walks and proofs on a highest-priority stream beside the render);
  step_issue_efficiency  the fast kernel against the issue-bound peak of its own step (was
                roofline_compute), with bound_frac / floor_bound_frac: the HBM-write fraction that
                step, and the LUT formulation's floor, allow.
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
CIRCLE = os.path.join(REPO, "tests", "golden", "data", "circle.csv")
LOC = (30.286502, 120.032669, 100.0)
FS = 2.6e6
WINDOW_S = 300.0
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters
METRIC = "IQ MSamples/s (and × real-time) at 2.6 MS/s, 12 sats, -b 16; 1/2/4/8 GPU"
BOX_CORES = 16                 # host threads for the planner/proofs (the box's CPU share per GPU)

# The fast kernel's compute rooflines, in channel-samples/s: every SIMD issuing
# nothing but the step loop at the top clock.  VALU: per wave channel-step v_lshl_add_u64 4.60 +
# v_lshrrev_b32_sdwa with an SGPR window 4.38 + v_alignbit_b32 4.37 + v_and_b32 2.75 SIMD cycles
# at 4 waves per SIMD (profiles/round2/issue_ubench2.log) + a quarter of a
# v_mfma_f32_16x16x32_f16, 3.5 (profiles/round3/mfma_issue_ubench.log: 57.3 vs 43.4 cycles per
# body); LDS: one conflict-free ds_read_b32 (2 LDS cycles for 64 channel-samples) per CU-cycle
# pair (MI355X_MICROARCH.md, LDS).  Same step loop for -b 16, -b 8 and -b 1.
SIMDS, CUS, CLOCK_MAX_HZ = 1024, 256, 2.4e9
VALU_CYC_PER_CHSTEP = 4.60 + 4.38 + 4.37 + 2.75 + 3.5
VALU_PEAK_CHS = SIMDS * 64 * CLOCK_MAX_HZ / VALU_CYC_PER_CHSTEP
LDS_PEAK_CHS = CUS * CLOCK_MAX_HZ * 64 / 2.0


# The LUT formulation's floor in hardware terms ("Where the plateau ends"): per
# channel-sample a phase advance, a chip-sign extraction, a LUT address and a LUT read cannot be
# fewer than one VOP2 op each for the first three (2.75 SIMD cycles apiece at 4 waves per SIMD,
# profiles/round2/issue_ubench2.log) plus the accumulate's share of the MFMA (2 cycles: a
# 16x16x32 f16 MFMA holds vector issue 8 cycles, MI355X_MICROARCH.md, per 4 channel-steps).
FLOOR_CYC_PER_CHSTEP = 3 * 2.75 + 2.0
FLOOR_PEAK_CHS = SIMDS * 64 * CLOCK_MAX_HZ / FLOOR_CYC_PER_CHSTEP


def compute_roofline(ch_samples, kern_ms, bytes_per_sample=None, ch_per_sample=None):
    """The fast kernel's issue efficiency: achieved channel-samples/s of one launch against the
    issue-bound peak of ITS OWN step (4 VALU + a quarter MFMA at the top clock) -- how well the
    chosen step issues, not whether it is the cheapest step -- and the LDS bound.  bound_frac:
    the HBM-write roofline fraction that this step allows at 100 % issue and 2.4 GHz
    (bytes_per_sample, ch_per_sample of the launch); floor_bound_frac: the same for the LUT
    formulation's floor (FLOOR_CYC_PER_CHSTEP)."""
    if kern_ms <= 0:
        return None
    a = ch_samples / (kern_ms * 1e-3)
    out = {"what": "issue efficiency of the 4-VALU + 1/4-MFMA step (not an HBM roofline)",
           "bound": "valu issue of this step", "achieved": round(a / 1e12, 4),
           "peak": round(VALU_PEAK_CHS / 1e12, 4),
           "unit": "T channel-samples/s", "frac": round(a / VALU_PEAK_CHS, 4),
           "lds_peak": round(LDS_PEAK_CHS / 1e12, 4), "lds_frac": round(a / LDS_PEAK_CHS, 4),
           "channel_samples_per_launch": int(ch_samples),
           "model": f"{VALU_CYC_PER_CHSTEP:.2f} SIMD cycles per wave channel-step, "
                    f"{SIMDS} SIMDs at {CLOCK_MAX_HZ / 1e9:.1f} GHz"}
    if bytes_per_sample and ch_per_sample:
        def hbm_frac(peak_chs):
            return round(peak_chs / ch_per_sample * bytes_per_sample / (HBM_PEAK_GBS * 1e9), 4)
        out.update({"bound_frac": hbm_frac(VALU_PEAK_CHS),
                    "floor_bound_frac": hbm_frac(FLOOR_PEAK_CHS),
                    "lds_bound_frac": hbm_frac(LDS_PEAK_CHS),
                    "channels_per_sample": round(ch_per_sample, 3),
                    "bound_model": f"HBM-write fraction at 100 % issue: this step "
                                   f"{VALU_CYC_PER_CHSTEP:.2f}, the formulation's floor "
                                   f"{FLOOR_CYC_PER_CHSTEP:.2f} SIMD cycles per wave "
                                   f"channel-step; one conflict-free ds_read_b32 per wave "
                                   f"channel-step for the LDS"})
    return out

# BASELINE.json configs[2..4] (per_config); configs[1] is the headline, configs[0] the CPU case
CONFIGS = [
    {"name": "configs[2]", "desc": "dynamic -u circle.csv -s 2600000 -b 8, 300 s",
     "kw": {"motion_file": CIRCLE}, "fs": 2.6e6, "fmt": 8, "window": 300.0},
    {"name": "configs[3]", "desc": "static -s 20000000 -b 16, 3600 s over 8 GPUs: the 450 s "
     "per-GPU share (4499 blocks x 2000000 samples)", "kw": {"llh": LOC}, "fs": 2.0e7,
     "fmt": 16, "window": 450.0},
    {"name": "configs[4]", "desc": "static -s 2600000 -b 1, 86400 s (863999 blocks)",
     "kw": {"llh": LOC}, "fs": 2.6e6, "fmt": 1, "window": 86400.0},
]


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process tree (cgroup v2 cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds=30, over_seconds=10):
    """The reference program (compiled from its own sources by oracle/Makefile) on a bounded
    sample of the static scenario to /dev/null: one process on one core, then one process per
    CPU the box grants (it is single-threaded by construction): min(affinity mask, ceil(cgroup
    cpu.max quota)) processes, each pinned to its own core -- `cores` is that number, the CPUs
    the aggregate actually had.  `oversubscribed` is one process per core of the whole affinity
    mask (a shorter sample), which the quota throttles, kept only for comparison.  Falls back to
    the repo's CPU restatement ("port") when the reference binary is absent."""
    ref = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim")
    port = os.path.join(REPO, "oracle", "_ref", "gss_oracle_cli")
    kind, exe = ("reference", ref) if os.path.exists(ref) else ("port", port)
    if not os.path.exists(exe):
        return None
    try:
        avail = sorted(os.sched_getaffinity(0))
    except AttributeError:
        avail = list(range(os.cpu_count() or 1))
    quota = cpu_quota()
    cores = len(avail) if quota is None else max(1, min(len(avail), int(-(-quota // 1))))
    env = dict(os.environ, GSS_THREADS="1")

    def run(n, sec):
        args = [exe, "-e", NAV, "-l", ",".join(map(str, LOC)), "-d", str(sec), "-s",
                str(int(FS)), "-b", "16", "-o", "/dev/null"]
        t0 = time.perf_counter()
        # pinned in the child before it runs the program (no launcher such as taskset, whose
        # own exec would be one more hop)
        ps = [subprocess.Popen(args, env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL,
                               preexec_fn=(lambda c=avail[i]: os.sched_setaffinity(0, {c})))
              for i in range(n)]
        ok = all(p.wait() == 0 for p in ps)
        return (time.perf_counter() - t0) if ok else None

    def rate(n, sec, wall):
        return n * (int(sec * 10) - 1) * FS / 10 / wall / 1e6

    blocks = int(seconds * 10) - 1
    w1 = run(1, seconds)
    wn = run(cores, seconds) if w1 is not None and cores > 1 else w1
    if w1 is None or wn is None:
        return None
    one, agg = rate(1, seconds, w1), rate(cores, seconds, wn)
    over = None
    if len(avail) > cores:
        wo = run(len(avail), over_seconds)
        if wo is not None:
            over = {"value": round(rate(len(avail), over_seconds, wo), 2),
                    "processes": len(avail),
                    "sample": f"static -d {over_seconds} -b 16 per process, {len(avail)} "
                              f"processes on the affinity mask under a {quota}-CPU quota: "
                              f"wall {wo:.2f} s"}
    return {"value": round(agg, 2), "unit": "MS/s", "cores": cores, "kind": kind,
            "cpu_quota": quota, "affinity_cores": len(avail),
            "single_core": {"value": round(one, 3), "cores": 1,
                            "x_realtime": round(one / (FS / 1e6), 2)},
            "x_realtime": round(agg / (FS / 1e6), 2),
            "oversubscribed": over,
            "sample": f"static -d {seconds} -b 16 -o /dev/null ({blocks} blocks x 260000 "
                      f"samples) per process; 1 process: wall {w1:.2f} s; {cores} concurrent "
                      f"processes, one per granted CPU (min(affinity {len(avail)}, quota "
                      f"{quota})), pinned to cores {avail[0]}..{avail[cores - 1]}: wall "
                      f"{wn:.2f} s"}


def host_state():
    """cgroup CPU accounting (cpu.stat), this process's threads and resident memory: recorded
    around each end-to-end leg (the bench-process e2e slowdown)"""
    st = {}
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()
            if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                st[k] = int(v)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/self/status"):
            if line.startswith(("Threads:", "VmRSS:", "VmHWM:")):
                k, v = line.split(":", 1)
                st[k] = int(v.split()[0])
    except (OSError, ValueError):
        pass
    st["t"] = time.perf_counter()
    return st


def host_delta(a, b):
    d = {k: b[k] - a[k] for k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec")
         if k in a and k in b}
    if "t" in a and "usage_usec" in d and b["t"] > a["t"]:
        d["cpus_used"] = round(d["usage_usec"] / 1e6 / (b["t"] - a["t"]), 2)
    for k in ("Threads", "VmRSS", "VmHWM"):
        if k in b:
            d[k + "_after"] = b[k]
    return d


def progress(msg):
    """a progress line on stderr (the JSON result is the last stdout line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def lib_sha16(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


PROFILE_TOL = 0.10     # a profile's kernel time must be within 10 % of the un-profiled run's


def load_traffic(workload, kernel, kern_ms, lib_sha):
    """HBM bytes per launch of `kernel` from a committed profile (profiles/pmc_traffic.json), only
    when it was taken on this workload and this kernel build (same library sha256) and its
    profiled kernel time (warm launches) is within PROFILE_TOL of THIS run's un-profiled HIP-event
    time kern_ms.  Fallback for live_traffic."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    if d.get("workload") != workload or not str(d.get("kernel", "")).startswith(kernel):
        return None, "profile of another workload"
    if d.get("lib_sha16") != lib_sha:
        return None, "profile of another build"
    prof_ms = (d.get("kernel_timed_avg_ns") or d.get("kernel_warm_avg_ns") or
               d.get("kernel_avg_ns") or 0) / 1e6
    if kern_ms <= 0 or abs(prof_ms - kern_ms) > PROFILE_TOL * kern_ms:
        return None, (f"committed profile kernel time {prof_ms:.3f} ms vs {kern_ms:.3f} ms of "
                      "this un-profiled run")
    return d.get("hbm_bytes_per_launch"), (f"{d.get('source')}; profiled kernel {prof_ms:.3f} ms "
                                           f"(this run un-profiled {kern_ms:.3f} ms)")


def live_traffic(fmt, window, threads, kern_ms, steps, warmup, timeout=150):
    """HBM bytes per launch of gss_lin_kernel measured on this box, for this build: three child
    runs of this bench with the same workload, steps and warm-up (no other legs) under rocprofv3
    -- kernel trace + stats, --pmc WRITE_SIZE, --pmc FETCH_SIZE, one pass each
    (MI355X_MICROARCH.md, HBM/rocprofv3: FETCH_SIZE x2 on gfx950, both KiB) -- parsed by
    tools/prof_summary.py.  Attached only when the profiled kernel time (warm launches of the
    trace) is within PROFILE_TOL of this run's own un-profiled HIP-event time kern_ms.  Returns
    (traffic or None, source text, profile summary dict or None); with env GSS_PROF_SAVE=<dir>
    the rocprofv3 outputs and the summary are kept there."""
    import shutil
    import signal
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import prof_summary as PS
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not found", None
    save = os.environ.get("GSS_PROF_SAVE")
    top = save or tempfile.mkdtemp(prefix="gss_pmc_", dir="/tmp")
    os.makedirs(top, exist_ok=True)
    child = [sys.executable, os.path.abspath(__file__), "--steps", str(steps), "--warmup",
             str(warmup), "--fmt", str(fmt), "--window", str(window), "--threads", str(threads),
             "--no-cpu-baseline", "--no-exact", "--no-configs", "--no-e2e", "--no-pmc",
             "--no-sustained", "--no-window"]
    env = dict(os.environ, TMPDIR="/tmp")
    env.pop("GSS_PROF_SAVE", None)
    passes = [("kt", ["--kernel-trace", "--stats"]),
              ("pmc_write", ["--pmc", "WRITE_SIZE", "--kernel-trace"]),
              ("pmc_fetch", ["--pmc", "FETCH_SIZE", "--kernel-trace"])]
    try:
        for name, opts in passes:
            # the rocprofv3 script run by this interpreter directly (its `#!/usr/bin/env python3`
            # line would be one more exec hop)
            cmd = [sys.executable, shutil.which("rocprofv3")] + opts + [
                "-d", os.path.join(top, name), "-o", name, "-f", "csv", "--"] + child
            outf = os.path.join(top, name + ".log")
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=open(outf, "w"),
                                 stderr=subprocess.DEVNULL, start_new_session=True)
            try:
                rc = p.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None, f"rocprofv3 {name} pass timed out", None
            if rc != 0:
                return None, f"rocprofv3 {name} pass exited {rc}", None
        ks, kd, cs = PS.kernel_stats(top), PS.kernel_durations(top), PS.counters(top)
        k = next((n for n in cs if n.startswith("gss_lin_kernel")), None)
        if k is None or "WRITE_SIZE" not in cs[k] or "FETCH_SIZE" not in cs[k] or k not in ks:
            return None, "rocprofv3 passes gave no gss_lin_kernel counters", None
        # the same launches as the timed region: dispatches warmup .. warmup + steps - 1
        prof_ms = (PS.timed_avg_ns(kd[k], steps, warmup) if kd.get(k) else ks[k]["avg_ns"]) / 1e6
        try:
            line = [l for l in open(os.path.join(top, "kt.log")) if l.startswith("{")][-1]
            child_ms = json.loads(line)["stages_ms"]["fast_path"]
        except (IndexError, KeyError, ValueError):
            child_ms = None
        traffic = round((cs[k]["WRITE_SIZE"] + 2 * cs[k]["FETCH_SIZE"]) * 1024)
        summary = {"kernel": k, "calls": ks[k]["calls"], "avg_ns": ks[k]["avg_ns"],
                   "warm_avg_ns": PS.warm_avg_ns(kd[k]) if kd.get(k) else None,
                   "timed_avg_ns": prof_ms * 1e6, "min_ns": ks[k]["min_ns"],
                   "max_ns": ks[k]["max_ns"], "profiled_run_event_ms": child_ms,
                   "unprofiled_event_ms": kern_ms, "steps": steps, "warmup": warmup,
                   "hbm_write_bytes": cs[k]["WRITE_SIZE"] * 1024,
                   "hbm_read_bytes_corrected": 2 * cs[k]["FETCH_SIZE"] * 1024,
                   "traffic": traffic, "other_kernels": {n: v["avg_ns"] for n, v in ks.items()
                                                         if n != k}}
        if save:
            json.dump(summary, open(os.path.join(top, "live_summary.json"), "w"), indent=1)
        if kern_ms <= 0 or abs(prof_ms - kern_ms) > PROFILE_TOL * kern_ms:
            return None, (f"live profile kernel time {prof_ms:.3f} ms vs {kern_ms:.3f} ms of "
                          "this un-profiled run"), summary
        return traffic, (f"live rocprofv3 passes on this box and build, {steps} steps + {warmup} "
                         f"warm-up as this run ({k}: write "
                         f"{cs[k]['WRITE_SIZE'] * 1024 / 1e9:.3f} GB + read "
                         f"{2 * cs[k]['FETCH_SIZE'] * 1024 / 1e9:.3f} GB per launch; profiled "
                         f"kernel {prof_ms:.3f} ms over its {steps} timed launches (after "
                         f"{warmup} warm-up), "
                         f"{ks[k]['avg_ns'] / 1e6:.3f} ms over all {ks[k]['calls']} with the "
                         f"warm-up; this run without the profiler {kern_ms:.3f} ms)"), summary
    finally:
        if not save:
            shutil.rmtree(top, ignore_errors=True)


def time_steps(torch, dev, dev_t, res, steps, warmup, stream):
    for _ in range(warmup):
        res.step(stream)
    torch.cuda.synchronize(dev_t)
    dev.timing_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        res.step(stream)
    torch.cuda.synchronize(dev_t)
    el = time.perf_counter() - t0
    n_lin, lin_ms = dev.timing_lin()
    return el, n_lin, lin_ms


def window_leg(torch, dev, dev_t, res, steps, warmup, stream, exact=None, anch=None,
               heads=None):
    """proof + render of the resident window per step (see the module docstring): the proof kernel
    rewrites the window's rows and fast flags in place (byte-identical rows: tests/
    test_gpu_proof.py), then the window renders from them; HIP events on the launch stream time
    the proof apart.  anch: the planner's chain anchors (resident like the rows), where the
    proofs' carrier walks start (gss_linearize_device_ex).
    heads (the window's walk inputs, SPEC_IN_DTYPE [nblk, 16]): a second pass, device_window,
    adds the planner's device work per step -- the carrier chain's speculative walks and their
    records (gss_spec_records_device: gss_spec_kernel + gss_spec_rec_kernel, resident in and out)
    -- so that spec + proof + render, the whole per-window GPU pipeline gss_run runs, is timed
    on the device (the host's chain between them excluded)."""
    import numpy as np
    import gpssim_amd as G
    st = torch.cuda.current_stream(dev_t)
    d_anch = None
    if anch is not None:
        d_anch = torch.from_numpy(anch.view("u1").reshape(-1).copy()).to(dev_t)

    def prove(lin=None, fast=None, on=None):
        lin = res.d_lin if lin is None else lin
        fast = res.d_fast if fast is None else fast
        dev.linearize_device(res.d_blk.data_ptr(), res.d_nch.data_ptr(), res.nblk, res.npb,
                             res.d_ca.data_ptr(), res.n_ca, res.d_nav.data_ptr(), res.n_nav,
                             lin.data_ptr(), fast.data_ptr(), stream if on is None else on,
                             anch_ptr=d_anch.data_ptr() if d_anch is not None else None)

    spec = None
    if heads is not None:
        nrow = heads.size
        d_heads = torch.from_numpy(np.ascontiguousarray(heads).reshape(-1).view(np.uint8)
                                   .copy()).to(dev_t)
        d_in = torch.empty(nrow * G.SPEC_IN_DTYPE.itemsize, dtype=torch.uint8, device=dev_t)
        d_spec = torch.empty(nrow * G.SPEC_DTYPE.itemsize, dtype=torch.uint8, device=dev_t)
        d_rec = torch.empty(nrow * G.SPEC_REC_DTYPE.itemsize, dtype=torch.uint8, device=dev_t)

        def spec(on=None):
            dev.spec_records_device(d_heads.data_ptr(), nrow, res.npb, d_in.data_ptr(),
                                    d_spec.data_ptr(), d_rec.data_ptr(),
                                    stream if on is None else on)

    def pipelined():
        """device_pipeline: gss_run's stream structure on resident windows: the walks + records
        and the proofs on a highest-priority stream (gss_run's spec and proof streams), the render
        on the launch stream (its compute stream); window i's proof follows its walks (in gss_run
        through the host's chain) and its render follows its proof, so in the steady state window
        i + 1 is walked and proven while window i renders.  GSS_BENCH_PIPE_STAGES=3 gives the
        proofs a stream of their own (window i + 2 walked, i + 1 proven, i rendered at once):
        measured slower, 2.19-2.27 against 2.13-2.15 ms per window (profiles/round6/pipeline/:
        the three stages share one chip's issue, and the proofs run 0.9 ms beside two kernels
        against 0.6 beside one).  The proofs alternate
        between two sets of lines and fast flags, so a proof never rewrites the set a render reads
        (proof i + 2 waits for render i; the walks of window i + 3 for it too: at most three
        windows in flight).  Events only, no host synchronisation.  Returns the ms per window over
        the timed steps (events on the render stream), the walks' and proofs' own ms per window
        under the render (events on their streams) and the two sets' agreement."""
        prio = int(os.environ.get("GSS_BENCH_PIPE_PRIO", "-1"))
        three = os.environ.get("GSS_BENCH_PIPE_STAGES", "2") == "3"
        sp = torch.cuda.Stream(device=dev_t, priority=prio)
        pp = torch.cuda.Stream(device=dev_t, priority=prio) if three else sp
        sets = [(res.d_lin, res.d_fast), (res.d_lin.clone(), res.d_fast.clone())]
        walked = [torch.cuda.Event() for _ in range(3)]
        proved = [torch.cuda.Event() for _ in range(2)]
        rendered = [torch.cuda.Event() for _ in range(3)]
        rs = torch.cuda.ExternalStream(stream, device=dev_t) if stream else st
        n = warmup + steps
        t = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n)]
        torch.cuda.synchronize(dev_t)
        po = 1 if three else 0                              # the proofs' and renders' lag
        for it in range(n + po + 1):
            i = it                                          # walk window i
            if i < n:
                if i >= 3:
                    sp.wait_event(rendered[(i - 3) % 3])
                ts[i][0].record(sp)
                spec(sp.cuda_stream)
                ts[i][1].record(sp)
                walked[i % 3].record(sp)
            i = it - po                                     # prove window i
            if 0 <= i < n:
                pp.wait_event(walked[i % 3])
                if i >= 2:
                    pp.wait_event(rendered[(i - 2) % 3])
                ts[i][2].record(pp)
                prove(*sets[i % 2], on=pp.cuda_stream)
                ts[i][3].record(pp)
                proved[i % 2].record(pp)
            i = it - po - 1                                 # render window i
            if 0 <= i < n:
                if i == warmup:
                    t[0].record(rs)
                rs.wait_event(proved[i % 2])
                res.step(stream, *sets[i % 2])
                rendered[i % 3].record(rs)
        t[1].record(rs)
        torch.cuda.synchronize(dev_t)
        same = bool(torch.equal(sets[0][0], sets[1][0]) and torch.equal(sets[0][1], sets[1][1]))
        spec_ms = sum(e[0].elapsed_time(e[1]) for e in ts[warmup:]) / steps
        proof_ms = sum(e[2].elapsed_time(e[3]) for e in ts[warmup:]) / steps
        return t[0].elapsed_time(t[1]) / steps, spec_ms, proof_ms, three, same

    def run(with_spec):
        for _ in range(warmup):
            if with_spec:
                spec()
            prove()
            res.step(stream)
        torch.cuda.synchronize(dev_t)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
        t0 = time.perf_counter()
        for i in range(steps):
            ev[i][0].record(st)
            if with_spec:
                spec()
            ev[i][1].record(st)
            prove()
            ev[i][2].record(st)
            res.step(stream)
            ev[i][3].record(st)
        torch.cuda.synchronize(dev_t)
        el = time.perf_counter() - t0
        part = [sum(e[j].elapsed_time(e[j + 1]) for e in ev) / steps for j in range(3)]
        return el, part

    samples = res.nblk * res.npb
    el, (_, proof_ms, render_ms) = run(False)
    out = {"value": round(samples * steps / el / 1e6, 2), "unit": "MS/s",
           "ms_per_step": round(el / steps * 1e3, 3), "proof_ms": round(proof_ms, 3),
           "render_ms": round(render_ms, 3), "steps": steps, "warmup": warmup,
           "workload": "the headline window: proof kernel (gss_linearize_device) + render "
                       "(gss_synth_lin_device) per step on resident rows",
           "anchors": d_anch is not None}
    if exact:
        out["vs_exact_path"] = round(out["value"] / exact["value"], 3)
    if spec is not None:
        el2, (spec_ms, proof2_ms, render2_ms) = run(True)
        dev_ms = spec_ms + proof2_ms + render2_ms
        bytes_step = res.n_fast * res.bb
        out["device_window"] = {
            "workload": "the headline window's whole GPU pipeline per step on resident rows: "
                        "the chain's speculative walks + records (gss_spec_records_device), "
                        "the proofs (gss_linearize_device_ex, anchors), the render",
            "value": round(samples * steps / el2 / 1e6, 2), "unit": "MS/s",
            "ms_per_step": round(el2 / steps * 1e3, 3),
            "spec_ms": round(spec_ms, 3), "proof_ms": round(proof2_ms, 3),
            "render_ms": round(render2_ms, 3), "device_ms": round(dev_ms, 3),
            "rows_walked": int(heads.size),
            "roofline": {"bound": "hbm", "achieved": round(bytes_step / (dev_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(bytes_step / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "note": "the window's output bytes over the three kernels' summed "
                                 "event time"}}
        want = res.out[:res.nblk * res.bb].clone()       # the serial pass's output
        pipe_ms, spec_ms_p, proof_ms_p, three, same = pipelined()
        same_out = bool(torch.equal(want, res.out[:res.nblk * res.bb]))
        del want
        out["device_pipeline"] = {
            "workload": ("the same three stages in gss_run's stream structure: window i + 2's "
                         "walks + records and window i + 1's proofs on two highest-priority "
                         "streams while window i renders (two sets of lines, events only)"
                         if three else
                         "the same three stages, window i + 1's walks + records and proofs on "
                         "one highest-priority stream while window i renders (two sets of "
                         "lines, events only)"),
            "stages": 3 if three else 2,
            "ms_per_window": round(pipe_ms, 3),
            "spec_ms_beside_render": round(spec_ms_p, 3),
            "proof_ms_beside_render": round(proof_ms_p, 3),
            "value": round(samples / (pipe_ms * 1e-3) / 1e6, 2), "unit": "MS/s",
            "vs_device_window": round(dev_ms / pipe_ms, 3),
            "lines_identical": same, "output_identical": same_out,
            "roofline": {"bound": "hbm", "achieved": round(bytes_step / (pipe_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(bytes_step / (pipe_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "note": "the window's output bytes per window of the pipelined steady "
                                 "state (events on the render stream)"}}
    return out


def per_config(G, torch, dev, dev_t, stream, steps, warmup, threads, e2e=True):
    from gpssim_amd.render import DeviceWindow
    from gpssim_amd.shard import blocks_per_rank
    out = []
    for c in CONFIGS:
        t0 = time.perf_counter()
        s = G.Scenario(NAV, duration=c["window"], samp_freq=c["fs"], data_format=c["fmt"],
                       **c["kw"])
        want = blocks_per_rank(c["window"])
        blk, nch = s.all_blocks(batch=2000, threads=threads)
        plan_s = time.perf_counter() - t0
        assert len(nch) == want, (c["name"], len(nch), want)
        res = DeviceWindow(torch, dev, dev_t, blk, nch, s.nav_table(), s.n_per_blk, c["fmt"],
                           threads=threads, batch=3000)
        el, n_lin, lin_ms = time_steps(torch, dev, dev_t, res, steps, warmup, stream)
        samples = res.nblk * res.npb
        msps = samples * steps / el / 1e6
        per_launch = (res.n_fast * res.bb) / len(res.batches)
        achieved = per_launch / (lin_ms * 1e-3) / 1e9 if lin_ms > 0 else 0.0
        comp = compute_roofline(res.ch_samples_fast / len(res.batches), lin_ms, res.bb / res.npb,
                                res.ch_samples_fast / max(1, res.n_fast * res.npb))
        out.append({
            "config": c["name"], "workload": c["desc"], "fmt": c["fmt"],
            "value": round(msps, 2), "unit": "MS/s", "x_realtime": round(msps / (c["fs"] / 1e6), 1),
            "ms_per_step": round(el / steps * 1e3, 3), "steps": steps,
            "blocks_fast_path": res.n_fast, "blocks_total": res.nblk,
            "launches_per_step": len(res.batches), "channels_max": res.nch_max,
            "bytes_per_step": res.nblk * res.bb,
            # the binding roofline: the step loop's VALU issue (the -b 8 / -b 1 outputs are 2 and
            # 0.25 B per sample, far below the HBM write bound); the HBM one beside it
            "roofline": dict(comp or {}, kernel_ms_per_launch=round(lin_ms, 3)),
            "roofline_hbm": {"bound": "hbm", "achieved": round(achieved, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(achieved / HBM_PEAK_GBS, 4),
                             "algorithmic_bytes_per_sample": res.bb / res.npb},
            "host_plan_s": round(plan_s, 3), "host_linearize_s": round(res.lin_s, 3),
            "proofs_on": res.proof})
        res.free(release=False)               # (released memory slows the next leg's downloads)
        del blk, nch, s
        progress(f"{c['name']}: {out[-1]['value']} MS/s")
        if e2e:
            # the same run end to end through gss_run (the CLI's path), one pass
            out[-1]["e2e"] = e2e_run(G, dev, threads, c["window"], fs=c["fs"], fmt=c["fmt"],
                                     kw=c["kw"], slope=False, desc=c["desc"])
    return out


def d2h_ceiling(nbytes, reps=8, trials=3):
    """device -> pinned host copy rate of one gss_run slot (the PCIe ceiling of e2e_run): the best
    of `trials` timings of `reps` back-to-back copies (one trial right after a long run has read
    as low as 0.78 of the link, which put that run above its "ceiling": round 6, s6ak)"""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(trials):
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes * reps / (time.perf_counter() - t0) / 1e9)
    del src, dst
    return round(best, 2)


E2E_SLOT_BYTES = 128 * 1040000  # gss_run slot size: 128 blocks at 2.6 MS/s -b 16 (133 MB)


def e2e_run(G, dev, threads, window=1800.0, batch=None, fs=FS, fmt=16, kw=None, slope=True,
            desc=None):
    """gss_run over a whole run into a discarding sink, wall-clocked (planner, proofs, uploads,
    kernels, D2H into pinned buffers and the sink, overlapped).  With `slope` the steady-state
    rate comes from the same run's sink calls (one per batch, in run order): bytes delivered
    after the first call up to the last, over the time between them; `startup_s` is the time to
    the first call.  Read against d2h_ceiling_GBps, the
    measured device -> pinned host copy rate of one slot in this process."""
    kw = kw if kw is not None else {"llh": LOC}
    bb = G.block_bytes(int(round(fs / 10)), fmt)
    if batch is None:
        batch = max(1, E2E_SLOT_BYTES // bb)

    s = G.Scenario(NAV, duration=window, samp_freq=fs, data_format=fmt, **kw)
    got = {"bytes": 0, "blocks": 0}
    marks = []                                       # (time, bytes so far) after each sink call

    def sink(mv, first, nb):
        got["bytes"] += len(mv)
        got["blocks"] += nb
        marks.append((time.perf_counter(), got["bytes"]))

    h0 = host_state()
    t0 = time.perf_counter()
    dev.run(s, sink, batch=batch, threads=threads)
    wall = time.perf_counter() - t0
    h1 = host_state()
    blocks, nbytes, n_per_blk = got["blocks"], got["bytes"], s.n_per_blk
    samples = blocks * n_per_blk
    ceiling = d2h_ceiling(batch * bb)
    out = {"value": round(samples / wall / 1e6, 2), "unit": "MS/s",
           "x_realtime": round(samples / wall / fs, 1), "wall_s": round(wall, 3),
           "blocks": blocks, "batch_blocks": batch, "threads": threads,
           "d2h_GBps": round(nbytes / wall / 1e9, 2), "d2h_ceiling_GBps": ceiling,
           "frac_of_d2h_ceiling": round(nbytes / wall / 1e9 / ceiling, 3) if ceiling else None,
           "workload": (desc or f"static -b {fmt}, {window:g} s") +
                       f" through gss_run (batch {batch} blocks), discarding sink",
           "host": host_delta(h0, h1)}
    if slope and len(marks) >= 8:
        # from the first sink call on: every later call's bytes were copied after the first
        # copy ended (one copy stream), so the slope cannot exceed the copy rate by more than
        # one slot; a later anchor can sit behind a backlog of finished slots and overstate it
        q = 0
        (tq, bq), (tl, bl) = marks[q], marks[-1]
        if tl > tq and bl > bq:
            rate = (bl - bq) / (tl - tq)                 # bytes/s in the run's steady part
            out.update({"steady_MSps": round(rate / bb * n_per_blk / 1e6, 1),
                        "steady_d2h_GBps": round(rate / 1e9, 2),
                        "steady_frac_of_d2h_ceiling": round(rate / 1e9 / ceiling, 3)
                        if ceiling else None,
                        "startup_s": round(marks[0][0] - t0, 3),
                        "steady_window": f"sink calls {q + 1}..{len(marks)} of {len(marks)}"})
    return out

GATHER_FS, GATHER_WINDOW_S = 2.0e7, 450.0   # configs[3]: 3600 s at 20 MS/s over 8 GPUs


def gather_leg(G, torch, td, dev, dev_t, rank, world, coll_t, walker, threads, window_s,
               host_wire, layout="stripe"):
    """BASELINE configs[3] as a whole-node run (N > 1 only): static -s 20000000 -b 16, each rank
    owning window_s seconds of one world * window_s run (weak scaling: 450 s per rank is
    configs[3]'s 3600 s at 8 GPUs), each rank's window planned (baton, chain run ahead); with the
    "stripe" layout (gpssim_amd.node.chunk_plan) the chunks' rows are handed round-robin to the
    ranks that render them (exchange_rows), so that rank 0 receives from every peer at once; the
    chunks are rendered and gathered in run order to rank 0 over RCCL point to point
    (render_chunks, chunk_source, ordered_gather) into a discarding sink.  Timed from the first
    render launch to the last byte at rank 0 (max over ranks): the node's data path, xGMI
    included, file system excluded."""
    from gpssim_amd.node import chunk_plan, chunk_source, exchange_rows, ordered_gather, \
        rank_blocks, render_chunks
    from gpssim_amd.render import DeviceWindow
    from gpssim_amd.shard import Baton, plan_window
    t0 = time.perf_counter()
    scn = G.Scenario(NAV, llh=LOC, duration=window_s * world, samp_freq=GATHER_FS,
                     data_format=16)
    nb_all, npb = scn.n_blocks, scn.n_per_blk
    bb = G.block_bytes(npb, 16)
    chunk = max(1, (256 << 20) // bb)
    b0, b1 = rank_blocks(nb_all, rank, world)
    blk, nch, ck, pt = plan_window(scn, b0, b1 - b0, baton=Baton(td, rank, world, device=coll_t),
                                   threads=threads, walker=walker,
                                   chain_threads=max(threads, BOX_CORES))
    plan = chunk_plan(nb_all, world, chunk, layout)
    nav = scn.nav_table()
    if layout == "stripe":
        blk, nch, nav, firsts = exchange_rows(plan, nb_all, rank, world, td, blk, nch, nav,
                                              device=coll_t)
        ck = None
    else:
        firsts = [c for r, c, nb in plan if r == rank]
    sizes = [nb for r, c, nb in plan if r == rank]
    win = DeviceWindow(torch, dev, dev_t, blk, nch, nav, npb, 16, ck=ck, threads=threads,
                       sizes=sizes or None)
    plan_s = time.perf_counter() - t0
    got = {"bytes": 0}

    def sink(t):
        got["bytes"] += t.numel()

    def make_buf(nb):
        return torch.empty(nb * bb, dtype=torch.uint8, device="cpu" if host_wire else dev_t)

    def once(sink0):
        """render + gather once into rank 0's sink0; wall seconds, max over ranks"""
        stats = {}
        td.barrier()
        torch.cuda.synchronize(dev_t)
        t1 = time.perf_counter()
        _, evs = render_chunks(torch, win, dev_t)
        get_chunk = chunk_source(torch, win, firsts, evs, dev_t,
                                 host_wire=host_wire and rank != 0)
        ordered_gather(plan, rank, td, get_chunk, make_buf, sink0 if rank == 0 else None,
                       stats=stats)
        if rank == 0 and hasattr(sink0, "close"):
            sink0.close()                         # the last chunk written
        torch.cuda.synchronize(dev_t)
        el = time.perf_counter() - t1
        t = torch.tensor([el], dtype=torch.float64, device=coll_t)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        return t.item(), stats

    el, stats = once(sink)
    # the same gather into a real file sink: rank 0 downloads each chunk into a ring of pinned
    # buffers and a writer thread os.write()s it to /dev/null (node.FileSink, as run_node)
    fsink = None
    if rank == 0:
        from gpssim_amd.node import FileSink
        fd_null = os.open(os.devnull, os.O_WRONLY)
        fsink = FileSink(torch, fd_null, chunk * bb)
    el_file, _ = once(fsink)
    if rank == 0:
        os.close(fd_null)
    t = torch.tensor([plan_s], dtype=torch.float64, device=coll_t)
    td.all_reduce(t, op=td.ReduceOp.MAX)
    plan_s = t.item()
    total = nb_all * bb
    win.free()
    return {"workload": f"static -s 20000000 -b 16, {window_s * world:g} s over {world} ranks "
                        f"({window_s:g} s = {b1 - b0} blocks planned per rank), rendered "
                        f"({layout} layout) and gathered in run order to rank 0 (chunks of "
                        f"{chunk} blocks), discarding sink",
            "wire": "gloo via host memory (rehearsal)" if host_wire else "RCCL point to point",
            "layout": layout, "bytes": total,
            "bytes_at_rank0": got["bytes"] if rank == 0 else None,
            "wall_s": round(el, 3), "GBps_at_rank0": round(total / el / 1e9, 2),
            "MSps": round(nb_all * npb / el / 1e6, 1), "host_plan_s_max": round(plan_s, 3),
            "recv_outstanding_max": stats.get("max_outstanding") if rank == 0 else None,
            "peers_outstanding_max": stats.get("max_peers_outstanding") if rank == 0 else None,
            "spec_rows_translated_rank": pt.get("spec_hits"),
            "file_sink": {"workload": "the same render + gather into node.FileSink (pinned "
                                      "ring, copy stream, writer thread) writing /dev/null",
                          "wall_s": round(el_file, 3),
                          "GBps_at_rank0": round(total / el_file / 1e9, 2),
                          "bytes_written": fsink.bytes if rank == 0 else None,
                          "vs_discarding": round(el / el_file, 3)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--window", type=float, default=WINDOW_S, help="seconds per GPU")
    ap.add_argument("--fmt", type=int, default=16, choices=[1, 8, 16])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact", action="store_true",
                    help="skip the exact-path run on the same batch (exact_path)")
    ap.add_argument("--no-configs", action="store_true", help="skip per_config")
    ap.add_argument("--no-window", action="store_true",
                    help="skip the proof + render leg (window)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the gss_run end-to-end run")
    ap.add_argument("--e2e-window", type=float, default=1800.0)
    ap.add_argument("--no-sustained", action="store_true",
                    help="skip the sustained-clock launches after the timed region")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 traffic passes (roofline.traffic)")
    ap.add_argument("--threads", type=int, default=BOX_CORES)
    ap.add_argument("--chain-threads", type=int, default=BOX_CORES,
                    help="threads of each rank's carrier-chain walk (the ranks' chains run one "
                         "after another: the baton)")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the whole-node gather leg (N > 1: configs[3] to rank 0)")
    ap.add_argument("--gather-layout", default="stripe", choices=["stripe", "block"],
                    help="gather leg: chunks rendered round-robin over the ranks (stripe, every "
                         "xGMI link into rank 0 at once) or each rank its own window (block)")
    ap.add_argument("--gather-window", type=float, default=GATHER_WINDOW_S,
                    help="seconds per rank of the gather leg's 20 MS/s run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    single = rank == 0 and world == 1

    # CPU baseline first: child processes, before this process touches the GPU
    cpu = None
    if single and not args.no_cpu_baseline:
        cpu = cpu_baseline()
        progress(f"cpu baseline: {cpu and cpu['value']} MS/s")

    import torch                      # loads the HIP runtime our library then shares
    import gpssim_amd as G
    from gpssim_amd.render import DeviceWindow

    dist = world > 1
    # GSS_BENCH_REHEARSE=1 (multi-rank rehearsal on a one-GPU box): every rank on GPU 0, gloo
    # collectives on host tensors; the data path is the same, the driver's runs use RCCL
    rehearse = dist and os.environ.get("GSS_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("gloo" if rehearse else "nccl")
    dev_t = torch.device("cuda", local)
    coll_t = torch.device("cpu") if rehearse else dev_t     # where collective tensors live

    # ---- host control plane for this rank's window (untimed setup) ----
    # planned once per node: each rank seeks to its window, produces its rows, and receives the
    # 16 slot carriers at its first block from rank r-1 (gpssim_amd.shard)
    # the carrier chain run ahead on this GPU (shard.device_walker) unless GSS_BENCH_HOST_CHAIN=1
    from gpssim_amd.shard import Baton, device_walker, plan_rank
    dev = G.Device(local)
    walker = None if os.environ.get("GSS_BENCH_HOST_CHAIN") == "1" else device_walker(dev, torch)
    baton = Baton(td, rank, world, device=coll_t) if dist else None
    t_plan0 = time.perf_counter()
    blk, nch, ck, nav, npb, plan_t = plan_rank(NAV, rank, world, args.window, llh=LOC,
                                               samp_freq=FS, data_format=args.fmt,
                                               threads=args.threads, baton=baton, walker=walker,
                                               chain_threads=args.chain_threads,
                                               anchors=single and not args.no_window)
    host_plan_s = time.perf_counter() - t_plan0
    progress(f"planned {len(nch)} blocks in {host_plan_s:.2f} s")
    if dist:
        # every rank's window planned before any renders: a rank's carrier chain (run ahead on
        # its GPU) then never shares the GPU with the proofs and renders of ranks planned before
        # it, which only happens in a one-GPU rehearsal (GSS_BENCH_REHEARSE)
        td.barrier()

    stream = torch.cuda.current_stream(dev_t).cuda_stream
    res = DeviceWindow(torch, dev, dev_t, blk, nch, nav, npb, args.fmt, ck=ck,
                       threads=args.threads, batch=len(nch))
    nblk = res.nblk

    if single and not args.no_exact and res.d_ck is None:
        # the exact path leg walks from the planner's checkpoints as in earlier rounds (rows
        # planned with the chain run ahead carry none)
        from gpssim_amd.render import block_checkpoints
        res.d_ck = torch.from_numpy(block_checkpoints(blk, nch, npb)).to(dev_t)

    def step_serial():
        dev.synth_device(res.d_blk.data_ptr(), res.d_nch.data_ptr(), res.nch_max,
                         res.d_ca.data_ptr(), res.n_ca, res.d_nav.data_ptr(), res.n_nav, nblk,
                         npb, args.fmt, res.out.data_ptr(), 0, 0, stream,
                         ck_ptr=res.d_ck.data_ptr())

    for _ in range(args.warmup):
        res.step(stream)
    torch.cuda.synchronize(dev_t)
    dev.timing_reset()
    if dist:
        td.barrier()
    torch.cuda.synchronize(dev_t)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res.step(stream)
    torch.cuda.synchronize(dev_t)
    if dist:
        td.barrier()
    elapsed = time.perf_counter() - t0
    n_launch, ck_ms, syn_ms = dev.timing()
    n_lin, lin_ms = dev.timing_lin()
    host_lin_s = res.lin_s
    # informational, after the timed region: the same launches continued until the shader clock
    # has finished ramping (clock ramp), i.e. the rate of a long run
    sustained_ms = None
    if single and args.steps >= 5 and not args.no_sustained:
        for _ in range(20):
            res.step(stream)
        torch.cuda.synchronize(dev_t)
        dev.timing_reset()
        for _ in range(args.steps):
            res.step(stream)
        torch.cuda.synchronize(dev_t)
        sustained_ms = round(dev.timing_lin()[1], 3)
    mine = [host_plan_s, plan_t["seek_s"], plan_t["rows_s"], plan_t["wait_s"],
            plan_t["chain_s"], host_lin_s, float(plan_t["rows_out"]),
            float(plan_t.get("spec_hits", -1)), plan_t.get("fix_s", -1.0),
            float(plan_t.get("spec_rewalked", -1))]
    per_rank = [mine]
    if dist:
        t = torch.tensor([elapsed, ck_ms, syn_ms, host_plan_s, lin_ms, host_lin_s],
                         dtype=torch.float64, device=coll_t)
        td.all_reduce(t, op=td.ReduceOp.MAX)
        elapsed, ck_ms, syn_ms, host_plan_s, lin_ms, host_lin_s = t.tolist()
        mt = torch.tensor(mine, dtype=torch.float64, device=coll_t)
        parts = [torch.empty_like(mt) for _ in range(world)]
        td.all_gather(parts, mt)
        per_rank = [p.tolist() for p in parts]
    host_plan_per_rank = [
        {"rank": r, "host_plan_s": round(v[0], 3), "seek_s": round(v[1], 3),
         "rows_s": round(v[2], 3), "baton_wait_s": round(v[3], 3),
         "carrier_chain_s": round(v[4], 3), "host_linearize_s": round(v[5], 3),
         "rows_produced": int(v[6]),
         "carrier_chain": ("speculated across ranks (walks on the GPU)" if v[9] >= 0 else
                           "run ahead on the GPU" if v[7] >= 0 else "host walk"),
         "spec_rows_translated": int(v[7]) if v[7] >= 0 else None,
         # the chain from the baton's arrival to the hand-off to rank r+1 (rank 0: its whole chain)
         "handoff_s": round(v[8], 3) if v[8] >= 0 else None,
         "spec_rows_rewalked": int(v[9]) if v[9] >= 0 else None}
        for r, v in enumerate(per_rank)]

    samples_rank = nblk * npb
    exact = None
    if single and not args.no_exact:
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
    window = None
    if single and not args.no_window and res.proof == "gpu":
        window = window_leg(torch, dev, dev_t, res, args.steps, args.warmup, stream, exact,
                            anch=plan_t.get("anch"), heads=plan_t.get("spec_heads"))
        progress(f"window (proof + render): {window['value']} MS/s, proof {window['proof_ms']} ms")
    ms_per_step = elapsed / args.steps * 1e3
    progress(f"timed {args.steps} steps: {ms_per_step:.3f} ms/step, kernel {lin_ms:.3f} ms")
    value = world * samples_rank * args.steps / elapsed / 1e6          # MS/s, whole job
    # the dominant kernel is gss_lin_kernel; its algorithmic bytes are the certified blocks'
    bytes_launch = res.n_fast * res.bb
    achieved = bytes_launch / (lin_ms * 1e-3) / 1e9 if lin_ms > 0 else 0.0
    comp_head = compute_roofline(res.ch_samples_fast, lin_ms, res.bb / npb,
                                 res.ch_samples_fast / max(1, res.n_fast * npb))
    workload = (f"static -l {LOC[0]},{LOC[1]},{LOC[2]:g} -s 2600000 -b {args.fmt}, "
                f"{args.window:g} s per GPU ({nblk} blocks x {npb} samples)")
    version = G.lib().gss_version().decode()
    sha = lib_sha16(G.LIB_PATH)
    # the buffers stay in torch's cache: memory returned to the driver is wiped by the copy
    # engines in the background, which slowed the e2e legs' downloads by up to 1/3 for seconds
    # (tools/e2e_bench_probe.py: 0.65 of the D2H ceiling after a release, 0.93 with the memory
    # kept)
    res.free(release=False)
    gather = None
    if dist and not args.no_gather:
        gather = gather_leg(G, torch, td, dev, dev_t, rank, world, coll_t, walker, args.threads,
                            args.gather_window, host_wire=rehearse, layout=args.gather_layout)
        progress(f"gather: {gather['GBps_at_rank0']} GB/s at rank 0")
    configs = e2e = None
    # the headline's end-to-end leg first, then the per-config legs (each after its own kernel
    # leg, whose memory stays cached)
    if single and not args.no_e2e:
        e2e = e2e_run(G, dev, args.threads, args.e2e_window, batch=128)
        progress(f"e2e: {e2e['value']} MS/s")
    if single and not args.no_configs:
        # the headline's steps and warm-up: the shader clock ramps over the first ~25 launches
        # after an idle spell, so a leg timed on fewer launches reads slower
        configs = per_config(G, torch, dev, dev_t, stream, args.steps, args.warmup, args.threads,
                             e2e=not args.no_e2e)
    # the live PMC passes last: their processes' device memory is wiped when they exit (above)
    traffic, traffic_src, prof = None, "not measured (--no-pmc)", None
    if single and not args.no_pmc:
        traffic, traffic_src, prof = live_traffic(args.fmt, args.window, args.threads, lin_ms,
                                                  args.steps, args.warmup)
    if traffic is None:
        t2, s2 = load_traffic(workload, "gss_lin_kernel", lin_ms, sha)
        if t2 is not None:
            traffic, traffic_src = t2, s2
        else:
            traffic_src = f"{traffic_src}; committed profile: {s2}"
    progress(f"traffic: {traffic_src[:120]}")

    out = {
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
        "dtype": ("int64 phases + f16 x f16 -> f32 MFMA accumulate (exact integer sums)"
                  if G.lib_mfma() else "int64 phases + int64 accumulate"),
        "build": G.build_info(),
        "data": "synthetic: deterministic static-receiver scenario (brdc3540.14n), no dataset",
        "config": {"workload": workload, "samples_per_gpu": samples_rank, "path": "lin",
                   "channels_max": res.nch_max, "parallelism": f"time-window shards x{world}"},
        "x_realtime": round(value / (FS / 1e6), 1),
        "stages_ms": {"fast_path": round(lin_ms, 3), "exact_leftovers_checkpoint": round(ck_ms, 3),
                      "exact_leftovers_synthesis": round(syn_ms, 3),
                      "launches_timed": max(n_launch, n_lin),
                      "fast_path_sustained": sustained_ms},
        "blocks_fast_path": res.n_fast, "blocks_total": nblk,
        "host_plan_s": round(host_plan_s, 3),
        "host_linearize_s": round(host_lin_s, 3),   # the proofs' time (on proofs_on)
        "proofs_on": "gpu (gss_linearize_device)",
        "host_plan_per_rank": host_plan_per_rank,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "profile": prof},
        "step_issue_efficiency": comp_head,
        "cpu_baseline": cpu,
        "per_config": configs,
        "gather": gather,
        "e2e": e2e,
        "exact_path": exact,
        "window": window,
        "lib": {"path": os.path.relpath(G.LIB_PATH, REPO), "version": version, "sha16": sha},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    dev.close()
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
