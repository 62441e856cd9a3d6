#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a bench.py live-profile directory (GSS_PROF_SAVE=<dir> python
bench.py ..., whose JSON line is in <dir>/bench.log): HBM bytes per launch of the fast kernel from
the PMC passes (WRITE_SIZE exact, FETCH_SIZE x2 for gfx950 wide reads; both KiB,
MI355X_MICROARCH.md §HBM), keyed by the bench workload string and library build, with the
profiled kernel time next to the un-profiled run's own event time (bench.py attaches the record
only when they agree within 10 %).
Usage: python tools/pmc_traffic.py gpurun_out/prof_<tag> [out.json]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "pmc_traffic.json")
    live = {}
    try:
        live = json.load(open(os.path.join(d, "live_summary.json")))
    except OSError:
        pass
    summ = json.loads(subprocess.check_output([sys.executable,
                                               os.path.join(REPO, "tools", "prof_summary.py"), d,
                                               str(live.get("steps") or 0),
                                               str(live.get("warmup") or 0)]))
    bench = None
    for name in ("bench", "kt", "pmc_write", "pmc_fetch"):
        try:
            for line in open(os.path.join(d, name + ".log")):
                if line.startswith("{") and '"metric"' in line:
                    bench = bench or json.loads(line)
        except OSError:
            pass
    k = next(n for n in summ if n.startswith("gss_lin_kernel"))
    e = summ[k]
    w, r = e["hbm_write_bytes"], e["hbm_read_bytes_corrected"]
    alg = None
    if bench:                 # -b 16: 4 B per sample; the fast path renders the certified blocks
        share = bench.get("blocks_fast_path", 0) / bench["blocks_total"]
        alg = round(bench["config"]["samples_per_gpu"] * 4 * share)
    res = {"workload": bench["config"]["workload"] if bench else None, "kernel": k,
           "hbm_bytes_per_launch": round(w + r), "hbm_write_bytes_per_launch": round(w),
           "hbm_read_bytes_per_launch": round(r), "algorithmic_bytes_per_launch": alg,
           "kernel_avg_ns": e.get("avg_ns"), "kernel_warm_avg_ns": e.get("warm_avg_ns"),
           "kernel_timed_avg_ns": e.get("timed_avg_ns"), "timed_launches": e.get("timed_launches"),
           "profiled_run_event_ms": live.get("profiled_run_event_ms"),
           "unprofiled_event_ms": (bench or {}).get("stages_ms", {}).get("fast_path"),
           "steps": live.get("steps"), "warmup": live.get("warmup"),
           "lib_sha16": (bench or {}).get("lib", {}).get("sha16"),
           "method": "rocprofv3 --kernel-trace --stats; --pmc WRITE_SIZE / --pmc FETCH_SIZE in "
                     "separate passes (--kernel-trace only), KiB x1024, FETCH_SIZE x2 (gfx950 "
                     "correction); the same bench command, steps and warm-up as the un-profiled "
                     "run; kernel_timed_avg_ns = dispatches warmup .. warmup + steps - 1, "
                     "the launches the bench times",
           "source": os.path.relpath(d, REPO)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
