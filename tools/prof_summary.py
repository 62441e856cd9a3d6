#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory: per-kernel average duration (kernel trace
stats) and per-dispatch PMC counters averaged per kernel, with the gfx950 corrections of
MI355X_MICROARCH.md §HBM (FETCH_SIZE reads half the bytes of wide streaming reads: x2;
WRITE_SIZE is exact for 16-B-per-lane streaming stores; both in KiB)."""
import csv
import collections
import glob
import json
import os
import sys


def short(name):
    """the kernel's name without its parameter list: 'void gss_lin_kernel<16>(...)' ->
    'gss_lin_kernel<16>', '(anonymous namespace)::k(...)' -> 'k'"""
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def kernel_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "kt", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    return out


def kernel_durations(d):
    """per-dispatch durations [ns] in dispatch order, per kernel (kernel trace of the kt pass)"""
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "*kernel_trace.csv")):
        try:
            rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
            for r in rows:
                out[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) -
                                                    int(r["Start_Timestamp"]))
        except (KeyError, ValueError):       # an unexpected trace layout: no per-dispatch data
            return {}
    return dict(out)


def warm_avg_ns(durs):
    """mean duration of the dispatches after the first (the cold warm-up launch)"""
    w = durs[1:] if len(durs) > 1 else durs
    return sum(w) / len(w) if w else 0.0


def timed_avg_ns(durs, steps, warmup=0):
    """mean duration of dispatches warmup .. warmup + steps - 1: the launches a bench run times
    after its warm-up (one launch per step).  Under sustained load the shader clock ramps up over
    the first ~25 launches (GRBM_GUI_ACTIVE per dispatch: 1.7 -> 2.3 GHz), so an average over all
    dispatches, warm-up included, is longer than the timed region's."""
    w = durs[warmup:warmup + steps] if steps and len(durs) >= warmup + steps else durs
    return sum(w) / len(w) if w else 0.0


# GRBM_GUI_ACTIVE counts the whole GPU's busy cycles over the counter window, which for a short
# dispatch is mostly the profiler's own window around it and for overlapping kernels includes the
# others' work: the effective clock is reported only for dispatches of >= 200 us and at most the
# chip's peak shader clock (2.4 GHz), else left out
CLK_MIN_NS = 200_000
CLK_MAX_GHZ = 2.4


def counters(d):
    """per kernel: each counter averaged over its dispatches, and "_clk": the clock the dispatches
    with GRBM_GUI_ACTIVE ran at, their per-XCD cycles summed over their own durations (the
    counter pass's timestamps of the same dispatches, not another pass's averages)"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    clk = collections.defaultdict(lambda: [0.0, 0.0])       # kernel -> [cycles, ns]
    for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("End_Timestamp"):
                ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                if ns >= CLK_MIN_NS:
                    clk[k][0] += float(r["Counter_Value"]) / 8
                    clk[k][1] += ns
            meta[k] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                       "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"]),
                       "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"])}
    res = {}
    for k, cs in acc.items():
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k]["_meta"] = meta[k]
        if clk[k][1] > 0 and clk[k][0] / clk[k][1] <= CLK_MAX_GHZ:
            res[k]["_clk"] = clk[k][0] / clk[k][1]
    return res


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0     # timed launches (bench --steps)
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 0    # launches before them (--warmup)
    ks = kernel_stats(d)
    kd = kernel_durations(d)
    cs = counters(d)
    summary = {}
    for k in sorted(set(ks) | set(cs)):
        e = dict(ks.get(k, {}))
        if k in kd:
            e["warm_avg_ns"] = warm_avg_ns(kd[k])
            if steps:
                e["timed_avg_ns"] = timed_avg_ns(kd[k], steps, warmup)
                e["timed_launches"] = min(steps, len(kd[k]))
        c = cs.get(k, {})
        e.update({"meta": c.get("_meta")})
        e["counters"] = {n: v for n, v in c.items() if not n.startswith("_")}
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c:
            e["hbm_read_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
            e["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1)
        if "_clk" in c:
            e["eff_clock_ghz"] = c["_clk"]
        if "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8                 # per-XCD GPU cycles of the dispatch
            if "SQ_ACTIVE_INST_VALU" in c:                 # 4 issue cycles per wave64 VALU op
                e["valu_issue_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024)
            if "SQ_LDS_IDX_ACTIVE" in c:
                e["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (cyc * 256)
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
        summary[k] = e
    json.dump(summary, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
