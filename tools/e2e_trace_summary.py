"""Summarise a GSS_RUN_TRACE=1 log of gss_run (stderr of tools/e2e_bench_probe.py or
tools/e2e_cfg_probe.py): per run (runs end at their 'trace spec total' line), the median and total
time of each stage per slot, the start-up (first rows to first drain) and the drain intervals.

usage: python tools/e2e_trace_summary.py TRACE_FILE"""
import statistics as st
import sys


def runs(path):
    cur = []
    for line in open(path):
        p = line.split()
        if not p or p[0] != "trace":
            continue
        cur.append(p)
        if p[1] == "spec" and p[2] == "total":
            yield cur
            cur = []
    if cur:
        yield cur


def nums(p):
    out = []
    for x in p:
        try:
            if "." in x:
                out.append(float(x))
        except ValueError:
            pass
    return out


def summary(ev):
    def span(kind):
        return [nums(p) for p in ev if p[1] == kind]
    rows = span("rows")        # produced t0 t1 wait
    plan = span("plan")        # t0 t1
    prove = span("prove")
    submit = span("submit")
    drain = span("drain")      # wait t0 t1 sink_end
    setup = span("setup")      # enter ready
    spec = [p for p in ev if p[1] == "spec" and p[2] == "nb"]
    out = {"slots": len(drain)}

    def ms(xs):
        return {"median_ms": round(st.median(xs) * 1e3, 3), "total_s": round(sum(xs), 3)} \
            if xs else None
    out["rows"] = ms([n[1] - n[0] for n in rows if len(n) >= 2])
    out["rows_wait"] = ms([n[2] for n in rows if len(n) >= 3])
    out["plan"] = ms([n[1] - n[0] for n in plan if len(n) >= 2])
    out["prove"] = ms([n[1] - n[0] for n in prove if len(n) >= 2])
    out["submit"] = ms([n[1] - n[0] for n in submit if len(n) >= 2])
    out["drain_wait"] = ms([n[1] - n[0] for n in drain if len(n) >= 2])
    if spec:
        out["spec_gpu_wait"] = ms([float(p[11]) for p in spec])
        out["spec_chain"] = ms([float(p[13]) for p in spec])
        out["spec_guess"] = ms([float(p[9]) for p in spec])
    if drain:
        ends = [n[2] for n in drain]
        iv = [b - a for a, b in zip(ends, ends[1:])]
        t_first = min([n[0] for n in rows if n] + [n[0] for n in plan if n] + [ends[0]] +
                      [n[0] for n in setup if n])
        if setup:
            out["setup_s"] = round(setup[0][1] - setup[0][0], 4)
        out["startup_s"] = round(ends[0] - t_first, 4)
        out["run_s"] = round(ends[-1] - t_first, 4)
        out["drain_interval"] = ms(iv)
    return out


if __name__ == "__main__":
    import json
    for i, ev in enumerate(runs(sys.argv[1])):
        print(json.dumps({"run": i, **summary(ev)}))
