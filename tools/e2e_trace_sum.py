#!/usr/bin/env python3
"""Summarise a GSS_RUN_TRACE=1 stderr log of gss_run (tools/gpu_e2e_trace.sh): per slot, the
planner's host-plane time (gss_scn_next), its proof time (gss_linearize), and the main thread's
wait for each slot's D2H; medians over the steady part of the run."""
import statistics
import sys

plan, scn, drain, prove = [], [], [], []
last_scn = None
for line in open(sys.argv[1]):
    f = line.split()
    if not f or f[0] != "trace":
        continue
    if f[1] == "scn_done":
        last_scn = float(f[2])
    elif f[1] == "plan":
        t0, t1 = float(f[6]), float(f[7])
        if last_scn is not None and t0 <= last_scn <= t1:
            scn.append((last_scn - t0, t1 - last_scn))
        plan.append(t1 - t0)
    elif f[1] == "prove":                        # proofs on the prover thread (gss_run)
        prove.append(float(f[7]) - float(f[6]))
    elif f[1] == "drain":
        drain.append((float(f[6]) - float(f[5]), float(f[8]) - float(f[6])))
steady = slice(2, -2)
med = lambda xs: statistics.median(xs) * 1e3 if xs else float("nan")
print(f"slots {len(plan)}")
if scn:
    print(f"planner per slot {med(plan[steady]):.2f} ms: host plane "
          f"{med([a for a, _ in scn[steady]]):.2f} ms + proofs {med([b for _, b in scn[steady]]):.2f} ms")
else:
    print(f"planner per slot {med(plan[steady]):.2f} ms (rows, chain, walks; proofs on the prover)")
if prove:
    print(f"prover per slot {med(prove[steady]):.2f} ms")
print(f"main thread: D2H wait per slot {med([a for a, _ in drain[steady]]):.2f} ms, sink "
      f"{med([b for _, b in drain[steady]]):.2f} ms")
