"""Diagnose a gss_run mode on a mid-run range: per-block hashes with the proofs on the GPU and on
the host, and which blocks differ (GPU box only).  Env as the streaming tests set it.

usage: GSS_RUN_SPEC=1 GSS_RUN_ROWS_AHEAD=1 python tools/diag_midrun.py [first] [n] [batch]"""
import hashlib
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "gps-sdr-sim_amd"), REPO, os.path.join(REPO, "tests")]
import gpssim_amd as G  # noqa: E402
from conftest import GOLDEN, NAV  # noqa: E402


def run(dev, proof, first, n, batch):
    os.environ["GSS_RUN_PROOF"] = proof
    s, _ = G.Scenario.from_cli(["-e", NAV, "-l", "-33.8688,151.2093,58", "-d", "65", "-b", "8",
                                "-i"])
    bb = G.block_bytes(s.n_per_blk, 8)
    out = []

    def sink(buf, f, nb):
        for i in range(nb):
            out.append((f + i, hashlib.sha256(buf[i * bb:(i + 1) * bb]).hexdigest()[:16]))
    dev.run(s, sink, first_block=first, n_blocks=n, batch=batch)
    return out


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 333
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    want = json.load(open(GOLDEN))["static_d65_b8_noiono"]["block_sha16"]
    dev = G.Device(0)
    out = {"first": first, "n": n, "batch": batch,
           "env": {k: v for k, v in os.environ.items() if k.startswith("GSS_RUN_")}}
    for proof in ("host", "gpu"):
        got = run(dev, proof, first, n, batch)
        bad = [b for b, x in got if x != want[b]]
        out[proof] = {"blocks": len(got), "n_wrong": len(bad), "wrong": bad[:12]}
    print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
