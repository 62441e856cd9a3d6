#!/usr/bin/env python3
"""Golden digests for the long BASELINE configurations, made by streaming the reference.

BASELINE.json configs[3] (static, 20 MS/s, -b 16, 3600 s: 288 GB) and configs[4] (static,
2.6 MS/s, -b 1, 86400 s: 56 GB) are too large to store or to hash on the GPU box sequentially.
This script runs the reference binary (oracle/_ref/gps-sdr-sim, compiled from
/root/reference/gpssim.c by oracle/Makefile) with `-o -` and records, from its stdout:

  block digests    sha256 of each 0.1 s block's bytes (gpssim.c:2276/2283/2287 writes),
  chunk digests    sha256 over the concatenated block digests of each 300-block (30 s) chunk,
  digest_of_blocks sha256 over all block digests concatenated (a checksum of checksums),
  sha256           the plain sha256 of the whole stream (same as `-o - | sha256sum`),
  head             the first 64 bytes of the stream (hex).

Only the chunk digests, the two totals and the digests of the first/last 8 blocks go into the
fixture (tests/golden/long_<name>.json); tests/test_gpu_long.py recomputes them on the GPU box
from the product's streaming driver (gss_run), hashing blocks in parallel.

Usage (in this container; CPU only, ~1 h for static20m, ~3.6 h for day_b1):
    python tests/golden/make_long_golden.py static20m|day_b1
"""
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim")
NAV = os.path.join(HERE, "data", "brdc3540.14n")
LOC = "30.286502,120.032669,100"
CHUNK = 300

CONFIGS = {
    # BASELINE configs[3]: the 8-GPU sharded scenario, as one stream
    "static20m": dict(args=["-d", "3600", "-s", "20000000", "-b", "16"], fs=20000000, fmt=16,
                      duration=3600.0),
    # BASELINE configs[4]: the 24 h 1-bit scenario
    "day_b1": dict(args=["-d", "86400", "-s", "2600000", "-b", "1"], fs=2600000, fmt=1,
                   duration=86400.0),
}


def block_bytes(fs, fmt):
    n = (int(fs) // 10 * 10) // 10
    return {16: 4 * n, 8: 2 * n, 1: n // 4}[fmt]


def main(name):
    cfg = CONFIGS[name]
    bb = block_bytes(cfg["fs"], cfg["fmt"])
    cmd = [REF, "-e", NAV, "-l", LOC] + cfg["args"] + ["-o", "-"]
    t0 = time.time()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, bufsize=0)
    whole = hashlib.sha256()
    all_dig = hashlib.sha256()
    chunk = hashlib.sha256()
    chunks, first, last = [], [], []
    head = None
    nblk = 0
    buf = bytearray(bb)
    mv = memoryview(buf)
    out = os.path.join(HERE, f"long_{name}.json")
    prog = out + ".progress"
    while True:
        got = 0
        while got < bb:
            r = p.stdout.readinto(mv[got:])
            if not r:
                break
            got += r
        if got == 0:
            break
        if got != bb:
            raise SystemExit(f"short block {nblk}: {got} of {bb} bytes")
        if head is None:
            head = bytes(buf[:64]).hex()
        whole.update(mv)
        d = hashlib.sha256(mv).digest()
        all_dig.update(d)
        chunk.update(d)
        if nblk < 8:
            first.append(d.hex())
        last = (last + [d.hex()])[-8:]
        nblk += 1
        if nblk % CHUNK == 0:
            chunks.append(chunk.hexdigest()[:16])
            chunk = hashlib.sha256()
            with open(prog, "w") as f:
                f.write(f"{nblk} blocks, {time.time() - t0:.0f} s\n")
    if nblk % CHUNK:
        chunks.append(chunk.hexdigest()[:16])
    rc = p.wait()
    if rc != 0:
        raise SystemExit(f"reference exited with {rc}")
    res = {
        "config": name,
        "command": "gps-sdr-sim -e brdc3540.14n -l " + LOC + " " + " ".join(cfg["args"]) + " -o -",
        "samp_freq": cfg["fs"], "fmt": cfg["fmt"], "duration": cfg["duration"],
        "blocks": nblk, "block_bytes": bb, "bytes": nblk * bb,
        "sha256": whole.hexdigest(),
        "digest_of_blocks": all_dig.hexdigest(),
        "chunk_blocks": CHUNK,
        "chunk_sha16": chunks,
        "first_block_sha": first,
        "last_block_sha": last,
        "head": head,
        "ref_wall_s": round(time.time() - t0, 1),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    if os.path.exists(prog):
        os.remove(prog)
    print(json.dumps({k: v for k, v in res.items() if k != "chunk_sha16"}))


if __name__ == "__main__":
    main(sys.argv[1])
