#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/gps-sdr-sim (the reference gpssim.c compiled by oracle/Makefile with the
reference's own flags) on the BASELINE.json configs, streaming its output through sha256:
  * full-output sha256 and byte count per config,
  * a per-block sha256 prefix list (16 hex chars) so a mismatch can be localised to a block,
  * the first 4096 samples of block 0 (raw bytes, hex) for quick diffs.
Also extracts the reference's 512-entry sin/cos tables (gpssim.c:15-83) as data (lut512.json).
Needs /root/reference (this container only); the GPU box uses the committed JSON.
Also records the reference's stderr text for two runs (stderr.json: banner, channel table,
-v details, progress lines).
Usage: python tests/golden/make_golden.py [--quick] [config names...]
"""
import hashlib
import json
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim")
REF_SRC = "/root/reference"
NAV = os.path.join(REF_SRC, "brdc3540.14n")
LOC = "30.286502,120.032669,100"

# name -> (argv tail, samples per block, fmt)
CONFIGS = {
    "static_d30_b16": (["-l", LOC, "-d", "30", "-s", "2600000", "-b", "16"], 260000, 16),
    "static_d30_b8": (["-l", LOC, "-d", "30", "-s", "2600000", "-b", "8"], 260000, 8),
    "static_d30_b1": (["-l", LOC, "-d", "30", "-s", "2600000", "-b", "1"], 260000, 1),
    "static_d30_s20M_b16": (["-l", LOC, "-d", "30", "-s", "20000000", "-b", "16"], 2000000, 16),
    "static_d300_b16": (["-l", LOC, "-d", "300", "-s", "2600000", "-b", "16"], 260000, 16),
    "circle_b8": (["-u", os.path.join(REF_SRC, "circle.csv"), "-s", "2600000", "-b", "8"], 260000, 8),
    "static_d65_b8_noiono": (["-l", "-33.8688,151.2093,58", "-d", "65", "-s", "2600000", "-b",
                              "8", "-i"], 260000, 8),
    "ecef_d35_s3M_b16": (["-c", "-2700000.0,-4290000.0,3860000.0", "-d", "35", "-s",
                          "3000000", "-b", "16"], 300000, 16),
}
# the rest of the CLI surface: NMEA input, valid -t, -T (the fall-through
# into -t's parser, gpssim.c:1804-1835), USER_MOTION_SIZE=4000 (gpssim.h:19-21) for rocket.csv,
# the LEO satellite.csv scenario with -i
DATA = os.path.join(REPO, "tests", "golden", "data")
REF_UM4000 = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim-um4000")
CONFIGS.update({
    "nmea_triumph_b8": (["-g", os.path.join(REF_SRC, "triumphv3.txt"), "-s", "2600000", "-b",
                         "8"], 260000, 8),
    "static_t0200_d30_b8": (["-l", LOC, "-t", "2014/12/20,02:00:00", "-d", "30", "-b", "8"],
                            260000, 8),
    "static_T1221_d30_b8": (["-l", LOC, "-T", "2014/12/21,00:00:00", "-d", "30", "-b", "8"],
                            260000, 8),
    "rocket_um4000_b8": (["-u", os.path.join(REF_SRC, "rocket.csv"), "-s", "2600000", "-b", "8"],
                         260000, 8),
    "satellite_i_b8": (["-u", os.path.join(REF_SRC, "satellite.csv"), "-i", "-s", "2600000",
                        "-b", "8"], 260000, 8),
})
# the integer-carrier build (FLOAT_CARR_PHASE off, gpssim.h:4; oracle/Makefile), which the
# product renders with --carrier=int
REF_INT = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim-intcarr")
CONFIGS.update({
    "intcarr_static_d30_b16": (["-l", LOC, "-d", "30", "-s", "2600000", "-b", "16"], 260000, 16),
    "intcarr_static_d65_b8": (["-l", LOC, "-d", "65", "-s", "2600000", "-b", "8"], 260000, 8),
    "intcarr_circle_b8": (["-u", os.path.join(REF_SRC, "circle.csv"), "-s", "2600000", "-b",
                           "8"], 260000, 8),
    "intcarr_static_d30_s20M_b1": (["-l", LOC, "-d", "30", "-s", "20000000", "-b", "1"],
                                   2000000, 1),
})
BINARY = {"rocket_um4000_b8": REF_UM4000, "intcarr_static_d30_b16": REF_INT,
          "intcarr_static_d65_b8": REF_INT, "intcarr_circle_b8": REF_INT,
          "intcarr_static_d30_s20M_b1": REF_INT}
# reference stderr (banner, channel table, -v details, progress), minus the timing line
STDERR = {
    "static_d31_v": ["-l", LOC, "-d", "31", "-b", "1", "-v"],
    "circle_d31": ["-u", os.path.join(REF_SRC, "circle.csv"), "-d", "31", "-b", "1"],
}
QUICK = {"static_d30_b16", "static_d30_b8", "static_d30_b1"}


def block_bytes(n, fmt):
    return n * 4 if fmt == 16 else n * 2 if fmt == 8 else n // 4


def run(name, tail, n, fmt):
    bb = block_bytes(n, fmt)
    argv = [BINARY.get(name, REF_BIN), "-e", NAV] + tail + ["-o", "-"]
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, cwd="/tmp")
    full = hashlib.sha256()
    blocks, head, total = [], None, 0
    while True:
        buf = p.stdout.read(bb)
        if not buf:
            break
        full.update(buf)
        total += len(buf)
        if head is None:
            head = buf[: min(len(buf), 4096 * (4 if fmt == 16 else 2 if fmt == 8 else 1))].hex()
        blocks.append(hashlib.sha256(buf).hexdigest()[:16])
    rc = p.wait()
    if rc != 0:
        raise SystemExit(f"{name}: reference exited {rc}")
    return {"argv": [os.path.basename(a) if a.startswith(REF_SRC) else a for a in tail],
            "n_per_blk": n, "fmt": fmt, "bytes": total, "blocks": len(blocks),
            "sha256": full.hexdigest(), "block_sha16": blocks, "head_hex": head,
            "user_motion_size": 4000 if name == "rocket_um4000_b8" else 3000,
            "carrier": "int" if name.startswith("intcarr_") else "float"}


def stderr_of(tail):
    """the reference's stderr for a run to /dev/null, without its CPU-time line"""
    argv = [REF_BIN, "-e", NAV] + tail + ["-o", "/dev/null"]
    p = subprocess.run(argv, capture_output=True, cwd="/tmp")
    if p.returncode != 0:
        raise SystemExit(f"{tail}: reference exited {p.returncode}")
    text = p.stderr.decode()
    return "".join(l for l in text.splitlines(True) if not l.startswith("Process time"))


def lut_fixture():
    src = open(os.path.join(REF_SRC, "gpssim.c")).read()
    out = {}
    for name in ("sinTable512", "cosTable512"):
        body = re.search(name + r"\[\]\s*=\s*\{([^}]*)\}", src).group(1)
        out[name] = [int(v) for v in body.replace("\n", " ").split(",") if v.strip()]
    return out


def main():
    quick = "--quick" in sys.argv
    if not os.path.exists(REF_BIN):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref"])
    path = os.path.join(HERE, "golden.json")
    gold = json.load(open(path)) if os.path.exists(path) else {}
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    for name, (tail, n, fmt) in CONFIGS.items():
        if (quick and name not in QUICK) or (only and name not in only):
            continue
        print("running", name, flush=True)
        gold[name] = run(name, tail, n, fmt)
        json.dump(gold, open(path, "w"), indent=1)
    if not quick:
        err = {name: {"argv": [os.path.basename(a) if a.startswith(REF_SRC) else a for a in tail],
                      "stderr": stderr_of(tail)} for name, tail in STDERR.items()}
        json.dump(err, open(os.path.join(HERE, "stderr.json"), "w"), indent=1)
    json.dump(lut_fixture(), open(os.path.join(HERE, "lut512.json"), "w"))
    print("done")


if __name__ == "__main__":
    main()
