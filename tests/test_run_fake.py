"""gss_run (csrc/hip/gss_run.hip, unchanged) on the CPU fake of the HIP runtime.

tests/helpers/fake_hip stands in for the HIP calls gss_run makes (streams drained by worker
threads, events as generation counters), tests/helpers/fake_dev.cpp for its device functions
(renders write a fingerprint of each block's rows and nav words), and run_fake.cpp drives
every mode of the run (host / gpu / split proofs, two runs on one handle, the two-rank
baton hand-off, a sink that stops) checking every byte the sink receives.  tools/sanitize.sh
runs the same program under TSan and ASan+UBSan; this is the plain build, so the CPU suite
catches an orchestration regression without a GPU.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAV = os.path.join(ROOT, "tests", "golden", "data", "brdc3540.14n")


@pytest.fixture(scope="module")
def run_fake(tmp_path_factory):
    if shutil.which("gcc") is None or shutil.which("g++") is None:
        pytest.skip("gcc/g++ not available")
    d = tmp_path_factory.mktemp("fake")
    cf = ["-O2", "-g", "-ffp-contract=off", "-fno-fast-math", "-D_FILE_OFFSET_BITS=64",
          "-I" + os.path.join(ROOT, "include")]
    inc = ["-I" + os.path.join(ROOT, "tests", "helpers"),
           "-I" + os.path.join(ROOT, "tests", "helpers", "fake_hip")]
    host = os.path.join(ROOT, "gps-sdr-sim_amd", "csrc", "host")
    objs = []
    srcs = [os.path.join(host, f) for f in sorted(os.listdir(host)) if f.endswith(".c")]
    srcs.append(os.path.join(ROOT, "gps-sdr-sim_amd", "csrc", "cli", "cli_args.c"))
    for s in srcs:
        o = str(d / (os.path.basename(s)[:-2] + ".o"))
        subprocess.run(["gcc"] + cf + ["-c", s, "-o", o], check=True)
        objs.append(o)
    cxx = [(os.path.join(ROOT, "gps-sdr-sim_amd", "csrc", "hip", "gss_run.hip"), True)]
    for f in ("fake_hip/fake_hip.cpp", "fake_dev.cpp", "run_fake.cpp"):
        cxx.append((os.path.join(ROOT, "tests", "helpers", f), False))
    for s, as_cxx in cxx:
        o = str(d / (os.path.basename(s).rsplit(".", 1)[0] + ".o"))
        cmd = ["g++", "-std=c++17"] + cf + inc + (["-x", "c++"] if as_cxx else []) + ["-c", s, "-o", o]
        subprocess.run(cmd, check=True)
        objs.append(o)
    exe = str(d / "run_fake")
    subprocess.run(["g++", "-o", exe] + objs + ["-lm", "-lpthread"], check=True)
    return exe


@pytest.mark.parametrize("args", [("35", "64", "1"), ("25", "16", "8")])
def test_gss_run_on_fake_device(run_fake, args):
    r = subprocess.run([run_fake, NAV, *args], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "all modes ok" in r.stdout
