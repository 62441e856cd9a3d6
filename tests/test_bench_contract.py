"""bench.py pieces that need no GPU: the metric is BASELINE.json's, the committed PMC traffic
record (profiles/pmc_traffic.json) is attached only to the workload, kernel and library build it
was measured on and only when its kernel time agrees with its own run's events, and the CPU
baseline runs the reference binary pinned per core without a launcher hop."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_metric_is_baselines():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert bench.METRIC == base["metric"]


def test_traffic_record_matches_its_build_only():
    rec = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    wl, sha = rec["workload"], rec["lib_sha16"]
    ms = rec["unprofiled_event_ms"]
    got, src = bench.load_traffic(wl, "gss_lin_kernel", ms, sha)
    assert got == rec["hbm_bytes_per_launch"] and "profiled kernel" in src
    # HBM bytes within a few % of the algorithmic bytes: no wasted re-reads
    assert 1.0 <= got / rec["algorithmic_bytes_per_launch"] < 1.05
    assert bench.load_traffic(wl, "gss_lin_kernel", ms, "0" * 16)[0] is None
    assert bench.load_traffic(wl + " x", "gss_lin_kernel", ms, sha)[0] is None
    assert bench.load_traffic(wl, "gss_synth_kernel", ms, sha)[0] is None
    # a run whose kernel time differs from the profile's by more than 10 % gets no traffic
    assert bench.load_traffic(wl, "gss_lin_kernel", ms * 0.8, sha)[0] is None


def test_committed_profile_agrees_with_unprofiled_run():
    """the profile's warm kernel time is within 10 % of the un-profiled run of the same build,
    steps and warm-up (bench.py live_traffic's rule), and not longer than its step"""
    rec = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    prof = rec["kernel_timed_avg_ns"] / 1e6
    assert abs(prof - rec["unprofiled_event_ms"]) <= 0.10 * rec["unprofiled_event_ms"]
    assert rec["steps"] >= 20 and rec["warmup"] >= 5


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "gss_oracle_cli")),
                    reason="oracle not built")
def test_cpu_baseline_short_sample():
    """one process per core of the affinity mask (no cap), plus the 1-core figure"""
    r = bench.cpu_baseline(seconds=1)
    assert r is not None and r["cores"] == len(os.sched_getaffinity(0)) and r["value"] > 0
    assert r["single_core"]["cores"] == 1 and r["kind"] in ("reference", "port")


def test_dtype_label_follows_the_build():
    """bench's dtype names the accumulation the loaded build uses (LIN_MFMA 1 or 2: matrix cores)"""
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import gpssim_amd as G
    info = G.build_info()
    assert info["lin_mfma"] in ("0", "1", "2")
    assert G.lib_mfma() == (info["lin_mfma"] != "0")
    assert info["lin_mfma"] == "2"                 # the shipped build: channel pairs on MFMA


def test_step_issue_efficiency_bounds():
    """the fast kernel's issue-efficiency line (was roofline_compute) says what it is and carries
    the HBM fraction its step and the formulation's floor allow: 19.6 SIMD
    cycles per wave channel-step at 11.3 channels and 4 B per sample bound the headline at
    ~0.355 of 8 TB/s; the floor and the LDS bound sit above it"""
    r = bench.compute_roofline(8.8e9, 1.466, 4.0, 11.3)
    assert "issue efficiency" in r["what"] and "not an HBM roofline" in r["what"]
    assert abs(r["bound_frac"] - 0.355) < 0.002
    assert r["bound_frac"] < r["floor_bound_frac"] < 1.0
    assert r["bound_frac"] < r["lds_bound_frac"] < 1.0
    # the kernel's HBM fraction over the step's bound = its issue efficiency
    hbm = 8.8e9 / 11.3 * 4.0 / 1.466e-3 / 8e12
    assert abs(hbm / r["bound_frac"] - r["frac"]) < 0.01
    assert "bound_frac" not in bench.compute_roofline(8.8e9, 1.466)    # without the shape
    assert bench.compute_roofline(8.8e9, 0.0) is None
