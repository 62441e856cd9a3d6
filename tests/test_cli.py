"""The CLI keeps the reference's option surface and error behaviour (gpssim.c:1650-1873)."""
import subprocess

import pytest

from conftest import LOC, NAV

import gpssim_amd as G


def run(args):
    return subprocess.run([G.CLI_PATH] + args, capture_output=True, text=True)


def test_usage_when_no_args():
    r = run([])
    assert r.returncode == 1 and "Usage: gps-sdr-sim [options]" in r.stderr


@pytest.mark.parametrize("args,msg", [
    (["-e", NAV, "-b", "4"], "ERROR: Invalid I/Q data format."),
    (["-e", NAV, "-s", "100000"], "ERROR: Invalid sampling frequency."),
    (["-e", NAV, "-t", "1970/01/01,00:00:00"], "ERROR: Invalid date and time."),
    (["-l", "1,2,3", "-d", "5"], "ERROR: GPS ephemeris file is not specified."),
    (["-e", NAV, "-l", "1,2,3", "-d", "-3"], "ERROR: Invalid duration."),
    (["-e", "/nope.14n", "-l", "1,2,3", "-d", "1"], "ERROR: ephemeris file not found."),
])
def test_cli_errors(args, msg):
    r = run(args)
    assert r.returncode == 1
    assert msg in r.stderr
