#!/usr/bin/env python3
"""Apply INTEGRATION.md §2 to a /tmp copy of the reference's gpssim.c and build it.

The reference stays untouched (/root/reference is read-only); its gpssim.c and gpssim.h are
copied to /tmp/gss_integ/ and edited there:
  1. two prototypes after `#include "gpssim.h"`;
  2. the sample loop and its pack/fwrite epilogue (gpssim.c:2190-2288: from
     `for (isamp=0; isamp<iq_buff_size; isamp++)` through the SC16 fwrite branch) become
     `gss_integ_block(chan, gain, iq_buff_size, data_format, delt, grx.sec, fp);`;
  3. `gss_integ_flush(fp);` before the reference's `tend = clock();`.
Then gcc builds it with the reference's flags together with tools/integration/gss_integ.c,
linked against gps-sdr-sim_amd/lib/libgpssim_amd.so, into oracle/_ref/gps-sdr-sim-integ
(git-ignored, travels to the GPU box; tests/test_gpu_parity.py runs it there).  A second build,
oracle/_ref/gps-sdr-sim-integ-intcarr, is the same patch on the reference's other carrier mode:
the one `#define FLOAT_CARR_PHASE` line of the gpssim.h copy dropped (as oracle/Makefile does for
its _ref/gps-sdr-sim-intcarr), so gss_integ.c's integer-carrier branch is built and tested too.
Usage: python tools/integration/build_integ.py [--check]   (--check: compile and link only)
"""
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
WORK = "/tmp/gss_integ"
OUT = os.path.join(REPO, "oracle", "_ref", "gps-sdr-sim-integ")
OUT_INT = OUT + "-intcarr"


def patch(src):
    inc = '#include "gpssim.h"\n'
    assert src.count(inc) == 1
    src = src.replace(inc, inc + "void gss_integ_block(channel_t *chan, const int *gain, "
                      "int iq_buff_size, int data_format, double delt, double grx_sec, "
                      "FILE *fp);\nvoid gss_integ_flush(FILE *fp);\n")
    start = src.index("for (isamp=0; isamp<iq_buff_size; isamp++)")
    sc16 = src.index("fwrite(iq_buff, 2, 2*iq_buff_size, fp);", start)
    end = src.index("}", sc16) + 1                       # the SC16 branch's closing brace
    src = (src[:start] +
           "gss_integ_block(chan, gain, iq_buff_size, data_format, delt, grx.sec, fp);"
           "  /* INTEGRATION.md: replaces gpssim.c:2190-2288 */" + src[end:])
    m = re.search(r"\n(\s*)tend = clock\(\);", src)
    src = src[:m.start()] + f"\n{m.group(1)}gss_integ_flush(fp);" + src[m.start():]
    return src


def build(work, out, drop_float_carr):
    os.makedirs(work, exist_ok=True)
    hdr = open(os.path.join(REF, "gpssim.h")).read()
    if drop_float_carr:
        hdr = re.sub(r"(?m)^#define FLOAT_CARR_PHASE.*\n", "", hdr)
        assert "#define FLOAT_CARR_PHASE" not in hdr
    open(os.path.join(work, "gpssim.h"), "w").write(hdr)
    open(os.path.join(work, "gpssim.c"), "w").write(
        patch(open(os.path.join(REF, "gpssim.c")).read()))
    lib = os.path.join(REPO, "gps-sdr-sim_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libgpssim_amd.so")):
        subprocess.check_call(["make", "-C", os.path.join(REPO, "gps-sdr-sim_amd")])
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["gcc", "-O3", "-Wall", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
           "-D_FILE_OFFSET_BITS=64", "-I" + work, "-I" + os.path.join(REPO, "include"),
           os.path.join(work, "gpssim.c"), os.path.join(HERE, "gss_integ.c"), "-L" + lib,
           "-lgpssim_amd", "-Wl,-rpath,$ORIGIN/../../gps-sdr-sim_amd/lib", "-lm", "-o", out]
    subprocess.check_call(cmd)
    print("built", out)


def main():
    if not os.path.exists(os.path.join(REF, "gpssim.c")):
        sys.exit("no reference sources at " + REF)
    build(WORK, OUT, False)
    build(WORK + "_intcarr", OUT_INT, True)


if __name__ == "__main__":
    main()
