#!/bin/bash
# Build measurement variants of the library into _var/<name>/ (another LIN_CH, or a variant
# source of the fast-path kernel): usage  [HOSTFLAGS="-D..."] bash tools/ablate.sh name "EXTRA_HIPFLAGS"
# SYNTH_SRC=<file> builds another version of gss_synth.hip (a measurement variant kept outside
# the product source, or a previous commit's: git show <rev>:gps-sdr-sim_amd/csrc/hip/gss_synth.hip;
# the ablation switches of rounds 2-4 -- LIN_ABLATE, LIN_STAMP, LIN_SWIN, LIN_MFMA, ... -- are in
# the source of commit 898e226).
# The variant is loaded by bench.py through GSS_LIB_PATH=_var/<name>/libgpssim_amd.so.
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p _var/$name/obj
HIPCC=/opt/rocm/bin/hipcc
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Iinclude -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form=1 $flags"
$HIPCC $F -c ${SYNTH_SRC:-gps-sdr-sim_amd/csrc/hip/gss_synth.hip} -o _var/$name/obj/gss_synth.o
$HIPCC $F -c gps-sdr-sim_amd/csrc/hip/gss_run.hip -o _var/$name/obj/gss_run.o
$HIPCC $F -c gps-sdr-sim_amd/csrc/hip/gss_producers.hip -o _var/$name/obj/gss_producers.o
$HIPCC $F -c gps-sdr-sim_amd/csrc/hip/gss_proof.hip -o _var/$name/obj/gss_proof.o
HOSTOBJ=gps-sdr-sim_amd/obj/host/*.o
if [ -n "$HOSTFLAGS" ]; then          # the host proof must agree with the kernel (e.g. GSS_LIN_CH)
    mkdir -p _var/$name/obj/host
    for f in gps-sdr-sim_amd/csrc/host/*.c gps-sdr-sim_amd/csrc/cli/cli_args.c; do
        gcc -O2 -fPIC -ffp-contract=off -fno-fast-math -D_FILE_OFFSET_BITS=64 -Iinclude $HOSTFLAGS \
            -c $f -o _var/$name/obj/host/$(basename ${f%.c}).o
    done
    HOSTOBJ=_var/$name/obj/host/*.o
fi
$HIPCC -shared -fPIC --offload-arch=gfx950 -Wl,--version-script=gps-sdr-sim_amd/exports.map \
    -o _var/$name/libgpssim_amd.so $HOSTOBJ \
    _var/$name/obj/gss_synth.o _var/$name/obj/gss_run.o _var/$name/obj/gss_producers.o \
    _var/$name/obj/gss_proof.o -lm -lpthread
