"""The fast kernel's hidden window registers, checked in the shipped code object (CPU only).

gss_lin_kernel<FMT> (gss_synth.hip) loads each channel's chunk windows with s_load_dwordx16 into
s[68:83] and s[84:99] from inline asm, registers the compiler never allocates because the kernel
is limited to LIN_SW_SGPRS = 68 SGPRs (amdgpu_num_sgpr).  Nothing but the asm statements may touch
them between the load and the copy out (LIN_SW_TAKE).  A toolchain or flag change that let the
allocator, a spill or the ABI use them would corrupt the output silently, and only the GPU parity
tests would notice.  So this test disassembles the library the tests load and checks, for every
instantiation of the kernel:

* the only instructions that write s68..s99 are those two s_load_dwordx16;
* the only instructions that read them are the s_mov_b64 copies of LIN_SW_TAKE;
* the kernel descriptor's SGPR count covers s99;
* the compiler's own SGPRs stay below s68 (every other SGPR operand is < 68, VCC and the
  special registers aside).
"""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "gps-sdr-sim_amd", "lib", "libgpssim_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")


def _sgprs(operand):
    out = set()
    for m in SREG.finditer(operand):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


@pytest.fixture(scope="module")
def lin_kernels(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (run __graft_entry__.build())")
    for tool in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump", "llvm-readelf"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not in {LLVM}")
    d = tmp_path_factory.mktemp("isa")
    fat, elf, junk = d / "fat.bin", d / "gfx950.elf", d / "lib.copy"
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}",
                           LIB, str(junk)])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                           f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                           f"--output={elf}"])
    dis = subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                   str(elf)], text=True)
    notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", str(elf)],
                                    text=True)
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur and line.strip() and not line.strip().startswith(";"):
            funcs[cur].append(line.split("//")[0].strip())
    sgpr_count = {}
    name = None
    for line in notes.splitlines():
        m = re.match(r"\s*\.name:\s+(\S+)", line)
        if m:
            name = m.group(1)
        m = re.match(r"\s*\.sgpr_count:\s+(\d+)", line)
        if m and name:
            sgpr_count[name] = int(m.group(1))
    lin = {k: v for k, v in funcs.items() if "gss_lin_kernel" in k}
    return lin, sgpr_count


def test_lin_kernels_present(lin_kernels):
    lin, _ = lin_kernels
    assert len(lin) == 3, sorted(lin)            # -b 16, -b 8, -b 1


def test_hidden_window_registers(lin_kernels):
    lin, sgpr_count = lin_kernels
    hidden = set(range(68, 100))
    for name, insts in lin.items():
        loads, copies = 0, 0
        for ins in insts:
            parts = ins.split(None, 1)
            op = parts[0]
            ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
            regs = [_sgprs(o) for o in ops]
            touched = set().union(*regs) if regs else set()
            if not touched & hidden:
                continue
            if op == "s_load_dwordx16" and regs[0] in (set(range(68, 84)), set(range(84, 100))):
                assert not (set().union(*regs[1:]) & hidden), ins
                loads += 1
                continue
            # LIN_SW_TAKE: s_mov_b64 <compiler SGPR pair>, <hidden pair>
            assert op == "s_mov_b64", f"{name}: {ins}"
            assert regs[1] <= hidden and not regs[0] & hidden, f"{name}: {ins}"
            copies += 1
        assert loads >= 2 and copies >= 16, (name, loads, copies)
        assert sgpr_count.get(name, 0) >= 100, (name, sgpr_count.get(name))


def test_compiler_sgprs_below_hidden_buffers(lin_kernels):
    lin, _ = lin_kernels
    for name, insts in lin.items():
        for ins in insts:
            parts = ins.split(None, 1)
            if len(parts) < 2 or parts[0] in ("s_load_dwordx16", "s_mov_b64"):
                continue
            for o in parts[1].split(","):
                assert not (_sgprs(o) & set(range(68, 106))), f"{name}: {ins}"
