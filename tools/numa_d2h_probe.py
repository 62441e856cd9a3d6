"""Device -> pinned host copy rate by the NUMA node of the pinned buffer (GPU box only).

For gss_run's D2H (bench.py e2e): where is the GPU (its PCI device's numa_node), which nodes
exist, and how fast do 133 MB copies (one gss_run slot at batch 128) land in pinned buffers bound
to each node (set_mempolicy MPOL_BIND around hipHostMalloc, pages checked with move_pages), one
buffer and three in rotation, with and without a busy compute stream beside the copies."""
import ctypes
import glob
import os
import time

import torch

libc = ctypes.CDLL(None, use_errno=True)
hip = ctypes.CDLL("libamdhip64.so")
SYS_set_mempolicy, SYS_move_pages = 238, 279          # x86-64
MPOL_DEFAULT, MPOL_BIND = 0, 2


def gpu_node():
    p = torch.cuda.get_device_properties(0)
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", 0)
    dev = getattr(p, "pci_device_id", 0)
    cands = glob.glob(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{dev:02x}.*/numa_node") \
        if bus is not None else []
    return (int(open(cands[0]).read()) if cands else None), (dom, bus, dev)


def set_policy(node):
    if node is None:
        return libc.syscall(SYS_set_mempolicy, MPOL_DEFAULT, None, 0)
    mask = (ctypes.c_ulong * 16)()
    mask[node // 64] = 1 << (node % 64)
    return libc.syscall(SYS_set_mempolicy, MPOL_BIND, mask, 1024)


def page_node(addr):
    pages = (ctypes.c_void_p * 1)(addr)
    status = (ctypes.c_int * 1)(-1)
    libc.syscall(SYS_move_pages, 0, 1, pages, None, status, 0)
    return status[0]


def pinned(nbytes, node):
    set_policy(node)
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0)
    set_policy(None)
    assert rc == 0, rc
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    return torch.frombuffer(buf, dtype=torch.uint8), p


def rate(dsts, src, reps=12, busy=False):
    cs = torch.cuda.Stream()
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16) if busy else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if busy:
        with torch.cuda.stream(cs):
            for _ in range(40):
                a = a @ a
                a = a / a.abs().max()
    for i in range(reps):
        dsts[i % len(dsts)].copy_(src, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    el = time.perf_counter() - t0
    torch.cuda.synchronize()
    return src.numel() * reps / el / 1e9


def main():
    node, pci = gpu_node()
    nodes = sorted(int(os.path.basename(d)[4:]) for d in glob.glob("/sys/devices/system/node/node*"))
    print(f"GPU pci {pci} numa_node {node}; nodes {nodes}; this thread on cpu "
          f"{libc.sched_getcpu()}; affinity {len(os.sched_getaffinity(0))} cpus")
    for n in nodes:
        cl = open(f"/sys/devices/system/node/node{n}/cpulist").read().strip()
        print(f"  node {n}: cpus {cl}")
    nbytes = 133 << 20
    src = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for n in [None] + nodes:
        bufs = [pinned(nbytes, n) for _ in range(3)]
        where = page_node(bufs[0][1].value)
        r1 = rate([bufs[0][0]], src)
        r3 = rate([b[0] for b in bufs], src)
        rb = rate([b[0] for b in bufs], src, busy=True)
        print(f"bind {'default' if n is None else n:>7}: pages on node {where}: x1 {r1:5.1f} GB/s"
              f"  x3 {r3:5.1f}  x3 beside a busy stream {rb:5.1f}", flush=True)
        for _, p in bufs:
            hip.hipHostFree(p)


if __name__ == "__main__":
    main()
