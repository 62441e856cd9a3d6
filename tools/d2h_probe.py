"""Device -> pinned host copy rates for gss_run's slot pattern (GPU box only): one pinned buffer
copied into repeatedly (bench.py's d2h_ceiling) against NSLOT buffers in rotation, and pinned
buffers from hipHostMalloc (as gss_run allocates them) against torch's pinned allocator."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")


def rate(dsts, src, nbytes, reps=12):
    for d in dsts:
        d.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        dsts[i % len(dsts)].copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def hip_pinned(nbytes):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0) == 0
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    return torch.frombuffer(buf, dtype=torch.uint8), p


for mb in (66, 133, 266):
    n = mb << 20
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    one = [torch.empty(n, dtype=torch.uint8, pin_memory=True)]
    three = one + [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    hb = [hip_pinned(n) for _ in range(3)]
    print(f"{mb:4d} MB  torch pinned x1 {rate(one, src, n):6.1f} GB/s  x3 {rate(three, src, n):6.1f}"
          f"  hipHostMalloc x1 {rate([hb[0][0]], src, n):6.1f}  x3 {rate([h[0] for h in hb], src, n):6.1f}",
          flush=True)
    for _, p in hb:
        hip.hipHostFree(p)
    del src, one, three
