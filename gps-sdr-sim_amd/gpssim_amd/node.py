"""Whole-node runs with one byte sink: `python -m gpssim_amd.node <gps-sdr-sim
options>` under torchrun, one process per GPU.

Every rank renders its contiguous block range of the run on its own GPU into HBM (the time-window
shard: [B r/N, B (r+1)/N), the partition the C CLI's pwrite path uses, gps_sdr_sim.c).  Each rank
plans only its own window (gpssim_amd.shard.plan_window: seek, deferred rows, the slot carriers
handed on from the rank before, the chain run ahead on its GPU).  Rank 0
then writes the whole run to the reference's sink -- a file, or stdout with `-o -`
(gpssim.c:2101-2111, 2276-2287) -- in run order: its own chunks straight from HBM, every other
rank's chunks received point to point over RCCL (xGMI) into two alternating receive buffers, the
next chunk in flight while the current one is copied to pinned host memory and written.  Chunks
are `GSS_CHUNK_BLOCKS` blocks (default: about 256 MB, 256 blocks at -b 16, 2.6 MS/s), so rank 0
holds two of them beside its own slice.  Rendering and sending overlap: a rank launches all its
chunks on a render stream of their own, and each chunk is sent (or written) as soon as its own
render event has passed, while the later chunks still render.  The gather is the only
collective; it moves each byte once.

With WORLD_SIZE == 1 it is the single-process run (gss_run, overlapped planner/GPU/sink).
Backend: nccl (RCCL) for GPU tensors; gloo moves the chunks through host memory (tests).
"""
import os
import sys
import time

from . import Device, Scenario, block_bytes


def rank_blocks(n_blocks, rank, world):
    """[first, last) blocks of `rank` (same partition as the C CLI, gps_sdr_sim.c run_rank)."""
    return n_blocks * rank // world, n_blocks * (rank + 1) // world


def default_chunk_blocks(bb):
    """blocks per gather chunk: GSS_CHUNK_BLOCKS, else about 256 MB of output"""
    env = os.environ.get("GSS_CHUNK_BLOCKS")
    return int(env) if env else max(1, (256 << 20) // bb)


def render_chunks(torch, win, dev_t):
    """Launch every batch (= gather chunk) of DeviceWindow win on a render stream of its own, in
    order; returns (stream, per-batch completion events)."""
    st = torch.cuda.Stream(dev_t)
    evs = []
    for i in range(len(win.batches)):
        win.step_batch(i, st.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(st)
        evs.append(ev)
    return st, evs


def chunk_source(torch, win, first_block, chunk_blocks, evs, dev_t, host_wire):
    """get_chunk(first, nb) for ordered_gather: the chunk's bytes in HBM once its render event
    has passed (the caller's stream waits for it, so a send or copy queued behind runs after it,
    while later chunks still render); host_wire: a host copy (gloo)"""
    bb = win.bb

    def get_chunk(first, nb):
        i = (first - first_block) // chunk_blocks
        torch.cuda.current_stream(dev_t).wait_event(evs[i])
        t = win.out[(first - first_block) * bb:(first - first_block + nb) * bb]
        return t.cpu() if host_wire else t
    return get_chunk


def chunk_plan(n_blocks, world, chunk_blocks):
    """The run's chunks in run order: [(owner rank, first block, blocks)]."""
    plan = []
    for r in range(world):
        b0, b1 = rank_blocks(n_blocks, r, world)
        for c in range(b0, b1, chunk_blocks):
            plan.append((r, c, min(chunk_blocks, b1 - c)))
    return plan


def ordered_gather(plan, rank, dist, get_chunk, make_buf, sink):
    """Rank 0 hands every chunk of `plan` to sink(tensor) in plan order: its own from
    get_chunk(first, blocks), the others received from their owner (dist.irecv into one of two
    buffers from make_buf(blocks), the next receive posted before the current chunk is written).
    Every other rank sends its own chunks, in order (dist.send).  Point-to-point only: with
    RCCL each chunk crosses xGMI once, GPU to GPU."""
    if rank != 0:
        for r, b0, nb in plan:
            if r == rank:
                dist.send(get_chunk(b0, nb), dst=0)
        return
    bufs = {}

    def post(i):
        r, b0, nb = plan[i]
        if r == 0:
            return None, None
        key = i % 2
        buf = bufs.get((key, nb))
        if buf is None:
            buf = make_buf(nb)
            bufs[(key, nb)] = buf
        return dist.irecv(buf, src=r), buf

    nxt = post(0) if plan else None
    for i, (r, b0, nb) in enumerate(plan):
        work, buf = nxt
        nxt = post(i + 1) if i + 1 < len(plan) else None
        if r == 0:
            sink(get_chunk(b0, nb))
        else:
            work.wait()
            sink(buf)


class FileSink:
    """Writes device (or host) uint8 tensors to a file descriptor in call order, through a
    pinned host staging buffer."""

    def __init__(self, torch, fd, cap):
        self.torch, self.fd = torch, fd
        self.host = torch.empty(cap, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        self.bytes = 0

    def __call__(self, t):
        n = t.numel()
        if t.is_cuda:
            self.host[:n].copy_(t, non_blocking=True)
            self.torch.cuda.current_stream(t.device).synchronize()
            mv = memoryview(self.host[:n].numpy())
        else:
            mv = memoryview(t.numpy())
        while len(mv):
            w = os.write(self.fd, mv)
            mv = mv[w:]
        self.bytes += n


def run_node(argv, rank, world, local, backend="nccl", chunk_blocks=None, threads=16):
    """The whole-node run of one gps-sdr-sim command line; returns rank 0's byte count."""
    import torch
    import torch.distributed as dist
    from .render import DeviceWindow
    from .shard import Baton, device_walker, plan_window

    scn, out_file = Scenario.from_cli(argv)
    n_blocks, npb, fmt = scn.n_blocks, scn.n_per_blk, scn.data_format
    bb = block_bytes(npb, fmt)
    chunk_blocks = chunk_blocks or default_chunk_blocks(bb)
    torch.cuda.set_device(local)
    dev_t = torch.device("cuda", local)
    dev = Device(local)
    b0, b1 = rank_blocks(n_blocks, rank, world)
    baton = Baton(dist, rank, world, device=dev_t if backend == "nccl" else "cpu")
    blk, nch, ck, _ = plan_window(scn, b0, b1 - b0, baton=baton, threads=threads,
                                  walker=device_walker(dev, torch))
    win = DeviceWindow(torch, dev, dev_t, blk, nch, scn.nav_table(), npb, fmt, ck=ck,
                       threads=threads, batch=chunk_blocks)
    wire_gpu = backend == "nccl"
    _, evs = render_chunks(torch, win, dev_t)
    get_chunk = chunk_source(torch, win, b0, chunk_blocks, evs, dev_t,
                             host_wire=not (wire_gpu or rank == 0))

    def make_buf(nb):
        return torch.empty(nb * bb, dtype=torch.uint8, device=dev_t if wire_gpu else "cpu")

    plan = chunk_plan(n_blocks, world, chunk_blocks)
    total = 0
    if rank == 0:
        fd = 1 if out_file == "-" else os.open(out_file, os.O_WRONLY | os.O_CREAT | os.O_TRUNC,
                                               0o644)
        sink = FileSink(torch, fd, chunk_blocks * bb)
        ordered_gather(plan, rank, dist, get_chunk, make_buf, sink)
        total = sink.bytes
        if fd != 1:
            os.close(fd)
    else:
        ordered_gather(plan, rank, dist, get_chunk, make_buf, None)
    torch.cuda.synchronize(dev_t)
    dist.barrier()
    win.free()
    dev.close()
    return total


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:                       # the single-process run: gss_run to the sink
        import subprocess
        from . import CLI_PATH
        return subprocess.call([CLI_PATH] + list(argv))
    import torch.distributed as dist
    backend = os.environ.get("GSS_BACKEND", "nccl")
    dist.init_process_group(backend)
    t0 = time.perf_counter()
    n = run_node(argv, rank, world, local, backend=backend)
    if rank == 0:
        dt = time.perf_counter() - t0
        print(f"\nDone! {n} bytes from {world} ranks in {dt:.1f} s", file=sys.stderr)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
