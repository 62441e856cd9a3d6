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

import numpy as np

from . import MAXCH, NAV_WORDS, Device, Scenario, block_bytes


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


def chunk_source(torch, win, firsts, evs, dev_t, host_wire):
    """get_chunk(first, nb) for ordered_gather: the chunk's bytes in HBM once its render event
    has passed (the caller's stream waits for it, so a send or copy queued behind runs after it,
    while later chunks still render); firsts: the first block of each of win's batches, in batch
    order (one batch = one gather chunk); host_wire: a host copy (gloo)"""
    bb = win.bb
    at = {f: i for i, f in enumerate(firsts)}

    def get_chunk(first, nb):
        i = at[first]
        b0, b1 = win.batches[i][:2]
        assert b1 - b0 == nb, "a gather chunk is one render batch"
        torch.cuda.current_stream(dev_t).wait_event(evs[i])
        t = win.out[b0 * bb:b1 * bb]
        return t.cpu() if host_wire else t
    return get_chunk


def chunk_plan(n_blocks, world, chunk_blocks, layout="block"):
    """The run's chunks in run order: [(render rank, first block, blocks)].  Chunks never cross
    a planning window (rank_blocks: rank r plans [B r/N, B (r+1)/N)).  layout "block": each rank
    renders the chunks of its own window, so rank 0 takes rank 1's whole window, then rank 2's,
    ... -- one peer, one xGMI link, at a time.  "stripe": chunk i of the run is rendered by rank
    i mod N (its rows handed over by exchange_rows), so any N consecutive chunks come from N
    different ranks and rank 0 receives over every link at once."""
    plan = []
    for r in range(world):
        b0, b1 = rank_blocks(n_blocks, r, world)
        for c in range(b0, b1, chunk_blocks):
            plan.append((r, c, min(chunk_blocks, b1 - c)))
    if layout == "stripe":
        plan = [(i % world, c, nb) for i, (_, c, nb) in enumerate(plan)]
    elif layout != "block":
        raise ValueError(f"unknown layout {layout!r}")
    return plan


def planner_of(first, n_blocks, world):
    """the rank whose planning window holds block `first`"""
    r = first * world // n_blocks
    while rank_blocks(n_blocks, r, world)[0] > first:
        r -= 1
    while rank_blocks(n_blocks, r, world)[1] <= first:
        r += 1
    return r


def _run_p2p(dist, ops):
    """post a list of dist.P2POp as one group (dist.batch_isend_irecv) and wait for all of them;
    a rank with nothing to exchange posts nothing (allowed: the group already has collectives
    behind it, the planners' baton and all_gathers)"""
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def exchange_rows(plan, n_blocks, rank, world, dist, blk, nch, nav, device="cpu"):
    """Hand each chunk's rows from the rank that planned it (its window: blk[n, 16], nch[n], its
    nav table) to the rank that renders it (plan from chunk_plan(layout="stripe")).  Returns this
    rank's render input: (blk, nch, nav, firsts) over the chunks it renders, in run order, with
    every row's nav_tbl moved into the returned table (the planners' tables concatenated in rank
    order); firsts: each chunk's first block.  Point to point only: per pair of ranks one message
    of the nav-table size, then one of the table and the rows (torch.distributed; `device`
    "cuda" for RCCL).  The carriers are already exact in the rows (plan_window's chain), so a
    chunk renders the same bytes on any rank."""
    import torch
    from . import CHAN_DTYPE
    my0, _ = rank_blocks(n_blocks, rank, world)
    row_b = CHAN_DTYPE.itemsize * MAXCH
    nav = np.ascontiguousarray(nav, np.uint32)
    # chunks by (planner, renderer), in run order
    pairs = {}
    for r, c, nb in plan:
        pairs.setdefault((planner_of(c, n_blocks, world), r), []).append((c, nb))

    def payload(q):
        parts = [nav.view(np.uint8).reshape(-1)]
        for c, nb in pairs.get((rank, q), []):
            parts.append(np.ascontiguousarray(blk[c - my0:c - my0 + nb]).view(np.uint8).reshape(-1))
            parts.append(np.ascontiguousarray(nch[c - my0:c - my0 + nb], np.int32)
                         .view(np.uint8).reshape(-1))
        return np.concatenate(parts)

    # With the stripe layout most pairs of ranks exchange in BOTH directions.  Each phase is one
    # dist.batch_isend_irecv: under NCCL/RCCL the group's sends and receives are posted together
    # (one ncclGroupStart/End), so two ranks' large sends to each other cannot each wait on a
    # receive queued behind the other (the ungrouped two-way send/recv deadlock); gloo posts them
    # one by one, which is already safe.
    sends = [q for q in range(world) if q != rank and (rank, q) in pairs]
    recvs = [p for p in range(world) if p != rank and (p, rank) in pairs]
    # phase 1: nav-table sizes to every renderer this rank plans for (and from every planner)
    sizes, keep = {}, []
    ops = []
    for q in sends:
        t = torch.tensor([len(nav)], dtype=torch.int64, device=device)
        keep.append(t)
        ops.append(dist.P2POp(dist.isend, t, q))
    for p in recvs:
        sizes[p] = torch.empty(1, dtype=torch.int64, device=device)
        ops.append(dist.P2POp(dist.irecv, sizes[p], p))
    _run_p2p(dist, ops)
    # phase 2: the tables and rows
    ops, bufs = [], {}
    for q in sends:
        t = torch.from_numpy(payload(q)).to(device)
        keep.append(t)
        ops.append(dist.P2POp(dist.isend, t, q))
    for p in recvs:
        n_nav = int(sizes[p].item())
        nbytes = n_nav * NAV_WORDS * 4 + sum(nb for c, nb in pairs[(p, rank)]) * (row_b + 4)
        bufs[p] = torch.empty(nbytes, dtype=torch.uint8, device=device)
        ops.append(dist.P2POp(dist.irecv, bufs[p], p))
    _run_p2p(dist, ops)
    # assemble: the planners' nav tables in rank order, rows re-pointed into them
    tables, rows = {}, {}
    for p in range(world):
        if p == rank:
            if (rank, rank) in pairs:
                tables[p] = nav
                for c, nb in pairs[(rank, rank)]:
                    rows[c] = (blk[c - my0:c - my0 + nb], np.asarray(nch[c - my0:c - my0 + nb],
                                                                     np.int32), p)
            continue
        if p not in bufs:
            continue
        raw = bufs[p].cpu().numpy()
        n_nav = int(sizes[p].item())
        o = n_nav * NAV_WORDS * 4
        tables[p] = raw[:o].view(np.uint32).reshape(n_nav, NAV_WORDS)
        for c, nb in pairs[(p, rank)]:
            b = raw[o:o + nb * row_b].view(CHAN_DTYPE).reshape(nb, MAXCH)
            o += nb * row_b
            n = raw[o:o + nb * 4].view(np.int32)
            o += nb * 4
            rows[c] = (b, n, p)
    base, off = {}, 0
    for p in sorted(tables):
        base[p] = off
        off += len(tables[p])
    mine = [(c, nb) for r, c, nb in plan if r == rank]
    out_blk = np.zeros((sum(nb for _, nb in mine), MAXCH), CHAN_DTYPE)
    out_nch = np.zeros(len(out_blk), np.int32)
    o = 0
    for c, nb in mine:
        b, n, p = rows[c]
        out_blk[o:o + nb] = b
        out_blk[o:o + nb]["nav_tbl"] += base[p]
        out_nch[o:o + nb] = n
        o += nb
    out_nav = (np.concatenate([tables[p] for p in sorted(tables)]) if tables
               else np.zeros((1, NAV_WORDS), np.uint32))
    return out_blk, out_nch, out_nav, [c for c, _ in mine]


def ordered_gather(plan, rank, dist, get_chunk, make_buf, sink, depth=2, stats=None):
    """Rank 0 hands every chunk of `plan` ([(render rank, first, blocks)], run order) to
    sink(tensor) in plan order: its own from get_chunk(first, blocks), every other rank's
    received from it.  Every other rank sends its own chunks in order (dist.send).  Rank 0 keeps
    up to `depth` receives in flight from EVERY peer at once, each into one of that peer's
    `depth` buffers (make_buf(blocks), sliced for a short chunk), re-posted as soon as the sink
    has taken the chunk it held; so with a layout whose consecutive chunks come from different
    ranks (chunk_plan "stripe") the peers' links all carry data together.  Point to point only:
    with RCCL each chunk crosses xGMI once, GPU to GPU.  stats (a dict, rank 0): the most
    receives and the most distinct peers that were outstanding at once."""
    if rank != 0:
        for r, b0, nb in plan:
            if r == rank:
                dist.send(get_chunk(b0, nb), dst=0)
        return
    from collections import deque
    queues, cap = {}, {}
    for i, (r, b0, nb) in enumerate(plan):
        if r != 0:
            queues.setdefault(r, deque()).append(i)
            cap[r] = max(cap.get(r, 0), nb)
    free = {r: deque(make_buf(cap[r]) for _ in range(min(depth, len(q))))
            for r, q in queues.items()}
    inflight = {}                         # plan index -> (work, buffer, its view)
    out = {r: 0 for r in queues}
    most, most_peers = 0, 0

    def fill(r):
        nonlocal most, most_peers
        q = queues[r]
        while q and free[r]:
            i = q.popleft()
            buf = free[r].popleft()
            view = buf[:plan[i][2] * (buf.numel() // cap[r])]
            inflight[i] = (dist.irecv(view, src=r), buf, view)
            out[r] += 1
        most = max(most, len(inflight))
        most_peers = max(most_peers, sum(1 for v in out.values() if v))

    for r in queues:
        fill(r)
    for i, (r, b0, nb) in enumerate(plan):
        if r == 0:
            sink(get_chunk(b0, nb))
            continue
        work, buf, view = inflight.pop(i)
        work.wait()
        sink(view)
        out[r] -= 1
        free[r].append(buf)
        fill(r)
    if stats is not None:
        stats.update(max_outstanding=most, max_peers_outstanding=most_peers, depth=depth)


class FileSink:
    """Writes device (or host) uint8 tensors to a file descriptor in call order, overlapped: the
    reference writes each block as it is made (gpssim.c:2276-2287); here chunk i+1's download
    runs while chunk i is written.

    `nbuf` pinned staging buffers of `cap` bytes rotate between the caller and one writer thread.
    A call takes a free buffer (waiting only while all of them are still being written), queues
    the device-to-host copy on a copy stream of its own behind the caller's stream (the chunk's
    render or receive), records an event and hands (buffer, length, event) to the writer, which
    waits for that event and os.write()s the bytes in call order.  The caller's stream then waits
    for the copy's event, so whatever the caller queues next into the same device memory (the
    next receive into a reused buffer) runs after the copy has read it -- no host wait.  A host
    tensor is copied into the staging buffer at once (the caller may reuse it on return).
    close() drains the queue; a write error is raised there (or by the next call)."""

    def __init__(self, torch, fd, cap, nbuf=3):
        import queue
        import threading
        self.torch, self.fd, self.cap = torch, fd, cap
        pin = torch.cuda.is_available()
        self.host = [torch.empty(cap, dtype=torch.uint8, pin_memory=pin) for _ in range(nbuf)]
        self.free = queue.Queue()
        for i in range(nbuf):
            self.free.put(i)
        self.todo = queue.Queue()
        self.streams = {}                         # device -> copy stream
        self.bytes = 0
        self.err = None
        self.writer = threading.Thread(target=self._write_loop, name="gss-file-sink", daemon=True)
        self.writer.start()

    def _write_loop(self):
        while True:
            item = self.todo.get()
            if item is None:
                return
            i, n, ev = item
            try:
                if self.err is None:
                    if ev is not None:
                        ev.synchronize()
                    mv = memoryview(self.host[i][:n].numpy())
                    while len(mv):
                        w = os.write(self.fd, mv)
                        mv = mv[w:]
            except BaseException as e:             # reported by the next call or close()
                self.err = e
            finally:
                self.free.put(i)

    def _check(self):
        if self.err is not None:
            raise self.err

    def __call__(self, t):
        self._check()
        n = t.numel()
        assert n <= self.cap, "chunk larger than the staging buffers"
        i = self.free.get()
        ev = None
        if t.is_cuda:
            torch = self.torch
            cur = torch.cuda.current_stream(t.device)
            cs = self.streams.get(t.device)
            if cs is None:
                cs = self.streams[t.device] = torch.cuda.Stream(t.device)
            cs.wait_stream(cur)                    # the chunk's producer first
            with torch.cuda.stream(cs):
                self.host[i][:n].copy_(t.reshape(-1), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
            t.record_stream(cs)
            cur.wait_event(ev)                     # the caller's next use of t after the copy
        else:
            self.host[i][:n].copy_(t.reshape(-1))
        self.todo.put((i, n, ev))
        self.bytes += n

    def close(self):
        """wait until every queued chunk is written; raises the writer's error if any"""
        if self.writer.is_alive():
            self.todo.put(None)
            self.writer.join()
        self._check()


def run_node(argv, rank, world, local, backend="nccl", chunk_blocks=None, threads=16,
             layout="stripe", stats=None):
    """The whole-node run of one gps-sdr-sim command line; returns rank 0's byte count.  layout:
    chunk_plan's ("stripe": planned by window, rendered round-robin by chunk, gathered over every
    link at once; "block": every rank renders its own window)."""
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
    wire = dev_t if backend == "nccl" else "cpu"
    baton = Baton(dist, rank, world, device=wire)
    blk, nch, ck, _ = plan_window(scn, b0, b1 - b0, baton=baton, threads=threads,
                                  walker=device_walker(dev, torch))
    plan = chunk_plan(n_blocks, world, chunk_blocks, layout)
    nav = scn.nav_table()
    if layout == "stripe":
        blk, nch, nav, firsts = exchange_rows(plan, n_blocks, rank, world, dist, blk, nch, nav,
                                              device=wire)
        ck = None
    else:
        firsts = [c for r, c, nb in plan if r == rank]
    sizes = [nb for r, c, nb in plan if r == rank]
    win = DeviceWindow(torch, dev, dev_t, blk, nch, nav, npb, fmt, ck=ck, threads=threads,
                       sizes=sizes or None)
    wire_gpu = backend == "nccl"
    _, evs = render_chunks(torch, win, dev_t)
    get_chunk = chunk_source(torch, win, firsts, evs, dev_t,
                             host_wire=not (wire_gpu or rank == 0))

    def make_buf(nb):
        return torch.empty(nb * bb, dtype=torch.uint8, device=dev_t if wire_gpu else "cpu")

    total = 0
    if rank == 0:
        fd = 1 if out_file == "-" else os.open(out_file, os.O_WRONLY | os.O_CREAT | os.O_TRUNC,
                                               0o644)
        sink = FileSink(torch, fd, chunk_blocks * bb)
        try:
            ordered_gather(plan, rank, dist, get_chunk, make_buf, sink, stats=stats)
        finally:
            sink.close()
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
    n = run_node(argv, rank, world, local, backend=backend,
                 layout=os.environ.get("GSS_GATHER_LAYOUT", "stripe"))
    if rank == 0:
        dt = time.perf_counter() - t0
        print(f"\nDone! {n} bytes from {world} ranks in {dt:.1f} s", file=sys.stderr)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
