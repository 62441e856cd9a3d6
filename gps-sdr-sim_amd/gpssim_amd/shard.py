"""Time-window sharding of one run across ranks, planned once per node.

Blocks are independent given their per-block parameters: the code state is recomputed every
block (gpssim.c:1331-1345), and the only state the sample loop carries across blocks is the
carrier phase (gpssim.c:2245-2250), one chain per channel slot, restarted where allocateChannel
re-initialises the slot (gpssim.c:1615-1626).  So every rank plans its own window in parallel:

  1. gss_scn_seek to its first block: only the 30 s updates before it are replayed (nav frames,
     ephemeris steps, allocation), never the per-block refresh of earlier blocks;
  2. gss_scn_next_deferred over its window: every row except the carrier phases, plus the slot
     chain each row continues;
  3. the 16 slot carriers at its first block arrive from rank r-1 (the baton: 128 bytes, point to
     point over torch.distributed); gss_carr_chain walks the carrier over its window, filling
     carr0 and the checkpoints, and the end state goes on to rank r+1.

Steps 1-2 cost the same on every rank; step 3 is the carrier-only walk, the one serial piece, and
each rank walks only its own window.  With a walker (plan_window(walker=...)) step 3 is the chain
run ahead (gss_run.hip chain_upfront_spec): per 4,096 blocks, the rows' starts from the exact
carriers at the chunk's first block (gss_carr_chain_starts), every row's segments walked from
guesses -- on the GPU (device_walker: gss_spec_device) or the host (host_walker: gss_spec_host)
-- and the exact chain from those walks (gss_carr_chain_spec), which takes one partial cycle per
row where a guess holds and the exact walk where it does not.  There is no data-path collective;
a whole-run file is rank slices at byte offset first_block * block_bytes.

Weak scaling (bench.py): every rank owns `window_s` seconds, i.e. blocks_per = window_s*10 - 1
blocks starting at r * blocks_per, of one run of world * window_s seconds.
"""
import time

import numpy as np

from . import (MAXCH, SPEC_DTYPE, SPEC_IN_DTYPE, Scenario, carr_chain, carr_chain_guess,
               carr_chain_spec, spec_host)

SPEC_CHUNK = 4096                # blocks per run-ahead chunk (gss_run.hip chain_upfront_spec)



def host_walker(threads=8):
    """speculative segment walks on the host (gss_spec_host)"""
    def walk(gi, n_per_blk):
        return spec_host(gi, n_per_blk, threads=threads)
    return walk


def device_walker(dev, torch):
    """speculative segment walks on the GPU (gss_spec_device): the rows sit in pinned host memory
    that the kernel's lanes read and write directly, as in gss_run"""
    bufs = {}

    def walk(gi, n_per_blk):
        flat = gi.reshape(-1)
        n = flat.size
        if bufs.get("n", 0) < n:
            bufs["in"] = torch.empty(n * SPEC_IN_DTYPE.itemsize, dtype=torch.uint8,
                                     pin_memory=True)
            bufs["out"] = torch.empty(n * SPEC_DTYPE.itemsize, dtype=torch.uint8,
                                      pin_memory=True)
            bufs["n"] = n
        h_in = bufs["in"].numpy()[:n * SPEC_IN_DTYPE.itemsize].view(SPEC_IN_DTYPE)
        h_in[:] = flat
        st = torch.cuda.current_stream()
        dev.spec_device(bufs["in"].data_ptr(), n, n_per_blk, bufs["out"].data_ptr(),
                        stream=st.cuda_stream)
        st.synchronize()
        flat[:] = h_in                   # the walkers' own segment guesses, written back
        return bufs["out"].numpy()[:n * SPEC_DTYPE.itemsize].view(SPEC_DTYPE).copy()
    return walk


def chain_run_ahead(carr, blk, nch, chain, n_per_blk, walker, threads=8, chunk=SPEC_CHUNK):
    """gss_carr_chain's result (blk["carr0"] filled in place, the carriers after the last block)
    from speculative walks: returns (end carriers, rows whose translation held)"""
    c = np.array(carr, np.float64, copy=True)
    hits = 0
    for b0 in range(0, len(nch), chunk):
        b1 = min(len(nch), b0 + chunk)
        gi = carr_chain_guess(c, blk[b0:b1], nch[b0:b1], chain[b0:b1], n_per_blk,
                              starts_only=True)
        spec = walker(gi, n_per_blk)
        c, h = carr_chain_spec(c, blk[b0:b1], nch[b0:b1], chain[b0:b1], n_per_blk, gi, spec,
                               threads=threads)
        hits += h
    return c, hits


def blocks_per_rank(window_s):
    """Blocks each rank synthesises for a window of window_s seconds (the run writes numd-1
    blocks, gpssim.c:2154, so a lone 300 s window is 2999 blocks)."""
    return int(round(window_s * 10)) - 1


def rank_range(rank, world, window_s):
    """[first, first + count) block range of `rank`."""
    n = blocks_per_rank(window_s)
    return rank * n, n


class Baton:
    """The slot carriers at a rank's first block, handed from rank r-1 to rank r (point to point
    over torch.distributed; `device` "cuda" for RCCL, "cpu" for gloo)."""

    def __init__(self, dist, rank, world, device="cpu"):
        import torch
        self.torch, self.dist, self.rank, self.world, self.device = torch, dist, rank, world, device

    def recv(self):
        t = self.torch.empty(MAXCH, dtype=self.torch.float64, device=self.device)
        self.dist.recv(t, src=self.rank - 1)
        return t.cpu().numpy()

    def send(self, carr):
        if self.rank + 1 < self.world:
            t = self.torch.from_numpy(np.ascontiguousarray(carr, np.float64)).to(self.device)
            self.dist.send(t, dst=self.rank + 1)


def plan_window(scn, first, count, baton=None, threads=8, batch=2000, with_ck=True, walker=None,
                chain_threads=None):
    """Rows of blocks [first, first + count) of Scenario scn (count < 0: to the end), planned
    without the blocks before `first` when a baton supplies the carriers there (rank > 0).
    Returns (blk, nch, ck or None, timings {seek_s, rows_s, wait_s, chain_s, spec_hits}).
    chain_threads (default: threads): the threads of the carrier chain's walk.  The ranks' rows
    are produced at the same time, each on its `threads`; their chains run one after another
    (each waits for the carriers of the rank before it), so on a box whose CPUs the ranks share
    the chain can take them all.
    Without a baton and first > 0 the prefix's carrier chain is planned here (a lone process).
    With a walker (host_walker / device_walker) the window's chain is run ahead
    (chain_run_ahead) and ck is None: the exact path walks the few uncertified blocks from their
    carr0 (DeviceWindow computes their checkpoints)."""
    t = {}
    t0 = time.perf_counter()
    carr = None
    if first > 0 and baton is None:          # no rank before us: walk the prefix ourselves
        done = scn.position()[0]
        while done < first:
            b, n = scn.next(min(batch, first - done), threads=threads)
            if len(n) == 0:
                break
            done += len(n)
        carr = scn.carrier()
    else:
        scn.seek(first, threads=threads)
    t["seek_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    parts = []
    done = 0
    while count < 0 or done < count:
        ask = batch if count < 0 else min(batch, count - done)
        b, n, c = scn.next_deferred(ask, threads=threads)
        if len(n) == 0:
            break
        parts.append((b, n, c))
        done += len(n)
    t["rows_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if carr is None:
        carr = baton.recv() if (baton is not None and baton.rank > 0) else scn.carrier()
    t["wait_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    if parts:
        blk = np.concatenate([p[0] for p in parts])
        nch = np.concatenate([p[1] for p in parts])
        chain = np.concatenate([p[2] for p in parts])
    else:
        from . import CHAIN_DTYPE, CHAN_DTYPE
        blk = np.zeros((0, MAXCH), CHAN_DTYPE)
        nch = np.zeros(0, np.int32)
        chain = np.zeros((0, MAXCH), CHAIN_DTYPE)
    ct = chain_threads or threads
    if walker is not None and len(nch):
        end, t["spec_hits"] = chain_run_ahead(carr, blk, nch, chain, scn.n_per_blk, walker,
                                              threads=ct)
        ck = None
    else:
        end, ck = carr_chain(carr, blk, nch, chain, scn.n_per_blk, carrier_int=scn.carrier_int,
                             with_ck=with_ck, threads=ct)
    t["chain_s"] = time.perf_counter() - t0
    if baton is not None:
        baton.send(end)
    return blk, nch, ck, t


def plan_rank(nav_file, rank, world, window_s, *, llh, samp_freq=2.6e6, data_format=16,
              threads=8, batch=2000, baton=None, walker=None, chain_threads=None):
    """Host plane for one rank: (blk[n, 16], nch[n], ck[n, 16, NCK] or None, nav rows,
    n_per_blk, timings) of its block range (ck: the carrier checkpoints).  With world > 1 pass a
    Baton: the rank then plans only its own window (module docstring)."""
    first, count = rank_range(rank, world, window_s)
    scn = Scenario(nav_file, llh=llh, duration=window_s * world if world > 1 else window_s,
                   samp_freq=samp_freq, data_format=data_format)
    blk, nch, ck, t = plan_window(scn, first, count, baton=baton, threads=threads, batch=batch,
                                  walker=walker, chain_threads=chain_threads)
    if len(nch) != count:
        raise RuntimeError(f"rank {rank}: planned {len(nch)} of {count} blocks")
    t["rows_out"] = int(scn.position()[1])
    return blk, nch, ck, scn.nav_table(), scn.n_per_blk, t
