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

from . import (ANCHOR_DTYPE, MAXCH, SPEC_DTYPE, SPEC_IN_DTYPE, Scenario, carr_anchors,
               carr_chain, carr_chain_anchored, carr_chain_guess, carr_chain_linked,
               carr_chain_spec, carr_line_end, spec_host, spec_links)

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


def chain_run_ahead(carr, blk, nch, chain, n_per_blk, walker, threads=8, chunk=SPEC_CHUNK,
                    anch=None, heads=None):
    """gss_carr_chain's result (blk["carr0"] filled in place, the carriers after the last block)
    from speculative walks: returns (end carriers, rows whose translation held).  anch
    (ANCHOR_DTYPE [nb, 16], optional): filled with the chain's anchors (the proofs' walk starts).
    heads (SPEC_IN_DTYPE [nb, 16], optional): filled with the rows' walk inputs as the walkers
    got them (start guesses, steps, previous rows; segment starts left to the walkers), e.g. to
    replay the window's walks on the device (bench.py device_window)."""
    c = np.array(carr, np.float64, copy=True)
    hits = 0
    for b0 in range(0, len(nch), chunk):
        b1 = min(len(nch), b0 + chunk)
        gi = carr_chain_guess(c, blk[b0:b1], nch[b0:b1], chain[b0:b1], n_per_blk,
                              starts_only=True)
        if heads is not None:
            heads[b0:b1] = gi
        spec = walker(gi, n_per_blk).reshape(gi.shape)
        if anch is None:
            c, h = carr_chain_spec(c, blk[b0:b1], nch[b0:b1], chain[b0:b1], n_per_blk, gi, spec,
                                   threads=threads)
        else:
            sub = blk[b0:b1]                 # a contiguous view: filled in place
            c, h, a = carr_chain_anchored(c, sub, nch[b0:b1], chain[b0:b1], n_per_blk, gi, spec,
                                          threads=threads)
            anch[b0:b1] = a
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
        self._pending = None

    def recv(self):
        t = self.torch.empty(MAXCH, dtype=self.torch.float64, device=self.device)
        self.dist.recv(t, src=self.rank - 1)
        return t.cpu().numpy()

    def send(self, carr):
        if self.rank + 1 < self.world:
            t = self.torch.from_numpy(np.ascontiguousarray(carr, np.float64)).to(self.device)
            self.dist.send(t, dst=self.rank + 1)

    def isend(self, carr):
        """send without waiting for rank r+1 to take it (it may still be in a collective);
        finish() completes it"""
        if self.rank + 1 < self.world:
            t = self.torch.from_numpy(np.ascontiguousarray(carr, np.float64)).to(self.device)
            self._pending = (t, self.dist.isend(t, dst=self.rank + 1))

    def finish(self):
        if self._pending is not None:
            self._pending[1].wait()
            self._pending = None

    def all_gather(self, vec):
        """every rank's float64 vector (same length on all ranks), in rank order"""
        t = self.torch.from_numpy(np.ascontiguousarray(vec, np.float64)).to(self.device)
        parts = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [p.cpu().numpy() for p in parts]


# ---- the chain speculated across ranks -----------------------------------------------------------
# A rank's window acts on the 16 slot carriers as x -> x + a (mod 1) per slot, or as a constant
# where allocateChannel re-initialises the slot inside the window (gpssim.c:1615-1626).  Every rank
# publishes that map (all_gather, 48 doubles) and composes the maps of the ranks before it into a
# prediction of its start, so its guesses and walks run before the baton arrives:
#   1. the lines' map (gss_carr_line_end): a start off by ~1e-13 cycle per block before it;
#   2. walks from that start, the chain from them (gss_carr_chain_spec, exact for that start) and
#      its map: exact but for the rounding differences where the start's error crossed a margin,
#      so the second prediction is off by ~1e-13 cycle in all;
#   3. the rows walked again from the first chain's carriers moved by the correction (rows after
#      a re-initialisation keep their walks: they do not depend on the start);
#   4. every row's walk folded with its predecessor's into a link record (gss_spec_links);
#   5. the baton: the exact start, and gss_carr_chain_linked from it -- a compare and two adds per
#      row where the translation holds (almost every row) and the exact walk where it does not --
#      whose end goes on to rank r+1 at once.  Exact in every case; only the time depends on the
#      guesses.
SPEC_WALK_ROWS = 1 << 18         # rows per walker call (bounds the pinned buffers)


def _live(nch):
    return np.arange(MAXCH)[None, :] < np.asarray(nch)[:, None]


def slot_resets(nch, chain):
    """[16] bool: slots the window re-initialises (their carrier after it is a constant)"""
    live = _live(nch)
    sl = chain["slot"][live].astype(np.int64)
    ok = (chain["reset"][live] != 0) & (sl >= 0) & (sl < MAXCH)
    out = np.zeros(MAXCH, bool)
    out[sl[ok]] = True
    return out


def _start_dependent(nch, chain):
    """[nb, 16] bool: live rows whose carrier depends on the window's start (no re-initialisation
    of their slot at or before their block)"""
    live = _live(nch)
    nb = len(nch)
    sl = np.where(live, chain["slot"], -1).astype(np.int64)
    rs = live & (chain["reset"] != 0) & (sl >= 0)
    bi = np.broadcast_to(np.arange(nb, dtype=np.int64)[:, None], sl.shape)
    first = np.full(MAXCH, nb, np.int64)
    np.minimum.at(first, sl[rs], bi[rs])
    return live & (sl >= 0) & (bi < first[np.clip(sl, 0, MAXCH - 1)])


def map_vec(start, end, resets):
    """this rank's published map: [start (rank 0's is the run's), add, reset flags]"""
    add = np.where(resets, end, np.mod(end - start, 1.0))
    return np.concatenate([np.asarray(start, np.float64), add, resets.astype(np.float64)])


def compose_start(maps, rank):
    """the predicted slot carriers at rank `rank`'s first block from the ranks' maps"""
    x = np.array(maps[0][:MAXCH], np.float64)
    for m in maps[:rank]:
        add, rs = m[MAXCH:2 * MAXCH], m[2 * MAXCH:] != 0
        x = np.where(rs, add, np.mod(x + add, 1.0))
    return x


def _walk_rows(gi_rows, n_per_blk, walker):
    """the walker over a 1-D array of rows, SPEC_WALK_ROWS at a time (gi_rows written back)"""
    spec = np.zeros(len(gi_rows), SPEC_DTYPE)
    for i in range(0, len(gi_rows), SPEC_WALK_ROWS):
        part = gi_rows[i:i + SPEC_WALK_ROWS]
        spec[i:i + len(part)] = walker(part, n_per_blk).reshape(-1)
    return spec


def chain_speculated(scn_carr, blk, nch, chain, n_per_blk, walker, baton, threads=8,
                     anchors=False):
    """The window's chain with the walks run before the baton (steps 1-4 above): fills
    blk["carr0"]; returns (end carriers, timings).  Every rank of the baton's group calls it (two
    all_gathers); rank 0 passes the run's initial carriers as scn_carr."""
    t = {}
    t0 = time.perf_counter()
    rank = baton.rank
    resets = slot_resets(nch, chain)
    nb = len(nch)
    zero = np.zeros(MAXCH)
    line_end = (carr_line_end(zero, blk, nch, chain, n_per_blk) if nb else zero)
    start0 = scn_carr if rank == 0 else zero
    maps = baton.all_gather(map_vec(start0, line_end, resets))
    x0 = np.array(scn_carr, np.float64) if rank == 0 else compose_start(maps, rank)
    gi = carr_chain_guess(x0, blk, nch, chain, n_per_blk, starts_only=True)
    spec = _walk_rows(gi.reshape(-1), n_per_blk, walker).reshape(gi.shape)
    first = blk if rank == 0 else blk.copy()
    e0, hits = carr_chain_spec(x0, first, nch, chain, n_per_blk, gi, spec, threads=threads)
    if rank == 0:                            # the exact chain
        t["fix_s"] = time.perf_counter() - t0
    maps = baton.all_gather(map_vec(x0 if rank else scn_carr, e0, resets))
    if rank == 0:
        # on to rank 1 after the last collective: from here on only the batons move, in rank
        # order, so that no backend (RCCL orders a rank's operations) can interleave a pending
        # send with a collective the receiver has not reached
        baton.isend(e0)
    rewalked = 0
    if rank > 0:
        x1 = compose_start(maps, rank)
        d = np.mod(x1 - x0 + 0.5, 1.0) - 0.5
        dep = _start_dependent(nch, chain) & (d[np.clip(chain["slot"], 0, MAXCH - 1)] != 0.0)
        if dep.any():
            gi2 = gi[dep]
            sl = chain["slot"][dep].astype(np.int64)
            gi2["g"] = np.mod(first["carr0"][dep] + d[sl], 1.0)
            gi2["k"] = 0
            spec[dep] = _walk_rows(gi2, n_per_blk, walker)
            gi[dep] = gi2
            rewalked = int(dep.sum())
        link = spec_links(nch, chain, n_per_blk, gi, spec, threads=threads)
        t["pre_s"] = time.perf_counter() - t0
        t1 = time.perf_counter()
        x = baton.recv()
        t["wait_s"] = time.perf_counter() - t1
        t1 = time.perf_counter()
        e0, hits = carr_chain_linked(x, blk, nch, chain, n_per_blk, gi, spec, link,
                                     threads=threads)
        baton.isend(e0)
        t["fix_s"] = time.perf_counter() - t1
    baton.finish()
    if anchors:                              # after the hand-off: off the ranks' serial path
        t["anch"] = carr_anchors(blk, nch, n_per_blk, gi, spec, threads=threads)
    t["chain_s"] = time.perf_counter() - t0 - t.get("wait_s", 0.0)
    t["spec_hits"] = hits
    t["spec_rewalked"] = rewalked
    return e0, t


def _concat(parts):
    if parts:
        return (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]),
                np.concatenate([p[2] for p in parts]))
    from . import CHAIN_DTYPE, CHAN_DTYPE
    return (np.zeros((0, MAXCH), CHAN_DTYPE), np.zeros(0, np.int32),
            np.zeros((0, MAXCH), CHAIN_DTYPE))


def plan_window(scn, first, count, baton=None, threads=8, batch=2000, with_ck=True, walker=None,
                chain_threads=None, speculate=True, anchors=False):
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
    carr0 (DeviceWindow computes their checkpoints).  With a walker and a baton over more than one
    rank the chain is speculated across ranks (chain_speculated; speculate=False: the baton
    first, then the chain run ahead).  anchors (with a walker): the chain's anchors in
    timings["anch"] (ANCHOR_DTYPE [count, 16]) for the proofs (gss_linearize_ex)."""
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
    speculate = (carr is None and walker is not None and baton is not None and baton.world > 1
                 and speculate)
    if speculate:
        blk, nch, chain = _concat(parts)
        end, tc = chain_speculated(scn.carrier() if baton.rank == 0 else None, blk, nch, chain,
                                   scn.n_per_blk, walker, baton, threads=chain_threads or threads,
                                   anchors=anchors)
        t.update(tc)
        t.setdefault("wait_s", 0.0)
        return blk, nch, None, t
    t0 = time.perf_counter()
    if carr is None:
        carr = baton.recv() if (baton is not None and baton.rank > 0) else scn.carrier()
    t["wait_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    blk, nch, chain = _concat(parts)
    ct = chain_threads or threads
    if walker is not None and len(nch):
        anch = np.zeros((len(nch), MAXCH), ANCHOR_DTYPE) if anchors else None
        heads = np.zeros((len(nch), MAXCH), SPEC_IN_DTYPE) if anchors else None
        end, t["spec_hits"] = chain_run_ahead(carr, blk, nch, chain, scn.n_per_blk, walker,
                                              threads=ct, anch=anch, heads=heads)
        if anchors:
            t["anch"] = anch
            t["spec_heads"] = heads
        ck = None
    else:
        end, ck = carr_chain(carr, blk, nch, chain, scn.n_per_blk, carrier_int=scn.carrier_int,
                             with_ck=with_ck, threads=ct)
    t["chain_s"] = time.perf_counter() - t0
    if baton is not None:
        baton.send(end)
    return blk, nch, ck, t


def plan_rank(nav_file, rank, world, window_s, *, llh, samp_freq=2.6e6, data_format=16,
              threads=8, batch=2000, baton=None, walker=None, chain_threads=None, speculate=True,
              anchors=False):
    """Host plane for one rank: (blk[n, 16], nch[n], ck[n, 16, NCK] or None, nav rows,
    n_per_blk, timings) of its block range (ck: the carrier checkpoints).  With world > 1 pass a
    Baton: the rank then plans only its own window (module docstring)."""
    first, count = rank_range(rank, world, window_s)
    scn = Scenario(nav_file, llh=llh, duration=window_s * world if world > 1 else window_s,
                   samp_freq=samp_freq, data_format=data_format)
    blk, nch, ck, t = plan_window(scn, first, count, baton=baton, threads=threads, batch=batch,
                                  walker=walker, chain_threads=chain_threads,
                                  speculate=speculate, anchors=anchors)
    if len(nch) != count:
        raise RuntimeError(f"rank {rank}: planned {len(nch)} of {count} blocks")
    t["rows_out"] = int(scn.position()[1])
    return blk, nch, ck, scn.nav_table(), scn.n_per_blk, t
