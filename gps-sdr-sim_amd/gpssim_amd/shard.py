"""Time-window sharding of one run across ranks.

Blocks are independent given their per-block parameters: the code state is recomputed every
block (gpssim.c:1331-1345) and the host planner supplies each block's exact carrier start
(gss_carr_advance), so rank r can synthesise any contiguous block range on its own.  There is no
data-path collective; a whole-run file is rank slices at byte offset first_block * block_bytes.

Weak scaling (bench.py): every rank owns `window_s` seconds, i.e. blocks_per = window_s*10 - 1
blocks starting at r * blocks_per, of one run of world * window_s seconds.  The host plane is
serial in the carrier chain, so each rank plans up to its own window (the carrier at a block
start depends on every earlier block).
"""
import numpy as np

from . import Scenario


def blocks_per_rank(window_s):
    """Blocks each rank synthesises for a window of window_s seconds (the run writes numd-1
    blocks, gpssim.c:2154, so a lone 300 s window is 2999 blocks)."""
    return int(round(window_s * 10)) - 1


def rank_range(rank, world, window_s):
    """[first, first + count) block range of `rank`."""
    n = blocks_per_rank(window_s)
    return rank * n, n


def plan_rank(nav_file, rank, world, window_s, *, llh, samp_freq=2.6e6, data_format=16,
              threads=8, batch=1000):
    """Host plane for one rank: (blk[n, 16], nch[n], ck[n, 16, NCK], nav rows, n_per_blk) of its
    block range (ck: the planner's carrier checkpoints)."""
    first, count = rank_range(rank, world, window_s)
    scn = Scenario(nav_file, llh=llh, duration=window_s * world if world > 1 else window_s,
                   samp_freq=samp_freq, data_format=data_format)
    done, keep_b, keep_n, keep_c = 0, [], [], []
    while done < first + count:
        if done < first:             # before the window only the carrier chain matters
            ask = min(batch, first - done)
            b, n = scn.next(ask, threads=threads)
            if len(n) == 0:
                break
            done += len(n)
            continue
        b, n, c = scn.next(min(batch, first + count - done), threads=threads, with_ck=True)
        if len(n) == 0:
            break
        lo = max(0, first - done)
        if lo < len(n):
            keep_b.append(b[lo:])
            keep_n.append(n[lo:])
            keep_c.append(c[lo:])
        done += len(n)
    blk = np.concatenate(keep_b)[:count]
    nch = np.concatenate(keep_n)[:count]
    ck = np.concatenate(keep_c)[:count]
    if len(nch) != count:
        raise RuntimeError(f"rank {rank}: planned {len(nch)} of {count} blocks")
    return blk, nch, ck, scn.nav_table(), scn.n_per_blk
