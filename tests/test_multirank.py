"""The N>1 path on CPU: time-window shards (gpssim_amd.shard, the decomposition bench.py runs under
torchrun) planned once per node by two gloo ranks -- each seeks to its own window, produces its
rows, and receives the 16 slot carriers at its first block from the rank before (the baton) --
synthesised per rank (CPU oracle as the byte producer; no GPU here), gathered over
torch.distributed, and compared block by block with the reference's golden hashes of one
single-process run.  Rank 1 must never produce a row of a block before its window."""
import hashlib
import json
import os
import socket
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAV = os.path.join(REPO, "tests", "golden", "data", "brdc3540.14n")
LOC = (30.286502, 120.032669, 100.0)
WINDOW_S = 0.5                       # 4 blocks per rank


def _paths():
    for p in (os.path.join(REPO, "gps-sdr-sim_amd"), os.path.join(REPO, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(rank, world, port, result_path, window_s=WINDOW_S, run_ahead=False):
    _paths()
    import numpy as np
    import torch
    import torch.distributed as dist
    import gpssim_amd as G
    import oracle
    from gpssim_amd.shard import Baton, host_walker, plan_rank, rank_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blk, nch, ck, nav, npb, t = plan_rank(NAV, rank, world, window_s, llh=LOC, threads=2,
                                          baton=Baton(dist, rank, world),
                                          walker=host_walker(2) if run_ahead else None)
    # the rank produced rows for its own window only (rank 1 seeked past rank 0's blocks)
    assert t["rows_out"] == len(nch) == rank_range(rank, world, window_s)[1]
    out, rc = oracle.synth(blk, nch, G.ca_table(), nav, npb, 16)
    assert rc == 0
    t = torch.from_numpy(np.ascontiguousarray(out))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    if rank == 0:
        bb = G.block_bytes(npb, 16)
        whole = torch.cat(parts).numpy().tobytes()
        hashes = [hashlib.sha256(whole[i * bb:(i + 1) * bb]).hexdigest()[:16]
                  for i in range(len(whole) // bb)]
        firsts = [rank_range(r, world, window_s)[0] for r in range(world)]
        json.dump({"hashes": hashes, "firsts": firsts}, open(result_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,window_s,gold,run_ahead", [
    (2, WINDOW_S, "static_d30_b16", False),
    # rank 1 starts at block 309: its seek replays the 30 s nav/allocation update after block
    # 299 (gpssim.c:2294-2345) and its own window crosses the one after block 599
    (2, 31.0, "static_d300_b16", False),
    # the same with each rank's chain run ahead (speculative walks, shard.chain_run_ahead)
    (2, 31.0, "static_d300_b16", True),
    # three ranks: the middle one both receives and hands on the baton
    (3, WINDOW_S, "static_d30_b16", False),
])
def test_two_rank_time_window_shards(tmp_path, golden, world, window_s, gold, run_ahead):
    import torch.multiprocessing as mp
    res = tmp_path / "r.json"
    mp.spawn(_worker, args=(world, _free_port(), str(res), window_s, run_ahead), nprocs=world,
             join=True)
    r = json.load(open(res))
    n = int(round(window_s * 10)) - 1
    assert r["firsts"] == [k * n for k in range(world)]
    want = golden[gold]["block_sha16"][: n * world]
    assert r["hashes"] == want


def _spec_worker(rank, world, port, result_path, window_s):
    """each rank plans its window with the chain speculated across ranks (host walker) and
    checks every carrier against the serial chain of a lone process walking the prefix"""
    _paths()
    import numpy as np
    import torch.distributed as dist
    import gpssim_amd as G
    from gpssim_amd.shard import Baton, host_walker, plan_window, rank_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = rank_range(rank, world, window_s)
    scn = G.Scenario(NAV, llh=LOC, duration=window_s * world, samp_freq=2.6e6, data_format=16)
    blk, nch, ck, t = plan_window(scn, first, count, baton=Baton(dist, rank, world), threads=2,
                                  walker=host_walker(2))
    ref = G.Scenario(NAV, llh=LOC, duration=window_s * world, samp_freq=2.6e6, data_format=16)
    rb, rn, _, _ = plan_window(ref, first, count, threads=2, with_ck=False)
    ok = bool(np.array_equal(rn, nch) and
              np.array_equal(rb["carr0"].view(np.uint64), blk["carr0"].view(np.uint64)))
    rows = int(nch.sum())
    res = [ok, rows, t["spec_hits"], t["spec_rewalked"], t.get("fix_s", 0.0)]
    import torch
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        json.dump(out, open(result_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,window_s", [(2, 40.0), (3, 40.0), (4, 25.0)])
def test_chain_speculated_across_ranks(tmp_path, world, window_s):
    """gpssim_amd.shard.chain_speculated: every rank's guesses and walks run before its baton
    (predicted starts from the ranks' published maps); carriers bit-identical to the serial
    chain, the walks' translations holding on almost every row, later ranks re-walking the rows
    whose start the second prediction moved."""
    import torch.multiprocessing as mp
    res = tmp_path / "r.json"
    mp.spawn(_spec_worker, args=(world, _free_port(), str(res), window_s), nprocs=world,
             join=True)
    out = json.load(open(res))
    for rank, (ok, rows, hits, rewalked, fix_s) in enumerate(out):
        assert ok, f"rank {rank}: carriers differ from the serial chain"
        assert hits >= 0.97 * rows, (rank, hits, rows)
        if rank > 0:
            assert rewalked > 0
