"""The N>1 path on CPU: time-window shards (gpssim_amd.shard, the decomposition bench.py runs under
torchrun) planned independently by two gloo ranks, synthesised per rank (CPU oracle as the
byte producer; no GPU here), gathered over torch.distributed, and compared block by block with
the reference's golden hashes of one single-process run.  Covers the rank partition, each rank's
independent host planning (the exact carrier chain up to its window) and the byte layout of the
concatenated slices."""
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


def _worker(rank, world, port, result_path):
    _paths()
    import numpy as np
    import torch
    import torch.distributed as dist
    import gpssim_amd as G
    import oracle
    from gpssim_amd.shard import plan_rank, rank_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blk, nch, ck, nav, npb = plan_rank(NAV, rank, world, WINDOW_S, llh=LOC, threads=2)
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
        firsts = [rank_range(r, world, WINDOW_S)[0] for r in range(world)]
        json.dump({"hashes": hashes, "firsts": firsts}, open(result_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_time_window_shards(tmp_path, golden):
    import torch.multiprocessing as mp
    world = 2
    res = tmp_path / "r.json"
    mp.spawn(_worker, args=(world, _free_port(), str(res)), nprocs=world, join=True)
    r = json.load(open(res))
    assert r["firsts"] == [0, 4]
    want = golden["static_d30_b16"]["block_sha16"][: 4 * world]
    assert r["hashes"] == want
