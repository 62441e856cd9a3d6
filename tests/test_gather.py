"""Whole-node single-sink output (gpssim_amd.node): the ordered chunked gather of the ranks' time
shards to rank 0.

* CPU, gloo, world sizes 2 and 3: ordered_gather over synthetic byte chunks whose content
  encodes (block, byte) -- rank 0's sink must see the run's bytes in run order, whatever the
  partition and chunk size (uneven ranks, a last short chunk, more ranks than chunks of a rank);
* GPU (-m gpu), gloo, two ranks on the one GPU: run_node renders the two halves of the static
  -d 3 -b 16 run and rank 0 writes the file; its blocks carry the reference's golden hashes.
"""
import hashlib
import os
import socket
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAV = os.path.join(REPO, "tests", "golden", "data", "brdc3540.14n")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _block_bytes(b, bb):
    """synthetic content of block b: every byte depends on the block and its offset"""
    import numpy as np
    return ((np.arange(bb, dtype=np.int64) * 7 + b * 131) % 251).astype(np.uint8)


def _gather_worker(rank, world, port, n_blocks, bb, chunk_blocks, out_path):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import numpy as np
    import torch
    import torch.distributed as dist
    from gpssim_amd.node import chunk_plan, ordered_gather, rank_blocks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = rank_blocks(n_blocks, rank, world)
    mine = torch.from_numpy(np.concatenate([_block_bytes(b, bb) for b in range(b0, b1)])
                            if b1 > b0 else np.zeros(0, np.uint8))

    def get_chunk(first, nb):
        return mine[(first - b0) * bb:(first - b0 + nb) * bb].clone()

    got = []
    ordered_gather(chunk_plan(n_blocks, world, chunk_blocks), rank, dist, get_chunk,
                   lambda nb: torch.empty(nb * bb, dtype=torch.uint8),
                   (lambda t: got.append(t.numpy().tobytes())) if rank == 0 else None)
    if rank == 0:
        open(out_path, "wb").write(b"".join(got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_blocks,chunk", [(2, 29, 4), (3, 10, 3), (3, 5, 8), (2, 1, 4)])
def test_ordered_gather_gloo(tmp_path, world, n_blocks, chunk):
    import numpy as np
    import torch.multiprocessing as mp
    bb = 40
    out = tmp_path / "run.bin"
    mp.spawn(_gather_worker, args=(world, _free_port(), n_blocks, bb, chunk, str(out)),
             nprocs=world, join=True)
    want = np.concatenate([_block_bytes(b, bb) for b in range(n_blocks)]).tobytes()
    assert out.read_bytes() == want


def test_chunk_plan_partition():
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd.node import chunk_plan
    plan = chunk_plan(863999, 8, 256)
    assert [p[1] for p in plan] == sorted(p[1] for p in plan)
    assert sum(p[2] for p in plan) == 863999
    assert all(plan[i][1] + plan[i][2] == plan[i + 1][1] for i in range(len(plan) - 1))
    assert sorted({p[0] for p in plan}) == list(range(8))


def _node_worker(rank, world, port, out_path):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import torch.distributed as dist
    from gpssim_amd.node import run_node
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    run_node(["-e", NAV, "-l", "30.286502,120.032669,100", "-d", "3", "-b", "16", "-o",
              out_path], rank, world, 0, backend="gloo", chunk_blocks=5, threads=4)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_node_run_two_ranks_one_sink(tmp_path, golden):
    import torch.multiprocessing as mp
    out = tmp_path / "gpssim.bin"
    mp.spawn(_node_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    data = out.read_bytes()
    bb = 1040000
    assert len(data) == 29 * bb
    hs = [hashlib.sha256(data[i * bb:(i + 1) * bb]).hexdigest()[:16] for i in range(29)]
    assert hs == golden["static_d30_b16"]["block_sha16"][:29]
