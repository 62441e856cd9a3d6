"""Whole-node single-sink output (gpssim_amd.node): the ordered chunked gather of the ranks' time
shards to rank 0.

* CPU, gloo, world sizes 2-4: ordered_gather over synthetic byte chunks whose content encodes
  (block, byte) -- rank 0's sink must see the run's bytes in run order, whatever the partition,
  chunk size and layout (uneven ranks, a last short chunk, more ranks than chunks of a rank,
  "block" and "stripe"); with every layout rank 0 must have had receives outstanding from
  min(world - 1, 2) or more peers at once (the per-peer receive windows), and with "stripe"
  from every peer;
* CPU, gloo, world sizes 3 and 4: exchange_rows hands each chunk's rows from its planner to its
  renderer byte for byte, with the nav rows re-pointed into the merged table; and again with
  every pair exchanging in both directions and each message past 8 MB (the grouped posting,
  batch_isend_irecv, that keeps the same call safe under RCCL);
* CPU: FileSink writes in call order from its writer thread while the caller reuses its buffers;
* GPU (-m gpu), two ranks on the one GPU, backend GSS_TEST_BACKEND (default gloo: RCCL needs a
  GPU per rank, so a whole-node driver run sets nccl and exercises the same test unchanged):
  run_node renders the static -d 3 -b 16 run in both layouts and rank 0 writes the file; its
  blocks carry the reference's golden hashes.
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


def _gather_worker(rank, world, port, n_blocks, bb, chunk_blocks, layout, out_path):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import json
    import numpy as np
    import torch
    import torch.distributed as dist
    from gpssim_amd.node import chunk_plan, ordered_gather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = chunk_plan(n_blocks, world, chunk_blocks, layout)

    def get_chunk(first, nb):             # this rank "renders" the chunks the plan gives it
        assert any(r == rank and c == first and n == nb for r, c, n in plan)
        return torch.from_numpy(np.concatenate([_block_bytes(b, bb)
                                                for b in range(first, first + nb)]))

    got, stats = [], {}
    ordered_gather(plan, rank, dist, get_chunk,
                   lambda nb: torch.empty(nb * bb, dtype=torch.uint8),
                   (lambda t: got.append(t.numpy().tobytes())) if rank == 0 else None,
                   stats=stats)
    if rank == 0:
        open(out_path, "wb").write(b"".join(got))
        open(out_path + ".json", "w").write(json.dumps(stats))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("layout", ["block", "stripe"])
@pytest.mark.parametrize("world,n_blocks,chunk", [(2, 29, 4), (3, 10, 3), (3, 5, 8), (2, 1, 4),
                                                  (4, 23, 2), (4, 41, 5)])
def test_ordered_gather_gloo(tmp_path, world, n_blocks, chunk, layout):
    import json
    import numpy as np
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd.node import chunk_plan
    bb = 40
    out = tmp_path / "run.bin"
    mp.spawn(_gather_worker, args=(world, _free_port(), n_blocks, bb, chunk, layout, str(out)),
             nprocs=world, join=True)
    want = np.concatenate([_block_bytes(b, bb) for b in range(n_blocks)]).tobytes()
    assert out.read_bytes() == want
    st = json.loads((tmp_path / "run.bin.json").read_text())
    plan = chunk_plan(n_blocks, world, chunk, layout)
    peers = {r for r, c, nb in plan if r != 0}
    # every peer with chunks had its first receive posted before rank 0's sink took anything
    assert st["max_peers_outstanding"] == len(peers)
    assert st["max_peers_outstanding"] >= min(len(peers), 2)
    assert st["max_outstanding"] >= min(len(peers), 2)
    if layout == "stripe":
        assert {r for r, c, nb in plan[:world]} == set(range(min(world, len(plan))))


def _exchange_worker(rank, world, port, n_blocks, chunk, out_dir):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import numpy as np
    import torch.distributed as dist
    from gpssim_amd import CHAN_DTYPE, MAXCH, NAV_WORDS
    from gpssim_amd.node import chunk_plan, exchange_rows, rank_blocks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = rank_blocks(n_blocks, rank, world)
    blk, nch, nav = _rows(b0, b1, rank)
    plan = chunk_plan(n_blocks, world, chunk, "stripe")
    ob, on, onav, firsts = exchange_rows(plan, n_blocks, rank, world, dist, blk, nch, nav)
    np.save(os.path.join(out_dir, f"blk{rank}.npy"), ob.view(np.uint8))
    np.save(os.path.join(out_dir, f"nch{rank}.npy"), on)
    np.save(os.path.join(out_dir, f"nav{rank}.npy"), onav)
    np.save(os.path.join(out_dir, f"first{rank}.npy"), np.asarray(firsts, np.int64))
    dist.barrier()
    dist.destroy_process_group()


def _rows(b0, b1, planner):
    """synthetic rows of blocks [b0, b1) as planner `planner` would hold them: every field a
    function of (block, channel), nav_tbl into a planner-sized table of distinct rows"""
    import numpy as np
    from gpssim_amd import CHAN_DTYPE, MAXCH, NAV_WORDS
    n_nav = 3 + planner * 2
    nav = (np.arange(n_nav * NAV_WORDS, dtype=np.uint32).reshape(n_nav, NAV_WORDS) +
           np.uint32(1000 * (planner + 1)))
    blk = np.zeros((b1 - b0, MAXCH), CHAN_DTYPE)
    for i, b in enumerate(range(b0, b1)):
        for k in range(MAXCH):
            blk[i, k]["carr0"] = b + k / 64
            blk[i, k]["gain"] = b * 16 + k
            blk[i, k]["ca_tbl"] = (b + k) % 32
            blk[i, k]["nav_tbl"] = (b * 7 + k) % n_nav
    nch = np.array([(b % 12) + 1 for b in range(b0, b1)], np.int32)
    return blk, nch, nav


@pytest.mark.parametrize("world,n_blocks,chunk", [(3, 20, 3), (4, 23, 2), (4, 3, 2)])
def test_exchange_rows_gloo(tmp_path, world, n_blocks, chunk):
    import numpy as np
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd import CHAN_DTYPE
    from gpssim_amd.node import chunk_plan, planner_of, rank_blocks
    mp.spawn(_exchange_worker, args=(world, _free_port(), n_blocks, chunk, str(tmp_path)),
             nprocs=world, join=True)
    plan = chunk_plan(n_blocks, world, chunk, "stripe")
    for r in range(world):
        ob = np.load(tmp_path / f"blk{r}.npy").view(CHAN_DTYPE).reshape(-1, 16)
        on = np.load(tmp_path / f"nch{r}.npy")
        onav = np.load(tmp_path / f"nav{r}.npy")
        firsts = list(np.load(tmp_path / f"first{r}.npy"))
        mine = [(c, nb) for q, c, nb in plan if q == r]
        assert firsts == [c for c, _ in mine]
        o = 0
        for c, nb in mine:
            p = planner_of(c, n_blocks, world)
            pb0, pb1 = rank_blocks(n_blocks, p, world)
            assert pb0 <= c and c + nb <= pb1              # a chunk never crosses a window
            wb, wn, wnav = _rows(pb0, pb1, p)
            got, want = ob[o:o + nb], wb[c - pb0:c - pb0 + nb]
            for f in ("carr0", "gain", "ca_tbl"):
                assert np.array_equal(got[f], want[f])
            assert np.array_equal(on[o:o + nb], wn[c - pb0:c - pb0 + nb])
            # the re-pointed nav rows are the planner's rows
            assert np.array_equal(onav[got["nav_tbl"].reshape(-1)],
                                  wnav[want["nav_tbl"].reshape(-1)])
            o += nb
        assert o == len(ob) == len(on)


def _rows_big(b0, b1, planner):
    """as _rows, vectorised, with a large nav table: a pair's message passes 8 MB"""
    import numpy as np
    from gpssim_amd import CHAN_DTYPE, MAXCH, NAV_WORDS
    n_nav = 20000 + planner * 3
    nav = (np.arange(n_nav * NAV_WORDS, dtype=np.uint32).reshape(n_nav, NAV_WORDS) *
           np.uint32(2654435761) + np.uint32(1000 * (planner + 1)))
    b = np.arange(b0, b1, dtype=np.int64)[:, None]
    k = np.arange(MAXCH, dtype=np.int64)[None, :]
    blk = np.zeros((b1 - b0, MAXCH), CHAN_DTYPE)
    blk["carr0"] = b + k / 64
    blk["code0"] = b * 1.5 - k
    blk["gain"] = b * 16 + k
    blk["ca_tbl"] = (b + k) % 32
    blk["nav_tbl"] = (b * 7 + k) % n_nav
    nch = ((np.arange(b0, b1) % 12) + 1).astype(np.int32)
    return blk, nch, nav


def _exchange_big_worker(rank, world, port, n_blocks, chunk, out_path):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import numpy as np
    import torch.distributed as dist
    from gpssim_amd.node import chunk_plan, exchange_rows, planner_of, rank_blocks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = rank_blocks(n_blocks, rank, world)
    blk, nch, nav = _rows_big(b0, b1, rank)
    plan = chunk_plan(n_blocks, world, chunk, "stripe")
    ob, on, onav, firsts = exchange_rows(plan, n_blocks, rank, world, dist, blk, nch, nav)
    mine = [(c, nb) for q, c, nb in plan if q == rank]
    ok = firsts == [c for c, _ in mine]
    o = 0
    for c, nb in mine:
        p = planner_of(c, n_blocks, world)
        pb0, pb1 = rank_blocks(n_blocks, p, world)
        wb, wn, wnav = _rows_big(pb0, pb1, p)
        got, want = ob[o:o + nb], wb[c - pb0:c - pb0 + nb]
        for f in ("carr0", "code0", "gain", "ca_tbl"):
            ok &= bool(np.array_equal(got[f], want[f]))
        ok &= bool(np.array_equal(on[o:o + nb], wn[c - pb0:c - pb0 + nb]))
        ok &= bool(np.array_equal(onav[got["nav_tbl"].reshape(-1)],
                                  wnav[want["nav_tbl"].reshape(-1)]))
        o += nb
    ok &= o == len(ob)
    open(f"{out_path}.{rank}", "w").write("ok" if ok else "bad")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 4])
def test_exchange_rows_large_two_way_gloo(tmp_path, world):
    """every pair of ranks exchanges rows in both directions (stripe layout), each message past
    8 MB: the grouped posting (batch_isend_irecv) must deliver every byte whatever the sizes"""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd import CHAN_DTYPE, MAXCH, NAV_WORDS
    from gpssim_amd.node import chunk_plan, planner_of
    n_blocks, chunk = world * 30000, 1000
    plan = chunk_plan(n_blocks, world, chunk, "stripe")
    per_pair = {}
    for r, c, nb in plan:
        p = planner_of(c, n_blocks, world)
        if p != r:
            per_pair[(p, r)] = per_pair.get((p, r), 0) + nb * (CHAN_DTYPE.itemsize * MAXCH + 4)
    pairs = {(p, r) for p, r in per_pair}
    assert all((r, p) in pairs for p, r in pairs)              # two-way for every pair
    assert min(per_pair.values()) + 20000 * NAV_WORDS * 4 > 8 << 20
    out = tmp_path / "x"
    mp.spawn(_exchange_big_worker, args=(world, _free_port(), n_blocks, chunk, str(out)),
             nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"x.{r}").read_text() == "ok"


def test_file_sink_overlapped(tmp_path):
    """FileSink: chunks written in call order by its writer thread, the caller free to reuse a
    chunk's memory on return, errors raised at close()"""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd.node import FileSink
    rng = np.random.default_rng(5)
    path = tmp_path / "o.bin"
    fd = os.open(str(path), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    sink = FileSink(torch, fd, 1 << 16, nbuf=2)
    want = []
    buf = torch.empty(1 << 16, dtype=torch.uint8)
    for i in range(200):
        n = int(rng.integers(1, 1 << 16))
        v = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8))
        buf[:n] = v
        want.append(v.numpy().tobytes())
        sink(buf[:n])
        buf.fill_(i & 255)                      # reused at once, as ordered_gather's buffers
    sink.close()
    os.close(fd)
    assert sink.bytes == sum(len(w) for w in want)
    assert path.read_bytes() == b"".join(want)
    # a failing write surfaces
    r, w = os.pipe()
    os.close(r)
    sink = FileSink(torch, w, 64, nbuf=2)
    import signal
    old = signal.signal(signal.SIGPIPE, signal.SIG_IGN)
    try:
        sink(torch.zeros(8, dtype=torch.uint8))
        with pytest.raises(OSError):
            sink.close()
    finally:
        signal.signal(signal.SIGPIPE, old)
        os.close(w)


def test_planner_of():
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd.node import planner_of, rank_blocks
    for n, w in [(863999, 8), (29, 3), (3, 4), (100, 7)]:
        for b in list(range(min(n, 60))) + [n - 1]:
            r = planner_of(b, n, w)
            lo, hi = rank_blocks(n, r, w)
            assert lo <= b < hi


def test_chunk_plan_partition():
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    from gpssim_amd.node import chunk_plan
    plan = chunk_plan(863999, 8, 256)
    assert [p[1] for p in plan] == sorted(p[1] for p in plan)
    assert sum(p[2] for p in plan) == 863999
    assert all(plan[i][1] + plan[i][2] == plan[i + 1][1] for i in range(len(plan) - 1))
    assert sorted({p[0] for p in plan}) == list(range(8))


def _node_worker(rank, world, port, out_path, backend, layout):
    sys.path.insert(0, os.path.join(REPO, "gps-sdr-sim_amd"))
    import json
    import torch.distributed as dist
    from gpssim_amd.node import run_node
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group(backend, rank=rank, world_size=world)
    stats = {}
    # nccl: one GPU per rank (a whole-node run); gloo: both ranks on GPU 0
    run_node(["-e", NAV, "-l", "30.286502,120.032669,100", "-d", "3", "-b", "16", "-o",
              out_path], rank, world, rank if backend == "nccl" else 0, backend=backend,
             chunk_blocks=5, threads=4, layout=layout, stats=stats)
    if rank == 0:
        open(out_path + ".json", "w").write(json.dumps(stats))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["block", "stripe"])
def test_node_run_two_ranks_one_sink(tmp_path, golden, layout):
    import json
    import torch.multiprocessing as mp
    backend = os.environ.get("GSS_TEST_BACKEND", "gloo")
    world = int(os.environ.get("GSS_TEST_WORLD", "2"))
    out = tmp_path / "gpssim.bin"
    mp.spawn(_node_worker, args=(world, _free_port(), str(out), backend, layout), nprocs=world,
             join=True)
    data = out.read_bytes()
    bb = 1040000
    assert len(data) == 29 * bb
    hs = [hashlib.sha256(data[i * bb:(i + 1) * bb]).hexdigest()[:16] for i in range(29)]
    assert hs == golden["static_d30_b16"]["block_sha16"][:29]
    st = json.loads(open(str(out) + ".json").read())
    assert st["max_peers_outstanding"] == world - 1
