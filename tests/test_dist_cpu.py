"""CPU (gloo, world_size 2): the frame-sharding helpers the multi-GPU bench and
stream path use (mvpose/dist.py) — balanced contiguous shards, weight
broadcast from rank 0, and the rank-ordered gather of per-frame results."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mvpose import dist as mdist


def test_shard_covers_exactly():
    for n in (0, 1, 7, 100000, 12501):
        for w in (1, 2, 3, 8):
            spans = [mdist.shard(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = torch.full((5,), float(rank))              # rank 0 holds the real weights
        mdist.broadcast_([w], src=0)

        def process(a, b):                              # stand-in for the GPU pipeline on [a, b)
            t = torch.arange(a, b, dtype=torch.float32)
            return {"kpts_3d": t[:, None, None].expand(-1, 17, 3) + w[0],
                    "idx": torch.arange(a, b, dtype=torch.int64)}
        out = mdist.process_sharded(process, n_total)
        if rank == 0:
            q.put((out["kpts_3d"][:, 0, 0].tolist(), out["idx"].tolist(), w.tolist()))
        else:
            q.put(("rank1", out is None, w.tolist()))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("n_total", [10, 11])
def test_gloo_two_ranks_broadcast_and_gather(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    root = next(r for r in res if r[0] != "rank1")
    other = next(r for r in res if r[0] == "rank1")
    vals, idx, w0 = root
    assert idx == list(range(n_total))
    assert vals == [float(i) for i in range(n_total)]   # weights broadcast from rank 0 (= 0.0)
    assert w0 == [0.0] * 5 and other[2] == [0.0] * 5 and other[1] is True
