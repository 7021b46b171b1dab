"""world_size-2 gloo run of the multi-GPU plumbing on CPU: request sharding,
weight-blob broadcast from rank 0, max-time / sum-count reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rwkvtts import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # weights: rank 0 synthesises, others receive
        blob = torch.zeros(4096, dtype=torch.uint8)
        if rank == 0:
            blob.copy_(torch.from_numpy(np.random.default_rng(7).integers(0, 256, 4096, dtype=np.uint8)))
        D.broadcast_blob(blob)
        digest = int(blob.to(torch.int64).sum())
        # requests: 10 ids sharded round-robin, "processed" (squared) locally
        mine = D.shard(list(range(10)), rank, world)
        results = [x * x for x in mine]
        elapsed, total = D.reduce_run(0.5 + rank, len(results))
        q.put((rank, digest, mine, results, elapsed, total))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shard_broadcast_reduce():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = int(np.random.default_rng(7).integers(0, 256, 4096, dtype=np.uint8).astype(np.int64).sum())
    assert all(o[1] == expect for o in out)                     # identical weights everywhere
    assert out[0][2] == [0, 2, 4, 6, 8] and out[1][2] == [1, 3, 5, 7, 9]
    assert D.unshard([o[3] for o in out]) == [x * x for x in range(10)]
    assert all(o[4] == 1.5 and o[5] == 10 for o in out)           # max time, summed count


def test_shard_unshard_roundtrip():
    items = list(range(37))
    for world in (1, 2, 3, 8):
        parts = [D.shard(items, r, world) for r in range(world)]
        assert sum(len(p) for p in parts) == 37
        assert D.unshard(parts) == items
    with pytest.raises(ValueError):
        D.shard(items, 2, 2)
