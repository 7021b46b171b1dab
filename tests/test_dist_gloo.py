"""world_size-2 gloo run of the multi-GPU plumbing on CPU: request sharding,
weight-blob broadcast from rank 0, max-time / sum-count reduction -- and real TTS requests routed
through it, each rank generating its shard with a CPU stand-in for its GPU engine (the oracle's
serial controller, test infrastructure) on the weights it received by broadcast."""
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


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shard_broadcast_reduce(world):
    port = _free_port()
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
    assert [o[2] for o in out] == [list(range(r, 10, world)) for r in range(world)]  # round-robin shards
    assert D.unshard([o[3] for o in out]) == [x * x for x in range(10)]
    assert all(o[4] == 0.5 + (world - 1) and o[5] == 10 for o in out)  # max time, summed count


def test_shard_unshard_roundtrip():
    items = list(range(37))
    for world in (1, 2, 3, 8):
        parts = [D.shard(items, r, world) for r in range(world)]
        assert sum(len(p) for p in parts) == 37
        assert D.unshard(parts) == items
    with pytest.raises(ValueError):
        D.shard(items, 2, 2)


def _tts_worker(rank, world, port, q):
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from rwkvtts import weights as W
        from helpers import make_request, synth_text, to_struct
        nbytes = W.blob_bytes(W.DIMS_TINY)
        blob = torch.zeros(nbytes, dtype=torch.uint8)
        if rank == 0:
            blob.copy_(torch.from_numpy(W.synth_blob(W.DIMS_TINY, seed=99)))
        D.broadcast_blob(blob)                       # rank 0 -> every rank (RCCL on the GPUs)
        engine = oracle.Model(blob.numpy())          # CPU stand-in for this rank's GPU engine
        reqs = [make_request(synth_text(3000 + i), seed=40 + i, max_tokens=8 + i) for i in range(7)]
        mine = D.shard(reqs, rank, world)
        results = []
        for r in mine:
            st, keep = to_struct(r)
            g, s_, _ = engine.generate(st)
            results.append((g, s_))
        parts = [None] * world
        dist.all_gather_object(parts, results)
        elapsed, total = D.reduce_run(1.0 + rank, sum(len(s_) for _, s_ in results))
        q.put((rank, D.unshard(parts), elapsed, total))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_routes_tts_requests():
    """7 requests sharded over 2 ranks, generated per rank on the broadcast weights, gathered back
    in request order: identical to generating all 7 serially on one engine."""
    import oracle
    from rwkvtts import weights as W
    from helpers import make_request, synth_text, to_struct
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tts_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    om = oracle.Model(W.synth_blob(W.DIMS_TINY, seed=99))
    reqs = [make_request(synth_text(3000 + i), seed=40 + i, max_tokens=8 + i) for i in range(7)]
    serial = []
    for r in reqs:
        st, keep = to_struct(r)
        g, s_, _ = om.generate(st)
        serial.append((g, s_))
    assert out[0][1] == serial and out[1][1] == serial
    assert out[0][2] == 2.0 and out[0][3] == sum(len(s_) for _, s_ in serial)
