"""world_size-2 request sharding with REAL HIP engines (SURVEY §8e, config 4's per-rank path):
two ranks on the one visible GPU, gloo for the collectives (two ranks cannot share a device in
RCCL), each rank receiving the weight blob by broadcast from rank 0, building its own engine on
device 0 and generating its round-robin shard; the gathered results, in request order, must equal
the oracle's serial runs. The ranks are forked from the session's fork server
(tests/conftest.py), so no rank is exec'ed from a process that has initialised HIP."""
import os
import socket

import numpy as np
import pytest

from conftest import forkserver_context

pytestmark = pytest.mark.gpu

N_REQ = 9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _requests():
    from helpers import make_request, synth_text
    return [make_request(synth_text(4000 + i), seed=70 + i, max_tokens=6 + 2 * i) for i in range(N_REQ)]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import rwkvtts
        from rwkvtts import dist as D
        from rwkvtts import weights as W
        nbytes = W.blob_bytes(W.DIMS_TINY)
        blob = torch.zeros(nbytes, dtype=torch.uint8)
        if rank == 0:
            blob.copy_(torch.from_numpy(W.synth_blob(W.DIMS_TINY, seed=99)))
        D.broadcast_blob(blob)
        rt = rwkvtts.SharedRwkvRuntime(blob.numpy(), device=0, max_slots=4, token_chunk_size=64, use_graphs=True)
        try:
            mine = D.shard(_requests(), rank, world)
            results = rt.generate_batch(mine)
            steps = rt.stats()["steps"]
        finally:
            rt.close()
        parts = [None] * world
        dist.all_gather_object(parts, results)
        elapsed, total = D.reduce_run(1.0 + rank, sum(len(s) for _, s in results))
        q.put((rank, D.unshard(parts), elapsed, total, steps))
    except Exception as e:  # reported to the parent instead of a silent hang
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_gloo_world2_real_engines():
    import oracle
    from rwkvtts import weights as W
    from helpers import to_struct
    world, port = 2, _free_port()
    ctx = forkserver_context()
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=240) for _ in range(world)), key=lambda o: o[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(isinstance(o[1], list) for o in out), out
    om = oracle.Model(W.synth_blob(W.DIMS_TINY, seed=99))
    serial = []
    for r in _requests():
        st, keep = to_struct(r)
        g, s, _ = om.generate(st)
        serial.append((g, s))
    assert out[0][1] == serial and out[1][1] == serial
    assert out[0][2] == 2.0 and out[0][3] == sum(len(s) for _, s in serial)
    assert all(o[4] > 0 for o in out)  # both ranks' engines ran decode steps
    assert all(p.exitcode == 0 for p in procs)
