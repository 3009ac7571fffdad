"""world_size-2 gloo rehearsal of the bench's multi-process path (CPU)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kube-arbitrator_amd"))
    from kbgpu import dist
    assert dist.init("gloo")
    dist.barrier()
    # rank r "placed" 1000*(r+1) tasks in (r+1) seconds
    q.put((rank, dist.aggregate(float(rank + 1), 1000 * (rank + 1))))
    dist.shutdown()


@pytest.mark.parametrize("world", [2])
def test_gloo_aggregate(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r] == (float(world), 1000 * world * (world + 1) // 2)
