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
    replicas = dist.aggregate(float(rank + 1), 1000 * (rank + 1))
    # node-axis shards of one cluster: every rank reports the same decisions
    sharded = dist.aggregate(float(rank + 1), 5000, sharded=True)
    # the communicator id travels from rank 0 (kbg_comm_unique_id) to every rank
    uid = dist.broadcast_bytes(bytes(range(128)) if rank == 0 else b"")
    q.put((rank, (replicas, sharded, uid)))
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
        replicas, sharded, uid = got[r]
        assert replicas == (float(world), 1000 * world * (world + 1) // 2)
        assert sharded == (float(world), 5000)
        assert uid == bytes(range(128))


def test_comm_fails_loudly_without_device():
    """No silent single-process fallback when RCCL / HIP cannot start."""
    import ctypes
    from kbgpu import _abi
    L = _abi.lib()
    if L.kbg_device_count() > 0:
        pytest.skip("a device is present")
    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * _abi.COMM_ID_BYTES)()
    assert L.kbg_comm_init(uid, 1, 0, 0, ctypes.byref(h)) == _abi.KBG_E_HIP
    assert not h.value
    assert L.kbg_comm_init(uid, 2, 2, 0, ctypes.byref(h)) == _abi.KBG_E_INVALID
