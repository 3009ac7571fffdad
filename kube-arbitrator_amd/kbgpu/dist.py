"""Multi-process plumbing for `bench.py --gpus N` (one process per GPU).

N > 1 shards ONE cluster's node axis across the ranks: every
rank opens the same snapshot through `kbg_session_open_sharded` on an RCCL
communicator (`ShardComm`) and the library all-gathers the per-shard
feasibility bitmaps of each batch over xGMI. torch.distributed ("nccl" =
RCCL on MI355X, "gloo" on CPU) only carries the communicator's unique id, the
bench's barriers and the max-over-ranks wall time.
"""
import ctypes
import os


def _td():
    """torch.distributed, imported on first use (HostComm ranks need no torch)."""
    import torch.distributed as dist
    return dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend):
    """Initialises the default process group from the torchrun environment."""
    dist = _td()
    rank, world, _ = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world)
    return dist.is_initialized()


def barrier():
    dist = _td()
    if dist.is_initialized():
        dist.barrier()


def broadcast_bytes(data, src=0):
    """Rank `src`'s bytes on every rank (the communicator id's side channel)."""
    dist = _td()
    if not dist.is_initialized():
        return data
    box = [data]
    dist.broadcast_object_list(box, src=src)
    return box[0]


class ShardComm:
    """kbg_comm: the RCCL clique of the node-axis shards, one rank per GPU."""

    transport = "rccl"

    def __init__(self, device, rank=None, world=None):
        from . import _abi
        L = _abi.lib()
        if rank is None:
            dist = _td()
            rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
        uid = (ctypes.c_uint8 * _abi.COMM_ID_BYTES)()
        if rank == 0:
            _abi.check(L.kbg_comm_unique_id(uid))
        uid_bytes = broadcast_bytes(bytes(uid))
        uid = (ctypes.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(uid_bytes)
        self.handle = ctypes.c_void_p()
        _abi.check(L.kbg_comm_init(uid, world, rank, device, ctypes.byref(self.handle)))
        self.rank, self.world, self.device = rank, world, device

    def ranks(self):
        """(ranks, this rank) as the transport itself counts them (RCCL: ncclCommCount / ncclCommUserRank;
        host: the processes that joined the segment)."""
        from . import _abi
        n, r = ctypes.c_int32(), ctypes.c_int32()
        _abi.check(_abi.lib().kbg_comm_ranks(self.handle, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    def close(self):
        if self.handle:
            from . import _abi
            _abi.lib().kbg_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()


class HostComm(ShardComm):
    """kbg_comm over the host transport (kbg_comm_init_host): the ranks are
    processes of this host, possibly sharing one GPU, exchanging every
    collective through POSIX shared memory. Every rank passes the same fresh
    `name`; the call returns once all `world` ranks joined."""

    transport = "host"

    def __init__(self, name, rank, world, device=0):
        from . import _abi
        self.handle = ctypes.c_void_p()
        _abi.check(_abi.lib().kbg_comm_init_host(name.encode(), world, rank, device, ctypes.byref(self.handle)))
        self.rank, self.world, self.device = rank, world, device


def aggregate(elapsed_s, decisions, sharded=False):
    """(max elapsed over ranks, placements of the whole job). Sharded ranks
    produce the same decisions for one cluster, so they count once;
    independent clusters (replicas) add up."""
    import torch
    dist = _td()
    if not dist.is_initialized():
        return elapsed_s, decisions
    dev = torch.device("cuda") if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    d = torch.tensor([float(decisions)], dtype=torch.float64, device=dev)
    dist.all_reduce(d, op=dist.ReduceOp.MAX if sharded else dist.ReduceOp.SUM)
    return float(t.item()), int(d.item())


def shutdown():
    dist = _td()
    if dist.is_initialized():
        dist.destroy_process_group()
