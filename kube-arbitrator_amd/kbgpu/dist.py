"""Multi-process plumbing for `bench.py --gpus N` (one process per GPU).

This round N > 1 runs independent replicas (one cluster per rank, weak
scaling): the only cross-rank traffic is the bench's own barrier and the
max-over-ranks wall time / sum-over-ranks placements reduction below.
Works with "nccl" (RCCL over xGMI) on MI355X and with "gloo" on CPU.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend):
    """Initialises the default process group from the torchrun environment."""
    rank, world, _ = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world)
    return dist.is_initialized()


def barrier():
    if dist.is_initialized():
        dist.barrier()


def aggregate(elapsed_s, decisions):
    """(max elapsed over ranks, total placements over ranks)."""
    if not dist.is_initialized():
        return elapsed_s, decisions
    dev = torch.device("cuda") if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    d = torch.tensor([float(decisions)], dtype=torch.float64, device=dev)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    return float(t.item()), int(d.item())


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
