"""The owner-resolve protocol of a sharded allocate (kbg_session.cpp
allocate_sharded) on the CPU: R ranks, each holding a
contiguous range of node rows, rank 0 running the ordering engine, one
broadcast of the batch, a sum-reduce of per-rank availability and min-reduce
rounds of packed winners — checked against the kbref oracle (decision log,
order, kinds, gang dispatch) and against each other (every rank returns the
same log).

Two transports drive the same protocol code: R threads in one process
(kbg_tool_sharded_allocate_local) and one rank per process over
torch.distributed gloo at world_size 2 (kbg_tool_sharded_allocate_rank, the
collectives are the test's callbacks). The device scan and select of each
rank's rows are replaced by a host walk of its mirror (tools/engine_bench.cpp
HostIO); the RCCL transport and the device scan are exercised on the GPU."""
import ctypes
import os
import subprocess

import pytest

from helpers import ROOT, run_oracle, build_tools

PKG = os.path.join(ROOT, "kube-arbitrator_amd")
TOOLS = os.path.join(PKG, "tools", "libkbg_tools.so")
COLL = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_uint32),
                        ctypes.c_int64)


def tools_lib():
    build_tools()
    L = ctypes.CDLL(TOOLS)
    L.kbg_tool_sharded_allocate_local.restype = ctypes.c_int32
    L.kbg_tool_sharded_allocate_rank.restype = ctypes.c_int32
    L.kbg_last_error.restype = ctypes.c_char_p
    return L


@pytest.fixture(scope="module")
def tools():
    return tools_lib()


def flat(fx):
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    s = _OrderedCache(cache_from_fixture(fx, FakeBinder()), fx).snapshot()
    return FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))


def options(opts):
    from kbgpu import _abi
    o = _abi.kbg_options()
    for k, v in opts.items():
        setattr(o, k, v)
    return o


def as_log(f, buf, n):
    from kbgpu import _abi
    tasks, names = f.task_objs, f.node_names
    return [{"task": tasks[buf[i].task].uid, "job": tasks[buf[i].task].job, "node": names[buf[i].node],
             "kind": "allocate" if buf[i].kind == _abi.KIND_ALLOCATE else "pipeline",
             "dispatched_at": buf[i].dispatched_at} for i in range(n)]


def run_local(tools, fx, R, opts):
    from kbgpu import _abi
    f = flat(fx)
    cap = max(1, sum(1 for t in f.task_objs)) + 1
    out = (_abi.kbg_decision * (cap * R))()
    n = (ctypes.c_int32 * R)()
    st = (ctypes.c_int64 * (5 * R))()
    rc = tools.kbg_tool_sharded_allocate_local(ctypes.byref(f.snap), ctypes.byref(options(opts)), R, out, cap, n, st)
    logs = []
    for r in range(R):
        base = ctypes.cast(ctypes.byref(out, r * cap * ctypes.sizeof(_abi.kbg_decision)),
                           ctypes.POINTER(_abi.kbg_decision))
        logs.append(as_log(f, base, n[r]))
    stats = [list(st[5 * r:5 * r + 5]) for r in range(R)]
    return rc, logs, stats


def check(tools, fx, R, opts):
    fx = dict(fx)
    fx.pop("actions", None)  # allocate only
    ref = run_oracle(fx)
    if ref["status"] not in ("ok", "ref_panic"):
        pytest.skip(ref["status"])
    from kbgpu.api import RefPanic
    try:
        rc, logs, stats = run_local(tools, fx, R, opts)
    except RefPanic:
        assert ref["status"] == "ref_panic"
        return None
    if rc == -2:  # KBG_E_UNSUPPORTED: pod affinity keeps the replicated resolve
        pytest.skip(tools.kbg_last_error().decode())
    if ref["status"] == "ref_panic":
        assert rc == -3, (rc, tools.kbg_last_error())
    else:
        assert rc == 0, (rc, tools.kbg_last_error())
    for r in range(1, R):
        assert logs[r] == logs[0], f"rank {r} log differs from rank 0"
    if ref["status"] != "ok":
        return stats
    rd = ref["decisions"]
    for i, (a, b) in enumerate(zip(rd, logs[0])):
        assert a == b, f"decision {i}: oracle {a} != sharded {b}"
    assert len(rd) == len(logs[0])
    return stats


@pytest.mark.parametrize("seed", range(40))
def test_owner_resolve_fuzz(tools, seed):
    from kbgpu import synth
    fx = synth.random_fixture(11000 + seed)
    R = 2 + seed % 3
    check(tools, fx, R, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 4, "full_scan": seed % 2})


@pytest.mark.parametrize("seed", range(16))
def test_owner_resolve_contended(tools, seed):
    """Near-full clusters: rows fail on the low ranks and move up, tasks fit
    nowhere (mispredictions cut the batch), Releasing (pipelines)."""
    from kbgpu import synth
    fx = synth.contended_fixture(12000 + seed, nodes=24, jobs=20, tasks=8)
    check(tools, fx, 2 + seed % 4, {"batch_tasks": 4 + seed % 13, "candidates": 1 + seed % 3, "full_scan": seed % 2})


@pytest.mark.parametrize("R", [2, 4, 8])
def test_owner_resolve_config1(tools, R):
    from kbgpu import synth
    stats = check(tools, synth.config_fixture(1), R, {})
    assert stats and stats[0][4] > 0  # task evaluations


@pytest.mark.parametrize("R,full", [(3, 0), (8, 1)])
def test_owner_resolve_config2(tools, R, full):
    """1k heterogeneous nodes, selectors, taints, 10k tasks over R ranks."""
    from kbgpu import synth
    stats = check(tools, synth.config_fixture(2), R, {"full_scan": full})
    assert stats and stats[0][0] >= stats[0][1]  # at least one round per batch


def _gloo_rank(rank, world, port, fx, opts, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from kbgpu import _abi
        L = tools_lib()
        f = flat(fx)

        def coll(_user, op, buf, n):
            t = torch.tensor([buf[i] for i in range(n)], dtype=torch.int64)
            if op == 0:
                dist.broadcast(t, src=0)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.MIN if op == 1 else dist.ReduceOp.SUM)
            for i, v in enumerate(t.tolist()):
                buf[i] = v & 0xffffffff
            return 0

        cb = COLL(coll)
        cap = len(f.task_objs) + 1
        out = (_abi.kbg_decision * cap)()
        n = ctypes.c_int32()
        st = (ctypes.c_int64 * 5)()
        rc = L.kbg_tool_sharded_allocate_rank(ctypes.byref(f.snap), ctypes.byref(options(opts)), world, rank, cb,
                                              None, out, cap, ctypes.byref(n), st)
        q.put((rank, rc, as_log(f, out, n.value), list(st)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("seed", [0, 1])
def test_owner_resolve_gloo_world2(seed):
    """Two processes, one rank each, the protocol's collectives over gloo."""
    import socket

    import torch.multiprocessing as mp
    from kbgpu import synth
    tools_lib()  # built before the ranks start
    fx = synth.config_fixture(1) if seed == 0 else synth.contended_fixture(13000, nodes=24, jobs=20, tasks=8)
    fx.pop("actions", None)
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    opts = {"batch_tasks": 64, "candidates": 2}
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, fx, opts, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, rc, log, st in res:
        assert rc == 0, (rank, rc)
        assert log == ref["decisions"], f"rank {rank}"
        assert st[0] >= st[1] >= 1  # rounds >= batches


@pytest.mark.parametrize("seed", range(24))
def test_owner_resolve_ports_and_dup_keys(tools, seed):
    """Host ports (class-mask bits cleared and restored by a rank's rollback)
    and colliding pod keys (a commit that leaves the node unchanged)."""
    from kbgpu import synth
    fx = (synth.contended_fixture(14000 + seed, nodes=16, jobs=16, tasks=8, ports=0.5) if seed % 2
          else synth.dupkey_fixture(seed))
    check(tools, fx, 2 + seed % 3, {"batch_tasks": 3 + seed % 11, "candidates": 1 + seed % 3, "full_scan": seed % 4 == 1})
