"""The scan service of a node-axis sharded allocate (SURVEY §8e,
kbg_session.cpp allocate_svc_root / allocate_serve) with its device side on
the MI355X: R device sessions on device 0, rank r holding the node rows of
64-node words [r*Wl, (r+1)*Wl) (tools/engine_bench.cpp
kbg_tool_svc_allocate_device). Rank 0 runs the single-GPU pipeline; every scan
is a launch message each rank answers with kbg_firstfit_kernel over its own
words into the (slot, rank) info column and the [slot][W] masks, summed over
the ranks; the other ranks replay rank 0's commits. Only the transport is the
in-process hub instead of RCCL (RCCL refuses two ranks on one device). Every
rank's decision log must equal the oracle's (allocate.go:119-162)."""
import ctypes
import hashlib
import json

import pytest

from helpers import load_golden, run_oracle
from test_shard_protocol import as_log, flat, options, tools_lib

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import _abi, synth  # noqa: E402


@pytest.fixture(scope="module")
def tools():
    L = tools_lib()
    L.kbg_tool_svc_allocate_device.restype = ctypes.c_int32
    if _abi.lib().kbg_device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")
    return L


def run_svc(tools, fx, R, opts, cycles=1):
    f = flat(fx)
    cap = len(f.task_objs) + 1
    out = (_abi.kbg_decision * (cap * R))()
    n = (ctypes.c_int32 * R)()
    st = (ctypes.c_int64 * (5 * R))()
    rc = tools.kbg_tool_svc_allocate_device(ctypes.byref(f.snap), ctypes.byref(options(opts)), R, 0, out, cap, n, st,
                                            None, cycles)
    assert rc == 0, (rc, tools.kbg_last_error())
    logs = []
    for r in range(R):
        base = ctypes.cast(ctypes.byref(out, r * cap * ctypes.sizeof(_abi.kbg_decision)),
                           ctypes.POINTER(_abi.kbg_decision))
        logs.append(as_log(f, base, n[r]))
    for r in range(1, R):
        assert logs[r] == logs[0], f"rank {r} log differs from rank 0"
    return logs[0], [list(st[5 * r:5 * r + 5]) for r in range(R)]


@pytest.mark.parametrize("R", [2, 3, 4, 8])
@pytest.mark.parametrize("cid", [1, 2])
def test_svc_ranks_config_parity(tools, cid, R):
    fx = synth.config_fixture(cid)
    ref = run_oracle(fx)
    log, _ = run_svc(tools, fx, R, {"full_scan": cid % 2})
    assert log == ref["decisions"]


@pytest.mark.parametrize("R", [2, 4, 8])
def test_svc_ranks_saturated_digest(tools, R):
    """C3's cluster filling up mid-cycle (tests/golden/digest_saturated.json),
    two cycles on the reset sessions: mispredictions, contended rescans and
    reused lists all run on rank 0 with every scan served by the ranks."""
    ref = load_golden("digest_saturated.json")
    log, _ = run_svc(tools, synth.saturated_config(), R, {}, cycles=2)
    rows = [[d["task"], d["job"], d["node"], d["kind"], d["dispatched_at"], ""] for d in log]
    assert len(rows) == ref["n_decisions"]
    assert hashlib.sha256(json.dumps(rows, separators=(",", ":")).encode()).hexdigest() == ref["decisions"]


@pytest.mark.slow
@pytest.mark.parametrize("R", [4, 8])
def test_svc_ranks_config4_digest(tools, R):
    """C4 (20k nodes x 500k tasks, SURVEY §8(e)'s meaningful scaling point:
    2.5k nodes per rank at R = 8) through the scan service: the decision
    log's digest equals the oracle's (tests/golden/digest_c4.json)."""
    ref = load_golden("digest_c4.json")
    log, _ = run_svc(tools, synth.config_fixture(4), R, {})
    rows = [[d["task"], d["job"], d["node"], d["kind"], d["dispatched_at"], ""] for d in log]
    assert len(rows) == ref["n_decisions"]
    assert hashlib.sha256(json.dumps(rows, separators=(",", ":")).encode()).hexdigest() == ref["decisions"]


@pytest.mark.parametrize("seed", range(0, 48, 3))
def test_svc_ranks_fuzz(tools, seed):
    fx = synth.random_fixture(15000 + seed) if seed % 2 else \
        synth.contended_fixture(16000 + seed, nodes=200, jobs=40, tasks=12)
    fx.pop("actions", None)  # allocate only
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    R = 2 + seed % 7
    log, _ = run_svc(tools, fx, R, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 4,
                                    "full_scan": seed % 2})
    assert log == ref["decisions"]


@pytest.mark.parametrize("seed", range(0, 30, 3))
def test_svc_ranks_affinity(tools, seed):
    """Pod-affinity class-mask words written by rank 0's commits reach every
    rank's table with the next message."""
    fx = synth.affinity_fixture(seed)
    fx.pop("actions", None)
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    log, _ = run_svc(tools, fx, 2 + seed % 5, {"batch_tasks": 1 + seed % 7})
    assert log == ref["decisions"]


@pytest.mark.parametrize("seed", range(0, 24, 3))
def test_svc_ranks_host_ports(tools, seed):
    fx = synth.contended_fixture(8000 + seed, nodes=12, jobs=14, tasks=8, ports=0.4)
    fx.pop("actions", None)
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    log, _ = run_svc(tools, fx, 2 + seed % 3, {})
    assert log == ref["decisions"]
