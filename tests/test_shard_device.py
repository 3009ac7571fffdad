"""The owner-resolve protocol of a node-axis sharded allocate (SURVEY §8e,
kbg_session.cpp allocate_sharded) with its device side on the MI355X: R real
device sessions on device 0, rank r holding the node rows of 64-node words
[r*Wl, (r+1)*Wl) (tools/engine_bench.cpp kbg_tool_sharded_allocate_device).
Every rank but 0 starts at a word w_lo > 0, so kbg_firstfit_kernel over its
own words [w_lo, w_hi), with its availability bit 1 << r per shape, runs
exactly as on rank r of an R-GPU clique; only the collectives are the
in-process hub instead of RCCL (RCCL refuses two ranks on one device).
First-fit is the global minimum index (allocate.go:119-162): every rank's
decision log must equal the oracle's."""
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
    L.kbg_tool_sharded_allocate_device.restype = ctypes.c_int32
    if _abi.lib().kbg_device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")
    return L


def run_device(tools, fx, R, opts):
    f = flat(fx)
    cap = len(f.task_objs) + 1
    out = (_abi.kbg_decision * (cap * R))()
    n = (ctypes.c_int32 * R)()
    st = (ctypes.c_int64 * (5 * R))()
    rc = tools.kbg_tool_sharded_allocate_device(ctypes.byref(f.snap), ctypes.byref(options(opts)), R, 0, out, cap, n,
                                                st)
    assert rc == 0, (rc, tools.kbg_last_error())
    logs = []
    for r in range(R):
        base = ctypes.cast(ctypes.byref(out, r * cap * ctypes.sizeof(_abi.kbg_decision)),
                           ctypes.POINTER(_abi.kbg_decision))
        logs.append(as_log(f, base, n[r]))
    for r in range(1, R):
        assert logs[r] == logs[0], f"rank {r} log differs from rank 0"
    return logs[0], [list(st[5 * r:5 * r + 5]) for r in range(R)]


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("cid", [1, 2])
def test_device_ranks_config_parity(tools, cid, R):
    fx = synth.config_fixture(cid)
    ref = run_oracle(fx)
    log, stats = run_device(tools, fx, R, {"full_scan": cid % 2})
    assert log == ref["decisions"]
    assert stats[0][0] >= stats[0][1] > 0  # owner rounds >= batches


@pytest.mark.parametrize("R", [2, 4, 8])
def test_device_ranks_saturated_digest(tools, R):
    """C3's cluster filling up mid-cycle: rows fail on the low ranks and move
    up, unpredicted failures cut batches (tests/golden/digest_saturated.json)."""
    ref = load_golden("digest_saturated.json")
    log, stats = run_device(tools, synth.saturated_config(), R, {})
    rows = [[d["task"], d["job"], d["node"], d["kind"], d["dispatched_at"], ""] for d in log]
    assert len(rows) == ref["n_decisions"]
    assert hashlib.sha256(json.dumps(rows, separators=(",", ":")).encode()).hexdigest() == ref["decisions"]
    assert stats[0][2] > 0  # mispredictions: the speculation machinery ran across ranks


@pytest.mark.parametrize("seed", range(0, 48, 3))
def test_device_ranks_fuzz(tools, seed):
    fx = synth.random_fixture(15000 + seed) if seed % 2 else \
        synth.contended_fixture(16000 + seed, nodes=200, jobs=40, tasks=12)
    fx.pop("actions", None)  # allocate only
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    R = 2 + seed % 7
    log, _ = run_device(tools, fx, R, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 4,
                                       "full_scan": seed % 2})
    assert log == ref["decisions"]
