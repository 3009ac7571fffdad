"""The host transport of a sharded session's communicator (kbg_comm.cpp
HostColl, kbgpu.h kbg_comm_init_host) across real processes, on the CPU.

Each rank is its own Python process that loads the developer tool library and
runs kbg_tool_hostcomm_selftest over host buffers: broadcast, sum / min / max
all-reduce and all-gather, each result checked on the rank against its closed
form, with payloads past the 4 MB staging chunk. The failure cases are the
ones a multi-rank protocol depends on: a rank that exits mid-protocol (fault
injection KBG_HOST_COMM_EXIT_AFTER), a peer that never joins (time limit),
ranks that disagree on the clique size, and a stale segment name — every
surviving rank must return KBG_E_RCCL / KBG_E_INVALID promptly instead of
hanging. The same transport under the device protocols (scan service,
replicated scans, victim scans) is tests/test_scan_service_procs.py (GPU)."""
import os
import subprocess
import sys
import time
import uuid

import pytest

from helpers import ROOT
from test_shard_protocol import tools_lib

PKG = os.path.join(ROOT, "kube-arbitrator_amd")
TOOLS = os.path.join(PKG, "tools", "libkbg_tools.so")

RANK = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
L.kbg_tool_hostcomm_selftest.restype = ctypes.c_int32
L.kbg_tool_hostcomm_selftest.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                         ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
L.kbg_last_error.restype = ctypes.c_char_p
ops = ctypes.c_int64(0)
rc = L.kbg_tool_hostcomm_selftest(sys.argv[2].encode(), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]),
                                  int(sys.argv[6]), ctypes.byref(ops))
print(rc, ops.value, L.kbg_last_error().decode(), flush=True)
"""


@pytest.fixture(scope="module", autouse=True)
def _tools():
    tools_lib()  # builds libkbg_tools.so


def launch(R, n, iters, env_of=lambda r: {}, ranks=None, name=None):
    name = name or f"t{os.getpid()}-{uuid.uuid4().hex[:12]}"
    procs = []
    for r in (range(R) if ranks is None else ranks):
        env = dict(os.environ, **env_of(r))
        procs.append(subprocess.Popen([sys.executable, "-c", RANK, TOOLS, name, str(R), str(r), str(n), str(iters)],
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True))
    return procs


def collect(procs, timeout=60):
    out = []
    for p in procs:
        try:
            so, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung")
        line = so.strip().splitlines()[-1] if so.strip() else ""
        parts = line.split(" ", 2)
        out.append((p.returncode, int(parts[0]) if parts and parts[0].lstrip("-").isdigit() else None,
                    int(parts[1]) if len(parts) > 1 and parts[1].isdigit() else None, parts[2] if len(parts) > 2 else so))
    return out


@pytest.mark.parametrize("R,n", [(2, 1000), (3, 77), (4, 300_000), (2, 1_500_000), (8, 4096)])
def test_collectives_across_processes(R, n):
    """Every collective's result equals its closed form on every rank;
    1.5M words per rank crosses the 4 MB chunk boundary."""
    res = collect(launch(R, n, 3))
    for r, (code, rc, ops, msg) in enumerate(res):
        assert code == 0 and rc == 0, (r, code, rc, msg)
        assert ops == 3 * 5, (r, ops)


def test_rank_exit_mid_protocol_fails_peers_promptly():
    """Rank 1 exits inside its 7th collective (fault injection): ranks 0 and 2
    return KBG_E_RCCL (5) naming the rank that left, well within the limit."""
    t0 = time.time()
    res = collect(launch(3, 5000, 4, env_of=lambda r: {"KBG_HOST_COMM_EXIT_AFTER": "7"} if r == 1 else
                         {"KBG_COMM_TIMEOUT_MS": "60000"}))
    assert time.time() - t0 < 30
    assert res[1][0] == 3  # the injected exit
    for r in (0, 2):
        code, rc, ops, msg = res[r]
        assert code == 0 and rc == -5, (r, res[r])
        assert ops == 6 and ("rank 1 exited or left" in msg or "aborted it" in msg), (r, res[r])


def test_root_exit_fails_servers():
    """The root (rank 0, which broadcasts) dies: every other rank errors out."""
    res = collect(launch(4, 2000, 4, env_of=lambda r: {"KBG_HOST_COMM_EXIT_AFTER": "3"} if r == 0 else {}))
    assert res[0][0] == 3
    for r in (1, 2, 3):  # the first rank to notice aborts the clique; the others may see that first
        assert res[r][1] == -5 and ("rank 0 exited or left" in res[r][3] or "aborted it" in res[r][3]), res[r]


def test_missing_peer_times_out():
    """A clique of 2 whose second rank never joins: the join gives up at
    KBG_COMM_TIMEOUT_MS with KBG_E_RCCL."""
    t0 = time.time()
    res = collect(launch(2, 10, 1, env_of=lambda r: {"KBG_COMM_TIMEOUT_MS": "1500"}, ranks=[0]))
    assert res[0][1] == -5 and "no progress" in res[0][3], res[0]
    assert time.time() - t0 < 20


def test_ranks_disagree_on_size():
    name = f"t{os.getpid()}-{uuid.uuid4().hex[:12]}"
    a = launch(2, 10, 1, env_of=lambda r: {"KBG_COMM_TIMEOUT_MS": "3000"}, ranks=[0], name=name)
    time.sleep(0.5)
    b = launch(3, 10, 1, env_of=lambda r: {"KBG_COMM_TIMEOUT_MS": "3000"}, ranks=[1], name=name)
    rb = collect(b)[0]
    assert rb[1] == -1 and "disagree" in rb[3], rb  # KBG_E_INVALID
    ra = collect(a)[0]
    assert ra[1] == -5, ra  # its peer never joined


def test_duplicate_rank_refused():
    name = f"t{os.getpid()}-{uuid.uuid4().hex[:12]}"
    a = launch(2, 10, 1, env_of=lambda r: {"KBG_COMM_TIMEOUT_MS": "3000"}, ranks=[0], name=name)
    time.sleep(0.5)
    b = launch(2, 10, 1, ranks=[0], name=name)
    rb = collect(b)[0]
    assert rb[1] == -1 and "already joined" in rb[3], rb
    assert collect(a)[0][1] == -5


def test_segment_is_unlinked_after_join():
    name = f"t{os.getpid()}-{uuid.uuid4().hex[:12]}"
    res = collect(launch(2, 10, 1, name=name))
    assert all(r[1] == 0 for r in res), res
    assert not os.path.exists(f"/dev/shm/kbg.{name}")
