"""One rank of a multi-process sharded session (tests/test_scan_service_procs.py).

    python tests/svc_procs_worker.py NAME R RANK CASES.json OUT.json

Joins the host-transport communicator NAME (kbgpu.dist.HostComm, kbgpu.h
kbg_comm_init_host) as rank RANK of R on device 0, then runs every case of
CASES.json through the product path — kbg_session_open_sharded and the
fixture's actions (kbgpu.fixture.run_fixture) — in lockstep with the other
ranks, and writes each case's outputs (or their digest) to OUT.json. This
process owns one device session, exactly like one GPU's rank of
`bench.py --gpus N`; only the transport under the collectives differs.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))

from kbgpu import _abi, synth  # noqa: E402
from kbgpu.actions import decision_list  # noqa: E402
from kbgpu.digest import digest_outputs  # noqa: E402
from kbgpu.dist import HostComm  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402


def make_fixture(c):
    g, a = c["gen"], c.get("arg")
    if g == "config":
        fx = synth.config_fixture(a)
    elif g == "saturated":
        fx = synth.saturated_config()
    elif g == "random":
        fx = synth.random_fixture(a)
    elif g == "contended":
        fx = synth.contended_fixture(a, **c.get("kw", {}))
    elif g == "affinity":
        fx = synth.affinity_fixture(a)
    else:
        raise ValueError(g)
    if c.get("allocate_only"):
        fx.pop("actions", None)
    return fx


def again(ssn, cap):
    """kbg_session_reset and one more allocate: its raw decision log."""
    L = _abi.lib()
    _abi.check(L.kbg_session_reset(ssn.handle))
    buf = (_abi.kbg_decision * cap)()
    n = ctypes.c_int32(0)
    code = L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n))
    if code not in (_abi.KBG_OK, _abi.KBG_E_REF_PANIC):
        _abi.check(code)
    return decision_list(buf, n.value)


def main():
    name, R, rank, cases_path, out_path = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    with open(cases_path) as f:
        cases = json.load(f)
    comm = HostComm(name, rank, R, device=0)
    n, r = comm.ranks()
    assert (n, r) == (R, rank), (n, r)
    results = []
    for c in cases:
        t0 = time.time()
        fx = make_fixture(c)
        rec = {"id": c["id"]}
        try:
            got, ssn = run_fixture(fx, dict(c.get("opts", {}), comm=comm))
        except _abi.KbgError as e:
            got, ssn = {"status": e.status, "error": str(e)}, None
        if ssn is not None:
            st = ssn.stats()
            rec["stats"] = {"shards": st.shards, "shard_index": st.shard_index, "scan_launches": st.scan_launches,
                            "owner_rounds": st.owner_rounds, "allocate_ms": st.allocate_ms}
            if got["status"] == "ok" and c.get("cycles", 1) > 1:
                first = list(ssn.decisions)
                rec["cycles_equal"] = all(again(ssn, max(1, ssn.flat.pending_all)) == first
                                          for _ in range(c["cycles"] - 1))
            ssn.close()
        rec["out"] = digest_outputs(got) if c.get("digest") else got
        rec["s"] = round(time.time() - t0, 3)
        results.append(rec)
        print(f"rank {rank}: {c['id']} {got['status']} {rec['s']} s", flush=True)
    comm.close()
    with open(out_path, "w") as f:
        json.dump(results, f)


if __name__ == "__main__":
    main()
