"""Developer tool: the per-rank critical path of a node-axis
sharded allocate cycle at R = 1, 2, 4, 8 ranks — the scan service
(kbg_tool_svc_allocate_device, the default) or, with PROTOCOL=owner, the
owner-resolve protocol —
measured with R device sessions of ONE process on one MI355X (the in-process
host transport of tests/test_shard_device.py, kbg_tool_sharded_allocate_device_t:
rank r holds the node rows of words [r*Wl, (r+1)*Wl) and runs
kbg_firstfit_kernel over them; the collectives are a host barrier exchange
instead of RCCL). R = 1 runs the same protocol on one rank (KBG_OWNER_RESOLVE=1).
The R sessions share one GPU and the job's CPU quota, so a rank's times are
an upper bound of what it would take on a GPU of its own.
python kube-arbitrator_amd/tools/shard_paths.py [config] [R ...]"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

FIELDS = ["allocate_ms", "engine_ms", "resolve_ms", "device_ms", "exchange_ms"]


def main(cid, ranks):
    owner = os.environ.get("PROTOCOL", "svc") == "owner"
    if owner:
        os.environ["KBG_OWNER_RESOLVE"] = "1"  # (R = 1 runs the protocol too)
    from kbgpu import _abi, synth
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    L = ctypes.CDLL(os.environ.get("TOOLS_LIB", os.path.join(HERE, "libkbg_tools.so")))
    fn = L.kbg_tool_sharded_allocate_device_t if owner else L.kbg_tool_svc_allocate_device
    fn.restype = ctypes.c_int32
    L.kbg_last_error.restype = ctypes.c_char_p
    fx = synth.config_fixture(cid)
    s = _OrderedCache(cache_from_fixture(fx, FakeBinder()), fx).snapshot()
    f = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    cap = len(f.task_objs) + 1
    for R in ranks:
        out = (_abi.kbg_decision * (cap * R))()
        n = (ctypes.c_int32 * R)()
        st = (ctypes.c_int64 * (5 * R))()
        tm = (ctypes.c_int64 * (6 * R))()
        o = _abi.kbg_options()
        rc = fn(ctypes.byref(f.snap), ctypes.byref(o), R, 0, out, cap, n, st, tm, int(os.environ.get("CYCLES", "3")))
        if rc != 0:
            print(json.dumps({"config": cid, "R": R, "error": rc, "msg": L.kbg_last_error().decode()}), flush=True)
            continue
        per = []
        for r in range(R):
            d = {k: tm[6 * r + i] / 1e6 for i, k in enumerate(FIELDS)}
            d.update(rank=r, scan_launches=tm[6 * r + 5], owner_rounds=st[5 * r], batches=st[5 * r + 1],
                     mispredictions=st[5 * r + 2], task_evaluations=st[5 * r + 4], decisions=n[r])
            per.append(d)
        print(json.dumps({"config": cid, "R": R, "protocol": "owner" if owner else "svc",
                          "cycle_ms": max(p["allocate_ms"] for p in per), "ranks": per}),
              flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(int(a[0]) if a else 4, [int(x) for x in a[1:]] or [1, 2, 4, 8])
