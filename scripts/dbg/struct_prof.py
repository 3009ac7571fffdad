"""Phase timings (KBG_PROFILE_OPEN=1) of one structural update on a C3
resident session, as bench.py's resident_session step makes it."""
import ctypes
import os
import sys
import time

sys.path.insert(0, "kube-arbitrator_amd")
os.environ.setdefault("KBG_PROFILE_OPEN", "1")
from kbgpu import _abi, synth  # noqa: E402
from kbgpu.cache import FakeBinder, cache_from_fixture  # noqa: E402
from kbgpu.fixture import _OrderedCache, fixture_tiers  # noqa: E402
from kbgpu.framework import open_session  # noqa: E402

cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
fx = synth.config_fixture(cid)
ssn = open_session(_OrderedCache(cache_from_fixture(fx, FakeBinder()), fx), fixture_tiers(fx), {})
L = _abi.lib()
T = len(ssn.flat.task_objs)
buf = (_abi.kbg_decision * (T + 64))()
n = ctypes.c_int32(0)
_abi.check(L.kbg_allocate(ssn.handle, buf, T + 64, ctypes.byref(n)))
tasks = ssn.flat.arrays["tasks"]
nd0 = ssn.flat.arrays["nodes"][0]
for rep in range(3):
    spec = _abi.kbg_node_spec(f"prof-node-{rep}".encode(), None, 0, 0, None)
    evs = (_abi.kbg_event * 11)()
    evs[0].kind, evs[0].node_spec = _abi.EV_NODE_ADD, ctypes.pointer(spec)
    evs[0].resource = _abi.kbg_resource(*[float(x) for x in nd0["allocatable"]])
    evs[0].max_task_num = int(nd0["max_task_num"])
    name = f"prof/job-{rep}".encode()
    evs[1].kind, evs[1].name, evs[1].queue, evs[1].min_available = _abi.EV_JOB_ADD, name, 0, 8
    new_job = len(ssn.jobs)  # (each rep deletes one job and adds one: the count stays)
    keep = []
    for a in range(8):
        e = evs[2 + a]
        e.kind, e.job, e.spec, e.status, e.node = _abi.EV_POD_ADD, new_job, int(tasks[0]["spec"]), 1, -1
        e.resource = _abi.kbg_resource(*[float(x) for x in tasks[0]["resreq"]])
        keep += [f"prof-{rep}-{a}".encode(), f"prof/{rep}-{a}".encode()]
        e.uid, e.pod_key = keep[-2], keep[-1]
    evs[10].kind, evs[10].job = _abi.EV_JOB_DELETE, 0
    t0 = time.perf_counter()
    _abi.check(L.kbg_session_update(ssn.handle, evs, 11))
    print(f"structural update {rep}: {ssn.stats().update_ms:.3f} ms (wall {1e3 * (time.perf_counter() - t0):.3f})",
          flush=True)
ssn.close()
