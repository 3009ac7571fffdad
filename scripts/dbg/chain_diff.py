"""Debug: structural chain round-by-round diff (tests/test_update_gpu.py chain)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, "kube-arbitrator_amd")
from test_update_gpu import _open, _replay, abi_cycle  # noqa
from kbgpu import synth, _abi  # noqa
from kbgpu.fixture import _OrderedCache, fixture_tiers  # noqa
from kbgpu.framework import open_session  # noqa

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
fx0 = synth.contended_fixture(11500 + seed, nodes=16, jobs=10, tasks=6)
ssn = _open(fx0)
allc = []
for r in range(3):
    ch = synth.structural(fx0, 100 * seed + r, {j.uid for j in ssn.jobs}, {t.uid for t in ssn.flat.task_objs},
                          [q.uid for q in ssn.queues])
    print("round", r, [(k, o.get("name")) for k, o in ch])
    ssn.update(ch)
    allc += ch
    got = abi_cycle(ssn, ["allocate"])
    order = {"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names), "queues": [q.uid for q in ssn.queues]}
    f = open_session(_OrderedCache(_replay(fx0, allc), {"sessionOrder": order}), fixture_tiers(fx0), {})
    fr = abi_cycle(f, ["allocate"])
    print(" jobs", [j.uid for j in f.jobs] == order["jobs"], "tasks",
          [t.uid for t in f.flat.task_objs] == [t.uid for t in ssn.flat.task_objs],
          "nodes", list(f.flat.node_names) == order["nodes"], "queues", [q.uid for q in f.queues] == order["queues"])
    print(" others", len(f.others), "S1 tasks", len(f.flat.task_objs))
    for k in got:
        if got[k] != fr[k]:
            a, b = got[k], fr[k]
            if isinstance(a, list):
                for i, (x, y) in enumerate(zip(a, b)):
                    if x != y:
                        print("  ", k, i, "got", x, "\n      fresh", y)
                if len(a) != len(b):
                    print("  ", k, "len", len(a), len(b))
            else:
                print("  ", k, a, b)
    f.close()
    _abi.check(_abi.lib().kbg_session_reset(ssn.handle))
