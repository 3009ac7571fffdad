"""Structural events of kbg_session_update on the CPU (no device): nodes,
PodGroups and queues that join or leave (include/kbgpu.h KBG_EV_NODE_ADD ...
QUEUE_DELETE; event_handlers.go:232-268,344-381,635-654, cache.go:549-597).
The batch the Python wrapper marshals (framework.Session.marshal) is
prechecked and applied by the library's own host code through the tool
library (kube-arbitrator_amd/tools/engine_bench.cpp kbg_tool_structural),
and the updated snapshot the library would open from must equal the snapshot
of the Python cache mirror replayed through the same events, in the wrapper's
renumbered order: nodes (Idle, Releasing, pods and their keys, ports, labels,
taints), jobs and their tasks in JobInfo.Tasks order, queues, Others, and the
node copies of every pod. The GPU side (tests/test_update_gpu.py
test_update_structural*) checks the cycles after such updates."""
import ctypes
import os
import subprocess

import pytest

from helpers import ROOT, build_tools

PKG = os.path.join(ROOT, "kube-arbitrator_amd")
TOOLS = os.path.join(PKG, "tools", "libkbg_tools.so")


@pytest.fixture(scope="module")
def tools():
    build_tools()
    L = ctypes.CDLL(TOOLS)
    L.kbg_tool_structural.restype = ctypes.c_int32
    return L


def _replay(fx0, changes):
    from kbgpu.cache import FakeBinder, cache_from_fixture
    cache = cache_from_fixture(fx0, FakeBinder())
    pods = {p["uid"]: p for p in fx0["pods"]}
    for kind, obj in changes:
        if kind == "pod_add":
            cache.add_pod(obj)
            pods[obj["uid"]] = obj
        elif kind == "pod_update":
            cache.update_pod(pods[obj["uid"]], obj)
            pods[obj["uid"]] = obj
        elif kind == "pod_delete":
            cache.delete_pod(obj)
            pods.pop(obj["uid"], None)
        else:
            getattr(cache, {"node_add": "add_node", "node_update": "update_node", "node_delete": "delete_node",
                            "pod_group_add": "add_pod_group", "pod_group_delete": "delete_pod_group",
                            "queue_add": "add_queue", "queue_delete": "delete_queue"}[kind])(obj)
    return cache


def _view(cache, fx):
    """A framework.Session over the cache's snapshot without a device handle
    (what marshal / _renumber read)."""
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.framework import Session
    from kbgpu.snapshot import FlatSnapshot
    c = _OrderedCache(cache, fx)
    snap = c.snapshot()
    v = Session.__new__(Session)
    v.cache, v.jobs, v.nodes, v.queues, v.others = c, snap.jobs, snap.nodes, snap.queues, snap.others
    v.job_index = {j.uid: j for j in v.jobs}
    v.node_index = {n.name: n for n in v.nodes}
    v.queue_index = {q.uid: q for q in v.queues}
    v.flat = FlatSnapshot(v.nodes, v.jobs, v.queues, v.others, fixture_tiers(fx))
    return v


def _res(r):
    return (r.milli_cpu, r.memory, r.milli_gpu)


def canon(sn):
    """A kbg_snapshot by content (string ids resolved; ports canonical)."""
    S = [sn.strings[i].decode() for i in range(sn.n_strings)]

    def port(p):
        return (S[p.host_ip] or "0.0.0.0", S[p.protocol] or "TCP", p.host_port)
    task_uid = [S[sn.tasks[t].uid] for t in range(sn.n_tasks)]
    named, pod_only = [], []
    for i in range(sn.n_nodes):
        nd = sn.nodes[i]
        labels = sorted((S[sn.labels[2 * (nd.label_off + k)]], S[sn.labels[2 * (nd.label_off + k) + 1]])
                        for k in range(nd.label_len))
        taints = [(S[sn.taints[nd.taint_off + k].key], S[sn.taints[nd.taint_off + k].value],
                   S[sn.taints[nd.taint_off + k].effect]) for k in range(nd.taint_len)]
        ports = sorted(port(sn.ports[nd.port_off + k]) for k in range(nd.port_len))
        keys = [S[sn.node_pod_keys[nd.key_off + k]] for k in range(nd.key_len)]
        pods = [(_res(sn.node_pods[nd.key_off + k].resreq), sn.node_pods[nd.key_off + k].status)
                for k in range(nd.key_len)] if sn.n_node_pods else None
        mine = [task_uid[sn.node_tasks[nd.task_off + k]] for k in range(nd.task_len)]
        row = (S[nd.name], nd.has_node, _res(nd.allocatable), _res(nd.idle), _res(nd.releasing), nd.max_task_num,
               nd.num_tasks, nd.unschedulable, labels, taints, ports, keys, pods, mine)
        (named if S[nd.name] else pod_only).append(row)
    tasks_of = {}
    for t in range(sn.n_tasks):
        k = sn.tasks[t]
        tasks_of.setdefault(k.job, []).append((S[k.uid], k.status, k.priority, _res(k.resreq), S[k.node_name],
                                               S[k.pod_key]))
    jobs = [(S[sn.jobs[j].uid], S[sn.queues[sn.jobs[j].queue].uid], sn.jobs[j].min_available, sn.jobs[j].priority,
             sn.jobs[j].creation_ns, tasks_of.get(j, [])) for j in range(sn.n_jobs)]
    queues = [(S[sn.queues[q].uid], sn.queues[q].weight) for q in range(sn.n_queues)]
    others = sorted(_res(sn.others[i]) for i in range(sn.n_others))
    return {"nodes": named, "pod_only_nodes": sorted(pod_only, key=repr), "jobs": jobs, "queues": queues,
            "others": others}


def check(tools, fx0, changes_of):
    """Returns the library status of the batch (0: applied and compared)."""
    from kbgpu import _abi
    from kbgpu.api import RefPanic
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.snapshot import SnapshotBlob
    try:
        v = _view(cache_from_fixture(fx0, FakeBinder()), fx0)
    except RefPanic as e:
        pytest.skip(f"S0: the reference cache panics: {e}")
    changes = changes_of(v)
    try:
        plan = v.marshal(changes)
    except ValueError as e:  # the wrapper's documented re-open cases
        pytest.skip(f"needs a re-open: {e}")
    lens = (ctypes.c_int32 * 4)(len(v.flat.task_objs) + len(plan.objs) + 1, len(v.flat.node_names) + len(plan.new_nodes),
                                len(v.jobs) + len(plan.new_jobs), len(v.queues) + len(plan.new_queues))
    maps = [(ctypes.c_int32 * max(1, lens[k]))() for k in range(4)]
    ptrs = (ctypes.POINTER(ctypes.c_int32) * 4)(*[ctypes.cast(m, ctypes.POINTER(ctypes.c_int32)) for m in maps])
    n_out = ctypes.c_int64(0)
    cap = 1 << 22
    out = (ctypes.c_uint8 * cap)()
    rc = tools.kbg_tool_structural(ctypes.byref(v.flat.snap), ctypes.byref(_abi.kbg_options()), plan.evs, plan.n_ev,
                                   out, ctypes.c_int64(cap), ctypes.byref(n_out), ptrs, lens)
    if rc >= 100:  # a session on S0 does not open (e.g. proportion's panic at OnSessionOpen)
        pytest.skip(f"S0 does not open (status {rc - 100})")
    if rc == _abi.KBG_E_REF_PANIC:  # the cache itself panics applying the batch: so must the Python mirror
        with pytest.raises(RefPanic):
            _view(_replay(fx0, changes), fx0)
        return 0
    if rc != 0:
        return rc
    blob = SnapshotBlob.decode(bytes(out[:n_out.value]))
    got = canon(blob.snap)
    # the wrapper's renumbered lists, then the replayed cache in that order
    task_objs = v.flat.task_objs + [None] * (plan.n_objs - len(v.flat.task_objs))
    for i, ti in plan.objs.items():
        task_objs[i] = ti
    v._renumber(task_objs, plan.new_nodes, plan.new_jobs, plan.new_queues, plan.pod_only,
                maps=[list(maps[k][:lens[k]]) for k in range(4)])
    order = {"jobs": [j.uid for j in v.jobs], "nodes": [n for n in v.flat.node_names if n],
             "queues": [q.uid for q in v.queues]}
    try:
        ref = _view(_replay(fx0, changes), dict(fx0, sessionOrder=order))
    except RefPanic as e:
        pytest.skip(f"S1: the reference cache panics: {e}")
    want = canon(ref.flat.snap)
    if not blob.snap.n_node_pods:  # the library drops every copy when one is unknown
        for k in ("nodes", "pod_only_nodes"):
            want[k] = [r[:12] + (None,) + r[13:] for r in want[k]]
    assert got["queues"] == want["queues"]
    assert [j[0] for j in got["jobs"]] == [j[0] for j in want["jobs"]]
    for a, b in zip(got["jobs"], want["jobs"]):
        assert a == b, a[0]
    assert [n[0] for n in got["nodes"]] == [n[0] for n in want["nodes"]]
    for a, b in zip(got["nodes"], want["nodes"]):
        assert a == b, a[0]
    assert got["pod_only_nodes"] == want["pod_only_nodes"]
    assert got["others"] == want["others"]
    # the wrapper's task list follows the library's task order
    assert [t.uid for t in v.flat.task_objs] == [t[0] for j in got["jobs"] for t in j[5]]
    blob.close()
    return 0


def _structural(fx0, seed):
    from kbgpu import synth

    def changes_of(v):
        return synth.structural(fx0, seed, {j.uid for j in v.jobs}, {t.uid for t in v.flat.task_objs},
                                [q.uid for q in v.queues])
    return changes_of


@pytest.mark.parametrize("seed", range(80))
def test_structural_host_fuzz(tools, seed):
    from kbgpu import synth
    fx0 = synth.random_fixture(11000 + seed) if seed % 3 else synth.contended_fixture(11000 + seed, nodes=12, jobs=8,
                                                                                      tasks=6)
    assert check(tools, fx0, _structural(fx0, seed)) == 0


@pytest.mark.parametrize("seed", range(20))
def test_structural_host_ports(tools, seed):
    """Host-port pods on nodes that leave, and jobs whose pods stay on their
    nodes as pods outside the session jobs (their node copies and ports)."""
    from kbgpu import synth
    fx0 = synth.contended_fixture(11300 + seed, nodes=10, jobs=10, tasks=6, ports=0.5)
    assert check(tools, fx0, _structural(fx0, seed)) == 0


def test_structural_host_c1(tools):
    from kbgpu import synth
    fx0 = synth.config_fixture(1)

    def changes_of(v):
        ch = _structural(fx0, 41)(v)
        return [(k, o) for k, o in ch if k != "queue_delete"]
    assert check(tools, fx0, changes_of) == 0


def test_structural_host_refusals(tools):
    """A pod event after its job left in the same batch: KBG_E_UNSUPPORTED,
    before anything applies (the status the library returns)."""
    from kbgpu import _abi, synth
    fx0 = synth.contended_fixture(11400, nodes=8, jobs=6, tasks=4)

    def changes_of(v):
        j = v.jobs[0]
        t = next(iter(j.tasks.values()))
        pg = next(g for g in fx0["podGroups"] if f"{g.get('namespace', '')}/{g['name']}" == j.uid)
        return [("pod_group_delete", pg), ("pod_delete", t.pod)]
    assert check(tools, fx0, changes_of) == _abi.KBG_E_UNSUPPORTED
