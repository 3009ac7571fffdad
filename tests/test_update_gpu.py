"""Resident sessions (kbg_session_update, include/kbgpu.h): open(S0) +
update(events) + the cycle's actions must equal open(S1) + the same actions,
where S1 is the snapshot of the cache after the same events
(event_handlers.go:40-188: a pod update is delete + add, node-side AddTask /
RemoveTask by PodKey, SetNode on a node update). The fresh-open side is also
checked against the kbref oracle on S1."""
import ctypes

import pytest

from helpers import churn_chain, compare_digests, compare_outputs, digest_outputs, load_golden, run_oracle

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import _abi, synth  # noqa: E402
from kbgpu.cache import FakeBinder, cache_from_fixture  # noqa: E402
from kbgpu.fixture import _OrderedCache, fixture_tiers, run_fixture  # noqa: E402
from kbgpu.framework import open_session  # noqa: E402
from kbgpu.api import pod_key  # noqa: E402

ENTRY = {"allocate": "kbg_allocate", "backfill": "kbg_backfill", "reclaim": "kbg_reclaim", "preempt": "kbg_preempt"}


def _open(fx, opts=None):
    return open_session(_OrderedCache(cache_from_fixture(fx, FakeBinder()), fx), fixture_tiers(fx), opts or {})


def abi_cycle(ssn, actions):
    """The cycle's actions through the C ABI; results in run_fixture's schema
    (decisions, binds, job / queue / node state), without the host replay."""
    L = _abi.lib()
    cap = max(1, len(ssn.flat.task_objs))
    buf = (_abi.kbg_decision * cap)()
    n = ctypes.c_int32(0)
    status = "ok"
    for a in actions:
        code = getattr(L, ENTRY[a])(ssn.handle, buf, cap, ctypes.byref(n))
        if code == _abi.KBG_E_REF_PANIC:
            return {"status": "ref_panic"}
        if code == _abi.KBG_E_UNSUPPORTED:
            return {"status": "unsupported"}
        _abi.check(code)
    acts = (ctypes.c_int32 * cap)()
    m = ctypes.c_int32(0)
    _abi.check(L.kbg_decision_actions_get(ssn.handle, acts, cap, ctypes.byref(m)))
    tasks, names = ssn.flat.task_objs, ssn.flat.node_names
    out = {"status": status, "decisions": [], "binds": {}, "jobs": [], "queues": [], "nodes": []}
    for i in range(n.value):
        d = buf[i]
        row = {"task": tasks[d.task].uid, "job": tasks[d.task].job, "node": names[d.node],
               "kind": "allocate" if d.kind == _abi.KIND_ALLOCATE else "pipeline", "dispatched_at": d.dispatched_at}
        if acts[i] != 0:
            row["action"] = _abi.ACTION_NAMES[acts[i]]
        out["decisions"].append(row)
        if d.dispatched_at >= 0:
            out["binds"][pod_key(tasks[d.task].pod)] = names[d.node]
    for j, job in enumerate(ssn.jobs):
        st = ssn.job_state(j)
        row = {"uid": job.uid, "ready_num": st.ready_num, "ready": bool(st.ready), "drf_share": st.drf_share}
        if st.fit_valid:
            from kbgpu.fixture import fit_error
            row["fit_error"] = fit_error(st.fit_nodes, st.fit_cpu, st.fit_memory, st.fit_gpu)
        out["jobs"].append(row)
    for q, queue in enumerate(ssn.queues):
        st = ssn.queue_state(q)
        if st.has_attr:
            out["queues"].append({"uid": queue.uid, "share": st.share,
                                  "deserved": [st.deserved.milli_cpu, st.deserved.memory, st.deserved.milli_gpu]})
    for i, nd in enumerate(ssn.nodes):
        st = ssn.node_state(i)
        out["nodes"].append({"name": nd.name, "idle": [st.idle.milli_cpu, st.idle.memory, st.idle.milli_gpu],
                             "releasing": [st.releasing.milli_cpu, st.releasing.memory, st.releasing.milli_gpu],
                             "ntasks": st.num_tasks})
    return out


def check_update(fx0, seed, opts=None, rounds=1, strict=False):
    from kbgpu.api import RefPanic
    actions = fx0.get("actions") or ["allocate"]
    try:
        ssn = _open(fx0, opts)
    except RefPanic as e:  # the cache itself panics building S0 (Resource.Sub underflow)
        pytest.skip(f"S0: the reference cache panics: {e}")
    except _abi.KbgError as e:  # only the documented refusals skip; a device or input error fails the test
        if e.status not in ("ref_panic", "unsupported"):
            raise
        pytest.skip(f"S0 does not open ({e.status}, documented refusal): {e}")
    try:
        fx = dict(fx0, sessionOrder={"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names)})
        ref0 = run_oracle(fx)
        for r in range(rounds):
            uids = {t.uid for t in ssn.flat.task_objs}
            decided = ref0.get("decisions", []) if ref0["status"] == "ok" else []
            changes, fx1 = synth.churn(fx, seed * 31 + r, uids, decided)
            try:
                ssn.update(changes)
            except _abi.KbgError as e:
                if e.status == "unsupported" and not strict:  # a documented refusal (kbgpu.h kbg_session_update)
                    pytest.skip(f"update refused (unsupported, documented): {e}")
                if e.status != "ref_panic":
                    raise
                # the cache or the next session open panics: so must a fresh open of S1
                fresh, fssn = run_fixture(fx1, opts)
                assert fresh["status"] == "ref_panic", fresh
                return
            got = abi_cycle(ssn, actions)
            fresh, fssn = run_fixture(fx1, opts)
            ref1 = run_oracle(fx1)
            compare_outputs(ref1, fresh)  # the fresh open of S1 agrees with the oracle
            assert got["status"] == fresh["status"], (got, fresh.get("error"))
            if fresh["status"] == "ok":
                assert got["decisions"] == fresh["decisions"]
                assert got["binds"] == fresh["binds"]
                assert got["nodes"] == fresh["nodes"]
                for a, b in zip(got["jobs"], fresh["jobs"]):
                    assert (a["uid"], a["ready_num"], a["ready"], a.get("fit_error")) == \
                           (b["uid"], b["ready_num"], b["ready"], b.get("fit_error")), (a, b)
                    if "drf_share" in b:
                        assert a["drf_share"] == b["drf_share"]
                for a, b in zip(got["queues"], fresh["queues"]):
                    assert a["uid"] == b["uid"] and a["share"] == b["share"] and a["deserved"] == b["deserved"]
            if fssn:
                fssn.close()
            _abi.check(_abi.lib().kbg_session_reset(ssn.handle))
            fx, ref0 = fx1, ref1
    finally:
        ssn.close()


@pytest.mark.parametrize("seed", range(120))
def test_update_fuzz(seed):
    fx = synth.random_fixture(7000 + seed)
    check_update(fx, seed, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2},
                 rounds=2)


@pytest.mark.parametrize("seed", range(30))
def test_update_contended(seed):
    check_update(synth.contended_fixture(8000 + seed, nodes=20, jobs=16, tasks=8), seed, rounds=2)


@pytest.mark.parametrize("seed", range(30))
def test_update_host_ports(seed):
    """Churn on clusters whose pods use host ports: a pod with ports that
    completes, is deleted or moves takes its own entries out of the node's
    used ports (node.Pods() no longer lists it, vendor predicates.go:1031-1051),
    so a port another pod on the node still lists stays used. No refusal."""
    check_update(synth.contended_fixture(8200 + seed, nodes=12, jobs=16, tasks=8, ports=0.5), seed, rounds=3,
                 strict=True)


@pytest.mark.parametrize("seed", range(30))
def test_update_affinity(seed):
    check_update(synth.affinity_fixture(9000 + seed), seed, rounds=2)


@pytest.mark.parametrize("cid", [1, 2])
def test_update_configs(cid):
    check_update(synth.config_fixture(cid), cid, rounds=3)


def _same_cycle(got, fresh):
    """An updated session's cycle (abi_cycle) against a fresh open's (run_fixture)."""
    assert got["status"] == fresh["status"], (got, fresh.get("error"))
    if fresh["status"] != "ok":
        return
    assert got["decisions"] == fresh["decisions"]
    assert got["binds"] == fresh["binds"]
    assert got["nodes"] == fresh["nodes"]
    for a, b in zip(got["jobs"], fresh["jobs"]):
        assert (a["uid"], a["ready_num"], a["ready"], a.get("fit_error")) == \
               (b["uid"], b["ready_num"], b["ready"], b.get("fit_error")), (a, b)
        if "drf_share" in b:
            assert a["drf_share"] == b["drf_share"]
    for a, b in zip(got["queues"], fresh["queues"]):
        assert a["uid"] == b["uid"] and a["share"] == b["share"] and a["deserved"] == b["deserved"]


@pytest.mark.slow
@pytest.mark.parametrize("cid", [3, 4])
def test_update_chain_at_scale(cid):
    """BASELINE C3 (5k x 100k, over-requested queues) and C4 (20k x 500k) as
    resident sessions over 3 churn rounds (helpers.churn_chain: ~20-30k
    events per round at C3): each snapshot S_r opened fresh must match the
    oracle's digest of S_r (tests/golden/digest_c{3,4}_churn.json), and the
    session opened once at S_0 and updated round by round must make the same
    cycle as the fresh open of S_r."""
    ref = load_golden(f"digest_c{cid}_churn.json")["steps"]
    state = {}

    def run(fx, changes):
        fresh, fssn = run_fixture(fx)
        if fssn:
            fssn.close()
        if not changes:  # S_0: the resident session starts here
            state["ssn"] = _open(fx)
            got = abi_cycle(state["ssn"], ["allocate"])
        else:
            _abi.check(_abi.lib().kbg_session_reset(state["ssn"].handle))
            try:
                state["ssn"].update(changes)
                got = abi_cycle(state["ssn"], ["allocate"])
            except _abi.KbgError as e:
                assert e.status == "ref_panic", e
                got = {"status": "ref_panic"}
        _same_cycle(got, fresh)
        return fresh

    try:
        for r, changes, fx, out in churn_chain(synth.config_fixture(cid), cid, len(ref) - 1, run):
            compare_digests(ref[r], digest_outputs(out))
            assert len(changes) == ref[r]["events"]
    finally:
        if "ssn" in state:
            state["ssn"].close()


@pytest.mark.parametrize("seed", range(12))
def test_update_without_reset_restarts_the_table(seed):
    """An update right after a cycle's actions (no kbg_session_reset): the
    node rows the actions committed — bound or not, touched by an event or
    not — go back to the updated snapshot, so the next cycle equals a fresh
    open's. Events here: none, or completions that miss most decided nodes."""
    fx0 = synth.random_fixture(17000 + seed) if seed % 2 else synth.config_fixture(2 if seed % 4 == 0 else 1)
    fx0.pop("actions", None)
    ssn = _open(fx0)
    try:
        fx = dict(fx0, sessionOrder={"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names)})
        first = abi_cycle(ssn, ["allocate"])
        if first["status"] != "ok":
            pytest.skip(first["status"])
        changes = []
        if seed % 3:
            mine = {t.uid for t in ssn.flat.task_objs}  # session tasks (pods of a PodGroup)
            running = [p for p in fx["pods"] if p.get("phase") == "Running" and p["uid"] in mine]
            changes = [("pod_update", dict(p, phase="Succeeded")) for p in running[:2]]
        pods = {p["uid"]: p for p in fx["pods"]}
        for kind, p in changes:  # the cache's delete + add: an updated pod moves to the end
            pods.pop(p["uid"])
            pods[p["uid"]] = p
        fx1 = dict(fx, pods=list(pods.values()))
        try:
            ssn.update(changes)  # no reset: the cycle's commits are still in the device table
        except _abi.KbgError as e:  # refused before any event applied: the session is as it was
            assert e.status == "unsupported", e
            _abi.check(_abi.lib().kbg_session_reset(ssn.handle))
            assert abi_cycle(ssn, ["allocate"]) == first
            return
        got = abi_cycle(ssn, ["allocate"])
        fresh, fssn = run_fixture(fx1)
        _same_cycle(got, fresh)
        assert got["decisions"] == first["decisions"] or changes  # no events: the same cycle again
        if fssn:
            fssn.close()
    finally:
        ssn.close()


def test_refused_update_leaves_the_session_unchanged():
    """KBG_E_INVALID found before any event applies (a deleted task, an index
    out of range) leaves the session as it was; the same batch without the
    bad event then applies."""
    fx = synth.config_fixture(1)
    ssn = _open(fx)
    try:
        before = abi_cycle(ssn, ["allocate"])
        pods = [p for p in fx["pods"]][:3]
        good = [("pod_delete", pods[0]), ("pod_update", dict(pods[1], phase="Succeeded"))]
        L = _abi.lib()
        evs = (_abi.kbg_event * 3)()
        idx = {t.uid: i for i, t in enumerate(ssn.flat.task_objs)}
        evs[0].kind, evs[0].task = _abi.EV_POD_DELETE, idx[pods[0]["uid"]]
        evs[1].kind, evs[1].task = _abi.EV_POD_DELETE, idx[pods[0]["uid"]]  # deleted by the event before it
        evs[2].kind, evs[2].task, evs[2].status, evs[2].node = _abi.EV_POD_UPDATE, idx[pods[1]["uid"]], 1 << 7, -1
        assert L.kbg_session_update(ssn.handle, evs, 3) == _abi.KBG_E_INVALID
        _abi.check(L.kbg_session_reset(ssn.handle))
        assert abi_cycle(ssn, ["allocate"]) == before  # nothing was applied
        _abi.check(L.kbg_session_reset(ssn.handle))
        ssn.update(good)
        assert abi_cycle(ssn, ["allocate"])["status"] == "ok"
    finally:
        ssn.close()


@pytest.mark.parametrize("bad", ["null_label", "negative_taints", "null_taints", "other_name", "renamed_twice"])
def test_refused_node_set_leaves_the_session_unchanged(bad):
    """A malformed KBG_EV_NODE_SET after a valid event: refused (KBG_E_INVALID)
    before anything applies, so the session is as it was (kbgpu.h: an invalid
    event leaves the session unchanged); not marked broken."""
    import ctypes
    fx = synth.config_fixture(1)
    ssn = _open(fx)
    try:
        before = abi_cycle(ssn, ["allocate"])
        L = _abi.lib()
        idx = {t.uid: i for i, t in enumerate(ssn.flat.task_objs)}
        node = 3
        name = ssn.flat.node_names[node].encode()
        labels = (ctypes.c_char_p * 2)(b"zone", None if bad == "null_label" else b"z9")
        taints = (ctypes.c_char_p * 3)(b"k", b"v", b"NoSchedule")
        spec = _abi.kbg_node_spec(b"some-other-node" if bad == "other_name" else name, labels, 1,
                                  -1 if bad == "negative_taints" else 1,
                                  None if bad == "null_taints" else taints)
        evs = (_abi.kbg_event * 3)()
        evs[0].kind, evs[0].task = _abi.EV_POD_DELETE, idx[fx["pods"][0]["uid"]]
        evs[1].kind, evs[1].node, evs[1].node_spec = _abi.EV_NODE_SET, node, ctypes.pointer(spec)
        n = 2
        if bad == "renamed_twice":  # the batch's second NODE_SET names the node differently
            spec2 = _abi.kbg_node_spec(b"renamed", labels, 1, 1, taints)
            evs[2].kind, evs[2].node, evs[2].node_spec = _abi.EV_NODE_SET, node, ctypes.pointer(spec2)
            n = 3
        for e in evs[:n]:
            e.resource = _abi.kbg_resource(32000.0, 128.0 * 2**30, 0.0)
            e.max_task_num = 110
        assert L.kbg_session_update(ssn.handle, evs, n) == _abi.KBG_E_INVALID
        _abi.check(L.kbg_session_reset(ssn.handle))
        assert abi_cycle(ssn, ["allocate"]) == before  # nothing was applied, the session still works
    finally:
        ssn.close()


def check_changes(fx0, changes, fx1, opts=None):
    """open(S0) + update(changes) + the cycle's actions against open(S1) with
    the updated session's node and job order, and S1 against the oracle."""
    from kbgpu.api import RefPanic
    actions = fx0.get("actions") or ["allocate"]
    try:
        ssn = _open(fx0, opts)
    except RefPanic as e:  # the cache itself panics building S0 (Resource.Sub underflow)
        pytest.skip(f"S0: the reference cache panics: {e}")
    except _abi.KbgError as e:  # only the documented refusals skip; a device or input error fails the test
        if e.status not in ("ref_panic", "unsupported"):
            raise
        pytest.skip(f"S0 does not open ({e.status}, documented refusal): {e}")
    try:
        order = {"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names)}
        try:
            ssn.update(changes)
        except _abi.KbgError as e:
            if e.status != "ref_panic":
                raise
            # the cache's clone panics on the new Node: so must a fresh open of S1
            fresh, _ = run_fixture(dict(fx1, sessionOrder=order), opts)
            assert fresh["status"] == "ref_panic", fresh
            return {"status": "ref_panic"}
        got = abi_cycle(ssn, actions)
        fx1 = dict(fx1, sessionOrder={"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names)})
        fresh, fssn = run_fixture(fx1, opts)
        compare_outputs(run_oracle(fx1), fresh)
        assert got["status"] == fresh["status"], (got, fresh.get("error"))
        if fresh["status"] == "ok":
            assert got["decisions"] == fresh["decisions"]
            assert got["binds"] == fresh["binds"]
            assert got["nodes"] == fresh["nodes"]
            for a, b in zip(got["jobs"], fresh["jobs"]):
                assert (a["uid"], a["ready_num"], a["ready"], a.get("fit_error")) == \
                       (b["uid"], b["ready_num"], b["ready"], b.get("fit_error")), (a, b)
        if fssn:
            fssn.close()
        return got
    finally:
        ssn.close()


def _late_nodes(seed, k=2):
    """random_fixture with `k` nodes withheld: the Running pods on them make
    the cache create NodeInfo(nil) entries (event_handlers.go:49-53), whose
    Node then arrives (cache.AddNode -> SetNode)."""
    import copy
    import random
    fx = synth.random_fixture(seed, max_nodes=12)
    rng = random.Random(seed)
    held = {p["nodeName"] for p in fx["pods"] if p.get("nodeName") and p["phase"] == "Running"}
    late = [n for n in fx["nodes"] if n["name"] in held][:k]
    if not late:
        pytest.skip("no node holds a Running pod")
    for n in late:  # room for what its pods hold, so the clone does not panic
        n["allocatable"] = dict(n["allocatable"], cpu="64", memory="256Gi", pods="110")
    fx1 = copy.deepcopy(fx)
    fx0 = copy.deepcopy(fx)
    names = {n["name"] for n in late}
    fx0["nodes"] = [n for n in fx0["nodes"] if n["name"] not in names]
    rng.shuffle(late)
    return fx0, [("node_add", copy.deepcopy(n)) for n in late], fx1


@pytest.mark.parametrize("seed", range(40))
def test_update_node_set_pod_only(seed):
    """A node the cache knew only from its pods gets its Node (KBG_EV_NODE_SET):
    the node takes its name, labels, taints and Allocatable, its pods stop
    being allocated pods on a node outside the session, and the static
    predicate is recompiled — the same cycle as a fresh open of the cache
    with the node from the start."""
    fx0, changes, fx1 = _late_nodes(5000 + seed)
    got = check_changes(fx0, changes, fx1, {"batch_tasks": 1 + seed % 7})
    assert got["status"] in ("ok", "ref_panic")


def _with_pods(fx, changed):
    """fx's pods after the cache's delete + add of each changed pod (it moves to the end)."""
    pods = {p["uid"]: p for p in fx["pods"]}
    for p in changed:
        pods.pop(p["uid"], None)
        pods[p["uid"]] = p
    return dict(fx, pods=list(pods.values()))


@pytest.mark.parametrize("case", ["pod_only", "after_node_add", "bind_onto"])
@pytest.mark.parametrize("seed", range(12))
def test_update_pod_on_pod_only_node(seed, case):
    """Pod events naming a node the cache knows only from its pods
    (sc.Nodes[NodeName] = NewNodeInfo(nil), event_handlers.go:40-61): a
    Running pod there completes (it leaves that NodeInfo), the same after the
    node's Node arrived earlier in the batch (the batch's later events name it
    by its Node's name), or a Pending pod is bound onto it. open(S0) +
    update ≡ open(S1) ≡ the oracle on S1."""
    import copy
    fx0, adds, fx_full = _late_nodes(5100 + seed, k=1)
    late = adds[0][1]["name"]
    from kbgpu.api import RefPanic
    try:
        snap0 = cache_from_fixture(fx0, FakeBinder()).snapshot()
    except RefPanic as e:
        pytest.skip(f"S0: the reference cache panics: {e}")
    uids = {t.uid for j in snap0.jobs for t in j.tasks.values()}

    def session_pod(p):  # a pod of a job the snapshot keeps (the update names session tasks)
        return p["uid"] in uids
    on_late = [p for p in fx0["pods"] if p.get("nodeName") == late and p["phase"] == "Running" and session_pod(p)]
    if case == "bind_onto":
        pend = [p for p in fx0["pods"] if p["phase"] == "Pending" and not p.get("nodeName") and session_pod(p)]
        if not pend:
            pytest.skip("fixture without a Pending session pod to bind")
        p = dict(copy.deepcopy(pend[0]), nodeName=late, phase="Running")
    else:
        if not on_late:
            pytest.skip("fixture without a Running session pod on the late node")
        p = dict(copy.deepcopy(on_late[0]), phase="Succeeded")
    if case == "after_node_add":
        changes = [adds[0], ("pod_update", p)]
        fx1 = _with_pods(dict(fx0, nodes=fx0["nodes"] + [adds[0][1]]), [p])
        fx1 = dict(fx1, nodes=[n for n in fx_full["nodes"] if n["name"] in {x["name"] for x in fx1["nodes"]}])
    else:
        changes = [("pod_update", p)]
        fx1 = _with_pods(fx0, [p])
    got = check_changes(fx0, changes, fx1, {"batch_tasks": 1 + seed % 5})
    assert got["status"] in ("ok", "ref_panic")


@pytest.mark.parametrize("seed", range(24))
def test_update_node_relabel(seed):
    """UpdateNode with new labels and taints (isNodeInfoUpdated,
    event_handlers.go:242-259): selectors, node affinity and taint tolerations
    see the new Node after the update."""
    import copy
    import random
    fx0 = synth.random_fixture(6000 + seed)
    rng = random.Random(seed)
    fx1 = copy.deepcopy(fx0)
    changes = []
    for n in rng.sample(fx1["nodes"], min(3, len(fx1["nodes"]))):
        labels = dict(n.get("labels") or {})
        if labels and rng.random() < 0.5:
            labels.pop(rng.choice(sorted(labels)))
        labels[rng.choice(["zone", "disk", "tier"])] = rng.choice(["a", "b", "ssd", "x"])
        n["labels"] = labels
        if rng.random() < 0.5:
            n["taints"] = list(n.get("taints") or []) + [{"key": "maint", "value": "", "effect": "NoSchedule"}]
        elif n.get("taints"):
            n["taints"] = []
        changes.append(("node_update", copy.deepcopy(n)))
    check_changes(fx0, changes, fx1, {"batch_tasks": 1 + seed % 5})


def _replay(fx0, changes):
    """The cache of fx0 after `changes` (event_handlers.go): what a fresh open
    of the updated cache sees, including what a fixture cannot say (pods
    whose node was deleted, PodGroup-less jobs that still hold pods)."""
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


def _fixture_after(fx0, changes):
    """fx0 after `changes` as a fixture, or None when a fixture cannot say it:
    a deleted node that pods still name (a fresh cache would make a
    NodeInfo(nil) for them; the live one has none)."""
    pods = {p["uid"]: p for p in fx0["pods"]}
    nodes = {n["name"]: n for n in fx0["nodes"]}
    groups = {(g.get("namespace", ""), g["name"]): g for g in fx0.get("podGroups", [])}
    queues = {q["name"]: q for q in fx0.get("queues", [])}
    gone = set()
    for kind, o in changes:
        if kind in ("pod_add", "pod_update"):
            pods.pop(o["uid"], None)
            pods[o["uid"]] = o
        elif kind == "pod_delete":
            pods.pop(o["uid"], None)
        elif kind in ("node_add", "node_update"):
            nodes[o["name"]] = o
            gone.discard(o["name"])
        elif kind == "node_delete":
            nodes.pop(o["name"], None)
            gone.add(o["name"])
        elif kind == "pod_group_add":
            groups[(o.get("namespace", ""), o["name"])] = o
        elif kind == "pod_group_delete":
            groups.pop((o.get("namespace", ""), o["name"]), None)
        elif kind == "queue_add":
            queues[o["name"]] = o
        elif kind == "queue_delete":
            queues.pop(o["name"], None)
    if any(p.get("nodeName") in gone for p in pods.values()):
        return None
    return dict(fx0, pods=list(pods.values()), nodes=list(nodes.values()), podGroups=list(groups.values()),
                queues=list(queues.values()))


def check_structural(fx0, changes_of, opts=None):
    """open(S0) + update(structural changes) + the cycle's actions against a
    fresh open of the replayed cache in the updated session's order."""
    from kbgpu.api import RefPanic
    actions = fx0.get("actions") or ["allocate"]
    try:
        ssn = _open(fx0, opts)
    except RefPanic as e:
        pytest.skip(f"S0: the reference cache panics: {e}")
    except _abi.KbgError as e:
        if e.status not in ("ref_panic", "unsupported"):
            raise
        pytest.skip(f"S0 does not open ({e.status}, documented refusal): {e}")
    fssn = None
    try:
        changes = changes_of(ssn)
        try:
            ssn.update(changes)
        except ValueError as e:  # the wrapper's documented re-open cases (a PodGroup of pods outside the session)
            pytest.skip(f"update needs a re-open: {e}")
        except _abi.KbgError as e:
            if e.status == "unsupported":
                pytest.skip(f"update refused (unsupported, documented): {e}")
            assert e.status == "ref_panic", e
            return {"status": "ref_panic"}
        got = abi_cycle(ssn, actions)
        order = {"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names),
                 "queues": [q.uid for q in ssn.queues]}
        try:
            fssn = open_session(_OrderedCache(_replay(fx0, changes), {"sessionOrder": order}), fixture_tiers(fx0),
                                opts or {})
        except RefPanic:
            assert got["status"] == "ref_panic", got
            return got
        assert [j.uid for j in fssn.jobs] == order["jobs"]
        assert [q.uid for q in fssn.queues] == order["queues"]
        assert [t.uid for t in fssn.flat.task_objs] == [t.uid for t in ssn.flat.task_objs]
        fresh = abi_cycle(fssn, actions)
        assert got == fresh
        fx1 = _fixture_after(fx0, changes)
        if fx1 is not None and not fx0.get("namespaces"):  # also pinned to the oracle on S1
            fx1 = dict(fx1, sessionOrder=order)
            out, fs = run_fixture(fx1, opts)
            try:
                compare_outputs(run_oracle(fx1), out)
                if out["status"] == "ok":
                    assert got["decisions"] == out["decisions"] and got["binds"] == out["binds"]
            finally:
                if fs:
                    fs.close()
        return got
    finally:
        ssn.close()
        if fssn:
            fssn.close()


@pytest.mark.parametrize("seed", range(60))
def test_update_structural(seed):
    """Nodes, PodGroups and queues that join or leave (KBG_EV_NODE_ADD ...
    QUEUE_DELETE, event_handlers.go:232-268,344-381,635-654): the session is
    renumbered (kbg_session_renumbering) and its next cycle equals a fresh
    open of the cache after the same events."""
    fx0 = synth.random_fixture(11000 + seed) if seed % 3 else synth.contended_fixture(11000 + seed, nodes=12, jobs=8,
                                                                                      tasks=6)

    def changes_of(ssn):
        return synth.structural(fx0, seed, {j.uid for j in ssn.jobs}, {t.uid for t in ssn.flat.task_objs},
                                [q.uid for q in ssn.queues])
    opts = {"batch_tasks": 1 + seed % 7, "full_scan": seed % 2, "shards": 1 + seed % 3}  # (in-process node shards)
    check_structural(fx0, changes_of, opts)


@pytest.mark.parametrize("seed", range(6))
def test_update_structural_chain(seed):
    """Structural and pod churn over several updates of one session: each
    round's cycle equals a fresh open of the replayed cache."""
    fx0 = synth.contended_fixture(11500 + seed, nodes=16, jobs=10, tasks=6)
    ssn = _open(fx0)
    changes_all = []
    try:
        for r in range(3):
            ch = synth.structural(fx0, 100 * seed + r, {j.uid for j in ssn.jobs},
                                  {t.uid for t in ssn.flat.task_objs}, [q.uid for q in ssn.queues])
            # (new names carry the round's seed: unique over the chain)
            try:
                ssn.update(ch)
            except (ValueError, _abi.KbgError) as e:
                if isinstance(e, _abi.KbgError) and e.status not in ("unsupported", "ref_panic"):
                    raise
                pytest.skip(f"round {r}: {e}")
            changes_all += ch
            got = abi_cycle(ssn, ["allocate"])
            order = {"jobs": [j.uid for j in ssn.jobs], "nodes": list(ssn.flat.node_names),
                     "queues": [q.uid for q in ssn.queues]}
            fssn = open_session(_OrderedCache(_replay(fx0, changes_all), {"sessionOrder": order}),
                                fixture_tiers(fx0), {})
            try:
                assert got == abi_cycle(fssn, ["allocate"]), r
            finally:
                fssn.close()
            _abi.check(_abi.lib().kbg_session_reset(ssn.handle))
    finally:
        ssn.close()


@pytest.mark.parametrize("cid", [1, pytest.param(3, marks=pytest.mark.slow)])
def test_update_structural_configs(cid):
    """BASELINE C1 and C3 with structural events: the rebuild from the
    session's own updated snapshot (update_ms reported) against a fresh open
    of the replayed cache."""
    fx0 = synth.config_fixture(cid)

    def changes_of(ssn):
        ch = synth.structural(fx0, 40 + cid, {j.uid for j in ssn.jobs}, {t.uid for t in ssn.flat.task_objs},
                              [q.uid for q in ssn.queues])
        return [(k, o) for k, o in ch if k != "queue_delete" or len(ssn.queues) > 1]  # (C1: one queue)
    got = check_structural(fx0, changes_of)
    assert got["status"] == "ok"


def test_refused_structural_leaves_the_session_unchanged():
    """Invalid structural events (a NODE_ADD of a name the session holds, a
    JOB_ADD into a queue the batch deleted, a pod event after its job left in
    the same batch) are refused before anything applies."""
    fx = synth.config_fixture(1)
    ssn = _open(fx)
    try:
        before = abi_cycle(ssn, ["allocate"])
        L = _abi.lib()
        name = ssn.flat.node_names[0].encode()
        spec = _abi.kbg_node_spec(name, None, 0, 0, None)
        evs = (_abi.kbg_event * 2)()
        evs[0].kind, evs[0].node_spec = _abi.EV_NODE_ADD, ctypes.pointer(spec)
        assert L.kbg_session_update(ssn.handle, evs, 1) == _abi.KBG_E_INVALID
        evs[0] = _abi.kbg_event(kind=_abi.EV_QUEUE_DELETE, queue=0)
        evs[1] = _abi.kbg_event(kind=_abi.EV_JOB_ADD, name=b"ns/new", queue=0)
        assert L.kbg_session_update(ssn.handle, evs, 2) == _abi.KBG_E_INVALID
        t = 0
        j = ssn.flat.job_index[ssn.flat.task_objs[t].job]
        evs[0] = _abi.kbg_event(kind=_abi.EV_JOB_DELETE, job=j)
        evs[1] = _abi.kbg_event(kind=_abi.EV_POD_DELETE, task=t)
        assert L.kbg_session_update(ssn.handle, evs, 2) == _abi.KBG_E_UNSUPPORTED
        n = ctypes.c_int32(-1)
        _abi.check(L.kbg_session_renumbering(ssn.handle, _abi.RENUM_TASKS, None, 0, ctypes.byref(n)))
        assert n.value == 0
        _abi.check(L.kbg_session_reset(ssn.handle))
        assert abi_cycle(ssn, ["allocate"]) == before
    finally:
        ssn.close()
