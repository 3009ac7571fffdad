"""Parity of the MI355X path against the kbref oracle (run on the GPU box).

Decisions must be bit-exact (task -> node, Allocate/Pipeline kind, order,
gang dispatch); drf/proportion shares within 1e-12 relative.
"""
import copy
import glob
import os

import pytest

from helpers import GOLDEN, compare_outputs, load_golden, run_oracle

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import synth  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402


def device_available():
    from kbgpu import _abi
    return _abi.lib().kbg_device_count() > 0


@pytest.fixture(scope="module", autouse=True)
def _need_device():
    if not device_available():
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")


@pytest.mark.parametrize("case", ["ref_allocate_case1", "ref_allocate_case2"])
def test_reference_allocate_cases(case):
    """pkg/scheduler/actions/allocate/allocate_test.go:140-300, through the device path."""
    fx = load_golden(case + ".json")
    got, ssn = run_fixture(fx)
    assert got["status"] == "ok"
    assert got["binds"] == fx["expected"]["binds"]
    compare_outputs(run_oracle(fx), got)
    ssn.close()


KATS = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "kat_*.json")))


@pytest.mark.parametrize("name", KATS)
def test_kats_through_device(name):
    """Every hand-derived KAT session through the device path, against the
    oracle (which tests/test_oracle_golden.py pins to the KAT's expectations)."""
    fx = load_golden(name)
    if fx.get("kind", "session") != "session":
        pytest.skip("data-model KAT")
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if "decisions" in fx.get("expected", {}) and got["status"] == "ok":
        assert [(d["task"], d["node"], d["kind"]) for d in got["decisions"]] \
            == [tuple(x) for x in fx["expected"]["decisions"]]
    if ssn:
        ssn.close()


def test_allocate_like_reference_test():
    """The allocate_test.go harness, verbatim in shape: cache -> OpenSession -> Execute -> binds."""
    from kbgpu import actions, framework
    from kbgpu.cache import FakeBinder, SchedulerCache
    from kbgpu.conf import PluginOption, Tier

    def res(cpu, mem):
        return {"cpu": cpu, "memory": mem, "nvidia.com/gpu": "0"}

    def pod(ns, n):
        return {"uid": f"{ns}-{n}", "namespace": ns, "name": n, "phase": "Pending",
                "annotations": {"scheduling.k8s.io/group-name": "pg1" if ns == "c1" else "pg2"},
                "containers": [{"requests": res("1", "1G")}]}

    binder = FakeBinder()
    cache = SchedulerCache(binder=binder)
    cache.add_node({"name": "n1", "allocatable": res("2", "4G")})
    for ns in ("c1", "c2"):
        for n in ("p1", "p2"):
            cache.add_pod(pod(ns, n))
    cache.add_pod_group({"namespace": "c1", "name": "pg1"})
    cache.add_pod_group({"namespace": "c2", "name": "pg2"})
    cache.add_queue({"name": "c1", "weight": 1})
    cache.add_queue({"name": "c2", "weight": 1})
    ssn = framework.open_session(cache, [Tier([PluginOption("drf"), PluginOption("proportion")])])
    actions.new().execute(ssn)
    framework.close_session(ssn)
    assert binder.binds == {"c2/p1": "n1", "c1/p1": "n1"}


@pytest.mark.parametrize("cid", [1, 2])
def test_config_parity(cid):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("actions", [None, ["reclaim", "allocate", "backfill", "preempt"]])
@pytest.mark.parametrize("full_scan", [0, 1])
def test_zero_nodes(actions, full_scan):
    """A session without nodes and with pending tasks: every task fails with
    "0 nodes are available" (job_info.go:329-358). The fused kernel gets no
    words to walk and must read neither the node table nor the class masks."""
    fx = synth.config_fixture(1)
    fx["nodes"] = []
    if actions:
        fx["actions"] = actions
    got, ssn = run_fixture(fx, {"full_scan": full_scan})
    compare_outputs(run_oracle(fx), got)
    assert got["decisions"] == []
    if ssn:
        ssn.close()


@pytest.mark.parametrize("opts", [
    {"batch_tasks": 1, "candidates": 1},
    {"batch_tasks": 7, "candidates": 2},
    {"batch_tasks": 64, "candidates": 4},
    {"batch_tasks": 4096, "candidates": 256},
    {"batch_tasks": 1, "candidates": 1, "full_scan": 1},
    {"batch_tasks": 7, "candidates": 2, "full_scan": 1},
    {"batch_tasks": 64, "candidates": 4, "full_scan": 1},
    {"batch_tasks": 2048, "candidates": 32, "full_scan": 1},
])
def test_batching_is_exact(opts):
    """Speculation, truncation and replay must not change any decision."""
    fx = synth.config_fixture(1)
    got, ssn = run_fixture(fx, opts)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(300))
def test_fuzz_parity(seed):
    fx = synth.random_fixture(seed)
    ref = run_oracle(fx)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_parity_heap_rule(seed):
    fx = synth.random_fixture(1000 + seed, max_nodes=6, max_jobs=14, max_tasks=5)
    fx["options"] = {"heapDownRule": "go1.13"}
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.slow
@pytest.mark.parametrize("full_scan", [0, 1])
def test_config3_full_parity(full_scan):
    """C3 (5k nodes x 100k tasks, 4 queues all over-requested: Overused
    queues, failing tasks) end to end against the oracle's digest
    (tests/golden/digest_c3.json; the oracle takes ~90 s on one core), both
    scan modes."""
    from helpers import compare_digests, digest_outputs
    ref = load_golden("digest_c3.json")
    got, ssn = run_fixture(synth.config_fixture(3), {"full_scan": full_scan})
    st = ssn.stats()
    ssn.close()
    compare_digests(ref, digest_outputs(got))
    assert st.task_evaluations == ref["evaluated"]
    if not full_scan:
        # grouped mode resolved re-predicted tasks against the stage's lists
        # after cuts (cut-time list reuse) instead of rescanning
        assert st.reused_batches > 0, st.reused_batches


def _open(fx, opts=None):
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.framework import open_session
    return open_session(_OrderedCache(cache_from_fixture(fx, FakeBinder()), fx), fixture_tiers(fx), opts or {})


@pytest.mark.parametrize("seed", list(range(0, 60, 3)) + ["c1"])
def test_select_replays_reference_node_loop(seed):
    """kbg_select (the node loop of allocate.go:119-162) on the oracle's own
    evaluation sequence, one task per call, reproduces every outcome."""
    import ctypes
    from kbgpu import _abi
    fx = synth.config_fixture(1) if seed == "c1" else synth.random_fixture(seed)
    fx.pop("actions", None)  # the node loop of allocate only
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    ssn = _open(fx)
    idx = {t.uid: i for i, t in enumerate(ssn.flat.task_objs)}
    decided = {d["task"]: (d["node"], d["kind"]) for d in ref["decisions"]}
    L = _abi.lib()
    node, kind, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    for uid in ref["evaluated"]:
        arr = (ctypes.c_int32 * 1)(idx[uid])
        _abi.check(L.kbg_select(ssn.handle, arr, 1, 1, ctypes.byref(node), ctypes.byref(kind), ctypes.byref(n)))
        assert n.value == 1
        if uid in decided:
            want_node, want_kind = decided[uid]
            assert ssn.flat.node_names[node.value] == want_node, uid
            assert ("allocate" if kind.value == _abi.KIND_ALLOCATE else "pipeline") == want_kind, uid
        else:
            assert node.value == -1, uid
    for i, nref in enumerate(ref["nodes"]):
        st = ssn.node_state(i)
        assert [st.idle.milli_cpu, st.idle.memory, st.idle.milli_gpu] == nref["idle"]
        assert st.num_tasks == nref["ntasks"]
    ssn.close()


def test_select_batch_stops_at_first_success():
    """One job pop: tasks tried in order until one is placed (allocate.go:105-171)."""
    import ctypes
    from kbgpu import _abi
    fx = load_golden("kat_tolerance_edge.json")  # a -> n1 (tolerance), b -> n2, c fits nowhere
    ssn = _open(fx)
    idx = {t.uid: i for i, t in enumerate(ssn.flat.task_objs)}
    L = _abi.lib()
    order = [idx["c"], idx["a"], idx["b"]]
    arr = (ctypes.c_int32 * 3)(*order)
    nodes, kinds, n = (ctypes.c_int32 * 3)(), (ctypes.c_int32 * 3)(), ctypes.c_int32()
    _abi.check(L.kbg_select(ssn.handle, arr, 3, 1, nodes, kinds, ctypes.byref(n)))
    assert n.value == 2  # c failed, a placed, b not evaluated
    assert nodes[0] == -1 and ssn.flat.node_names[nodes[1]] == "n1"
    ssn.close()


def test_apply_matches_node_accounting():
    """kbg_apply = NodeInfo.AddTask (node_info.go:101-129) on the device table."""
    import ctypes
    from kbgpu import _abi
    fx = synth.config_fixture(1)
    ref = run_oracle(fx)
    ssn = _open(fx)
    tasks = {t.uid: t for t in ssn.flat.task_objs}
    names = {n: i for i, n in enumerate(ssn.flat.node_names)}
    L = _abi.lib()
    for d in ref["decisions"]:
        r = tasks[d["task"]].resreq
        res = _abi.kbg_resource(r.milli_cpu, r.memory, r.milli_gpu)
        _abi.check(L.kbg_apply(ssn.handle, names[d["node"]], ctypes.byref(res),
                               _abi.KIND_ALLOCATE if d["kind"] == "allocate" else _abi.KIND_PIPELINE))
    for i, nref in enumerate(ref["nodes"]):
        st = ssn.node_state(i)
        assert [st.idle.milli_cpu, st.idle.memory, st.idle.milli_gpu] == nref["idle"]
        assert st.num_tasks == nref["ntasks"]
    # the device table must agree with the host mirror: every further task now fits nowhere it should not
    ssn.close()


@pytest.fixture
def general_scan(monkeypatch):
    """Sessions opened under this fixture use the reference's LessEqual
    expression on the device instead of integer thresholds."""
    monkeypatch.setenv("KBG_FORCE_GENERAL_SCAN", "1")


@pytest.mark.parametrize("cid", [1, 2])
def test_general_scan_config_parity(cid, general_scan):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx)
    assert ssn.stats().int_scan == 0
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(0, 100, 3))
def test_general_scan_fuzz_parity(seed, general_scan):
    fx = synth.random_fixture(seed)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


def test_int_scan_is_the_default_on_integer_sessions():
    fx = synth.config_fixture(2)
    got, ssn = run_fixture(fx)
    assert ssn.stats().int_scan == 1
    ssn.close()


@pytest.mark.parametrize("seed", range(60))
def test_backfill_parity(seed):
    """backfill.go:40-71 after (or without) allocate: first node whose PredicateFn
    passes, pod caps 2-5 on most nodes, panics on overcommitted Idle."""
    fx = synth.random_fixture(2000 + seed, max_nodes=10, max_jobs=12, max_tasks=12, be_frac=0.6)
    fx["actions"] = ["allocate", "backfill"] if seed % 4 else ["backfill"]
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 7, "candidates": 1 + seed % 3, "full_scan": seed % 2})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("be_req", [{}, {"cpu": "5m"}])
def test_backfill_config2(shards, be_req):
    """C2 with every 7th pod BestEffort: allocate then backfill over 1k nodes.
    Requests of 5m drive a full node's Idle below the tolerance on the second
    BestEffort pod, where Resource.Sub panics (resource_info.go:100-110)."""
    fx = synth.config_fixture(2)
    for i, p in enumerate(fx["pods"]):
        if i % 7 == 3:
            p["containers"] = [{"requests": dict(be_req)}]
    fx["actions"] = ["allocate", "backfill"]
    ref = run_oracle(fx)
    if be_req:
        assert ref["status"] == "ref_panic"
    else:
        assert sum(1 for d in ref["decisions"] if d.get("action") == "backfill") > 1000
    got, ssn = run_fixture(fx, {"shards": shards})
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(150))
def test_contended_reclaim_preempt_parity(seed):
    """reclaim.go / preempt.go / statement.go on clusters full of running gang
    jobs: evictions (order, preemptor), pipelines, discarded statements'
    node-side residue, shares and readiness against the oracle."""
    fx = synth.contended_fixture(seed)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("nodes,jobs,pending", [(300, 120, 8), (1000, 400, 20)])
def test_config5_scaled_parity(nodes, jobs, pending):
    """The C5 generator (95% full cluster, reclaim, allocate, backfill,
    preempt) at reduced size: evictions, pipelines and allocations exact."""
    fx = synth.contended_config(nodes=nodes, jobs=jobs, pending_jobs=pending)
    ref = run_oracle(fx)
    assert ref["status"] == "ok" and ref["evictions"], ref.get("error")
    got, ssn = run_fixture(fx)
    compare_outputs(ref, got)
    ssn.close()


@pytest.mark.slow
def test_config5_full_parity():
    """C5 (10k nodes x 200k tasks) end to end against the oracle."""
    fx = synth.config_fixture(5)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(60))
def test_contended_large_parity(seed):
    """Bigger contended clusters: many tries per preemptor shape, so the host
    keeps the victim scan's stop maps across evictions, pipelines and
    discarded statements before the next scan."""
    fx = synth.contended_fixture(5000 + seed, nodes=40, jobs=30, tasks=10, queues=3)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(300))
def test_affinity_fuzz_parity(seed):
    """Inter-pod (anti)affinity folded into the class masks (kbg_affinity.cpp):
    monotone losses re-checked by the resolver, affinity gains cutting the
    batch, FitError counts rewound with the counts, across batch sizes and
    both scan modes."""
    fx = synth.affinity_fixture(seed)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("nodes,jobs,tasks", [(300, 60, 20), (600, 100, 20)])
def test_affinity_config_scaled_parity(nodes, jobs, tasks):
    """C3's generator with spread (host anti-affinity) and co-located (zone
    affinity) jobs, at a size the oracle's per-pair podLister walk finishes."""
    fx = synth.affinity_config(nodes=nodes, jobs=jobs, tasks_per_job=tasks)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(200))
def test_dupkey_fuzz_parity(seed):
    """Colliding pod keys (synth.dupkey_fixture): a placement onto a node that
    already holds the PodKey is logged and dispatched but leaves the node
    unchanged (node_info.go:101-106, session.go:205-293), across allocate,
    backfill, reclaim and preempt, batch sizes and both scan modes."""
    fx = synth.dupkey_fixture(seed)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(120))
def test_victim_affinity_parity(seed):
    """reclaim/preempt (reclaim.go, preempt.go) on contended clusters whose
    jobs carry required pod (anti)affinity on the zone or the host: the
    victim scan's class masks follow evictions, pipelines and discarded
    statements through kbg_affinity.cpp's counts."""
    fx = synth.contended_fixture(7000 + seed, nodes=12, jobs=14, tasks=8, aff=0.5)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(100))
def test_victim_host_ports_parity(seed):
    """reclaim/preempt with host ports: an eviction frees the victim's port
    atoms, a pipelined preemptor takes them (predicates.go host-port check)."""
    fx = synth.contended_fixture(8000 + seed, nodes=12, jobs=14, tasks=8, ports=0.4)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(12))
def test_victim_big_node_parity(seed):
    """Nodes with 130-250 Running pods: the victim scan walks the candidates in
    several 64-wide chunks (kbg_victim_big_kernel), evictions exact."""
    fx = synth.contended_fixture(9000 + seed, big=True, nodes=2, jobs=50, tasks=24)
    running = {}
    for p in fx["pods"]:
        if p["phase"] == "Running":
            running[p["nodeName"]] = running.get(p["nodeName"], 0) + 1
    assert max(running.values()) > 128
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


# seeds of synth.contended_dupkey_fixture whose oracle run discards a statement
# holding a pipeline onto a node that already had its pod key (oracle stats
# dup_discards > 0; the first 300 seeds)
DUP_DISCARD_SEEDS = [66, 73, 89, 106, 117, 154, 179, 208, 212, 227, 240, 253, 273, 295]


@pytest.mark.parametrize("seed", DUP_DISCARD_SEEDS + [0, 1, 2, 3, 4, 5])
def test_dupkey_statement_discard_parity(seed):
    """A discarded preempt statement whose pipeline found its pod key already
    on the node: unpipeline's RemoveTask removes the pod that held the key
    (statement.go:156-192, node_info.go:131-157), and the holder's own
    unevict then adds it back as Running. No KBG_E_UNSUPPORTED."""
    fx = synth.contended_dupkey_fixture(seed)
    ref = run_oracle(fx)
    if seed in DUP_DISCARD_SEEDS:
        assert ref["stats"]["dup_discards"] > 0
    got, ssn = run_fixture(fx)
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


# seeds of synth.contended_dupkey_fixture(seed, ports=0.4) whose oracle run
# discards such a statement (the first 900 seeds): the holders carry host ports
DUP_DISCARD_PORT_SEEDS = [79, 89, 126, 231, 293, 369, 444, 469, 509, 570, 598, 669, 681, 793, 816, 884]


@pytest.mark.parametrize("seed", DUP_DISCARD_PORT_SEEDS)
def test_dupkey_statement_discard_ports_parity(seed):
    """The discarded statement's RemoveTask by key takes the holder's host
    ports out of node.Pods(); its unevict adds the holder back
    (statement.go:81-108), so its ports are used again and a later pipeline
    onto a conflicting port must fail as the reference's does
    (predicates.go:144-155, vendor cache/node_info.go:593-605)."""
    fx = synth.contended_dupkey_fixture(seed, ports=0.4)
    ref = run_oracle(fx)
    assert ref["stats"]["dup_discards"] > 0
    got, ssn = run_fixture(fx)
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", [7] + list(range(24)))
def test_dupkey_pending_holder_parity(seed):
    """Pending pods sharing a pod key (synth.contended_dupkey_fixture with
    pending_dups): the key's holder can be a pod placed earlier in the same
    cycle, whose Allocated or Pipelined copy a discarded statement's
    RemoveTask by key takes off the node (node_info.go:131-157); its own
    unpipeline then finds nothing. Seed 7's oracle run has such a discard."""
    fx = synth.contended_dupkey_fixture(seed, pending_dups=0.6)
    ref = run_oracle(fx)
    if seed == 7:
        assert ref["stats"]["dup_discards_placed"] > 0
    got, ssn = run_fixture(fx)
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(10))
def test_victim_huge_node_parity(seed):
    """Nodes with more than kMaxNodeCandidates (1024) Running pods, which the
    reference walks like any other (preempt.go:169-236): left out of the
    device victim scans and evaluated on the host when a stop search reaches
    them (host_stop), evictions exact. No KBG_E_UNSUPPORTED."""
    fx = synth.contended_fixture(9500 + seed, big=True, huge=True, nodes=2, jobs=240, tasks=30)
    running = {}
    for p in fx["pods"]:
        if p["phase"] == "Running":
            running[p["nodeName"]] = running.get(p["nodeName"], 0) + 1
    assert max(running.values()) > 1024
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", list(range(0, 60, 4)))
def test_select_replays_with_affinity(seed):
    """kbg_select on affinity fixtures: a placement that creates an affinity
    gain for later tasks is seen by the next call (the gain rescan)."""
    import ctypes
    from kbgpu import _abi
    fx = synth.affinity_fixture(seed)
    fx["actions"] = ["allocate"]
    ref = run_oracle(fx)
    if ref["status"] != "ok":
        pytest.skip(ref["status"])
    ssn = _open(fx)
    idx = {t.uid: i for i, t in enumerate(ssn.flat.task_objs)}
    decided = {d["task"]: (d["node"], d["kind"]) for d in ref["decisions"]}
    L = _abi.lib()
    node, kind, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    for uid in ref["evaluated"]:
        arr = (ctypes.c_int32 * 1)(idx[uid])
        _abi.check(L.kbg_select(ssn.handle, arr, 1, 1, ctypes.byref(node), ctypes.byref(kind), ctypes.byref(n)))
        if uid in decided:
            assert ssn.flat.node_names[node.value] == decided[uid][0], uid
        else:
            assert node.value == -1, uid
    ssn.close()


def test_staging_reuse_under_overlap():
    """A resident-session churn fixture (update fuzz seed 83, round 2) whose
    allocate runs 3-task batches with the next scan in flight: the pinned
    delta staging must not be rewritten before the stream has copied it
    (stage_acquire / stage_release), or a lost node delta shows up as a
    backfill onto a full node. Repeated in one process, where the stream runs
    behind the host."""
    fx = load_golden("fx_staging_race.json")
    ref = run_oracle(fx)
    for it in range(120):
        opts = {"batch_tasks": 3, "candidates": 4, "full_scan": 1} if it % 2 else \
               {"batch_tasks": 1 + it % 9, "candidates": 1 + it % 5, "full_scan": it % 4 == 0}
        opts["full_scan"] = int(opts["full_scan"])
        got, ssn = run_fixture(fx, opts)
        compare_outputs(ref, got)
        if ssn:
            ssn.close()


@pytest.mark.parametrize("seed", range(0, 40, 2))
def test_predictor_engine_is_final(seed, monkeypatch):
    """At the end of a cycle the predictor's engine is the committed state
    (its last epoch had no cut), so the truth engine's backlog is dropped:
    KBG_CHECK_TRUTH=1 waits for it and compares the two engines field by
    field on contended and saturated cycles (cuts, reused lists)."""
    monkeypatch.setenv("KBG_CHECK_TRUTH", "1")
    fx = synth.contended_fixture(12000 + seed, nodes=16, jobs=20, tasks=10) if seed % 4 else \
        synth.saturated_config(nodes=64, jobs=40, tasks_per_job=12, seed=seed)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()
