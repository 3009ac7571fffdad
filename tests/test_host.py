"""Host-side logic that needs no GPU: the session mirror, marshaling, config."""
import json

import pytest

from helpers import load_golden


def test_quantities_match_reference_rounding():
    from kbgpu import api
    fx = load_golden("kat_quantity.json")
    got = [[api.milli_value(q), api.value(q)] for q in fx["quantities"]]
    assert got == fx["expected"]["values"]


@pytest.mark.parametrize("case", ["ref_nodeinfo_add", "ref_nodeinfo_remove"])
def test_nodeinfo_mirror(case):
    """pkg/scheduler/api/node_info_test.go through the Python mirror."""
    from kbgpu import api
    fx = load_golden(case + ".json")
    node = api.NodeInfo(fx["node"])
    pods = {f"{p['namespace']}/{p['name']}": p for p in fx["pods"]}
    for op in fx["ops"]:
        t = api.TaskInfo(pods[op["pod"]])
        if op["op"] == "add":
            node.add_task(t)
        else:
            key = api.pod_key(t.pod)
            old = node.tasks.pop(key)
            node.idle.add(old.resreq)
            node.used.sub(old.resreq)
    exp = fx["expected"]
    assert list(node.idle.as_tuple()) == exp["idle"] and list(node.used.as_tuple()) == exp["used"]
    assert sorted(node.tasks) == exp["tasks"]


@pytest.mark.parametrize("case", ["ref_jobinfo_add", "ref_jobinfo_delete1", "ref_jobinfo_delete2"])
def test_jobinfo_mirror(case):
    """pkg/scheduler/api/job_info_test.go through the Python mirror."""
    from kbgpu import api
    fx = load_golden(case + ".json")
    job = api.JobInfo(fx["uid"])
    pods = {f"{p['namespace']}/{p['name']}": p for p in fx["pods"]}
    for op in fx["ops"]:
        t = api.TaskInfo(pods[op["pod"]])
        if op["op"] == "add":
            job.add_task_info(t)
        else:
            job.delete_task_info(t)
    exp = fx["expected"]
    assert list(job.allocated.as_tuple()) == exp["allocated"]
    assert list(job.total_request.as_tuple()) == exp["total_request"]
    assert {str(k): sorted(v) for k, v in job.task_status_index.items()} == exp["status_index"]


def test_snapshot_semantics():
    """cache.Snapshot: jobs without a PodGroup feed Others; missing queues drop jobs."""
    from kbgpu.cache import cache_from_fixture
    fx = {"nodes": [{"name": "n1", "allocatable": {"cpu": "4", "memory": "4Gi"}}],
          "pods": [{"uid": "a", "namespace": "x", "name": "a", "phase": "Running", "nodeName": "n1",
                    "containers": [{"requests": {"cpu": "1"}}], "controller": "rc"},
                   {"uid": "b", "namespace": "x", "name": "b", "phase": "Pending",
                    "annotations": {"scheduling.k8s.io/group-name": "pg"}, "containers": [{"requests": {"cpu": "1"}}]},
                   {"uid": "c", "namespace": "y", "name": "c", "phase": "Pending",
                    "annotations": {"scheduling.k8s.io/group-name": "pg"}, "containers": [{"requests": {"cpu": "1"}}]}],
          "podGroups": [{"namespace": "x", "name": "pg", "queue": "q"}, {"namespace": "y", "name": "pg", "queue": "nope"}],
          "queues": [{"name": "q", "weight": 1}]}
    s = cache_from_fixture(fx).snapshot()
    assert [j.uid for j in s.jobs] == ["x/pg"]
    assert [t.uid for t in s.others] == ["a"]
    assert s.nodes[0].idle.milli_cpu == 3000


def test_flat_snapshot_layout():
    """The marshaled arrays carry what the device path needs, in session order."""
    from kbgpu import synth
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    from kbgpu.api import RefPanic
    for seed in range(7, 100):
        fx = synth.random_fixture(seed)
        try:
            s = cache_from_fixture(fx).snapshot()
            break
        except RefPanic:  # overcommitted node: the reference panics in AddPod
            continue
    flat = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    A = flat.arrays
    strs = flat.interner.strings
    assert [strs[i] for i in A["nodes"]["name"]] == [n.name for n in s.nodes]
    assert len(A["tasks"]) == sum(len(j.tasks) for j in s.jobs)
    for row, t in zip(A["tasks"], flat.task_objs):
        assert strs[row["uid"]] == t.uid and row["status"] == t.status
        assert tuple(row["resreq"]) == t.resreq.as_tuple()
    assert flat.snap.n_plugins == sum(len(t.plugins) for t in fixture_tiers(fx))


def test_scheduler_conf_default():
    from kbgpu.conf import load_scheduler_conf
    actions, tiers = load_scheduler_conf()
    assert actions == ["allocate", "backfill"]
    assert [[p.name for p in t.plugins] for t in tiers] == [["priority", "gang"], ["drf", "predicates", "proportion"]]


def test_fit_error_format():
    from kbgpu.fixture import fit_error
    assert fit_error(0, 0, 0, 0) == "0 nodes are available"
    assert fit_error(12, 10, 2, 0) == "0/12 nodes are available, 10 insufficient cpu, 2 insufficient memory."


def test_synth_is_deterministic():
    from kbgpu import synth
    assert json.dumps(synth.config_fixture(2)) == json.dumps(synth.config_fixture(2))
    assert json.dumps(synth.random_fixture(5)) == json.dumps(synth.random_fixture(5))
