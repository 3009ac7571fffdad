"""The Python input builder (kbgpu/cache.py, the SchedulerCache mirror that
feeds kbg_snapshot) against the reference's own cache tests
(pkg/scheduler/cache/cache_test.go TestAddPod / TestAddNode, restated as data
in tests/golden/ref_cache_*.json): node accounting, including a node that pods
named before it was added (NodeInfo(nil), then SetNode), and job membership
by the controller owner reference."""
import glob
import json
import os

import pytest

from helpers import GOLDEN

REF = sorted(glob.glob(os.path.join(GOLDEN, "ref_cache_*.json")))


def res(r):
    return [r.milli_cpu, r.memory, r.milli_gpu]


@pytest.mark.parametrize("path", REF, ids=[os.path.basename(p) for p in REF])
def test_cache_ops(path):
    from kbgpu.api import pod_key
    from kbgpu.cache import SchedulerCache
    fx = json.load(open(path))
    nodes = {n["name"]: n for n in fx["nodes"]}
    pods = {pod_key(p): p for p in fx["pods"]}
    c = SchedulerCache()
    for op in fx["ops"]:
        if op["op"] == "add_node":
            c.add_node(nodes[op["node"]])
        else:
            c.add_pod(pods[op["pod"]])
    exp = fx["expected"]
    got_nodes = {name: {"idle": res(ni.idle), "used": res(ni.used), "releasing": res(ni.releasing),
                        "allocatable": res(ni.allocatable), "tasks": sorted(ni.tasks)}
                 for name, ni in c.nodes.items()}
    assert got_nodes == exp["nodes"]
    got_jobs = {}
    for uid, job in c.jobs.items():
        idx = {str(s): sorted(t.uid for t in ts.values()) for s, ts in job.task_status_index.items() if ts}
        got_jobs[uid] = {"status_index": idx, "allocated": res(job.allocated), "total_request": res(job.total_request)}
    assert got_jobs == exp["jobs"]
