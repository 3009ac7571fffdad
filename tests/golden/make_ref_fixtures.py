"""Restates the reference's own unit-test cases as JSON fixtures (data only).

Each fixture carries the inputs of one reference test case and the expected
outputs that test asserts, with the file:line it comes from. Nothing from the
reference is executed (there is no Go toolchain); the values below
are transcribed from the test sources.

Run:  python tests/golden/make_ref_fixtures.py   (rewrites tests/golden/ref_*.json)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def res(cpu, mem, gpu="0"):
    # allocate_test.go:41-55 buildResourceList / buildResourceListWithGPU
    return {"cpu": cpu, "memory": mem, "nvidia.com/gpu": gpu}


def alloc_pod(ns, n, nn, phase, req, group):
    # allocate_test.go:71-98 buildPod: UID "<ns>-<n>", group annotation, one container
    return {
        "uid": f"{ns}-{n}", "namespace": ns, "name": n, "nodeName": nn, "phase": phase,
        "annotations": {"scheduling.k8s.io/group-name": group},
        "labels": {}, "nodeSelector": {},
        "containers": [{"requests": req}],
    }


def api_pod(ns, n, nn, phase, req, owner=None):
    # pkg/scheduler/api/test_utils.go:71-98 buildPod (owner references, no annotation)
    p = {"uid": f"{ns}-{n}", "namespace": ns, "name": n, "nodeName": nn, "phase": phase,
         "containers": [{"requests": {"cpu": req[0], "memory": req[1]}}]}
    if owner:
        p["controller"] = owner
    return p


DRF_PROPORTION = [[{"name": "drf"}, {"name": "proportion"}]]  # allocate_test.go:272-283

FIXTURES = {
    # pkg/scheduler/actions/allocate/allocate_test.go:153-184
    "ref_allocate_case1": {
        "source": "pkg/scheduler/actions/allocate/allocate_test.go:153-184",
        "tiers": DRF_PROPORTION,
        "nodes": [{"name": "n1", "allocatable": res("2", "4Gi")}],
        "pods": [
            alloc_pod("c1", "p1", "", "Pending", res("1", "1G"), "pg1"),
            alloc_pod("c1", "p2", "", "Pending", res("1", "1G"), "pg1"),
        ],
        "podGroups": [{"namespace": "c1", "name": "pg1"}],
        "queues": [{"name": "c1", "weight": 1}],
        "expected": {"binds": {"c1/p1": "n1", "c1/p2": "n1"}},
    },
    # pkg/scheduler/actions/allocate/allocate_test.go:185-237
    "ref_allocate_case2": {
        "source": "pkg/scheduler/actions/allocate/allocate_test.go:185-237",
        "tiers": DRF_PROPORTION,
        "nodes": [{"name": "n1", "allocatable": res("2", "4G")}],
        "pods": [
            alloc_pod("c1", "p1", "", "Pending", res("1", "1G"), "pg1"),
            alloc_pod("c1", "p2", "", "Pending", res("1", "1G"), "pg1"),
            alloc_pod("c2", "p1", "", "Pending", res("1", "1G"), "pg2"),
            alloc_pod("c2", "p2", "", "Pending", res("1", "1G"), "pg2"),
        ],
        "podGroups": [{"namespace": "c1", "name": "pg1"}, {"namespace": "c2", "name": "pg2"}],
        "queues": [{"name": "c1", "weight": 1}, {"name": "c2", "weight": 1}],
        "expected": {"binds": {"c2/p1": "n1", "c1/p1": "n1"}},
    },
    # pkg/scheduler/api/node_info_test.go:35-80 TestNodeInfo_AddPod
    "ref_nodeinfo_add": {
        "source": "pkg/scheduler/api/node_info_test.go:35-80",
        "kind": "nodeinfo_ops",
        "node": {"name": "n1", "allocatable": {"cpu": "8000m", "memory": "10G"}},
        "pods": [api_pod("c1", "p1", "n1", "Running", ("1000m", "1G")),
                 api_pod("c1", "p2", "n1", "Running", ("2000m", "2G"))],
        "ops": [{"op": "add", "pod": "c1/p1"}, {"op": "add", "pod": "c1/p2"}],
        "expected": {"idle": [5000, 7e9, 0], "used": [3000, 3e9, 0], "releasing": [0, 0, 0],
                     "allocatable": [8000, 10e9, 0], "tasks": ["c1/p1", "c1/p2"]},
    },
    # pkg/scheduler/api/node_info_test.go:82-135 TestNodeInfo_RemovePod
    "ref_nodeinfo_remove": {
        "source": "pkg/scheduler/api/node_info_test.go:82-135",
        "kind": "nodeinfo_ops",
        "node": {"name": "n1", "allocatable": {"cpu": "8000m", "memory": "10G"}},
        "pods": [api_pod("c1", "p1", "n1", "Running", ("1000m", "1G")),
                 api_pod("c1", "p2", "n1", "Running", ("2000m", "2G")),
                 api_pod("c1", "p3", "n1", "Running", ("3000m", "3G"))],
        "ops": [{"op": "add", "pod": "c1/p1"}, {"op": "add", "pod": "c1/p2"}, {"op": "add", "pod": "c1/p3"},
                {"op": "remove", "pod": "c1/p2"}],
        "expected": {"idle": [4000, 6e9, 0], "used": [4000, 4e9, 0], "releasing": [0, 0, 0],
                     "allocatable": [8000, 10e9, 0], "tasks": ["c1/p1", "c1/p3"]},
    },
    # pkg/scheduler/api/job_info_test.go:35-101 TestAddTaskInfo
    "ref_jobinfo_add": {
        "source": "pkg/scheduler/api/job_info_test.go:35-101",
        "kind": "jobinfo_ops",
        "uid": "uid",
        "pods": [api_pod("c1", "p1", "", "Pending", ("1000m", "1G"), "uid"),
                 api_pod("c1", "p2", "n1", "Running", ("2000m", "2G"), "uid"),
                 api_pod("c1", "p3", "n1", "Pending", ("1000m", "1G"), "uid"),
                 api_pod("c1", "p4", "n1", "Pending", ("1000m", "1G"), "uid")],
        "ops": [{"op": "add", "pod": "c1/p1"}, {"op": "add", "pod": "c1/p2"},
                {"op": "add", "pod": "c1/p3"}, {"op": "add", "pod": "c1/p4"}],
        # status bits: Pending=1, Bound=16, Running=32 (pkg/scheduler/api/types.go:23-58)
        "expected": {"allocated": [4000, 4e9, 0], "total_request": [5000, 5e9, 0],
                     "status_index": {"1": ["c1-p1"], "16": ["c1-p3", "c1-p4"], "32": ["c1-p2"]}},
    },
    # pkg/scheduler/api/job_info_test.go:103-197 TestDeleteTaskInfo case 1
    "ref_jobinfo_delete1": {
        "source": "pkg/scheduler/api/job_info_test.go:103-146,159-173",
        "kind": "jobinfo_ops",
        "uid": "owner1",
        "pods": [api_pod("c1", "p1", "", "Pending", ("1000m", "1G"), "owner1"),
                 api_pod("c1", "p2", "n1", "Running", ("2000m", "2G"), "owner1"),
                 api_pod("c1", "p3", "n1", "Running", ("3000m", "3G"), "owner1")],
        "ops": [{"op": "add", "pod": "c1/p1"}, {"op": "add", "pod": "c1/p2"}, {"op": "add", "pod": "c1/p3"},
                {"op": "remove", "pod": "c1/p2"}],
        "expected": {"allocated": [3000, 3e9, 0], "total_request": [4000, 4e9, 0],
                     "status_index": {"1": ["c1-p1"], "32": ["c1-p3"]}},
    },
    # pkg/scheduler/api/job_info_test.go:103-197 TestDeleteTaskInfo case 2
    "ref_jobinfo_delete2": {
        "source": "pkg/scheduler/api/job_info_test.go:125-134,174-194",
        "kind": "jobinfo_ops",
        "uid": "owner2",
        "pods": [api_pod("c1", "p1", "", "Pending", ("1000m", "1G"), "owner2"),
                 api_pod("c1", "p2", "n1", "Pending", ("2000m", "2G"), "owner2"),
                 api_pod("c1", "p3", "n1", "Running", ("3000m", "3G"), "owner2")],
        "ops": [{"op": "add", "pod": "c1/p1"}, {"op": "add", "pod": "c1/p2"}, {"op": "add", "pod": "c1/p3"},
                {"op": "remove", "pod": "c1/p2"}],
        "expected": {"allocated": [3000, 3e9, 0], "total_request": [4000, 4e9, 0],
                     "status_index": {"1": ["c1-p1"], "32": ["c1-p3"]}},
    },
    # pkg/scheduler/cache/cache_test.go:128-186 TestAddPod (nodes, then pods; job from the controller owner)
    "ref_cache_addpod": {
        "source": "pkg/scheduler/cache/cache_test.go:128-186",
        "kind": "cache_ops",
        "nodes": [{"name": "n1", "allocatable": {"cpu": "2000m", "memory": "10G"}}],
        "pods": [api_pod("c1", "p1", "", "Pending", ("1000m", "1G"), "j1"),
                 api_pod("c1", "p2", "n1", "Running", ("1000m", "1G"), "j1")],
        "ops": [{"op": "add_node", "node": "n1"}, {"op": "add_pod", "pod": "c1/p1"}, {"op": "add_pod", "pod": "c1/p2"}],
        "expected": {"nodes": {"n1": {"idle": [1000, 9e9, 0], "used": [1000, 1e9, 0], "releasing": [0, 0, 0],
                                      "allocatable": [2000, 10e9, 0], "tasks": ["c1/p2"]}},
                     "jobs": {"j1": {"status_index": {"1": ["c1-p1"], "32": ["c1-p2"]},
                                     "allocated": [1000, 1e9, 0], "total_request": [2000, 2e9, 0]}}},
    },
    # pkg/scheduler/cache/cache_test.go:188-236 TestAddNode (pods first: the node is a NodeInfo(nil)
    # until AddNode's SetNode; pods without a controller join no job)
    "ref_cache_addnode": {
        "source": "pkg/scheduler/cache/cache_test.go:188-236",
        "kind": "cache_ops",
        "nodes": [{"name": "n1", "allocatable": {"cpu": "2000m", "memory": "10G"}}],
        "pods": [api_pod("c1", "p1", "", "Pending", ("1000m", "1G")),
                 api_pod("c1", "p2", "n1", "Running", ("1000m", "1G"))],
        "ops": [{"op": "add_pod", "pod": "c1/p1"}, {"op": "add_pod", "pod": "c1/p2"}, {"op": "add_node", "node": "n1"}],
        "expected": {"nodes": {"n1": {"idle": [1000, 9e9, 0], "used": [1000, 1e9, 0], "releasing": [0, 0, 0],
                                      "allocatable": [2000, 10e9, 0], "tasks": ["c1/p2"]}},
                     "jobs": {}},
    },
}


def main():
    for name, fx in FIXTURES.items():
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, indent=1, sort_keys=False)
            f.write("\n")
    print("wrote", len(FIXTURES), "fixtures")


if __name__ == "__main__":
    main()
