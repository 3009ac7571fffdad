"""Fake-cache builder: the SchedulerCache semantics the allocate path consumes.

Mirrors the parts of pkg/scheduler/cache that define a session's contents:
AddNode/AddPod/AddPodGroup/AddPDB/AddQueue/AddNamespace
(event_handlers.go:40-61,232-240,344-358,458-470,635-640,726-736) and
Snapshot (cache.go:549-597). Informers, resync and the apiserver are out of
scope; Bind goes to a caller-supplied binder (allocate_test.go:99-115 style).
Go map iteration order is replaced by insertion order.
"""
from .api import FAILED, RUNNING, SUCCEEDED, JobInfo, NodeInfo, QueueInfo, TaskInfo


class ClusterInfo:
    def __init__(self):
        self.nodes = []
        self.jobs = []
        self.queues = []
        self.others = []


class FakeBinder:
    """Records binds like allocate_test.go:99-115, without the blocking channel (F11)."""

    def __init__(self):
        self.binds = {}
        self.order = []
        self.evicts = []

    def bind(self, pod, hostname):
        key = f"{pod.get('namespace', '')}/{pod['name']}"
        self.binds[key] = hostname
        self.order.append(key)

    def evict(self, pod, reason):  # the fake Evictor: records (pod key, reason)
        self.evicts.append((f"{pod.get('namespace', '')}/{pod['name']}", reason))


class SchedulerCache:
    def __init__(self, binder=None, default_queue=""):
        self.nodes = {}
        self.jobs = {}
        self.queues = {}
        self.binder = binder or FakeBinder()
        self.default_queue = default_queue

    # event_handlers.go:40-61
    def _add_task(self, pi):
        if pi.job:
            if pi.job not in self.jobs:
                self.jobs[pi.job] = JobInfo(pi.job)
            self.jobs[pi.job].add_task_info(pi)
        if pi.node_name:
            if pi.node_name not in self.nodes:
                self.nodes[pi.node_name] = NodeInfo(None)
            if pi.status not in (SUCCEEDED, FAILED):
                self.nodes[pi.node_name].add_task(pi)

    def add_pod(self, pod):
        self._add_task(TaskInfo(pod))

    # event_handlers.go:105-130: the job side, then the node side (RemoveTask by
    # PodKey: whatever pod holds the key leaves the node); False on an error
    def _delete_task(self, pi):
        ok = True
        if pi.job:
            job = self.jobs.get(pi.job)
            ok = job is not None and job.delete_task_info(pi)
        if pi.node_name:
            node = self.nodes.get(pi.node_name)
            if node is not None and not node.remove_task(pi):
                ok = False
        return ok

    def delete_pod(self, pod):  # :132-152 (the cache's own copy of the task when it has one)
        pi = TaskInfo(pod)
        job = self.jobs.get(pi.job)
        task = job.tasks.get(pi.uid, pi) if job is not None else pi
        if not self._delete_task(task):
            return False
        job = self.jobs.get(pi.job)
        if job is not None and job.pod_group is None and job.pdb is None and not job.tasks:  # JobTerminated
            del self.jobs[pi.job]
        return True

    def update_pod(self, old_pod, new_pod):  # :96-101: deletePod's error stops the update
        if not self.delete_pod(old_pod):
            return False
        self.add_pod(new_pod)
        return True

    def update_node(self, node):  # :249-259 (every churn node update changes Allocatable)
        if node["name"] in self.nodes:
            self.nodes[node["name"]].set_node(node)

    def add_node(self, node):  # :232-240
        if node["name"] in self.nodes:  # a pod named the node first: NodeInfo(nil) gets its Node (SetNode)
            self.nodes[node["name"]].set_node(node)
        else:
            self.nodes[node["name"]] = NodeInfo(node)

    def delete_node(self, node):  # :262-268 (its pods stay in their jobs, NodeName unchanged)
        self.nodes.pop(node["name"], None)

    def delete_pod_group(self, pg):  # :361-381: UnsetPodGroup; the job stays until it has no pods
        job = self.jobs.get(f"{pg.get('namespace', '')}/{pg['name']}")
        if job is not None:
            job.pod_group = None

    def delete_queue(self, q):  # :650-654
        self.queues.pop(q["name"], None)

    def add_pod_group(self, pg):  # :344-358
        jid = f"{pg.get('namespace', '')}/{pg['name']}"
        if jid not in self.jobs:
            self.jobs[jid] = JobInfo(jid)
        self.jobs[jid].set_pod_group(pg, self.default_queue)

    def add_pdb(self, pdb):  # :458-470
        jid = pdb.get("controller", "")
        if jid not in self.jobs:
            self.jobs[jid] = JobInfo(jid)
        self.jobs[jid].set_pdb(pdb, self.default_queue)

    def add_queue(self, q):  # :635-640
        qi = QueueInfo(q["name"], q.get("weight", 0))
        self.queues[qi.uid] = qi

    def add_namespace(self, name):  # :726-736
        self.queues[name] = QueueInfo(name, 1)

    def bind(self, task, hostname):  # cache.go:408-444 (session-visible part)
        self.binder.bind(task.pod, hostname)

    def evict(self, task, reason):  # cache.go:369-405 (the evictor side)
        self.binder.evict(task.pod, reason)

    def snapshot(self):  # cache.go:549-597
        s = ClusterInfo()
        s.nodes = [n.clone() for n in self.nodes.values()]
        s.queues = [q.clone() for q in self.queues.values()]
        qids = {q.uid for q in s.queues}
        for job in self.jobs.values():
            if job.pod_group is None and job.pdb is None:
                s.others.extend(t.clone() for t in job.task_status_index.get(RUNNING, {}).values())
                continue
            if job.queue not in qids:
                continue
            s.jobs.append(job.clone())
        return s


def cache_from_fixture(fx, binder=None):
    """Builds a SchedulerCache from a fixture dict in the order the reference
    test harness adds objects (allocate_test.go:258-272): nodes, pods,
    podgroups, PDBs, queues, namespaces."""
    opts = fx.get("options") or {}
    c = SchedulerCache(binder=binder, default_queue=opts.get("defaultQueue", ""))
    for n in fx.get("nodes", []):
        c.add_node(n)
    seen = set()
    for p in fx.get("pods", []):
        if p["uid"] in seen:
            raise ValueError(f"duplicate pod uid {p['uid']}")
        seen.add(p["uid"])
        c.add_pod(p)
    for g in fx.get("podGroups", []):
        c.add_pod_group(g)
    for d in fx.get("pdbs", []):
        c.add_pdb(d)
    for q in fx.get("queues", []):
        c.add_queue(q)
    for n in fx.get("namespaces", []):
        c.add_namespace(n if isinstance(n, str) else n["name"])
    return c
