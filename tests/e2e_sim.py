"""Multi-cycle restatement of the reference's e2e specs (test infrastructure).

The reference's behavioural tests of the scheduling path are Ginkgo e2e specs
against a live 3-node kubeadm-dind cluster (`test/e2e/job.go:27-368`,
`predicates.go:29-193`, `queue.go:27-70`, scheduler started by
`hack/run-e2e.sh:30` with `example/kube-batch-conf.yaml`). They cannot run here
(no cluster, no network), but what they assert is a state the scheduler's
loop reaches within a minute of polling. `Cluster` replays that loop on a
fake cluster: every cycle is one `Scheduler.runOnce` (`scheduler.go:83-93`:
snapshot, the conf's actions, close) run by a caller-supplied runner (the
kbref oracle on the CPU, the MI355X path on the GPU), and between cycles the
parts of Kubernetes the e2e cluster supplies are modelled:

- the binder / kubelet: a bound pod runs from the next cycle on
  (`cache.Bind`, `cache.go:408-444`); a pipelined task binds nothing;
- the evictor: an evicted pod terminates (Running with a deletionTimestamp,
  i.e. Releasing, for its 3 s grace period = 3 one-second cycles,
  `cache.go:110-123`, then gone), and its batch Job creates a
  Pending replacement at once (the Job controller does not count terminating
  pods as active);
- ReplicaSet pods (`util.go:490-535`, default scheduler, no PodGroup) are
  placed first-fit on untainted nodes and terminate like evicted pods when
  the ReplicaSet is deleted;
- the e2e context (`util.go:75-130`): namespace `test`, queues `q1`, `q2` and
  `test` (weight 1, queue CRDs), priority classes master-pri = 100 and
  worker-pri = 1; nodes: 3 untainted workers plus a master tainted
  NoSchedule (`hack/run-e2e.sh:6`, NUM_NODES=3).

`clusterSize` / `computeNode` / `clusterNodeNumber` restate `util.go:566-690`.
The wait helpers (`waitTasksReady`, `waitPodGroupPending`,
`waitPodGroupUnschedulable`, `podGroupEvicted`, `util.go:342-470`) become
predicates on the cluster state, polled between cycles (`Cluster.wait`).
"""
import copy

GROUP = "scheduling.k8s.io/group-name"
CPU = {"half": {"cpu": "500m"}, "one": {"cpu": "1000m"}, "two": {"cpu": "2000m"}}
PRIORITY = {"master-pri": 100, "worker-pri": 1}
CONF_ACTIONS = ["reclaim", "allocate", "backfill", "preempt"]  # example/kube-batch-conf.yaml:1
CONF_TIERS = [[{"name": "priority"}, {"name": "gang"}],
              [{"name": "drf"}, {"name": "predicates"}, {"name": "proportion"}]]  # :2-9
MASTER_TAINT = {"key": "node-role.kubernetes.io/master", "value": "", "effect": "NoSchedule"}


class WaitTimeout(AssertionError):
    """A wait helper's condition did not hold within its poll budget."""


def milli_cpu(req):
    v = (req or {}).get("cpu", "0")
    return int(v[:-1]) if v.endswith("m") else int(float(v) * 1000)


class Cluster:
    def __init__(self, worker_cpu=(4000, 4000, 4000), system_cpu=(250, 0, 0), runner=None, grace=3, ns_queues=False):
        # cycles a terminating pod stays Releasing: the evictor deletes with a
        # 3 s grace period (cache.go:110-123) and a cycle runs every second
        # (--schedule-period 1s, cmd/kube-batch/app/options/options.go:64)
        self.grace = grace
        self.runner = runner  # fixture -> output in the oracle's schema (one Scheduler.runOnce)
        self.nodes = [{"name": "master", "allocatable": {"cpu": "4", "memory": "16Gi", "pods": "110"},
                       "labels": {"kubernetes.io/hostname": "master"}, "taints": [dict(MASTER_TAINT)]}]
        for i, c in enumerate(worker_cpu):
            self.nodes.append({"name": f"node-{i + 1}", "allocatable": {"cpu": f"{c}m", "memory": "16Gi",
                                                                         "pods": "110"},
                               "labels": {"kubernetes.io/hostname": f"node-{i + 1}"}})
        # queue CRDs q1, q2 and the context namespace's (util.go:180-216), or —
        # ENABLE_NAMESPACES_AS_QUEUE, which hack/run-e2e.sh:11-15 toggles at
        # random — every namespace a queue of weight 1 (event_handlers.go:726-736)
        self.ns_queues = ns_queues
        self.queues = [] if ns_queues else [{"name": "q1", "weight": 1}, {"name": "q2", "weight": 1},
                                            {"name": "test", "weight": 1}]
        self.namespaces = ["kube-system", "test", "q1", "q2"] if ns_queues else []
        self.pods, self.pgs = [], []
        self.templates = {}  # pod uid -> template the Job controller recreates it from
        self.terminating = {}  # uid -> scheduling cycles left before the pod is gone
        self.uid = 0
        self.clock = 0
        self.evictions = []  # (victim uid, group, cycle)
        self.last = None
        self.cycles = 0
        # kube-system pods (no scheduler of ours, no PodGroup): part of node usage
        for i, c in enumerate(system_cpu):
            if c:
                self._pod("kube-system", f"sys-{i}", {"cpu": f"{c}m"}, None, node=f"node-{i + 1}",
                          phase="Running")

    # ------------------------------------------------------------ objects
    def _pod(self, ns, name, req, group, node="", phase="Pending", **kw):
        self.uid += 1
        p = {"uid": f"u{self.uid:05d}", "namespace": ns, "name": f"{name}-{self.uid}", "phase": phase,
             "nodeName": node, "containers": [{"requests": dict(req or {})}]}
        if group:
            p["annotations"] = {GROUP: group}
        for k, v in kw.items():
            if v is not None:
                p[k] = copy.deepcopy(v)
        self.pods.append(p)
        return p

    def create_job(self, name, tasks, ns=None, queue="", min_member=None):
        """createJobEx (util.go:279-340): one batch Job per task spec, one
        PodGroup with MinMember = sum of the tasks' min (or the override), in
        getNS's namespace (util.go:262-277: the job's queue when namespaces
        are queues, else the context's)."""
        if ns is None:
            ns = queue if (self.ns_queues and queue) else "test"
        self.clock += 1
        mn = 0
        for i, t in enumerate(tasks):
            tmpl = {"ns": ns, "name": f"{name}-{i}", "req": t.get("req"), "group": name,
                    "priority": PRIORITY.get(t.get("pri")), "labels": t.get("labels"),
                    "affinity": t.get("affinity")}
            if t.get("hostport"):
                tmpl["ports"] = [{"hostPort": t["hostport"], "containerPort": t["hostport"]}]
            for _ in range(t["rep"]):
                self._from_template(tmpl)
            mn += t["min"]
        self.pgs.append({"namespace": ns, "name": name, "minMember": mn if min_member is None else min_member,
                         "queue": queue, "creationTimestamp": self.clock})

    def _from_template(self, tmpl):
        p = self._pod(tmpl["ns"], tmpl["name"], tmpl["req"], tmpl["group"], priority=tmpl["priority"],
                      labels=tmpl["labels"], affinity=tmpl["affinity"])
        if tmpl.get("ports"):
            p["containers"][0]["ports"] = copy.deepcopy(tmpl["ports"])
        self.templates[p["uid"]] = tmpl
        return p

    def _free(self, node):
        alloc = milli_cpu(node["allocatable"])
        used = sum(milli_cpu(p["containers"][0]["requests"]) for p in self.pods
                   if p["nodeName"] == node["name"] and p["uid"] not in self.terminating)
        return alloc - used

    def create_replicaset(self, name, rep, req):
        """createReplicaSet (util.go:490-535): pods of the default scheduler,
        placed first-fit on untainted nodes, Running once placed."""
        for _ in range(rep):
            for n in self.nodes:
                if not n.get("taints") and self._free(n) >= milli_cpu(req):
                    self._pod("test", name, req, None, node=n["name"], phase="Running", labels={"rs": name})
                    break
            else:
                raise AssertionError(f"replicaset {name}: no room for a pod")

    def delete_replicaset(self, name):
        for p in self.pods:
            if (p.get("labels") or {}).get("rs") == name and p["uid"] not in self.terminating:
                self._terminate(p)

    def taint_all(self, taints):  # util.go taintAllNodes (workers; the master keeps its own)
        for n in self.nodes:
            if n["name"] != "master":
                n["taints"] = copy.deepcopy(taints)

    def untaint_all(self):
        for n in self.nodes:
            if n["name"] != "master":
                n.pop("taints", None)

    def _terminate(self, p):
        p["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        self.terminating[p["uid"]] = self.grace

    # ------------------------------------------------------------ cycles
    def fixture(self):
        fx = {"actions": list(CONF_ACTIONS), "tiers": copy.deepcopy(CONF_TIERS), "nodes": copy.deepcopy(self.nodes),
              "pods": copy.deepcopy(self.pods), "podGroups": copy.deepcopy(self.pgs),
              "queues": copy.deepcopy(self.queues)}
        if self.namespaces:
            fx["namespaces"] = list(self.namespaces)
        return fx

    def cycle_once(self):
        self.cycle(self.runner)

    def cycle(self, runner):
        """One Scheduler.runOnce, then the cluster's reaction to its binds and
        evictions."""
        gone = {u for u, k in self.terminating.items() if k <= 1}  # their grace ends with this cycle
        out = runner(self.fixture())
        assert out["status"] == "ok", out.get("error")
        self.cycles += 1
        self.last = out
        by_key = {f"{p['namespace']}/{p['name']}": p for p in self.pods}
        by_uid = {p["uid"]: p for p in self.pods}
        self.pods = [p for p in self.pods if p["uid"] not in gone]
        self.terminating = {u: k - 1 for u, k in self.terminating.items() if u not in gone}
        for key, node in out["binds"].items():
            p = by_key[key]
            p["nodeName"], p["phase"] = node, "Running"
        for ev in out.get("evictions", []):
            p = by_uid[ev["task"]]
            self.evictions.append((p["uid"], (p.get("annotations") or {}).get(GROUP), self.cycles))
            self._terminate(p)
            tmpl = self.templates.get(p["uid"])
            if tmpl:  # the batch Job replaces a pod that is going away
                self._from_template(tmpl)

    def wait(self, cond, max_cycles=60):
        """wait.Poll(..., oneMinute, cond) of the e2e helpers: true as soon as
        `cond` holds between two cycles (checked before the first one too),
        not at a steady state — preemption under the conf's tiers can
        oscillate (gang's tier decides Preemptable alone, session_plugins.go:
        100-140, so a preemptee can lose every task above MinAvailable)."""
        for _ in range(max_cycles + 1):
            if cond():
                return
            self.cycle(self.runner)
        raise WaitTimeout(f"condition not reached within {max_cycles} cycles")

    def settle(self, cycles=4):
        """A few more cycles (the state a spec asserts without a wait)."""
        for _ in range(cycles):
            self.cycle(self.runner)

    # ------------------------------------------------------------ e2e helpers
    def size(self, req):
        """clusterSize (util.go:566-615): slots of `req` on untainted nodes."""
        n = 0
        for nd in self.nodes:
            if not nd.get("taints"):
                n += max(0, self._free(nd)) // milli_cpu(req)
        return n

    def compute_node(self, req):
        """computeNode (util.go:635-690): the first untainted node with room."""
        for nd in self.nodes:
            if not nd.get("taints"):
                k = max(0, self._free(nd)) // milli_cpu(req)
                if k > 0:
                    return nd["name"], k
        return "", 0

    def node_number(self):  # clusterNodeNumber (util.go:618-633)
        return sum(1 for nd in self.nodes if not nd.get("taints"))

    def group_pods(self, pg):
        return [p for p in self.pods if (p.get("annotations") or {}).get(GROUP) == pg]

    def running(self, pg, pri=None):
        """taskPhase / taskPhaseEx with Running|Succeeded (util.go:342-398,
        449-457): a count of `pod.Status.Phase` alone, so a pod in its
        eviction grace period (deletionTimestamp set, containers still up:
        phase Running) counts, as it does against the live cluster."""
        return sum(1 for p in self.group_pods(pg) if p["phase"] == "Running"
                   and (pri is None or p.get("priority") == PRIORITY[pri]))

    def pending(self, pg):
        return sum(1 for p in self.group_pods(pg) if p["phase"] == "Pending")

    def min_member(self, pg):
        return next(g["minMember"] for g in self.pgs if g["name"] == pg)

    def unschedulable(self, pg):
        """The Unschedulable condition gang's OnSessionClose sets on a job that
        is not ready (gang.go:169-190), in the last cycle."""
        return any(j["uid"].endswith("/" + pg) and not j["ready"] for j in self.last["jobs"])

    def evicted(self, pg, since_cycle=0):  # podGroupEvicted (util.go:419-438)
        return any(g == pg and c > since_cycle for _, g, c in self.evictions)

    def nodes_of(self, pg):
        return [p["nodeName"] for p in self.group_pods(pg) if p["phase"] == "Running"]
