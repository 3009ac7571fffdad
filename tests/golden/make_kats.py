"""Hand-derived known-answer fixtures (KATs) for paths the reference's own
tests do not pin. Each expected value below was derived by
reading the cited reference code, not by running any implementation.

Run: python tests/golden/make_kats.py   (rewrites tests/golden/kat_*.json)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def pod(uid, name, req, ns="ns", group="pg1", phase="Pending", node="", **kw):
    p = {"uid": uid, "namespace": ns, "name": name, "phase": phase, "nodeName": node,
         "containers": [{"requests": req}]}
    if group:
        p["annotations"] = {"scheduling.k8s.io/group-name": group}
    p.update(kw)
    return p


def node(name, cpu, mem="64Gi", pods="110", **kw):
    alloc = {"cpu": cpu, "memory": mem}
    if pods is not None:
        alloc["pods"] = pods
    n = {"name": name, "allocatable": alloc}
    n.update(kw)
    return n


Q = [{"name": "q", "weight": 1}]
GI = 1024 ** 3


def pg(name="pg1", ns="ns", minMember=0, created=0, queue="q"):
    return {"namespace": ns, "name": name, "minMember": minMember, "queue": queue, "creationTimestamp": created}


KATS = {
    # resource_info.go:142-146: |idle - req| < 10 mCPU counts as a fit and
    # drives Idle to -9 (Sub only panics beyond the tolerance, :100-110).
    # Next task: LessEqual(1m, -9m) is false (|-9-1| = 10 is not < 10).
    "kat_tolerance_edge": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "1", "1Gi"), node("n2", "1", "1Gi")],
        "pods": [pod("a", "pa", {"cpu": "1009m", "memory": "1Mi"}),
                 pod("b", "pb", {"cpu": "1m", "memory": "20Mi"}),
                 pod("c", "pc", {"cpu": "1011m", "memory": "1Mi"})],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["a", "n1", "allocate"], ["b", "n2", "allocate"]],
                     "binds": {"ns/pa": "n1", "ns/pb": "n2"}},
    },
    # allocate.go:131-161: Idle misses, Releasing fits -> Pipeline (no dispatch,
    # session.go:205-241); gang counts Pipelined as ready (gang.go:44-55).
    # The releasing pod (Running + deletionTimestamp) holds 2 CPU / 1Gi.
    "kat_pipeline": {
        "tiers": [[{"name": "gang"}], [{"name": "predicates"}]],
        "nodes": [node("n1", "2", "4Gi")],
        "pods": [pod("r", "old", {"cpu": "2", "memory": "1Gi"}, ns="other", group=None, phase="Running",
                     node="n1", deletionTimestamp="2026-01-01T00:00:00Z"),
                 pod("t1", "p1", {"cpu": "1", "memory": "512Mi"}),
                 pod("t2", "p2", {"cpu": "1", "memory": "512Mi"}),
                 pod("t3", "p3", {"cpu": "1", "memory": "512Mi"})],
        "podGroups": [pg(minMember=2)], "queues": Q,
        "expected": {"decisions": [["t1", "n1", "pipeline"], ["t2", "n1", "pipeline"]], "binds": {},
                     "ready": {"ns/pg1": True}},
    },
    # gang.go:129-163 job order + session.go:283-290 dispatch: pg1 (older) goes
    # first until ready (3 of 4), then non-ready pg2 ranks ahead of ready pg1;
    # FitError (job_info.go:329-358) of pg1's failed last task a4: cpu only
    # (FitDelta skips dims the task does not request, resource_info.go:116-129).
    "kat_gang_dispatch": {
        "tiers": [[{"name": "priority"}, {"name": "gang"}], [{"name": "drf"}, {"name": "predicates"}]],
        "nodes": [node("n1", "4", "4Gi")],
        "pods": [pod(f"a{i}", f"a{i}", {"cpu": "1"}, group="pg1") for i in range(1, 5)] +
                [pod("b1", "b1", {"cpu": "1"}, group="pg2")],
        "podGroups": [pg("pg1", minMember=3, created=0), pg("pg2", minMember=1, created=100)], "queues": Q,
        "expected": {"decisions": [["a1", "n1", "allocate"], ["a2", "n1", "allocate"], ["a3", "n1", "allocate"],
                                   ["b1", "n1", "allocate"]],
                     "binds": {"ns/a1": "n1", "ns/a2": "n1", "ns/a3": "n1", "ns/b1": "n1"},
                     "ready": {"ns/pg1": True, "ns/pg2": True},
                     "fit_error": {"ns/pg1": "0/1 nodes are available, 1 insufficient cpu.",
                                   "ns/pg2": "0 nodes are available"}},
    },
    # priority.go:37-53: higher pod priority first, default priority 1
    # (job_info.go:79), ties by UID (session_plugins.go:266-276).
    "kat_priority_order": {
        "tiers": [[{"name": "priority"}], [{"name": "predicates"}]],
        "nodes": [node("n1", "2")],
        "pods": [pod("a", "pa", {"cpu": "1"}, priority=1), pod("b", "pb", {"cpu": "1"}, priority=10),
                 pod("c", "pc", {"cpu": "1"}, priority=5), pod("d", "pd", {"cpu": "1"})],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["b", "n1", "allocate"], ["c", "n1", "allocate"]]},
    },
    # Static predicates: selector (labels/selector.go:849-866, invalid key =>
    # match all), unschedulable (predicates.go:105-110), taints NoSchedule/
    # NoExecute only (predicates.go:1489-1517), node affinity terms
    # (helpers.go:302-331: empty term list matches nothing, a term with an
    # invalid operator is skipped), Gt on a non-integer label fails, matchFields
    # metadata.name, empty-key Exists toleration tolerates everything.
    "kat_selector_taints": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "10", labels={"zone": "a", "size": "4"},
                       taints=[{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}]),
                  node("n2", "10", labels={"zone": "a", "size": "8"},
                       taints=[{"key": "soft", "value": "", "effect": "PreferNoSchedule"}]),
                  node("n3", "10", labels={"zone": "b"}, unschedulable=True),
                  node("n4", "10", labels={"zone": "b", "size": "x"})],
        "pods": [
            pod("a", "pa", {"cpu": "1"}, nodeSelector={"zone": "b"}),
            pod("b", "pb", {"cpu": "1"}, tolerations=[{"key": "dedicated", "operator": "Equal", "value": "gpu",
                                                      "effect": "NoSchedule"}]),
            pod("c", "pc", {"cpu": "1"}),
            pod("d", "pd", {"cpu": "1"}, nodeSelector={"bad key!": "x"}),
            pod("e", "pe", {"cpu": "1"}, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "NotIn", "values": ["a"]}]}]}}}),
            pod("f", "pf", {"cpu": "1"}, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": [{"key": "size", "operator": "Gt", "values": ["5"]}]}]}}}),
            pod("g", "pg", {"cpu": "1"}, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": []}}}),
            pod("h", "ph", {"cpu": "1"}, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "in", "values": ["b"]}]},
                                      {"matchExpressions": [{"key": "zone", "operator": "Exists"}]}]}}}),
            pod("i", "pi", {"cpu": "1"}, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchFields": [{"key": "metadata.name", "operator": "In",
                                                        "values": ["n4"]}]}]}}}),
            pod("j", "pj", {"cpu": "1"}, tolerations=[{"operator": "Exists"}]),
        ],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["a", "n4", "allocate"], ["b", "n1", "allocate"], ["c", "n2", "allocate"],
                                   ["d", "n2", "allocate"], ["e", "n4", "allocate"], ["f", "n2", "allocate"],
                                   ["h", "n2", "allocate"], ["i", "n4", "allocate"], ["j", "n1", "allocate"]]},
    },
    # F10: without a "pods" allocatable MaxTaskNum is 0 and the cap rejects the
    # node (predicates.go:125-127); with pods=1 the second task is rejected.
    "kat_pod_cap": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4", pods=None), node("n2", "4", pods="1")],
        "pods": [pod("t1", "p1", {"cpu": "1"}), pod("t2", "p2", {"cpu": "1"})],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["t1", "n2", "allocate"]]},
    },
    # F9: a second water-fill round subtracts cumulative deserved
    # (proportion.go:119-140): qb becomes met in round 2 with deserved 8 CPU
    # while remaining is 4 CPU -> Resource.Sub panics.
    "kat_proportion_panic": {
        "tiers": [[{"name": "proportion"}]],
        "nodes": [node("n1", "10", "10Gi")],
        "pods": [pod("a", "pa", {"cpu": "1", "memory": "1Gi"}, group="pga"),
                 pod("b", "pb", {"cpu": "8", "memory": "8Gi"}, group="pgb")],
        "podGroups": [pg("pga", queue="qa"), pg("pgb", queue="qb")],
        "queues": [{"name": "qa", "weight": 1}, {"name": "qb", "weight": 1}],
        "expected": {"status": "ref_panic"},
    },
    # A pod bound to an unknown node creates a NodeInfo with Node == nil
    # (event_handlers.go:51-54); the predicates closure dereferences it when
    # the scan reaches it (predicates.go:122-123). n1 fails first because the
    # same bound pod names a node outside ssn.NodeIndex (vendor
    # predicates.go:1273-1282), so every predicate call errors.
    "kat_nil_node_panic": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4")],
        "pods": [pod("r", "run", {"cpu": "1"}, group="pg1", phase="Running", node="ghost"),
                 pod("t", "pt", {"cpu": "500m"})],
        "podGroups": [pg()], "queues": Q,
        "expected": {"status": "ref_panic"},
    },
    # Same cluster without predicates: the nil node is a zero-resource node.
    "kat_nil_node_nopred": {
        "tiers": [[{"name": "drf"}]],
        "nodes": [node("n1", "4")],
        "pods": [pod("r", "run", {"cpu": "1"}, group="pg1", phase="Running", node="ghost"),
                 pod("t", "pt", {"cpu": "500m"})],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["t", "n1", "allocate"]], "binds": {"ns/pt": "n1"}},
    },
    # allocate.go:88-96: BestEffort pods are skipped; gang minMember 2 is then
    # not reached, so nothing is dispatched (session.go:283-290).
    "kat_besteffort": {
        "tiers": [[{"name": "gang"}], [{"name": "predicates"}]],
        "nodes": [node("n1", "4")],
        "pods": [pod("a", "pa", {"cpu": "5m"}), pod("b", "pb", {"cpu": "1"})],
        "podGroups": [pg(minMember=2)], "queues": Q,
        "expected": {"decisions": [["b", "n1", "allocate"]], "binds": {}, "ready": {"ns/pg1": False}},
    },
    # proportion.go:146-159,188-193: queue order by share, overused queues are
    # dropped from the queue heap (allocate.go:71-74).
    "kat_overused": {
        "tiers": [[{"name": "proportion"}]],
        "nodes": [node("n1", "4", "4Gi")],
        "pods": [pod(f"a{i}", f"a{i}", {"cpu": "1"}, group="pga") for i in range(1, 5)] +
                [pod(f"b{i}", f"b{i}", {"cpu": "1"}, group="pgb") for i in range(1, 5)],
        "podGroups": [pg("pga", queue="qa"), pg("pgb", queue="qb")],
        "queues": [{"name": "qa", "weight": 1}, {"name": "qb", "weight": 3}],
        "expected": {"decisions": [["a1", "n1", "allocate"], ["b1", "n1", "allocate"], ["b2", "n1", "allocate"],
                                   ["b3", "n1", "allocate"]]},
    },
    # k8s Quantity -> (MilliValue, Value), both rounding up.
    "kat_quantity": {
        "kind": "quantity",
        "quantities": ["1", "500m", "1.5", "1Gi", "1G", "100Mi", "1e3", "0.1m", "2.5Ki", "1n", "0"],
        "expected": {"values": [[1000, 1], [500, 1], [1500, 2], [1073741824000, 1073741824],
                                [1000000000000, 1000000000], [104857600000, 104857600], [1000000, 1000],
                                [1, 1], [2560000, 2560], [1, 1], [0, 0]]},
    },
    # vendor predicates.go:1031-1051 PodFitsHostPorts over NewNodeInfo(node.Pods()...),
    # host_ports.go CheckConflict: "" ip = 0.0.0.0 and "" protocol = TCP (sanitize);
    # a 0.0.0.0 side conflicts with every ip of the same (protocol, port), two
    # concrete ips only when equal; hostPort <= 0 never conflicts. The pods on
    # a node include pods outside any session job (web, dns: no PodGroup).
    #   a 10.0.0.2:80/TCP  -> n1 (only 10.0.0.1:80 there)
    #   b 0.0.0.0:80/TCP   -> n1 has TCP 80 -> n2
    #   c 10.0.0.1:53/UDP  -> n1 (no UDP 53 on n1)
    #   d 10.0.0.3:80/TCP  -> n1 (no 0.0.0.0:80 or 10.0.0.3:80 there)
    #   e 10.0.0.1:53/UDP  -> n1 has it (c), n2 has 0.0.0.0:53/UDP -> n3
    #   f :0 + 10.0.0.1:80 -> n1 has it, n2 has 0.0.0.0:80 (b) -> n3 (e is UDP)
    #   g 0.0.0.0:80/UDP   -> n1
    "kat_host_ports": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "8"), node("n2", "8"), node("n3", "8")],
        "pods": [pod("web", "web", {"cpu": "1"}, ns="sys", group=None, phase="Running", node="n1",
                     containers=[{"requests": {"cpu": "1"},
                                  "ports": [{"hostIP": "10.0.0.1", "hostPort": 80, "protocol": "TCP"}]}]),
                 pod("dns", "dns", {"cpu": "1"}, ns="sys", group=None, phase="Running", node="n2",
                     containers=[{"requests": {"cpu": "1"}, "ports": [{"hostPort": 53, "protocol": "UDP"}]}])]
                + [pod(u, "p" + u, {"cpu": "1"}, containers=[{"requests": {"cpu": "1"}, "ports": ports}])
                   for u, ports in (("a", [{"hostIP": "10.0.0.2", "hostPort": 80}]),
                                    ("b", [{"hostPort": 80}]),
                                    ("c", [{"hostIP": "10.0.0.1", "hostPort": 53, "protocol": "UDP"}]),
                                    ("d", [{"hostIP": "10.0.0.3", "hostPort": 80, "protocol": "TCP"}]),
                                    ("e", [{"hostIP": "10.0.0.1", "hostPort": 53, "protocol": "UDP"}]),
                                    ("f", [{"hostPort": 0}, {"hostIP": "10.0.0.1", "hostPort": 80}]),
                                    ("g", [{"hostIP": "0.0.0.0", "hostPort": 80, "protocol": "UDP"}]))],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["a", "n1", "allocate"], ["b", "n2", "allocate"], ["c", "n1", "allocate"],
                                   ["d", "n1", "allocate"], ["e", "n3", "allocate"], ["f", "n3", "allocate"],
                                   ["g", "n1", "allocate"]]},
    },
    # backfill.go:40-71 after allocate (conf "allocate, backfill"): w (1 CPU)
    # takes n1's last pod slot (cap 2 with the running pod) but pg1 needs 2
    # (gang.go:72-78), so it is not dispatched; backfill puts BestEffort x
    # (pg1) on n2 (n1 is at its pod cap, predicates.go:125-127) through
    # ssn.Allocate, pg1 becomes ready and both are bound (session.go:283-290);
    # y, z (pg2) follow on n2.
    "kat_backfill": {
        "actions": ["allocate", "backfill"],
        "tiers": [[{"name": "gang"}], [{"name": "predicates"}]],
        "nodes": [node("n1", "4", pods="2"), node("n2", "4")],
        "pods": [pod("r", "run", {"cpu": "1"}, ns="sys", group=None, phase="Running", node="n1"),
                 pod("w", "pw", {"cpu": "1"}), pod("x", "px", {}),
                 pod("y", "py", {}, group="pg2"), pod("z", "pz", {}, group="pg2")],
        "podGroups": [pg(minMember=2), pg("pg2")], "queues": Q,
        "expected": {"decisions": [["w", "n1", "allocate"], ["x", "n2", "allocate"], ["y", "n2", "allocate"],
                                   ["z", "n2", "allocate"]],
                     "binds": {"ns/pw": "n1", "ns/px": "n2", "ns/py": "n2", "ns/pz": "n2"}},
    },
    # reclaim.go:41-188 with gang + proportion in one tier (session_plugins.go:59-98
    # intersects them). CPU-only requests, so memory shares are Share(0,0)=0.
    # proportion.go:102-144: total 4 CPU, q1 requests 4, q2 requests 2 -> both
    # met in round 1 at 2 CPU deserved; q1 holds 4 (share 2, overused), q2 0.
    # q2 pops first; b1 (1 CPU) on n1: gang keeps all of a1..a4 (A ready 4,
    # MinMember 1); proportion's running allocation 4000 -> 3000 (victim: 2000
    # <= 3000), 2000 (victim), 1000 (no), 0 (no) -> victims [a1, a2]; a1 covers
    # the request (LessEqual), so only a1 is evicted and b1 is pipelined onto
    # n1 (session.go:205-241). Job B is not pushed back (reclaim.go:96-101).
    "kat_reclaim": {
        "actions": ["reclaim"],
        "tiers": [[{"name": "gang"}, {"name": "proportion"}, {"name": "predicates"}]],
        "nodes": [node("n1", "4", "8Gi")],
        "pods": [pod(u, "p" + u, {"cpu": "1"}, group="pgA", ns="na", phase="Running", node="n1")
                 for u in ("a1", "a2", "a3", "a4")]
                + [pod(u, "p" + u, {"cpu": "1"}, group="pgB", ns="nb") for u in ("b1", "b2")],
        "podGroups": [pg("pgA", ns="na", minMember=1, queue="q1"), pg("pgB", ns="nb", minMember=1, queue="q2")],
        "queues": [{"name": "q1", "weight": 1}, {"name": "q2", "weight": 1}],
        "expected": {"decisions": [["b1", "n1", "pipeline"]], "evictions": [["a1", "b1"]],
                     "nodes": {"n1": [[0, 8 * GI, 0], [0, 0, 0], 5]}},
    },
    # preempt.go:43-171, within one queue: P (MinMember 2) preempts V
    # (MinMember 2, 4 running on the full node). gang decides in tier 1
    # (priority has no preemptable fn): V stays >= 2 without the victim while
    # it has 4 then 3 ready tasks. p1 evicts v1 (one victim covers 1 CPU) and
    # is pipelined; P is not ready (1 < 2) so p2 goes next and evicts v2; P is
    # ready, the statement commits (statement.go:207-217).
    "kat_preempt": {
        "actions": ["preempt"],
        "tiers": [[{"name": "priority"}, {"name": "gang"}], [{"name": "drf"}, {"name": "predicates"}]],
        "nodes": [node("n1", "4", "8Gi")],
        "pods": [pod(u, "p" + u, {"cpu": "1"}, group="pgV", phase="Running", node="n1")
                 for u in ("v1", "v2", "v3", "v4")]
                + [pod(u, "p" + u, {"cpu": "1"}, group="pgP") for u in ("p1", "p2")],
        "podGroups": [pg("pgV", minMember=2), pg("pgP", minMember=2)], "queues": Q,
        "expected": {"decisions": [["p1", "n1", "pipeline"], ["p2", "n1", "pipeline"]],
                     "evictions": [["v1", "p1"], ["v2", "p2"]],
                     "nodes": {"n1": [[0, 8 * GI, 0], [0, 0, 0], 6]}},
    },
    # The same with P needing 3: after p1, p2 P is still short, the statement
    # is discarded (statement.go:194-205). unpipeline removes p1, p2 from the
    # node (Releasing += 1 CPU each, node_info.go:131-157); unevict's
    # node.AddTask finds v1, v2 still there as Releasing and fails
    # (node_info.go:101-106), so the node keeps 2 CPU Releasing while the job
    # sees them Running again. Nothing is committed.
    "kat_preempt_discard": {
        "actions": ["preempt"],
        "tiers": [[{"name": "priority"}, {"name": "gang"}], [{"name": "drf"}, {"name": "predicates"}]],
        "nodes": [node("n1", "4", "8Gi")],
        "pods": [pod(u, "p" + u, {"cpu": "1"}, group="pgV", phase="Running", node="n1")
                 for u in ("v1", "v2", "v3", "v4")]
                + [pod(u, "p" + u, {"cpu": "1"}, group="pgP") for u in ("p1", "p2")],
        "podGroups": [pg("pgV", minMember=2), pg("pgP", minMember=3)], "queues": Q,
        "expected": {"decisions": [], "evictions": [],
                     "nodes": {"n1": [[0, 8 * GI, 0], [2000, 0, 0], 4]}},
    },
    # Inter-pod anti-affinity of an existing pod (vendor predicates.go:1244-1332,
    # kube-batch predicates.go:185-198 with meta == nil). Running e (ns, app=db,
    # job pg0 of the session, so the podLister sees it, predicates.go:45-65)
    # forbids (zone, a) to pods its term selects: app=web in e's own namespace
    # (GetNamespacesFromPodAffinityTerm, topologies.go:28-37). w1 skips n1, n2
    # (zone a) for n3; w2 (app=other) and w3 (namespace other) are not selected.
    "kat_pod_anti_affinity_existing": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4", labels={"zone": "a"}), node("n2", "4", labels={"zone": "a"}),
                  node("n3", "4", labels={"zone": "b"})],
        "pods": [pod("e", "e", {"cpu": "1"}, group="pg0", phase="Running", node="n1", labels={"app": "db"},
                     affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "zone"}]}}),
                 pod("w1", "w1", {"cpu": "1"}, labels={"app": "web"}),
                 pod("w2", "w2", {"cpu": "1"}, labels={"app": "other"}),
                 pod("w3", "w3", {"cpu": "1"}, ns="other", group="pg2", labels={"app": "web"})],
        "podGroups": [pg("pg0"), pg(), pg("pg2", ns="other", created=100)], "queues": Q,
        "expected": {"decisions": [["w1", "n3", "allocate"], ["w2", "n1", "allocate"], ["w3", "n1", "allocate"]],
                     "binds": {"ns/w1": "n3", "ns/w2": "n1", "other/w3": "n1"}},
    },
    # The pod's own affinity (vendor predicates.go:1402-1456). a1: no allocated
    # pod matches the term's selector and a1 matches its own term, so it may go
    # anywhere (the "first pod of a series" rule) -> n1, which it fills. a2: a1
    # now matches, so the node must share a1's zone: n2 (zone b) fails, n3
    # (zone a) takes it. c1's term selects nothing and c1 does not match it
    # itself (targetPodMatchesAffinityOfPod): it fits nowhere.
    "kat_pod_affinity_first_pod": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "1", labels={"zone": "a"}), node("n2", "4", labels={"zone": "b"}),
                  node("n3", "4", labels={"zone": "a"})],
        "pods": [pod(u, u, {"cpu": "1"}, labels={"app": "cache"},
                     affinity={"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"app": "cache"}}, "topologyKey": "zone"}]}})
                 for u in ("a1", "a2")]
                + [pod("c1", "c1", {"cpu": "1"}, group="pg2", labels={"app": "other"},
                       affinity={"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                           {"labelSelector": {"matchLabels": {"app": "nothing"}}, "topologyKey": "zone"}]}})],
        "podGroups": [pg(), pg("pg2", created=100)], "queues": Q,
        "expected": {"decisions": [["a1", "n1", "allocate"], ["a2", "n3", "allocate"]],
                     "binds": {"ns/a1": "n1", "ns/a2": "n3"}},
    },
    # Own anti-affinity on a per-node topology key: one app=spread pod per
    # node. s2 sees s1 on n1 (both as s1's existing anti term, :1244-1332, and
    # as its own, :1428-1436); s3 finds both nodes taken.
    "kat_pod_anti_affinity_spread": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4", labels={"host": "n1"}), node("n2", "4", labels={"host": "n2"})],
        "pods": [pod(u, u, {"cpu": "1"}, labels={"app": "spread"},
                     affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"app": "spread"}}, "topologyKey": "host"}]}})
                 for u in ("s1", "s2", "s3")],
        "podGroups": [pg()], "queues": Q,
        "expected": {"decisions": [["s1", "n1", "allocate"], ["s2", "n2", "allocate"]],
                     "binds": {"ns/s1": "n1", "ns/s2": "n2"}},
    },
    # Errors fail the predicate. x1's anti term has an invalid operator
    # (LabelSelectorAsSelector, helpers.go:46-59): with any allocated pod in
    # the podLister the error is reached (:1428-1435). y1's affinity term has an
    # empty topologyKey: the running e matches its selector, so
    # podMatchesPodAffinityTerms returns the error (:1205-1208). z1 is plain.
    "kat_pod_affinity_errors": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4", labels={"zone": "a"})],
        "pods": [pod("e", "e", {"cpu": "1"}, group="pg0", phase="Running", node="n1", labels={"app": "db"}),
                 pod("x1", "x1", {"cpu": "1"}, affinity={"podAntiAffinity": {
                     "requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchExpressions": [{"key": "app", "operator": "Foo", "values": ["a"]}]},
                          "topologyKey": "zone"}]}}),
                 pod("y1", "y1", {"cpu": "1"}, affinity={"podAffinity": {
                     "requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": ""}]}}),
                 pod("z1", "z1", {"cpu": "1"})],
        "podGroups": [pg("pg0"), pg()], "queues": Q,
        "expected": {"decisions": [["z1", "n1", "allocate"]], "binds": {"ns/z1": "n1"}},
    },
    # An allocated pod whose anti term fails to build its selector makes
    # getMatchingAntiAffinityTopologyPairsOfPods return the error for every
    # incoming pod on every node (:1270-1289, :1310-1314): nothing is placed.
    "kat_pod_anti_affinity_poison": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "4", labels={"zone": "a"}), node("n2", "4", labels={"zone": "b"})],
        "pods": [pod("e", "e", {"cpu": "1"}, group="pg0", phase="Running", node="n1",
                     affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"bad key!": "x"}}, "topologyKey": "zone"}]}}),
                 pod("p1", "p1", {"cpu": "1"})],
        "podGroups": [pg("pg0"), pg()], "queues": Q,
        "expected": {"decisions": [], "binds": {}},
    },
    # NodeInfo.AddTask keys the node's tasks by PodKey "<ns>/<name>"
    # (node_info.go:101-106, api/helpers.go:27-33): t1 is a new pod named like
    # the Running r still on n1, so ssn.Allocate logs t1 -> n1 and runs the
    # handlers but AddTask returns "already on node" and Idle stays 1 CPU
    # (session.go:243-293); t2 then fits the same CPU. Without the key rule
    # t2 would find Idle 0 and fit nowhere.
    "kat_dup_pod_key": {
        "tiers": [[{"name": "predicates"}]],
        "nodes": [node("n1", "2")],
        "pods": [pod("r", "p1", {"cpu": "1"}, group="pg0", phase="Running", node="n1"),
                 pod("t1", "p1", {"cpu": "1"}),
                 pod("t2", "p2", {"cpu": "1"})],
        "podGroups": [pg("pg0"), pg()], "queues": Q,
        "expected": {"decisions": [["t1", "n1", "allocate"], ["t2", "n1", "allocate"]],
                     "binds": {"ns/p1": "n1", "ns/p2": "n1"},
                     "nodes": {"n1": [[0.0, 64.0 * GI, 0.0], [0.0, 0.0, 0.0], 2]}},
    },
    # kat_preempt_discard with the key's holder placed in the same statement:
    # p1 and p2 share the pod key ns/px, pgP needs 3 and p3 (selector matches
    # nothing) fits nowhere. p1 evicts one of v1..v4 (pgV, 4 running, min 2)
    # and is pipelined (Releasing 1 -> 0, node_info.go:117-118); p2 evicts
    # another (gang: 3 still ready) and its pipeline's AddTask finds ns/px
    # taken by p1's copy (node_info.go:101-106), node unchanged. The discard
    # runs backwards (statement.go:194-205): unpipeline(p2)'s RemoveTask by key
    # removes p1's Pipelined copy (Releasing += 1 CPU, node_info.go:145-146),
    # the second victim's unevict finds it still there, unpipeline(p1)'s
    # RemoveTask finds no ns/px (an error, no change), the first victim's
    # unevict as well. n1: Releasing 2 CPU (both victims), 4 pods, nothing
    # committed.
    "kat_preempt_discard_placed_holder": {
        "actions": ["preempt"],
        "tiers": [[{"name": "priority"}, {"name": "gang"}], [{"name": "drf"}, {"name": "predicates"}]],
        "nodes": [node("n1", "4", "8Gi")],
        "pods": [pod(u, "p" + u, {"cpu": "1"}, group="pgV", phase="Running", node="n1")
                 for u in ("v1", "v2", "v3", "v4")]
                + [pod("p1", "px", {"cpu": "1"}, group="pgP"), pod("p2", "px", {"cpu": "1"}, group="pgP"),
                   pod("p3", "p3", {"cpu": "1"}, group="pgP", nodeSelector={"zone": "nowhere"})],
        "podGroups": [pg("pgV", minMember=2), pg("pgP", minMember=3, created=10)], "queues": Q,
        "expected": {"decisions": [], "evictions": [], "binds": {},
                     "nodes": {"n1": [[0, 8 * GI, 0], [2000, 0, 0], 4]}},
    },
    # The podLister Filter (kube-batch predicates.go:67-89, vendor
    # cache/node_info.go:692-702): a pod whose spec names node n but that is
    # missing from n's pods is left out of n's inter-pod affinity checks.
    # One queue, action preempt; gang decides readiness (its victim fn
    # disabled), drf picks victims (its job order disabled, so pgP — created
    # first — precedes pgW: session_plugins.go JobOrderFn's timestamp
    # fallback). Cluster CPU 7: n1 (3) runs h (app=db, key ns/px, pgH), v1
    # (pgV, 3 tasks), y1 (pgY, 2 tasks); n2 (4) runs p0 (pgP), v2, v3, y2.
    # p (key ns/px): drf (drf.go:80-105) takes a preemptee whose job keeps a
    # share >= pgP's with p, 2/7: on n1 only v1 (pgV 2/7; pgY 1/7, pgH 0).
    # p evicts v1 and is pipelined: AddTask refuses the taken key
    # (node_info.go:101-106). p2 (selector matches nothing) fails; pgP (min 3)
    # has p0 + p = 2 and the statement is discarded (statement.go:194-205):
    # RemoveTask by key takes h off n1 (Idle +1), v1's unevict finds it still
    # Releasing. w (anti-affinity to app=db per host) on n1: h's spec still
    # names n1 but n1's pods lack it, so the Filter drops it and n1 passes;
    # drf takes y1 (pgY keeps 1/7 = pgW's share with w). w is pipelined, pgW
    # is ready, the statement commits. Without the Filter n1 fails and w goes
    # to n2. n1: Idle 1 CPU, Releasing 1 (v1 then y1 released, w took one).
    "kat_podlister_filter": {
        "actions": ["preempt"],
        "tiers": [[{"name": "priority"}, {"name": "gang", "disablePreemptable": True}],
                  [{"name": "drf", "disableJobOrder": True}, {"name": "predicates"}]],
        "nodes": [node("n1", "3", labels={"kubernetes.io/hostname": "n1"}),
                  node("n2", "4", labels={"kubernetes.io/hostname": "n2"})],
        "pods": [pod("h", "px", {"cpu": "1"}, group="pgH", phase="Running", node="n1", labels={"app": "db"}),
                 pod("v1", "v1", {"cpu": "1"}, group="pgV", phase="Running", node="n1"),
                 pod("y1", "y1", {"cpu": "1"}, group="pgY", phase="Running", node="n1"),
                 pod("p0", "p0", {"cpu": "1"}, group="pgP", phase="Running", node="n2"),
                 pod("v2", "v2", {"cpu": "1"}, group="pgV", phase="Running", node="n2"),
                 pod("v3", "v3", {"cpu": "1"}, group="pgV", phase="Running", node="n2"),
                 pod("y2", "y2", {"cpu": "1"}, group="pgY", phase="Running", node="n2"),
                 pod("p", "px", {"cpu": "1"}, group="pgP"),
                 pod("p2", "p2", {"cpu": "1"}, group="pgP", nodeSelector={"zone": "nowhere"}),
                 pod("w", "w", {"cpu": "1"}, group="pgW",
                     affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                         {"labelSelector": {"matchLabels": {"app": "db"}},
                          "topologyKey": "kubernetes.io/hostname"}]}})],
        "podGroups": [pg("pgH", minMember=1), pg("pgV", minMember=1), pg("pgY", minMember=1),
                      pg("pgP", minMember=3, created=10), pg("pgW", minMember=1, created=20)],
        "queues": Q,
        "expected": {"decisions": [["w", "n1", "pipeline"]], "evictions": [["y1", "w"]], "binds": {},
                     "nodes": {"n1": [[1000, 64 * GI, 0], [1000, 0, 0], 3],
                               "n2": [[0, 64 * GI, 0], [0, 0, 0], 4]}},
    },
}


def main():
    for name, fx in KATS.items():
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fx, f, indent=1)
            f.write("\n")
    print("wrote", len(KATS), "KATs")


if __name__ == "__main__":
    main()
