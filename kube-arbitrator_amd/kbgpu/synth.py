"""Seeded synthetic sessions in the fixture schema (k8s-like objects).

`config_fixture(cid)` builds BASELINE.json's configs C1-C4 as SURVEY §8(d)
specifies them (seed 20261015 + config id); `random_fixture(seed)` builds
small adversarial sessions for parity fuzzing (tight capacity, releasing
pods, BestEffort pods, priorities, selectors/affinity/taints, gang minimums,
several queues, random tiers and disable flags).
The same dicts feed the kbref oracle (as JSON) and the device path.
"""
import random

BASE_SEED = 20261015
GI = 1024 ** 3

CONFIGS = {
    1: dict(nodes=100, jobs=20, tasks_per_job=50, mix="c1", queues=[("default", 1)],
            tiers=[[{"name": "priority"}, {"name": "gang"}],
                   [{"name": "drf"}, {"name": "predicates"}, {"name": "nodeorder"}]]),
    2: dict(nodes=1000, jobs=200, tasks_per_job=50, mix="hetero", queues=[("q1", 1), ("q2", 1)], tiers=None),
    3: dict(nodes=5000, jobs=2000, tasks_per_job=50, mix="hetero", queues=[("q1", 1), ("q2", 2), ("q3", 3), ("q4", 4)],
            tiers=None, over=1.15),
    4: dict(nodes=20000, jobs=10000, tasks_per_job=50, mix="hetero4", queues=[("q1", 1), ("q2", 2), ("q3", 3), ("q4", 4)],
            tiers=None),
}

# C5: contended cluster at ~95% CPU utilisation (reclaim, allocate, backfill, preempt)
C5 = dict(nodes=10000, jobs=4000, tasks_per_job=50, pending_jobs=200, util=0.95,
          queues=[("q1", 1), ("q2", 2), ("q3", 3), ("q4", 4)])

NODE_TYPES = {  # (type, cpu cores, memory GiB, gpus)
    "cpu": (32, 128, 0),
    "mem": (64, 256, 0),
    "gpu": (96, 512, 8),
}


def _node(i, rng, mix):
    name = f"node-{i:05d}"
    if mix == "c1":
        ntype, (cpu, mem, gpu) = "cpu", NODE_TYPES["cpu"]
    else:
        ntype = ("cpu", "mem", "gpu")[rng.randrange(3)]
        cpu, mem, gpu = NODE_TYPES[ntype]
        if mix == "hetero4":
            mem = min(mem, 256)  # keep Σ memory < 2^53 at 20k nodes
    alloc = {"cpu": str(cpu), "memory": f"{mem}Gi", "nvidia.com/gpu": str(gpu), "pods": "110"}
    n = {"name": name, "allocatable": alloc,
         "labels": {"zone": f"z{i % 4}", "type": ntype, "rack": f"r{i % 50}", "cores": str(cpu)}}
    if mix != "c1":
        taints = []
        if ntype == "gpu":
            taints.append({"key": "dedicated", "value": "gpu", "effect": "NoSchedule"})
        if rng.random() < 0.05:
            taints.append({"key": "maint", "value": "", "effect": "NoExecute"})
        if taints:
            n["taints"] = taints
        if rng.random() < 0.02:
            n["unschedulable"] = True
    return n


def config_fixture(cid):
    """BASELINE config `cid` (1-5) as a fixture dict."""
    if cid == 5:
        return contended_config()
    if cid == 6:  # not a BASELINE config: C3 with inter-pod (anti)affinity (scale check)
        return affinity_config()
    c = CONFIGS[cid]
    if c.get("over"):
        return over_requested_config(cid)
    rng = random.Random(BASE_SEED + cid)
    nodes = [_node(i, rng, c["mix"]) for i in range(c["nodes"])]
    queues = [{"name": q, "weight": w} for q, w in c["queues"]]
    pods, pgs = [], []
    for j in range(c["jobs"]):
        ns = f"ns{j % 8}"
        pg = f"pg-{j:05d}"
        q = queues[rng.randrange(len(queues))]["name"]
        cpu = ("500m", "1", "2")[rng.randrange(3)]
        mem = ("1Gi", "2Gi", "4Gi")[rng.randrange(3)]
        req = {"cpu": cpu, "memory": mem}
        spec = {}
        if c["mix"] != "c1":
            r = rng.random()
            if r < 0.10:  # GPU job: 1 GPU + tolerate the dedicated taint
                req["nvidia.com/gpu"] = "1"
                spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"}]
            elif r < 0.40:  # 30%: node selector on zone or type
                spec["nodeSelector"] = ({"zone": f"z{rng.randrange(4)}"} if rng.random() < 0.5
                                        else {"type": ("cpu", "mem")[rng.randrange(2)]})
            elif r < 0.45:  # 5%: required node affinity
                k = rng.randrange(3)
                if k == 0:
                    expr = {"key": "rack", "operator": "In", "values": [f"r{x}" for x in rng.sample(range(50), 10)]}
                elif k == 1:
                    expr = {"key": "zone", "operator": "NotIn", "values": [f"z{rng.randrange(4)}"]}
                else:
                    expr = {"key": "cores", "operator": "Gt", "values": ["40"]}
                spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                    "nodeSelectorTerms": [{"matchExpressions": [expr]}]}}}
        min_member = 50 if cid == 1 else (1, 25, 50)[rng.randrange(3)]
        pgs.append({"namespace": ns, "name": pg, "minMember": min_member, "queue": q,
                    "creationTimestamp": (1_700_000_000 + j) * 1_000_000_000})
        for t in range(c["tasks_per_job"]):
            p = {"uid": f"uid-{j:05d}-{t:03d}", "namespace": ns, "name": f"{pg}-{t:03d}", "phase": "Pending",
                 "annotations": {"scheduling.k8s.io/group-name": pg}, "containers": [{"requests": dict(req)}]}
            p.update(spec)
            pods.append(p)
    return {"name": f"C{cid}", "tiers": c["tiers"], "nodes": nodes, "pods": pods, "podGroups": pgs, "queues": queues}


def over_requested_config(cid=3):
    """BASELINE config 3 as SURVEY §8(d) specifies it: 5k nodes of the C2 mix,
    2k gang PodGroups x 50 pending tasks, `minAvailable` in {1, 25, 50}, 4
    proportion queues of weights {1, 2, 3, 4}, ALL over-requested: every
    queue's request exceeds its deserved share (total x w / 10) in every
    dimension (cpu, memory, GPU), so the proportion water-fill ends after one
    round (proportion.go:102-144, no F9 hazard), demand exceeds capacity by
    the factor `over`, queues become Overused (allocate.go:71-74,
    proportion.go:188-193) and tasks fail once the cluster fills.
    Jobs go to the queues in the weighted pattern q1 q2 q2 q3 q3 q3 q4 q4 q4 q4
    (job j by j % 10), so each queue holds w / 10 of the jobs; one job in ten
    is a GPU job (2 GPUs per task, tolerates the GPU nodes' taint), one per
    pattern residue in every block of 100 jobs; 30% of the others carry a
    zone / type node selector and 5% a required node affinity. A job's tasks
    share one (cpu, memory) request, drawn per job and scaled so the total
    requested is `over` x the cluster's allocatable in cpu and memory."""
    c = CONFIGS[cid]
    rng = random.Random(BASE_SEED + cid)
    nodes = [_node(i, rng, c["mix"]) for i in range(c["nodes"])]
    queues = [{"name": q, "weight": w} for q, w in c["queues"]]
    pattern = [q for q, w in c["queues"] for _ in range(w)]  # weights in jobs out of every len(pattern)
    total_cpu = sum(int(n["allocatable"]["cpu"]) * 1000 for n in nodes)        # milli
    total_mem = sum(int(n["allocatable"]["memory"][:-2]) * 1024 for n in nodes)  # Mi
    total_gpu = sum(int(n["allocatable"]["nvidia.com/gpu"]) for n in nodes)
    J, T = c["jobs"], c["tasks_per_job"]
    base = []
    for j in range(J):
        gpu_job = (j // len(pattern)) % len(pattern) == j % len(pattern)
        base.append((rng.choice((1, 2, 3, 4, 6, 8)), rng.choice((2, 3, 4, 5, 6)), gpu_job, rng.random(), rng.random(),
                     rng.randrange(4), rng.randrange(2), rng.randrange(3), rng.sample(range(50), 10), rng.random()))
    cpu_scale = c["over"] * total_cpu / (T * sum(b[0] for b in base))
    mem_scale = c["over"] * total_mem / (T * sum(b[0] * b[1] for b in base))
    n_gpu_tasks = T * sum(1 for b in base if b[2])
    gpus_per_task = max(1, -(-int(c["over"] * total_gpu) // max(1, n_gpu_tasks)))
    pods, pgs = [], []
    for j, (units, mem_per, gpu_job, r, r2, zone, typ, aff_kind, racks, mm) in enumerate(base):
        ns = f"ns{j % 8}"
        pg = f"pg-{j:05d}"
        q = pattern[j % len(pattern)]
        cpu = max(50, int(units * cpu_scale) // 50 * 50)
        mem = max(64, int(units * mem_per * mem_scale) // 64 * 64)
        req = {"cpu": f"{cpu}m", "memory": f"{mem}Mi"}
        spec = {}
        if gpu_job:
            req["nvidia.com/gpu"] = str(gpus_per_task)
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"}]
        elif r < 0.30:
            spec["nodeSelector"] = {"zone": f"z{zone}"} if r2 < 0.5 else {"type": ("cpu", "mem")[typ]}
        elif r < 0.35:
            expr = ({"key": "rack", "operator": "In", "values": [f"r{x}" for x in racks]} if aff_kind == 0 else
                    {"key": "zone", "operator": "NotIn", "values": [f"z{zone}"]} if aff_kind == 1 else
                    {"key": "cores", "operator": "Gt", "values": ["40"]})
            spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": [expr]}]}}}
        pgs.append({"namespace": ns, "name": pg, "minMember": (1, 25, 50)[int(mm * 3)], "queue": q,
                    "creationTimestamp": (1_700_000_000 + j) * 1_000_000_000})
        for t in range(T):
            p = {"uid": f"uid-{j:05d}-{t:03d}", "namespace": ns, "name": f"{pg}-{t:03d}", "phase": "Pending",
                 "annotations": {"scheduling.k8s.io/group-name": pg}, "containers": [{"requests": dict(req)}]}
            p.update(spec)
            pods.append(p)
    return {"name": f"C{cid}", "tiers": c["tiers"], "nodes": nodes, "pods": pods, "podGroups": pgs, "queues": queues}


def queue_demand(fx):
    """Per queue: (weight, requested, total x weight / sum of weights) in
    (milli-cpu, Mi, GPU) — the first water-fill round of proportion.go:102-144
    (no Others: every pod belongs to a PodGroup)."""
    def q(v, unit):
        v = str(v)
        if v.endswith("m"):
            return int(v[:-1]) / 1000 * unit
        if v.endswith("Mi"):
            return int(v[:-2])
        if v.endswith("Gi"):
            return int(v[:-2]) * 1024
        return float(v) * unit
    tot = [0.0, 0.0, 0.0]
    for n in fx["nodes"]:
        a = n["allocatable"]
        tot[0] += q(a["cpu"], 1000)
        tot[1] += q(a["memory"], 1)
        tot[2] += q(a.get("nvidia.com/gpu", "0"), 1)
    pgq = {(g["namespace"], g["name"]): g["queue"] for g in fx["podGroups"]}
    req = {}
    for p in fx["pods"]:
        r = p["containers"][0]["requests"]
        k = pgq[(p["namespace"], p["annotations"]["scheduling.k8s.io/group-name"])]
        acc = req.setdefault(k, [0.0, 0.0, 0.0])
        acc[0] += q(r.get("cpu", "0"), 1000)
        acc[1] += q(r.get("memory", "0"), 1)
        acc[2] += q(r.get("nvidia.com/gpu", "0"), 1)
    W = sum(x["weight"] for x in fx["queues"])
    return {x["name"]: (x["weight"], req.get(x["name"], [0, 0, 0]), [t * x["weight"] / W for t in tot])
            for x in fx["queues"]}


def saturated_config(nodes=5000, jobs=2000, tasks_per_job=50, demand=1.08, seed=7):
    """C3's cluster (not a BASELINE config: the stress case the verdict asks
    for) with a request drawn per task instead of per job, and total demand
    about `demand` x the schedulable CPU, so the cluster fills up during the
    cycle: many (class, request) shapes fail mid-batch at the default K,
    which cuts batches and replays the ordering engine, and late tasks walk
    long infeasible prefixes. 10% of the jobs are GPU jobs (1-2 GPUs, tolerate
    the dedicated taint), 30% carry a zone / type selector."""
    rng = random.Random(BASE_SEED + 200 + seed)
    nds = [_node(i, rng, "hetero") for i in range(nodes)]
    usable = sum(int(n["allocatable"]["cpu"]) * 1000 for n in nds
                 if not n.get("unschedulable") and n["labels"]["type"] != "gpu")
    queues = [{"name": q, "weight": w} for q, w in (("q1", 1), ("q2", 2), ("q3", 3), ("q4", 4))]
    cpus = (250, 500, 1000, 1500, 2000, 3000, 4000, 6000)
    mems = (0.5, 1, 2, 3, 4, 6, 8, 12, 16)
    mean_cpu = sum(cpus) / len(cpus)
    scale = demand * usable / (0.9 * jobs * tasks_per_job * mean_cpu)  # GPU jobs land on the GPU nodes
    pods, pgs = [], []
    for j in range(jobs):
        ns = f"ns{j % 8}"
        pg = f"pg-{j:05d}"
        spec = {}
        r = rng.random()
        gpu_job = r < 0.10
        if gpu_job:
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"}]
        elif r < 0.40:
            spec["nodeSelector"] = ({"zone": f"z{rng.randrange(4)}"} if rng.random() < 0.5
                                    else {"type": ("cpu", "mem")[rng.randrange(2)]})
        pgs.append({"namespace": ns, "name": pg, "minMember": (1, 25, 50)[rng.randrange(3)],
                    "queue": queues[rng.randrange(4)]["name"],
                    "creationTimestamp": (1_700_000_000 + j) * 1_000_000_000})
        for t in range(tasks_per_job):
            cpu = max(100, int(rng.choice(cpus) * scale) // 50 * 50)
            req = {"cpu": f"{cpu}m", "memory": f"{int(rng.choice(mems) * 1024)}Mi"}
            if gpu_job:
                req["nvidia.com/gpu"] = str(rng.choice((1, 1, 2)))
            p = {"uid": f"uid-{j:05d}-{t:03d}", "namespace": ns, "name": f"{pg}-{t:03d}", "phase": "Pending",
                 "annotations": {"scheduling.k8s.io/group-name": pg}, "containers": [{"requests": req}]}
            if rng.random() < 0.2:
                p["priority"] = rng.choice((5, 10))
            p.update(spec)
            pods.append(p)
    return {"name": f"saturated-{seed}", "tiers": None, "nodes": nds, "pods": pods, "podGroups": pgs,
            "queues": queues}


def churn(fx, seed, session_uids, decided=(), bind=0.6, done=0.08, delete=0.03, add=0.02, node_frac=0.02):
    """Cache events between two scheduling cycles of session `fx`
    (kbg_session_update, event_handlers.go): binds of the last cycle's
    Allocate decisions confirmed (the pod Running on its node), completions
    (Running -> Succeeded: the pod leaves its node, stays in its job),
    deletions, new pods of existing jobs (a copy of a job's pod under a new
    UID and name) and node allocatable growth. Returns (changes, fx1): the
    event list in order, and the fixture of the cache after them — updated pods
    move to the end of the pod order (the cache's delete + add), and
    `sessionOrder.jobs` keeps the job order (jobs persist in the cache)."""
    rng = random.Random(seed)
    pods = {p["uid"]: dict(p) for p in fx["pods"]}  # insertion order = cache order
    changes = []

    def update(p):
        pods.pop(p["uid"], None)
        pods[p["uid"]] = p
        changes.append(("pod_update", p))

    for d in decided:  # cache.Bind confirmed: the pod runs where the last cycle put it
        if d["kind"] == "allocate" and rng.random() < bind:
            p = dict(pods[d["task"]], phase="Running", nodeName=d["node"])
            update(p)
    for uid in list(pods):
        p = pods[uid]
        if uid not in session_uids or p.get("phase") != "Running":
            continue
        if rng.random() < done:
            update(dict(p, phase="Succeeded"))
    for uid in list(pods):
        if uid in session_uids and rng.random() < delete:
            changes.append(("pod_delete", pods.pop(uid)))
    groups = {}
    for p in pods.values():
        g = (p.get("annotations") or {}).get("scheduling.k8s.io/group-name")
        if g and p["uid"] in session_uids:
            groups.setdefault((p.get("namespace", ""), g), p)
    keys = sorted(groups)
    for i in range(int(add * len(pods)) + 1):
        if not keys:
            break
        base = groups[keys[rng.randrange(len(keys))]]
        p = dict(base, uid=f"new-{seed}-{i:05d}", name=f"{base['name']}-n{seed}-{i}", phase="Pending", nodeName="")
        p.pop("deletionTimestamp", None)
        pods[p["uid"]] = p
        changes.append(("pod_add", p))
    nodes = [dict(n) for n in fx["nodes"]]
    for n in nodes:
        if rng.random() < node_frac and "cpu" in n["allocatable"]:
            cpu = n["allocatable"]["cpu"]
            cores = int(cpu[:-1]) // 1000 if cpu.endswith("m") else int(float(cpu))
            n["allocatable"] = dict(n["allocatable"], cpu=str(cores + rng.choice((1, 2, 8))))
            changes.append(("node_update", n))
    fx1 = dict(fx, pods=list(pods.values()), nodes=nodes)
    return changes, fx1


def structural(fx, seed, session_jobs, session_uids, session_queues):
    """Structural cache events between two cycles of session `fx`
    (kbg_session_update KBG_EV_NODE_ADD ... QUEUE_DELETE): new nodes, a
    deleted node (its pods stay in their jobs on no NodeInfo), a new PodGroup
    with pods (one of them may run on a new node), a deleted PodGroup (its
    pods stay in the cache outside the session jobs), a new queue with a job,
    a deleted queue (its jobs leave the session), then completions of
    unaffected Running pods. Returns the change list in event order."""
    rng = random.Random(seed)
    changes = []
    pods = {p["uid"]: p for p in fx["pods"]}
    groups = {(g.get("namespace", ""), g["name"]): g for g in fx.get("podGroups", [])}
    sess = [k for k in groups if f"{k[0]}/{k[1]}" in session_jobs]
    gone_nodes, gone_jobs, gone_queues = set(), set(), set()
    new_nodes = []
    for i in range(rng.randint(0, 2)):
        base = rng.choice(fx["nodes"])
        n = dict(base, name=f"nx{seed}-{i}")
        new_nodes.append(n["name"])
        changes.append(("node_add", n))
    if fx["nodes"] and rng.random() < 0.6:
        n = rng.choice(fx["nodes"])
        gone_nodes.add(n["name"])
        changes.append(("node_delete", n))
    if sess and rng.random() < 0.6:
        k = rng.choice(sess)
        gone_jobs.add(f"{k[0]}/{k[1]}")
        changes.append(("pod_group_delete", groups[k]))
    if session_queues and rng.random() < 0.4:
        q = rng.choice(sorted(session_queues))
        gone_queues.add(q)
        changes.append(("queue_delete", {"name": q}))
        for k, g in groups.items():  # (the default queue's jobs too: their queue is the job's own field)
            if f"{k[0]}/{k[1]}" in session_jobs and g.get("queue") == q:
                gone_jobs.add(f"{k[0]}/{k[1]}")
    queues = [q for q in session_queues if q not in gone_queues]
    if rng.random() < 0.5:
        q = {"name": f"qx{seed}", "weight": rng.randint(1, 4)}
        changes.append(("queue_add", q))
        queues.append(q["name"])
    # a new job: a copy of a session job's pods under a new PodGroup
    live_pods = [p for p in pods.values() if p["uid"] in session_uids]
    if live_pods and queues and rng.random() < 0.8:
        base = rng.choice(live_pods)
        ns = base.get("namespace", "")
        gname = f"pgx{seed}"
        changes.append(("pod_group_add", {"namespace": ns, "name": gname, "minMember": rng.randint(1, 3),
                                          "queue": rng.choice(queues), "creationTimestamp": 10 ** 12 + seed}))
        for i in range(rng.randint(1, 4)):
            p = dict(base, uid=f"px{seed}-{i}", name=f"px{seed}-{i}", phase="Pending", nodeName="",
                     annotations=dict(base.get("annotations") or {}, **{"scheduling.k8s.io/group-name": gname}))
            p.pop("deletionTimestamp", None)
            if new_nodes and i == 0 and rng.random() < 0.5:
                p = dict(p, phase="Running", nodeName=new_nodes[0])
            changes.append(("pod_add", p))
    # completions of Running session pods the structural events left alone
    left = [p for p in live_pods if p.get("phase") == "Running" and p.get("nodeName") not in gone_nodes]
    job_of = {}
    for p in left:
        g = (p.get("annotations") or {}).get("scheduling.k8s.io/group-name")
        job_of[p["uid"]] = f"{p.get('namespace', '')}/{g}" if g else None
    left = [p for p in left if job_of[p["uid"]] not in gone_jobs and job_of[p["uid"]] in session_jobs]
    for p in rng.sample(left, min(len(left), rng.randint(0, 2))):
        changes.append(("pod_update", dict(p, phase="Succeeded")))
    return changes


# ------------------------------------------------------------------ fuzz
_OPS = ("In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt")


def random_fixture(seed, max_nodes=24, max_jobs=10, max_tasks=8, be_frac=0.06):
    rng = random.Random(seed)
    nn = rng.randint(1, max_nodes)
    zones = ["a", "b", "c"]
    nodes = []
    for i in range(nn):
        cpu = rng.choice([1, 2, 4, 8, 16])
        mem = rng.choice([1, 2, 4, 8, 32])
        gpu = rng.choice([0, 0, 0, 1, 4])
        alloc = {"cpu": str(cpu), "memory": f"{mem}Gi", "nvidia.com/gpu": str(gpu)}
        if rng.random() < 0.93:
            alloc["pods"] = str(rng.choice([2, 3, 5, 110]))
        labels = {"zone": rng.choice(zones), "size": str(cpu)}
        if rng.random() < 0.3:
            labels["ssd"] = "true"
        if rng.random() < 0.1:
            labels["size"] = "x12"  # non-integer: Gt/Lt must fail on it
        n = {"name": f"n{i:02d}", "allocatable": alloc, "labels": labels}
        if rng.random() < 0.2:
            n["taints"] = [{"key": rng.choice(["dedicated", "maint"]), "value": rng.choice(["", "gpu"]),
                            "effect": rng.choice(["NoSchedule", "NoExecute", "PreferNoSchedule"])}]
        if rng.random() < 0.08:
            n["unschedulable"] = True
        nodes.append(n)
    queues = [{"name": f"q{i}", "weight": rng.choice([1, 1, 2, 3])} for i in range(rng.randint(1, 3))]
    pods, pgs = [], []
    uid = 0

    def mk_pod(ns, name, phase, node, req, group=None, controller=None):
        nonlocal uid
        uid += 1
        p = {"uid": f"u{uid:04d}-{rng.randrange(100):02d}", "namespace": ns, "name": name, "phase": phase,
             "nodeName": node, "containers": [{"requests": req}]}
        if group:
            p["annotations"] = {"scheduling.k8s.io/group-name": group}
        if controller:
            p["controller"] = controller
        return p

    def rand_req(best_effort_ok=True):
        if best_effort_ok and rng.random() < be_frac:
            return {"cpu": "5m"}  # BestEffort (all dims below the tolerance)
        r = {"cpu": rng.choice(["100m", "500m", "1", "2", "3"]), "memory": rng.choice(["256Mi", "1Gi", "2Gi", "3Gi"])}
        if rng.random() < 0.15:
            r["nvidia.com/gpu"] = rng.choice(["1", "2"])
        return r

    def rand_ports():  # v1.ContainerPort host ports (vendor cache/host_ports.go semantics)
        return [{"hostPort": rng.choice([80, 443, 0]), "protocol": rng.choice(["", "TCP", "UDP"]),
                 "hostIP": rng.choice(["", "0.0.0.0", "10.0.0.1", "10.0.0.2"])} for _ in range(rng.randint(1, 2))]

    # remaining capacity per node, so that bound pods rarely overcommit a node
    # (an overcommitted node makes the reference panic in AddPod; ~3% keep that path)
    free = {n["name"]: [int(n["allocatable"]["cpu"]) * 1000, int(n["allocatable"]["memory"][:-2]) * 1024]
            for n in nodes}

    def fits(node_name, req):
        cpu = req.get("cpu", "0")
        mc = int(float(cpu[:-1])) if cpu.endswith("m") else int(float(cpu) * 1000)
        mem = req.get("memory", "0")
        mm = int(mem[:-2]) if mem.endswith("Mi") else (int(mem[:-2]) * 1024 if mem.endswith("Gi") else 0)
        f = free[node_name]
        if (f[0] >= mc and f[1] >= mm) or rng.random() < 0.03:
            f[0] -= mc
            f[1] -= mm
            return True
        return False

    # existing pods on nodes (Running / deleting -> Releasing)
    for i in range(rng.randint(0, nn)):
        node = rng.choice(nodes)
        if not fits(node["name"], {"cpu": "500m", "memory": "512Mi"}):
            continue
        p = mk_pod("default", f"run{i}", "Running", node["name"], {"cpu": "500m", "memory": "512Mi"},
                   group=None if rng.random() < 0.5 else "pg-run", controller="rc-1" if rng.random() < 0.5 else None)
        if rng.random() < 0.35:
            p["deletionTimestamp"] = "2026-01-01T00:00:00Z"
        if rng.random() < 0.2:
            p["containers"][0]["ports"] = rand_ports()
        pods.append(p)
    nj = rng.randint(1, max_jobs)
    for j in range(nj):
        ns = rng.choice(["c1", "c2"])
        pg = f"pg{j}"
        ntask = rng.randint(1, max_tasks)
        pgs.append({"namespace": ns, "name": pg, "minMember": rng.randint(0, ntask + 1),
                    "queue": rng.choice(queues)["name"] if rng.random() < 0.9 else "",
                    "creationTimestamp": rng.choice([0, 100, 200, 300]) * 1_000_000_000})
        job_req = rand_req()
        spec = {}
        r = rng.random()
        if r < 0.25:
            spec["nodeSelector"] = {"zone": rng.choice(zones)}
            if rng.random() < 0.1:
                spec["nodeSelector"]["bad key!"] = "x"  # invalid => selector matches everything
        elif r < 0.5:
            terms = []
            for _ in range(rng.randint(0, 2)):
                exprs = []
                for _ in range(rng.randint(0, 2)):
                    op = rng.choice(_OPS)
                    if op in ("In", "NotIn"):
                        vals = rng.sample(zones, rng.randint(1, 2))
                        key = "zone"
                    elif op in ("Gt", "Lt"):
                        vals = [rng.choice(["2", "4", "x"])]
                        key = "size"
                    else:
                        vals = []
                        key = rng.choice(["ssd", "zone", "gpu"])
                    exprs.append({"key": key, "operator": op, "values": vals})
                term = {"matchExpressions": exprs}
                if rng.random() < 0.3:
                    term["matchFields"] = [{"key": "metadata.name", "operator": rng.choice(["In", "NotIn"]),
                                            "values": [rng.choice(nodes)["name"]]}]
                terms.append(term)
            spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution":
                                                 {"nodeSelectorTerms": terms}}}
        if rng.random() < 0.3:
            spec["tolerations"] = [{"key": rng.choice(["dedicated", "maint", ""]),
                                    "operator": rng.choice(["Equal", "Exists", ""]),
                                    "value": rng.choice(["", "gpu"]),
                                    "effect": rng.choice(["", "NoSchedule", "NoExecute"])}]
        ports = rand_ports() if rng.random() < 0.2 else None
        for t in range(ntask):
            req = job_req if rng.random() < 0.7 else rand_req()
            phase, node = "Pending", ""
            if rng.random() < 0.1:
                cand = rng.choice(nodes)["name"]
                if fits(cand, req):
                    phase, node = "Running", cand
            p = mk_pod(ns, f"{pg}-t{t}", phase, node, req, group=pg)
            if rng.random() < 0.25:
                p["priority"] = rng.choice([1, 5, 10])
            p.update(spec)
            if ports:
                p["containers"][0]["ports"] = ports
            pods.append(p)
    plugins = ["priority", "gang", "drf", "predicates", "proportion", "nodeorder"]
    rng.shuffle(plugins)
    keep = [p for p in plugins if rng.random() < 0.85]
    cut = rng.randint(0, len(keep))
    flags = ["disableJobOrder", "disableJobReady", "disableTaskOrder", "disableQueueOrder", "disablePredicate"]

    def opt(name):
        o = {"name": name}
        if rng.random() < 0.1:
            o[rng.choice(flags)] = True
        return o

    tiers = [[opt(p) for p in keep[:cut]], [opt(p) for p in keep[cut:]]]
    tiers = [t for t in tiers if t]
    fx = {"name": f"fuzz-{seed}", "tiers": tiers, "nodes": nodes, "pods": pods, "podGroups": pgs, "queues": queues}
    if rng.random() < 0.2:
        fx["namespaces"] = ["c1", "c2"]
    r = rng.random()  # conf actions (util.go:30-61): the default "allocate, backfill", the full set, or one
    if r < 0.4:
        fx["actions"] = ["allocate", "backfill"]
    elif r < 0.5:
        fx["actions"] = ["backfill"]
    elif r < 0.7:
        fx["actions"] = ["reclaim", "allocate", "backfill", "preempt"]
    elif r < 0.8:
        fx["actions"] = ["preempt"]
    elif r < 0.9:
        fx["actions"] = ["reclaim"]
    return fx


def dupkey_fixture(seed, **kw):
    """random_fixture with colliding pod keys (PodKey = "<ns>/<name>",
    api/helpers.go:27-33): some Running / deleting pods take the namespace and
    name of a Pending pod (a StatefulSet pod recreated while its predecessor
    is still on a node), and some Pending pods share a name with a Pending
    pod of another job in their namespace. NodeInfo.AddTask refuses a key the
    node already holds (node_info.go:101-106): the decision is logged, the
    node is left unchanged."""
    fx = random_fixture(seed, **kw)
    rng = random.Random(seed * 7919 + 1)
    pods = fx["pods"]
    pending = [p for p in pods if p["phase"] == "Pending"]
    placed = [p for p in pods if p["phase"] == "Running"]
    if pending:
        for p in placed:
            if rng.random() < 0.6:
                q = rng.choice(pending)
                p["namespace"], p["name"] = q["namespace"], q["name"]
        for _ in range(max(1, len(pending) // 4)):
            a, b = rng.choice(pending), rng.choice(pending)
            if a is not b and a["namespace"] == b["namespace"]:
                b["name"] = a["name"]
    fx["name"] = f"dupkey-{seed}"
    return fx


def contended_fixture(seed, nodes=8, jobs=8, tasks=6, queues=3, aff=0.0, ports=0.0, big=False, huge=False):
    """A cluster already full of Running gang jobs in several queues, with
    Pending jobs of every queue: the regime of reclaim and preempt
    (BASELINE config 5 in miniature). Tasks of a job share one request so the
    reference's eviction loop (preempt.go:214-226) stays panic-free most of
    the time; mixed sizes still occur."""
    rng = random.Random(seed)
    qs = [{"name": f"q{i}", "weight": rng.choice([1, 2, 3])} for i in range(queues)]
    nds = []
    for i in range(nodes):
        alloc = {"cpu": str(rng.choice([4, 8])), "memory": f"{rng.choice([8, 16])}Gi",
                 "pods": str(rng.choice([4, 8, 110]))}
        if big:  # nodes that hold hundreds of small pods (victim scans in several 64-candidate chunks)
            alloc = {"cpu": "64", "memory": "256Gi", "pods": str(rng.choice([300, 600, 1100]))}
        if huge:  # more Running pods than one device victim scan takes (kbg_device.hpp kMaxNodeCandidates)
            alloc = {"cpu": "256", "memory": "1Ti", "pods": "3000"}
        nds.append({"name": f"n{i:02d}", "allocatable": alloc,
                    "labels": {"zone": rng.choice(["a", "b"]), "host": f"n{i:02d}"}})
    free = {n["name"]: [int(n["allocatable"]["cpu"]) * 1000, int(n["allocatable"]["pods"])] for n in nds}
    used_ports = {}
    pods, pgs = [], []
    uid = 0
    uniform = rng.random() < 0.7  # one request size for every job: evictions free exactly what a pipeline needs
    base = (rng.choice([500, 1000, 2000]), rng.choice(["0", "512Mi", "1Gi"]))
    if big or huge:
        base = (rng.choice([50, 100, 200]), "0")
        uniform = True
    for j in range(jobs):
        ns = rng.choice(["c1", "c2"])
        pg = f"pg{j}"
        q = rng.choice(qs)["name"]
        n_t = rng.randint(1, tasks)
        pgs.append({"namespace": ns, "name": pg, "minMember": rng.randint(0, n_t), "queue": q,
                    "creationTimestamp": rng.choice([0, 100, 200]) * 1_000_000_000})
        cpu, mem = base if uniform else (rng.choice([500, 1000, 2000]), rng.choice(["0", "512Mi", "1Gi"]))
        req = {"cpu": f"{cpu}m", "memory": mem}
        running = rng.random() < 0.6
        app = f"app{rng.randrange(3)}"
        job_aff = None
        if rng.random() < aff:  # required pod (anti)affinity on the zone or the host
            term = {"labelSelector": {"matchLabels": {"app": rng.choice([app, f"app{rng.randrange(3)}"])}},
                    "topologyKey": rng.choice(["zone", "host"])}
            job_aff = {rng.choice(["podAffinity", "podAntiAffinity", "podAntiAffinity"]):
                       {"requiredDuringSchedulingIgnoredDuringExecution": [term]}}
        job_ports = None
        if rng.random() < ports:
            job_ports = [{"hostPort": rng.choice([80, 443]), "protocol": rng.choice(["", "UDP"]),
                          "hostIP": rng.choice(["", "10.0.0.1"])}]
        for t in range(n_t):
            uid += 1
            phase, node = "Pending", ""
            if running:
                cands = [n["name"] for n in nds if free[n["name"]][0] >= cpu and free[n["name"]][1] > 0
                         and not (job_ports and used_ports.get(n["name"]))]
                if cands:
                    node = rng.choice(cands)
                    free[node][0] -= cpu
                    free[node][1] -= 1
                    phase = "Running"
                    if job_ports:
                        used_ports[node] = True
            p = {"uid": f"u{uid:04d}", "namespace": ns, "name": f"{pg}-t{t}", "phase": phase, "nodeName": node,
                 "annotations": {"scheduling.k8s.io/group-name": pg},
                 "containers": [{"requests": dict(req) if rng.random() < 0.95 or not uniform else {"cpu": "5m"}}]}
            if rng.random() < 0.3:
                p["priority"] = rng.choice([1, 5, 10])
            if rng.random() < 0.15:
                p["nodeSelector"] = {"zone": rng.choice(["a", "b"])}
            if aff:
                p["labels"] = {"app": app}
                if job_aff:
                    p["affinity"] = job_aff
            if job_ports:
                p["containers"][0]["ports"] = job_ports
            pods.append(p)
    plugins = ["priority", "gang", "drf", "predicates", "proportion"]
    rng.shuffle(plugins)
    cut = rng.randint(0, len(plugins))
    flags = ["disablePreemptable", "disableReclaimable", "disableJobOrder", "disableJobReady"]

    def opt(name):
        o = {"name": name}
        if rng.random() < 0.1:
            o[rng.choice(flags)] = True
        return o

    tiers = [t for t in ([opt(p) for p in plugins[:cut]], [opt(p) for p in plugins[cut:]]) if t]
    acts = rng.choice([["reclaim"], ["preempt"], ["reclaim", "allocate", "backfill", "preempt"],
                       ["allocate", "preempt"]])
    return {"name": f"contended-{seed}", "tiers": tiers, "nodes": nds, "pods": pods, "podGroups": pgs,
            "queues": qs, "actions": acts}


def contended_dupkey_fixture(seed, ports=0.0, pending_dups=0.0):
    """contended_fixture with half of the Running pods renamed after a Pending
    pod (PodKey = "<ns>/<name>" shared: a StatefulSet pod recreated while its
    predecessor still runs): preempt pipelines a pod onto the node that holds
    its key — AddTask refuses it (node_info.go:101-106) — and when the
    statement is discarded, unpipeline's RemoveTask removes by key the pod
    that held it (statement.go:156-192, node_info.go:131-157). `ports`: the
    share of pod specs with host ports (contended_fixture), so the holder's
    ports leave node.Pods() with it and come back with its unevict.
    `pending_dups`: the share of Pending pods renamed after another Pending
    pod of their namespace, so the key's holder can be a pod placed earlier in
    the same cycle (its node copy Allocated or Pipelined)."""
    fx = contended_fixture(8800 + seed, nodes=6, jobs=10, tasks=6, ports=ports)
    rng = random.Random(seed)
    pods = fx["pods"]
    pend = [p for p in pods if p["phase"] == "Pending"]
    run = [p for p in pods if p["phase"] == "Running"]
    if pend and run:
        for p in run:
            if rng.random() < 0.5:
                q = rng.choice(pend)
                p["namespace"], p["name"] = q["namespace"], q["name"]
    if pending_dups:
        for p in pend:
            q = rng.choice(pend)
            if rng.random() < pending_dups and q is not p and q["namespace"] == p["namespace"]:
                p["name"] = q["name"]
    fx["name"] = (f"contended-dupkey-{seed}" + (f"-ports{ports}" if ports else "")
                  + (f"-pdups{pending_dups}" if pending_dups else ""))
    return fx


def contended_config(**over):
    """BASELINE config 5: 10k nodes x 200k tasks, the cluster ~95% full (CPU)
    of Running gang jobs spread round-robin over the nodes, most of them in the
    two low-weight queues (which therefore exceed their proportion share), and
    200 Pending jobs (10k tasks, pod priority 10 against 1) spread over all four
    queues. Every task requests the same 3200m / 6Gi, so the reference's
    eviction loop never underflows (preempt.go:221-226, reclaim.go:152-165) and
    a pipelined task always fits the Releasing its victim freed. Runs the
    actions "reclaim, allocate, backfill, preempt" under the default tiers
    (util.go:30-40), so gang's victim fns (tier 1) decide both actions."""
    c = dict(C5, **over)  # smaller instances of the same generator for parity tests
    rng = random.Random(BASE_SEED + 5)
    nodes = [_node(i, rng, "hetero4") for i in range(c["nodes"])]
    for n in nodes:  # keep every node usable: the packer below ignores taints and selectors
        n.pop("taints", None)
        n.pop("unschedulable", None)
    queues = [{"name": q, "weight": w} for q, w in c["queues"]]
    cpu, req = 3200, {"cpu": "3200m", "memory": "6Gi"}
    room = [int(n["allocatable"]["cpu"]) * 1000 // cpu for n in nodes]
    cursor = 0
    n_run = c["jobs"] - c["pending_jobs"]
    pods, pgs = [], []
    for j in range(c["jobs"]):
        ns = f"ns{j % 8}"
        pg = f"pg-{j:05d}"
        running = j < n_run
        if running:
            q = ("q1", "q1", "q2", "q2", "q2", "q3", "q4")[rng.randrange(7)]
        else:
            q = queues[rng.randrange(4)]["name"]
        pgs.append({"namespace": ns, "name": pg, "minMember": (1, 25, 50)[rng.randrange(3)], "queue": q,
                    "creationTimestamp": (1_700_000_000 + j) * 1_000_000_000})
        for t in range(c["tasks_per_job"]):
            p = {"uid": f"uid-{j:05d}-{t:03d}", "namespace": ns, "name": f"{pg}-{t:03d}", "phase": "Pending",
                 "annotations": {"scheduling.k8s.io/group-name": pg}, "containers": [{"requests": dict(req)}],
                 "priority": 1 if running else 10}
            if running:
                for _ in range(len(nodes)):  # round-robin over the nodes with room
                    k = cursor
                    cursor = (cursor + 1) % len(nodes)
                    if room[k] > 0:
                        room[k] -= 1
                        p["phase"], p["nodeName"] = "Running", nodes[k]["name"]
                        break
            pods.append(p)
    return {"name": "C5", "tiers": None, "nodes": nodes, "pods": pods, "podGroups": pgs, "queues": queues,
            "actions": ["reclaim", "allocate", "backfill", "preempt"]}


def affinity_fixture(seed, max_nodes=16, max_jobs=8, max_tasks=6):
    """Small sessions exercising inter-pod (anti)affinity (vendor
    predicates.go:1155-1466): pod labels over a few apps and namespaces,
    required pod affinity / anti-affinity terms with matchLabels,
    matchExpressions, nil and empty selectors, explicit namespaces, zone / rack
    / host topology keys (some nodes lack them), the occasional empty
    topologyKey or invalid selector, running pods that carry terms, and
    allocate or allocate + backfill."""
    rng = random.Random(seed)
    nn = rng.randint(2, max_nodes)
    nodes = []
    for i in range(nn):
        labels = {"host": f"n{i:02d}"}
        if rng.random() < 0.9:
            labels["zone"] = rng.choice(["a", "b", "c"])
        if rng.random() < 0.7:
            labels["rack"] = f"r{rng.randrange(4)}"
        nodes.append({"name": f"n{i:02d}", "labels": labels,
                      "allocatable": {"cpu": str(rng.choice([2, 4, 8])), "memory": "16Gi",
                                      "pods": str(rng.choice([3, 110]))}})
    apps = ["web", "db", "cache"]
    nss = ["c1", "c2"]

    def selector():
        r = rng.random()
        if r < 0.08:
            return None  # nil: selects nothing
        if r < 0.14:
            return {}  # empty: selects everything
        if r < 0.18:
            return {"matchExpressions": [{"key": "app", "operator": "Foo", "values": ["web"]}]}  # build error
        if r < 0.6:
            return {"matchLabels": {"app": rng.choice(apps)}}
        op = rng.choice(["In", "NotIn", "Exists", "DoesNotExist"])
        e = {"key": rng.choice(["app", "tier"]), "operator": op}
        if op in ("In", "NotIn"):
            e["values"] = rng.sample(apps, rng.randint(1, 2))
        return {"matchExpressions": [e]}

    def terms():
        out = []
        for _ in range(rng.choice([1, 1, 1, 2])):
            t = {"topologyKey": rng.choice(["zone", "zone", "rack", "host", "nokey", ""] if rng.random() < 0.15
                                           else ["zone", "rack", "host"])}
            sel = selector()
            if sel is not None:
                t["labelSelector"] = sel
            if rng.random() < 0.25:
                t["namespaces"] = rng.sample(nss, rng.randint(1, 2))
            out.append(t)
        return out

    def affinity():
        r = rng.random()
        a = {}
        if r < 0.45:
            a["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": terms()}
        if 0.3 < r < 0.8:
            a["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": terms()}
        return a or None

    pods, pgs = [], []
    uid = 0

    def mk(ns, name, group, phase="Pending", node="", app=None, aff=None, req=None):
        nonlocal uid
        uid += 1
        p = {"uid": f"u{uid:04d}", "namespace": ns, "name": name, "phase": phase, "nodeName": node,
             "annotations": {"scheduling.k8s.io/group-name": group},
             "containers": [{"requests": req or {"cpu": rng.choice(["500m", "1"]), "memory": "1Gi"}}]}
        labels = {}
        if app:
            labels["app"] = app
        if rng.random() < 0.3:
            labels["tier"] = rng.choice(["front", "back"])
        if labels:
            p["labels"] = labels
        if aff:
            p["affinity"] = aff
        return p

    pgs.append({"namespace": "c1", "name": "pg-run", "minMember": 0, "queue": "q1"})
    for i in range(rng.randint(0, nn)):
        node = rng.choice(nodes)["name"]
        pods.append(mk("c1", f"run{i}", "pg-run", "Running", node, rng.choice(apps + [None]),
                       affinity() if rng.random() < 0.3 else None, {"cpu": "500m", "memory": "512Mi"}))
    for j in range(rng.randint(1, max_jobs)):
        ns = rng.choice(nss)
        nt = rng.randint(1, max_tasks)
        pgs.append({"namespace": ns, "name": f"pg{j}", "minMember": rng.randint(0, nt), "queue": "q1",
                    "creationTimestamp": rng.choice([0, 100, 200]) * 1_000_000_000})
        app = rng.choice(apps + [None])
        aff = affinity() if rng.random() < 0.7 else None
        be = rng.random() < 0.1
        for t in range(nt):
            pods.append(mk(ns, f"pg{j}-{t}", f"pg{j}", app=app if rng.random() < 0.9 else rng.choice(apps),
                           aff=aff, req={"cpu": "5m"} if be else None))
    plugins = [{"name": "predicates"}] + [{"name": p} for p in rng.sample(["gang", "drf", "priority", "proportion"],
                                                                            rng.randint(0, 3))]
    rng.shuffle(plugins)
    cut = rng.randint(1, len(plugins))
    tiers = [t for t in (plugins[:cut], plugins[cut:]) if t]
    fx = {"name": f"affinity-{seed}", "tiers": tiers, "nodes": nodes, "pods": pods, "podGroups": pgs,
          "queues": [{"name": "q1", "weight": 1}]}
    if rng.random() < 0.4:
        fx["actions"] = ["allocate", "backfill"]
    return fx


def affinity_config(nodes=5000, jobs=2000, tasks_per_job=50, seed=6):
    """C3's cluster and jobs with inter-pod (anti)affinity on top (not a
    BASELINE config; a scale check of kbg_affinity.cpp): every pod is labelled
    with its job; 40% of the jobs spread over hosts (required anti-affinity to
    their own pods on the node's name label), 20% co-locate in one zone
    (required affinity to their own pods on the zone label), the rest plain."""
    fx = config_fixture(3)
    rng = random.Random(BASE_SEED + 100 + seed)
    fx = dict(fx, name="C3-affinity")
    fx["nodes"] = fx["nodes"][:nodes]
    for n in fx["nodes"]:
        n["labels"] = dict(n["labels"], host=n["name"])
    pods = [p for p in fx["pods"] if int(p["uid"].split("-")[1]) < jobs and int(p["uid"].split("-")[2]) < tasks_per_job]
    kind = {}
    for p in pods:
        j = p["annotations"]["scheduling.k8s.io/group-name"]
        if j not in kind:
            r = rng.random()
            kind[j] = "spread" if r < 0.4 else ("colocate" if r < 0.6 else "plain")
        p["labels"] = {"job": j}
        term = {"labelSelector": {"matchLabels": {"job": j}}}
        if kind[j] == "spread":
            p["affinity"] = dict(p.get("affinity") or {}, podAntiAffinity={
                "requiredDuringSchedulingIgnoredDuringExecution": [dict(term, topologyKey="host")]})
        elif kind[j] == "colocate":
            p["affinity"] = dict(p.get("affinity") or {}, podAffinity={
                "requiredDuringSchedulingIgnoredDuringExecution": [dict(term, topologyKey="zone")]})
    fx["pods"] = pods
    names = {p["annotations"]["scheduling.k8s.io/group-name"] for p in pods}
    fx["podGroups"] = [g for g in fx["podGroups"] if g["name"] in names]
    return fx
