"""framework: Session, plugin/action registries (pkg/scheduler/framework).

`open_session` / `close_session` mirror framework.OpenSession / CloseSession
(framework.go:26-54). The plugins named in the tiers (drf, proportion, gang,
priority, predicates) run their OnSessionOpen inside the device library
(kbg_session_open), which also uploads the node table to HBM. Every tier
entry goes to the library with KBG_PLUGIN_REGISTERED set when this process's
registry has a builder for its name (kbg_options.plugin_registry = 1): names
without one are skipped, exactly like GetPluginBuilder misses
(framework.go:30-35), and a registered plugin the library does not implement
refuses the session (KBG_E_UNSUPPORTED: run the reference path). `Session.allocate` / `Session.pipeline` /
`Session.dispatch` replay device decisions into the host objects with the
reference's bookkeeping (session.go:205-316).
"""
import ctypes
import os

import numpy as np

from . import _abi
from .api import ALLOCATED, BINDING, PIPELINED, RELEASING, pod_key
from .snapshot import FlatSnapshot

KNOWN_PLUGINS = ("priority", "gang", "drf", "predicates", "proportion")

_plugin_builders = {n: n for n in KNOWN_PLUGINS}
_actions = {}


def register_plugin_builder(name, builder=None):  # plugins.go:28-33
    _plugin_builders[name] = builder or name


def cleanup_plugin_builders():  # plugins.go:35-40
    _plugin_builders.clear()


def get_plugin_builder(name):  # plugins.go:42-49
    return _plugin_builders.get(name)


def register_action(action):  # plugins.go:53-58
    _actions[action.name()] = action


def get_action(name):  # plugins.go:60-66
    return _actions.get(name)


class Session:
    """framework.Session (session.go:35-61) plus the device handle."""

    def __init__(self, cache, tiers, options=None):
        snap = cache.snapshot()
        self.cache = cache
        self.jobs = snap.jobs  # JobValid is a no-op at openSession time
        self.job_index = {j.uid: j for j in self.jobs}
        self.nodes = snap.nodes
        self.node_index = {n.name: n for n in self.nodes}
        self.queues = snap.queues
        self.queue_index = {q.uid: q for q in self.queues}
        self.others = snap.others
        self.tiers = tiers
        self.plugins = [p.name for t in tiers for p in t.plugins if get_plugin_builder(p.name) is not None]
        self.flat = FlatSnapshot(self.nodes, self.jobs, self.queues, self.others, self.tiers,
                                 registered=lambda name: get_plugin_builder(name) is not None)
        self.handle = ctypes.c_void_p()
        opts = _abi.kbg_options()
        opts.device = -1
        opts.plugin_registry = 1
        options = dict(options or {})
        comm = options.pop("comm", None)  # dist.ShardComm: node-axis shard of an RCCL clique
        for k, v in options.items():
            setattr(opts, k, v)
        L = _abi.lib()
        if comm is not None:
            _abi.check(L.kbg_session_open_sharded(ctypes.byref(self.flat.snap), ctypes.byref(opts), comm.handle,
                                                  ctypes.byref(self.handle)))
        else:
            _abi.check(L.kbg_session_open(ctypes.byref(self.flat.snap), ctypes.byref(opts),
                                          ctypes.byref(self.handle)))
        self.decisions = []
        self.action_of = []  # action name of each decision of the cycle
        self.evictions = []  # (task, by, action) committed evictions (cache.Evict)

    # ---- session.go:205-241
    def pipeline(self, task, hostname):
        job = self.job_index.get(task.job)
        if job is not None:
            job.update_task_status(task, PIPELINED)
        task.node_name = hostname
        node = self.node_index.get(hostname)
        if node is not None:
            node.add_task(task)

    # ---- session.go:243-293 (the JobReady/dispatch decision comes from the device log)
    def allocate(self, task, hostname):
        job = self.job_index.get(task.job)
        if job is not None:
            job.update_task_status(task, ALLOCATED)
        task.node_name = hostname
        node = self.node_index.get(hostname)
        if node is not None:
            node.add_task(task)

    # ---- session.go:295-316
    def dispatch(self, task):
        self.cache.bind(task, task.node_name)
        job = self.job_index.get(task.job)
        if job is not None:
            job.update_task_status(task, BINDING)

    # ---- session.go:318-352 / statement.go: the resource side of evictions and of
    # the pipelines that follow them lives in the device session (node Idle /
    # Releasing, including what discarded statements leave behind); the host
    # objects record the statuses, the node membership and the cache's Evict.
    def evict(self, task, reason):
        job = self.job_index.get(task.job)
        if job is not None:
            job.update_task_status(task, RELEASING)
        node = self.node_index.get(task.node_name)
        if node is not None:
            held = node.tasks.get(pod_key(task.pod))
            if held is not None:
                held.status = RELEASING
        self.cache.evict(task, reason)

    def pipeline_replay(self, task, hostname):
        job = self.job_index.get(task.job)
        if job is not None:
            job.update_task_status(task, PIPELINED)
        task.node_name = hostname
        node = self.node_index.get(hostname)
        if node is not None and pod_key(task.pod) not in node.tasks:
            node.tasks[pod_key(task.pod)] = task.clone()

    def sync_node_resources(self):
        """Idle / Releasing of every host NodeInfo from the device session,
        after an action whose statements changed them (reclaim, preempt), so
        later actions' replays account from the same values."""
        for i, name in enumerate(self.flat.node_names):
            node = self.node_index.get(name)
            if node is None or node.node is None:
                continue
            st = self.node_state(i)
            for mine, dev in ((node.idle, st.idle), (node.releasing, st.releasing)):
                mine.milli_cpu, mine.memory, mine.milli_gpu = dev.milli_cpu, dev.memory, dev.milli_gpu

    def update(self, changes):
        """kbg_session_update: cache events since the session's snapshot,
        applied to the resident session (include/kbgpu.h). `changes` is a list
        of ("pod_update", pod) | ("pod_delete", pod) | ("pod_add", pod) |
        ("node_add", node) | ("node_update", node) | ("node_delete", node) |
        ("pod_group_add", pg) | ("pod_group_delete", pg) | ("queue_add", q) |
        ("queue_delete", q) in event order, objects as the informer delivers
        them (event_handlers.go). New pods must use a pod spec the session
        already has. Structural changes (a node, PodGroup or queue joins or
        leaves; a pod naming a node the cache does not know, which makes a
        NodeInfo(nil), event_handlers.go:49-53) renumber the session: the
        wrapper's task, node, job and queue lists follow the library's
        renumbering (kbg_session_renumbering). The host-side objects are not
        replayed: read results through the C ABI (decisions, job / queue /
        node state)."""
        plan = self.marshal(changes)
        _abi.check(_abi.lib().kbg_session_update(self.handle, plan.evs, plan.n_ev))
        self._accept(plan)

    def marshal(self, changes):
        """The kbg_event batch of `changes` against this session's current
        numbering (update's first half; host-only, also used by the CPU tests
        of the structural path through the tool library)."""
        from types import SimpleNamespace
        from .api import JobInfo, NodeInfo, QueueInfo, TaskInfo, pod_key
        flat = self.flat
        tidx = {t.uid: i for i, t in enumerate(flat.task_objs) if t is not None}
        nidx = {n: i for i, n in enumerate(flat.node_names) if n}
        pod_only = dict(flat.pod_only_names)  # NodeName -> index of a node the cache knows only from pods
        jidx = dict(flat.job_index)
        qidx = dict(flat.queue_index)
        n_nodes, n_jobs, n_queues = len(flat.node_names), len(self.jobs), len(self.queues)
        new_nodes, new_jobs, new_queues = {}, {}, {}  # new index -> NodeInfo / JobInfo / QueueInfo
        # at most two events per change: a pod naming a node new to the cache makes it first
        evs = (_abi.kbg_event * max(1, 2 * len(changes)))()
        n_ev = 0
        keep = []
        objs = {}  # task index -> its TaskInfo after the events (applied once the library accepts them)
        n_objs = len(flat.task_objs)
        renamed = {}  # pod-only node index -> the name its Node gave it

        def ev():
            nonlocal n_ev
            n_ev += 1
            return evs[n_ev - 1]

        def job_of(j):
            return self.jobs[j] if j < len(self.jobs) else new_jobs[j]

        def node_spec(e, obj):
            ni = NodeInfo(obj)
            e.resource = _abi.kbg_resource(*ni.allocatable.as_tuple())
            e.max_task_num = ni.allocatable.max_task_num
            e.unschedulable = 1 if obj.get("unschedulable") else 0
            labels = [x.encode() for kv in (obj.get("labels") or {}).items() for x in kv]
            taints = [str(t.get(f, "")).encode() for t in (obj.get("taints") or []) for f in ("key", "value", "effect")]
            la = (ctypes.c_char_p * max(1, len(labels)))(*labels)
            ta = (ctypes.c_char_p * max(1, len(taints)))(*taints)
            spec = _abi.kbg_node_spec(obj["name"].encode(), la, len(labels) // 2, len(taints) // 3, ta)
            keep.extend([la, ta, spec])
            e.node_spec = ctypes.pointer(spec)

        def node_of(name):
            """kbg_event.node of a pod's NodeName: the session node of that name,
            else the node the cache knows only from pods carrying it
            (sc.Nodes[NodeName]); a name the cache does not know makes that
            node (NewNodeInfo(nil), event_handlers.go:49-53): KBG_EV_NODE_ADD."""
            nonlocal n_nodes
            if not name:
                return -1
            i = nidx.get(name)
            if i is None:
                i = pod_only.get(name)
            if i is None:
                e = ev()
                e.kind = _abi.EV_NODE_ADD
                keep.append(name.encode())
                e.node_name = keep[-1]
                i = pod_only[name] = n_nodes
                new_nodes[i] = NodeInfo(None)
                n_nodes += 1
            return i

        def pod_node(e, name):
            e.node = node_of(name)
            if e.node >= 0 and name not in nidx:
                keep.append(name.encode())  # a node known only from pods: its NodeName
                e.node_name = keep[-1]

        for kind, obj in changes:
            if kind in ("node_update", "node_add"):
                # cache.AddNode / UpdateNode -> SetNode with the whole Node (the library
                # compares labels and taints and rebuilds only when they change)
                name = obj["name"]
                idx = nidx.get(name)
                if idx is None:
                    idx = pod_only.get(name)
                    if idx is None:
                        if kind == "node_update":  # updateNode: "node does not exist" (event_handlers.go:249-259)
                            continue
                        e = ev()  # a new node: NewNodeInfo(node), last in the session's node order
                        e.kind = _abi.EV_NODE_ADD
                        node_spec(e, obj)
                        nidx[name] = n_nodes
                        new_nodes[n_nodes] = NodeInfo(obj)
                        n_nodes += 1
                        continue
                    pod_only.pop(name, None)
                    if idx in new_nodes:  # made by a pod earlier in the batch
                        new_nodes[idx] = NodeInfo(obj)
                    else:
                        renamed[idx] = name
                    nidx[name] = idx  # later events of the batch name the node by its Node's name
                e = ev()
                e.kind = _abi.EV_NODE_SET
                e.node = idx
                if os.environ.get("KBG_PY_NODE_UPDATE") == "1" and idx not in renamed:  # (A/B: Allocatable only)
                    ni = NodeInfo(obj)
                    e.kind = _abi.EV_NODE_UPDATE
                    e.resource = _abi.kbg_resource(*ni.allocatable.as_tuple())
                    e.max_task_num = ni.allocatable.max_task_num
                    e.unschedulable = 1 if obj.get("unschedulable") else 0
                    continue
                node_spec(e, obj)
                continue
            if kind == "node_delete":  # deleteNode (event_handlers.go:262-268); an unknown name is an error there
                name = obj["name"]
                idx = nidx.pop(name, None)
                if idx is None:
                    idx = pod_only.pop(name, None)
                if idx is None:
                    continue
                e = ev()
                e.kind, e.node = _abi.EV_NODE_DELETE, idx
                continue
            if kind in ("pod_group_add", "pod_group_delete"):
                jid = f"{obj.get('namespace', '')}/{obj['name']}"
                if kind == "pod_group_delete":  # UnsetPodGroup: the job leaves ssn.Jobs
                    j = jidx.pop(jid, None)
                    if j is not None:
                        e = ev()
                        e.kind, e.job = _abi.EV_JOB_DELETE, j
                        self._outside_jobs().add(jid)  # its pods stay in the cache, outside the session jobs
                    continue
                if jid in jidx:
                    raise ValueError(f"PodGroup {jid!r}: an update of a session job's PodGroup needs a re-open")
                if jid in self._outside_jobs():
                    raise ValueError(f"PodGroup {jid!r}: the cache holds pods of it outside the session jobs "
                                     "(they predate the PodGroup): re-open")
                job = JobInfo(jid)
                job.set_pod_group(obj, getattr(self.cache, "default_queue", ""))
                if job.queue not in qidx:
                    raise ValueError(f"PodGroup {jid!r}: queue {job.queue!r} is not a session queue (re-open when it "
                                     "exists)")
                e = ev()
                e.kind = _abi.EV_JOB_ADD
                keep.append(jid.encode())
                e.name = keep[-1]
                e.queue = qidx[job.queue]
                e.min_available = job.min_available
                e.priority = job.priority
                e.creation_ns = job.creation_timestamp
                jidx[jid] = n_jobs
                new_jobs[n_jobs] = job
                n_jobs += 1
                continue
            if kind in ("queue_add", "queue_delete"):
                qi = QueueInfo(obj["name"], obj.get("weight", 0))
                if kind == "queue_delete":
                    q = qidx.pop(qi.uid, None)
                    if q is not None:
                        e = ev()
                        e.kind, e.queue = _abi.EV_QUEUE_DELETE, q
                        for jid in [k for k, j in jidx.items() if job_of(j).queue == qi.uid]:
                            jidx.pop(jid)  # its jobs leave ssn.Jobs (cache.go:584-588)
                            self._outside_jobs().add(jid)
                    continue
                if qi.uid in qidx:
                    raise ValueError(f"queue {qi.uid!r}: an update of a session queue needs a re-open")
                e = ev()
                e.kind = _abi.EV_QUEUE_ADD
                keep.append(qi.uid.encode())
                e.name = keep[-1]
                e.weight = qi.weight
                qidx[qi.uid] = n_queues
                new_queues[n_queues] = qi
                n_queues += 1
                continue
            ti = TaskInfo(obj)
            if kind in ("pod_update", "pod_delete"):
                if kind == "pod_update":
                    node_of(ti.node_name)  # a NodeInfo(nil) first, when the name is new to the cache
                e = ev()
                e.kind = _abi.EV_POD_UPDATE if kind == "pod_update" else _abi.EV_POD_DELETE
                e.task = tidx[obj["uid"]]
                e.status = ti.status
                if kind == "pod_update":
                    pod_node(e, ti.node_name)
                objs[e.task] = ti
            elif kind == "pod_add":
                if ti.job not in jidx:
                    raise ValueError(f"pod {ti.uid!r}: job {ti.job!r} is not a session job (re-open)")
                node_of(ti.node_name)
                e = ev()
                e.kind = _abi.EV_POD_ADD
                e.job = jidx[ti.job]
                e.spec = flat.spec_index(obj)
                e.status = ti.status
                e.priority = ti.priority
                pod_node(e, ti.node_name)
                e.resource = _abi.kbg_resource(*ti.resreq.as_tuple())
                keep += [ti.uid.encode(), pod_key(obj).encode()]
                e.uid, e.pod_key = keep[-2], keep[-1]
                tidx[ti.uid] = n_objs
                objs[n_objs] = ti
                n_objs += 1
            else:
                raise ValueError(f"unknown change {kind}")
        return SimpleNamespace(evs=evs, n_ev=n_ev, keep=keep, objs=objs, n_objs=n_objs, renamed=renamed, tidx=tidx,
                               new_nodes=new_nodes, new_jobs=new_jobs, new_queues=new_queues, pod_only=pod_only)

    def _accept(self, plan):
        """update's second half, once the library applied the batch: the
        wrapper's lists follow it (renumbered after a structural batch)."""
        flat = self.flat
        evs, n_ev, objs, n_objs, tidx = plan.evs, plan.n_ev, plan.objs, plan.n_objs, plan.tidx
        new_nodes, new_jobs, new_queues, pod_only = plan.new_nodes, plan.new_jobs, plan.new_queues, plan.pod_only
        for i, name in plan.renamed.items():  # the NodeInfo the cache made from a pod has its Node's name now
            flat.node_names[i] = name
            flat.pod_only_names.pop(name, None)
            self.nodes[i].name = name
            self.node_index[name] = self.nodes[i]
        task_objs = flat.task_objs + [None] * (n_objs - len(flat.task_objs))
        for i, ti in objs.items():
            task_objs[i] = ti
        structural = any(evs[k].kind >= _abi.EV_NODE_ADD for k in range(n_ev))
        if structural:
            self._renumber(task_objs, new_nodes, new_jobs, new_queues, pod_only)
        else:
            flat.task_objs = task_objs
        from .api import PENDING
        live = set(tidx)  # (deleted pods keep their index; counts only size output buffers)
        flat.pending_all = max(flat.pending_all, sum(1 for t in flat.task_objs
                                                     if t is not None and t.uid in live and t.status == PENDING))
        flat.pending_count = max(flat.pending_count, flat.pending_all)

    def _outside_jobs(self):
        """JobIDs with pods the snapshot holds outside the session jobs
        (Others, pods on nodes): a PodGroup for one of them needs a re-open."""
        if getattr(self, "_outside", None) is None:
            mine = {t.uid for t in self.flat.task_objs if t is not None}
            out = {t.job for t in self.others}
            out |= {t.job for n in self.nodes for t in n.tasks.values() if t.uid not in mine}
            self._outside = out
        return self._outside

    def _renumber(self, task_objs, new_nodes, new_jobs, new_queues, pod_only, maps=None):
        """The wrapper's lists after a structural update, by the library's
        old -> new index maps (kbg_session_renumbering; `maps`: given)."""
        L = _abi.lib()
        flat = self.flat

        def renum(kind):
            if maps is not None:
                return np.asarray(maps[kind], dtype=np.int64)
            n = ctypes.c_int32(0)
            _abi.check(L.kbg_session_renumbering(self.handle, kind, None, 0, ctypes.byref(n)))
            buf = (ctypes.c_int32 * max(1, n.value))()
            _abi.check(L.kbg_session_renumbering(self.handle, kind, buf, n.value, ctypes.byref(n)))
            return np.frombuffer(buf, dtype=np.int32, count=n.value).astype(np.int64)

        def remap(old, r):
            # out[r[i]] = old[i] for every kept i (r[i] >= 0); positions no old
            # entry maps to stay None. In numpy: a C4 session has 500k tasks.
            if r.size == 0 or r.max() < 0:
                return []
            out = np.full(int(r.max()) + 1, None, dtype=object)
            n = min(len(old), r.size)
            if n:
                src = np.fromiter(old if n == len(old) else old[:n], dtype=object, count=n)
                rr = r[:n]
                keep = rr >= 0
                out[rr[keep]] = src[keep]
            return out.tolist()

        rt, rn, rj, rq = (renum(k) for k in (_abi.RENUM_TASKS, _abi.RENUM_NODES, _abi.RENUM_JOBS, _abi.RENUM_QUEUES))
        flat.task_objs = remap(task_objs, rt)
        nodes = list(self.nodes) + [new_nodes[i] for i in sorted(new_nodes)]
        names = list(flat.node_names) + [new_nodes[i].name for i in sorted(new_nodes)]
        self.nodes = remap(nodes, rn)
        flat.node_names = remap(names, rn)
        self.node_index = {n.name: n for n in self.nodes if n.name}
        flat.pod_only_names = {nm: int(rn[i]) for nm, i in pod_only.items() if i < len(rn) and rn[i] >= 0}
        jobs = list(self.jobs) + [new_jobs[i] for i in sorted(new_jobs)]
        self.jobs = remap(jobs, rj)
        self.job_index = {j.uid: j for j in self.jobs}
        flat.job_index = {j.uid: i for i, j in enumerate(self.jobs)}
        queues = list(self.queues) + [new_queues[i] for i in sorted(new_queues)]
        self.queues = remap(queues, rq)
        self.queue_index = {q.uid: q for q in self.queues}
        flat.queue_index = {q.uid: i for i, q in enumerate(self.queues)}

    def job_state(self, j):
        st = _abi.kbg_job_state()
        _abi.check(_abi.lib().kbg_job_state_get(self.handle, j, ctypes.byref(st)))
        return st

    def queue_state(self, q):
        st = _abi.kbg_queue_state()
        _abi.check(_abi.lib().kbg_queue_state_get(self.handle, q, ctypes.byref(st)))
        return st

    def node_state(self, n):
        st = _abi.kbg_node_state()
        _abi.check(_abi.lib().kbg_node_state_get(self.handle, n, ctypes.byref(st)))
        return st

    def stats(self):
        st = _abi.kbg_stats()
        _abi.check(_abi.lib().kbg_stats_get(self.handle, ctypes.byref(st)))
        return st

    def close(self):
        if self.handle:
            _abi.lib().kbg_session_close(self.handle)
            self.handle = ctypes.c_void_p()


def open_session(cache, tiers, options=None):
    return Session(cache, tiers, options)


def close_session(ssn):
    ssn.close()
