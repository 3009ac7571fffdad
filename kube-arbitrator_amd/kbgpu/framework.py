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
        ("node_update", node) in event order, pods and nodes as the informer
        delivers them. New pods must use a pod spec the session already has.
        The host-side objects (jobs / nodes of this wrapper) are not replayed:
        read results through the C ABI (decisions, job / queue / node state)."""
        from .api import NodeInfo, TaskInfo, pod_key
        tidx = {t.uid: i for i, t in enumerate(self.flat.task_objs)}
        nidx = {n: i for i, n in enumerate(self.flat.node_names) if n}

        def node_of(name):
            """kbg_event.node of a pod's NodeName: the session node of that name,
            else the node the cache knows only from pods carrying it (sc.Nodes[NodeName])."""
            if not name:
                return -1
            i = nidx.get(name)
            return i if i is not None else self.flat.pod_only_names.get(name, -1)
        evs = (_abi.kbg_event * max(1, len(changes)))()
        keep = []
        objs = {}  # task index -> its TaskInfo after the events (applied once the library accepts them)
        n_objs = len(self.flat.task_objs)
        renamed = {}  # pod-only node index -> the name its Node gave it
        for k, (kind, obj) in enumerate(changes):
            e = evs[k]
            if kind in ("node_update", "node_add"):
                # cache.AddNode / UpdateNode -> SetNode with the whole Node (the library
                # compares labels and taints and rebuilds only when they change)
                ni = NodeInfo(obj)
                name = obj["name"]
                idx = nidx.get(name)
                if idx is None or self.flat.node_names[idx] != name:
                    idx = self.flat.pod_only_names.get(name)
                    if idx is None:
                        raise ValueError(f"node {name!r}: not a node of the session (a new node needs a re-open)")
                    renamed[idx] = name
                    nidx[name] = idx  # later events of the batch name the node by its Node's name
                e.kind = _abi.EV_NODE_SET
                e.node = idx
                if os.environ.get("KBG_PY_NODE_UPDATE") == "1" and idx not in renamed:  # (A/B: Allocatable only)
                    e.kind = _abi.EV_NODE_UPDATE
                    e.resource = _abi.kbg_resource(*ni.allocatable.as_tuple())
                    e.max_task_num = ni.allocatable.max_task_num
                    e.unschedulable = 1 if obj.get("unschedulable") else 0
                    continue
                e.resource = _abi.kbg_resource(*ni.allocatable.as_tuple())
                e.max_task_num = ni.allocatable.max_task_num
                e.unschedulable = 1 if obj.get("unschedulable") else 0
                labels = [x.encode() for kv in (obj.get("labels") or {}).items() for x in kv]
                taints = [str(t.get(f, "")).encode() for t in (obj.get("taints") or []) for f in ("key", "value", "effect")]
                la = (ctypes.c_char_p * max(1, len(labels)))(*labels)
                ta = (ctypes.c_char_p * max(1, len(taints)))(*taints)
                spec = _abi.kbg_node_spec(name.encode(), la, len(labels) // 2, len(taints) // 3, ta)
                keep += [la, ta, spec]
                e.node_spec = ctypes.pointer(spec)
                continue
            ti = TaskInfo(obj)
            if kind in ("pod_update", "pod_delete"):
                e.kind = _abi.EV_POD_UPDATE if kind == "pod_update" else _abi.EV_POD_DELETE
                e.task = tidx[obj["uid"]]
                e.status = ti.status
                e.node = node_of(ti.node_name)
                if e.node >= 0 and e.node not in renamed and not self.flat.node_names[e.node]:
                    keep.append(ti.node_name.encode())  # a node known only from pods: its NodeName
                    e.node_name = keep[-1]
                objs[e.task] = ti
            elif kind == "pod_add":
                e.kind = _abi.EV_POD_ADD
                e.job = self.flat.job_index[ti.job]
                e.spec = self.flat.spec_index(obj)
                e.status = ti.status
                e.priority = ti.priority
                e.node = node_of(ti.node_name)
                if e.node >= 0 and e.node not in renamed and not self.flat.node_names[e.node]:
                    keep.append(ti.node_name.encode())
                    e.node_name = keep[-1]
                e.resource = _abi.kbg_resource(*ti.resreq.as_tuple())
                keep += [ti.uid.encode(), pod_key(obj).encode()]
                e.uid, e.pod_key = keep[-2], keep[-1]
                tidx[ti.uid] = n_objs
                objs[n_objs] = ti
                n_objs += 1
            else:
                raise ValueError(f"unknown change {kind}")
        _abi.check(_abi.lib().kbg_session_update(self.handle, evs, len(changes)))
        for i, name in renamed.items():  # the NodeInfo the cache made from a pod has its Node's name now
            self.flat.node_names[i] = name
            self.flat.pod_only_names.pop(name, None)
            self.nodes[i].name = name
            self.node_index[name] = self.nodes[i]
        for i in range(len(self.flat.task_objs), n_objs):
            self.flat.task_objs.append(None)
        for i, ti in objs.items():
            self.flat.task_objs[i] = ti
        from .api import PENDING
        live = set(tidx)  # (deleted pods keep their index; counts only size output buffers)
        self.flat.pending_all = max(self.flat.pending_all, sum(1 for t in self.flat.task_objs
                                                               if t.uid in live and t.status == PENDING))
        self.flat.pending_count = max(self.flat.pending_count, self.flat.pending_all)

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
