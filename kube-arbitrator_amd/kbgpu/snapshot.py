"""Marshals an opened session into the flat kbg_snapshot of include/kbgpu.h.

This is the work a Go cgo adapter would do in front of the device path
(INTEGRATION.md): intern every string, flatten ssn.Nodes / ssn.Jobs /
ssn.Queues / ssn.Others and each pod's predicate inputs into plain arrays.
"""
import ctypes
import json

import numpy as np

from . import _abi
from .api import PENDING, pod_key


class Interner:
    def __init__(self):
        self.ids = {}
        self.strings = []

    def __call__(self, s):
        s = "" if s is None else str(s)
        i = self.ids.get(s)
        if i is None:
            i = len(self.strings)
            self.ids[s] = i
            self.strings.append(s)
        return i


def container_ports(pod):
    """GetContainerPorts(pod) (vendor scheduler/util/utils.go:30-41) as (hostIP, protocol, hostPort)."""
    return [(pt.get("hostIP") or "", pt.get("protocol") or "", int(pt.get("hostPort") or 0))
            for c in pod.get("containers", []) for pt in (c.get("ports") or [])]


def pod_terms(pod, kind):
    """RequiredDuringSchedulingIgnoredDuringExecution terms of the pod's
    podAffinity / podAntiAffinity (vendor predicates.go:1216-1242)."""
    aff = pod.get("affinity") or {}
    pa = aff.get(kind) if isinstance(aff, dict) else None
    return list((pa or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []) if isinstance(pa, dict) else []


def _spec_key(pod, with_identity):
    aff = pod.get("affinity") or None
    key = [pod.get("nodeSelector") or {}, aff, pod.get("tolerations") or [], container_ports(pod)]
    if with_identity:  # other pods' affinity terms select by namespace and labels
        key += [pod.get("namespace") or "", pod.get("labels") or {}]
    return json.dumps(key, sort_keys=True)


class FlatSnapshot:
    """Owns the arrays behind one kbg_snapshot (keeps them alive for the call)."""

    def __init__(self, nodes, jobs, queues, others, tiers, registered=None):
        S = Interner()
        self.interner = S
        # queues
        self.queue_index = {q.uid: i for i, q in enumerate(queues)}
        qs = (_abi.kbg_queue * max(1, len(queues)))()
        for i, q in enumerate(queues):
            qs[i].uid = S(q.uid)
            qs[i].weight = q.weight
        # nodes
        nd = np.zeros(len(nodes), dtype=np.dtype(_abi.kbg_node))
        labels, taints, ports, node_keys, node_pods = [], [], [], [], []
        for i, n in enumerate(nodes):
            obj = n.node or {}
            r = nd[i]
            r["name"] = S(n.name)
            r["has_node"] = 1 if n.node is not None else 0
            r["allocatable"] = n.allocatable.as_tuple()
            r["idle"] = n.idle.as_tuple()
            r["releasing"] = n.releasing.as_tuple()
            r["max_task_num"] = n.allocatable.max_task_num
            r["num_tasks"] = len(n.tasks)
            r["unschedulable"] = 1 if obj.get("unschedulable") else 0
            r["label_off"] = len(labels) // 2
            for k, v in (obj.get("labels") or {}).items():
                labels += [S(k), S(v)]
            r["label_len"] = len(labels) // 2 - r["label_off"]
            r["taint_off"] = len(taints)
            for t in obj.get("taints") or []:
                taints.append((S(t.get("key")), S(t.get("value")), S(t.get("effect"))))
            r["taint_len"] = len(taints) - r["taint_off"]
            # NodeInfo.UsedPorts over node.Pods(): only hostPort > 0 is recorded
            # (host_ports.go Add); one entry per pod and port, so a pod that
            # leaves the node (kbg_session_update) takes exactly its own entries
            r["port_off"] = len(ports)
            for t in n.tasks.values():
                p0 = len(ports)
                for ip, proto, port in container_ports(t.pod):
                    if port > 0:
                        ports.append((S(ip or "0.0.0.0"), S(proto or "TCP"), port))
                # the node's copy as RemoveTask reads it (kbgpu.h kbg_node_pod)
                node_pods.append((t.resreq.as_tuple(), t.status, len(ports) - p0))
            r["port_len"] = len(ports) - r["port_off"]
            # NodeInfo.Tasks keys (PodKey) of every pod on the node, in order
            r["key_off"] = len(node_keys)
            node_keys.extend(S(k) for k in n.tasks.keys())
            r["key_len"] = len(node_keys) - r["key_off"]
        self.node_names = [n.name for n in nodes]
        # a node the cache knows only from its pods (Node nil, Name ""): the NodeName they carry -> its index
        self.pod_only_names = {}
        for i, n in enumerate(nodes):
            if n.node is None:
                for t in n.tasks.values():
                    if t.node_name:
                        self.pod_only_names.setdefault(t.node_name, i)
        # jobs + tasks + specs (node task lists are filled once task indices exist)
        jb = np.zeros(len(jobs), dtype=np.dtype(_abi.kbg_job))
        task_rows, self.task_objs = [], []
        spec_ids = {}
        specs, terms, reqs, values, tols, selectors = [], [], [], [], [], []
        pterms, plabels = [], []
        any_terms = any(pod_terms(t.pod, "podAffinity") or pod_terms(t.pod, "podAntiAffinity")
                        for job in jobs for t in job.tasks.values())

        def add_reqs(exprs):
            off = len(reqs)
            for e in exprs or []:
                voff = len(values)
                values.extend(S(v) for v in (e.get("values") or []))
                reqs.append((S(e.get("key")), S(e.get("operator")), voff, len(values) - voff))
            return off, len(reqs) - off

        def add_pod_terms(pod, kind):
            off = len(pterms)
            for t in pod_terms(pod, kind):
                ls = t.get("labelSelector")
                moff = len(selectors) // 2
                eoff, elen = len(reqs), 0
                if isinstance(ls, dict):
                    for k, v in (ls.get("matchLabels") or {}).items():
                        selectors.extend((S(k), S(v)))
                    eoff, elen = add_reqs(ls.get("matchExpressions"))
                noff = len(values)
                values.extend(S(n) for n in (t.get("namespaces") or []))
                pterms.append((1 if isinstance(ls, dict) else 0, moff, len(selectors) // 2 - moff, eoff, elen,
                               noff, len(values) - noff, S(t.get("topologyKey"))))
            return off, len(pterms) - off

        def spec_of(pod):
            key = _spec_key(pod, any_terms)
            sid = spec_ids.get(key)
            if sid is not None:
                return sid
            sel_off = len(selectors) // 2
            for k, v in (pod.get("nodeSelector") or {}).items():
                selectors.extend((S(k), S(v)))
            sel_len = len(selectors) // 2 - sel_off  # (pod terms append matchLabels pairs to the same array)
            aff = pod.get("affinity") or {}
            na = aff.get("nodeAffinity") if isinstance(aff, dict) else None
            req = na.get("requiredDuringSchedulingIgnoredDuringExecution") if isinstance(na, dict) else None
            term_off = len(terms)
            if req is not None:
                for t in req.get("nodeSelectorTerms") or []:
                    row = []
                    for part in ("matchExpressions", "matchFields"):
                        row += list(add_reqs(t.get(part)))
                    terms.append(tuple(row))
            tol_off = len(tols)
            for t in pod.get("tolerations") or []:
                tols.append((S(t.get("key")), S(t.get("operator")), S(t.get("value")), S(t.get("effect"))))
            cports = container_ports(pod)
            has_ports = any(port > 0 for _, _, port in cports)
            port_off = len(ports)
            for ip, proto, port in cports:
                ports.append((S(ip), S(proto), port))
            aff_off, aff_len = add_pod_terms(pod, "podAffinity")
            anti_off, anti_len = add_pod_terms(pod, "podAntiAffinity")
            lab_off = len(plabels) // 2
            if any_terms:
                for k, v in (pod.get("labels") or {}).items():
                    plabels.extend((S(k), S(v)))
            specs.append((sel_off, sel_len, 1 if req is not None else 0, term_off,
                          len(terms) - term_off, tol_off, len(tols) - tol_off, 1 if has_ports else 0,
                          1 if aff_len or anti_len else 0, port_off, len(ports) - port_off,
                          S(pod.get("namespace") or ""), lab_off, len(plabels) // 2 - lab_off,
                          aff_off, aff_len, anti_off, anti_len))
            sid = len(specs) - 1
            spec_ids[key] = sid
            return sid

        self._spec_ids, self._any_terms = spec_ids, any_terms
        for j, job in enumerate(jobs):
            r = jb[j]
            r["uid"] = S(job.uid)
            r["queue"] = self.queue_index[job.queue]
            r["min_available"] = job.min_available
            r["priority"] = job.priority
            r["creation_ns"] = job.creation_timestamp
            for t in job.tasks.values():
                task_rows.append((S(t.uid), j, t.status, t.priority, t.resreq.as_tuple(), spec_of(t.pod), S(t.node_name),
                                  S(pod_key(t.pod)), 0))
                self.task_objs.append(t)
        # NodeInfo.Tasks order of the session-job tasks on each node (preempt/reclaim victims)
        task_index = {t.uid: i for i, t in enumerate(self.task_objs)}
        node_tasks = []
        for i, n in enumerate(nodes):
            nd[i]["task_off"] = len(node_tasks)
            node_tasks.extend(task_index[t.uid] for t in n.tasks.values() if t.uid in task_index)
            nd[i]["task_len"] = len(node_tasks) - nd[i]["task_off"]
        tk = np.zeros(len(task_rows), dtype=np.dtype(_abi.kbg_task))
        for i, row in enumerate(task_rows):
            tk[i] = row
        self.job_index = {job.uid: j for j, job in enumerate(jobs)}
        self.pending_count = sum(1 for t in self.task_objs if t.status == PENDING and not t.resreq.is_empty())
        self.pending_all = sum(1 for t in self.task_objs if t.status == PENDING)

        def arr(ctype, rows):
            a = (ctype * max(1, len(rows)))()
            for i, row in enumerate(rows):
                a[i] = ctype(*row)
            return a

        self._keep = []
        oth = arr(_abi.kbg_resource, [t.resreq.as_tuple() for t in others])
        plugin_rows, tier_sizes = [], []
        for tier in tiers:
            tier_sizes.append(len(tier.plugins))
            for p in tier.plugins:  # KBG_PLUGIN_REGISTERED: this process has a builder for the name
                reg = _abi.PLUGIN_REGISTERED if registered is not None and registered(p.name) else 0
                plugin_rows.append((S(p.name), p.flags() | reg))
        self.strings_c = (ctypes.c_char_p * max(1, len(S.strings)))(*[s.encode("utf-8") for s in S.strings])
        self.arrays = dict(
            nodes=nd, jobs=jb, tasks=tk, queues=qs, others=oth,
            specs=arr(_abi.kbg_spec, specs), terms=arr(_abi.kbg_term, terms), reqs=arr(_abi.kbg_requirement, reqs),
            values=np.asarray(values or [0], dtype=np.int32), tols=arr(_abi.kbg_toleration, tols),
            labels=np.asarray(labels or [0, 0], dtype=np.int32), taints=arr(_abi.kbg_taint, taints),
            selectors=np.asarray(selectors or [0, 0], dtype=np.int32),
            plugins=arr(_abi.kbg_plugin_option, plugin_rows), tier_sizes=np.asarray(tier_sizes or [0], dtype=np.int32),
            ports=arr(_abi.kbg_host_port, ports), node_tasks=np.asarray(node_tasks or [0], dtype=np.int32),
            pod_terms=arr(_abi.kbg_pod_term, pterms), pod_labels=np.asarray(plabels or [0, 0], dtype=np.int32),
            node_pod_keys=np.asarray(node_keys or [0], dtype=np.int32), node_pods=arr(_abi.kbg_node_pod, node_pods))
        A = self.arrays

        def ptr(a, ctype):
            if isinstance(a, np.ndarray):
                return a.ctypes.data_as(ctypes.POINTER(ctype))
            return ctypes.cast(a, ctypes.POINTER(ctype))

        snap = _abi.kbg_snapshot()
        snap.strings = ctypes.cast(self.strings_c, ctypes.POINTER(ctypes.c_char_p))
        snap.n_strings = len(S.strings)
        snap.nodes, snap.n_nodes = ptr(A["nodes"], _abi.kbg_node), len(nodes)
        snap.jobs, snap.n_jobs = ptr(A["jobs"], _abi.kbg_job), len(jobs)
        snap.queues, snap.n_queues = ptr(A["queues"], _abi.kbg_queue), len(queues)
        snap.tasks, snap.n_tasks = ptr(A["tasks"], _abi.kbg_task), len(task_rows)
        snap.others, snap.n_others = ptr(A["others"], _abi.kbg_resource), len(others)
        snap.specs, snap.n_specs = ptr(A["specs"], _abi.kbg_spec), len(specs)
        snap.terms, snap.n_terms = ptr(A["terms"], _abi.kbg_term), len(terms)
        snap.reqs, snap.n_reqs = ptr(A["reqs"], _abi.kbg_requirement), len(reqs)
        snap.values, snap.n_values = ptr(A["values"], ctypes.c_int32), len(values)
        snap.tolerations, snap.n_tolerations = ptr(A["tols"], _abi.kbg_toleration), len(tols)
        snap.labels, snap.n_labels = ptr(A["labels"], ctypes.c_int32), len(labels) // 2
        snap.taints, snap.n_taints = ptr(A["taints"], _abi.kbg_taint), len(taints)
        snap.selectors, snap.n_selectors = ptr(A["selectors"], ctypes.c_int32), len(selectors) // 2
        snap.plugins, snap.n_plugins = ptr(A["plugins"], _abi.kbg_plugin_option), len(plugin_rows)
        snap.tier_sizes, snap.n_tiers = ptr(A["tier_sizes"], ctypes.c_int32), len(tier_sizes)
        snap.ports, snap.n_ports = ptr(A["ports"], _abi.kbg_host_port), len(ports)
        snap.node_tasks, snap.n_node_tasks = ptr(A["node_tasks"], ctypes.c_int32), len(node_tasks)
        snap.pod_terms, snap.n_pod_terms = ptr(A["pod_terms"], _abi.kbg_pod_term), len(pterms)
        snap.pod_labels, snap.n_pod_labels = ptr(A["pod_labels"], ctypes.c_int32), len(plabels) // 2
        snap.node_pod_keys, snap.n_node_pod_keys = ptr(A["node_pod_keys"], ctypes.c_int32), len(node_keys)
        snap.node_pods, snap.n_node_pods = ptr(A["node_pods"], _abi.kbg_node_pod), len(node_pods)
        self.snap = snap


    def spec_index(self, pod):
        """Index of the session spec a new pod of the same predicate inputs
        would use (kbg_session_update POD_ADD); KeyError when it has none."""
        return self._spec_ids[_spec_key(pod, self._any_terms)]


# ---- wire format (include/kbgpu.h "Snapshot wire format")
def encode(snap):
    """The kbg_snapshot `snap` as the library's wire-format bytes."""
    L = _abi.lib()
    n = ctypes.c_int64(0)
    _abi.check(L.kbg_snapshot_encode(ctypes.byref(snap), None, 0, ctypes.byref(n)))
    buf = (ctypes.c_uint8 * max(1, n.value))()
    _abi.check(L.kbg_snapshot_encode(ctypes.byref(snap), buf, n.value, ctypes.byref(n)))
    return bytes(buf[:n.value])


class SnapshotBlob:
    """A decoded wire-format snapshot owned by the library; .snap is the
    kbg_snapshot to hand to kbg_session_open."""

    def __init__(self, handle):
        self.handle = handle
        self.snap = _abi.lib().kbg_snapshot_blob_get(handle).contents
        # the view points into library-owned memory that close() frees: keep
        # the owner reachable from the view (`blob.snap` alone stays valid)
        self.snap._owner = self

    @classmethod
    def decode(cls, data):
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        _abi.check(_abi.lib().kbg_snapshot_decode(buf, len(data), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def load(cls, path):
        h = ctypes.c_void_p()
        _abi.check(_abi.lib().kbg_snapshot_load(str(path).encode(), ctypes.byref(h)))
        return cls(h)

    def close(self):
        if self.handle:
            _abi.lib().kbg_snapshot_blob_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()
