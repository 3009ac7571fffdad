"""Runs a JSON fixture (the schema the kbref oracle reads) through the device
path and reports the same fields the oracle prints, for parity checks."""
from . import _abi, actions
from .api import RefPanic
from .cache import FakeBinder, cache_from_fixture
from .conf import tiers_from_list, load_scheduler_conf
from .framework import get_action, open_session


def fixture_tiers(fx):
    if fx.get("tiers") is None:
        return load_scheduler_conf()[1]
    return tiers_from_list(fx["tiers"])


def session_order(ssn, fx):
    """Applies an explicit `sessionOrder` before marshaling."""
    so = fx.get("sessionOrder") or {}

    def reorder(items, keys, key):
        if not keys:
            return items
        pos = {k: i for i, k in enumerate(keys)}
        first = [x for x in sorted(items, key=lambda x: pos.get(key(x), 1 << 30)) if key(x) in pos]
        return first + [x for x in items if key(x) not in pos]

    return (reorder(ssn.nodes, so.get("nodes"), lambda n: n.name),
            reorder(ssn.jobs, so.get("jobs"), lambda j: j.uid),
            reorder(ssn.queues, so.get("queues"), lambda q: q.uid))


class _OrderedCache:
    """Wraps a SchedulerCache so snapshot() honours the fixture's sessionOrder."""

    def __init__(self, cache, fx):
        self._c = cache
        self._fx = fx

    def __getattr__(self, k):
        return getattr(self._c, k)

    def snapshot(self):
        s = self._c.snapshot()
        s.nodes, s.jobs, s.queues = session_order(s, self._fx)
        return s


def fit_error(nodes, cpu, memory, gpu):
    """JobInfo.FitError (job_info.go:329-358) from NodesFitDelta counts."""
    if nodes == 0:
        return "0 nodes are available"
    reasons = [f"{v} insufficient {k}" for k, v in (("cpu", cpu), ("memory", memory), ("GPU", gpu)) if v > 0]
    return f"0/{nodes} nodes are available, {', '.join(sorted(reasons))}."


def run_fixture(fx, options=None):
    """Returns (result dict in the oracle's output schema, session)."""
    opts = dict(options or {})
    if (fx.get("options") or {}).get("heapDownRule") == "go1.13":
        opts["heap_rule"] = 1
    binder = FakeBinder()
    try:
        cache = _OrderedCache(cache_from_fixture(fx, binder), fx)
        ssn = open_session(cache, fixture_tiers(fx), opts)
    except RefPanic as e:  # Resource.Sub underflow while building the cache/snapshot
        return {"status": "ref_panic", "error": str(e)}, None
    except _abi.KbgError as e:
        return {"status": e.status, "error": str(e)}, None
    status = "ok"
    try:
        for name in fx.get("actions") or ["allocate"]:  # conf "actions" (util.go:30-61)
            action = get_action(name)
            if action is None:
                return {"status": "bad_input", "error": f"unsupported action {name}"}, ssn
            status = action.execute(ssn).status
    except _abi.KbgError as e:
        if e.status == "unsupported":
            return {"status": "unsupported", "error": str(e)}, ssn
        if e.status != "ref_panic":
            raise
        return {"status": "ref_panic", "error": str(e)}, ssn
    return session_output(ssn, binder.binds, status), ssn


def session_output(ssn, binds, status="ok"):
    """The session's outputs in the oracle's output schema, after its actions
    have been replayed through it (actions.replay): the decision log, the
    binds the fake binder recorded, evictions, job / queue / node states (the
    latter three read from the library)."""
    tasks, names = ssn.flat.task_objs, ssn.flat.node_names
    out = {"status": status, "decisions": [], "binds": dict(binds), "jobs": [], "queues": [], "nodes": [],
           "evictions": [{"task": t.uid, "by": by.uid, "action": act} for t, by, act in ssn.evictions]}
    for (t, nd, kind, disp), act in zip(ssn.decisions, ssn.action_of):
        d = {"task": tasks[t].uid, "job": tasks[t].job, "node": names[nd],
             "kind": "allocate" if kind == _abi.KIND_ALLOCATE else "pipeline", "dispatched_at": disp}
        if act != "allocate":
            d["action"] = act
        out["decisions"].append(d)
    has_drf = any(p.name == "drf" for t in ssn.tiers for p in t.plugins)
    for j, job in enumerate(ssn.jobs):
        st = ssn.job_state(j)
        row = {"uid": job.uid, "queue": job.queue, "ready_num": st.ready_num, "min_available": job.min_available,
               "ready": bool(st.ready), "allocated": list(job.allocated.as_tuple())}
        if has_drf:
            row["drf_share"] = st.drf_share
        if st.fit_valid:
            row["fit_error"] = fit_error(st.fit_nodes, st.fit_cpu, st.fit_memory, st.fit_gpu)
        out["jobs"].append(row)
    for q, queue in enumerate(ssn.queues):
        st = ssn.queue_state(q)
        if st.has_attr:
            out["queues"].append({"uid": queue.uid, "share": st.share,
                                  "deserved": [st.deserved.milli_cpu, st.deserved.memory, st.deserved.milli_gpu],
                                  "allocated": [st.allocated.milli_cpu, st.allocated.memory, st.allocated.milli_gpu],
                                  "request": [st.request.milli_cpu, st.request.memory, st.request.milli_gpu]})
    for i, n in enumerate(ssn.nodes):
        st = ssn.node_state(i)
        out["nodes"].append({"name": n.name, "idle": [st.idle.milli_cpu, st.idle.memory, st.idle.milli_gpu],
                             "releasing": [st.releasing.milli_cpu, st.releasing.memory, st.releasing.milli_gpu],
                             "ntasks": st.num_tasks})
    return out
