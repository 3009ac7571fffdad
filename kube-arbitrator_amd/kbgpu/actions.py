"""The allocate, backfill, reclaim and preempt actions
(pkg/scheduler/actions/{allocate/allocate.go:27-178, backfill/backfill.go:26-73,
reclaim/reclaim.go:27-191, preempt/preempt.go:30-253}).

`execute(ssn)` runs the action's Execute on the MI355X path (kbg_allocate /
kbg_backfill) and replays the new part of the cycle's decision log through
the session in reference order: ssn.Allocate / ssn.Pipeline per decision,
then ssn.dispatch for every task the decision's JobReady check bound
(session.go:283-290) — a backfill decision can dispatch Allocate decisions of
its job made by the allocate action earlier in the cycle.
"""
import ctypes

from . import _abi
from .framework import register_action


class ActionResult:
    def __init__(self, decisions, status, error):
        self.decisions = decisions  # the cycle's log: (task_index, node_index, kind, dispatched_at)
        self.status = status
        self.error = error


AllocateResult = ActionResult


def decision_list(buf, n):
    """The first n kbg_decision records as (task, node, kind, dispatched_at)."""
    return [(buf[i].task, buf[i].node, buf[i].kind, buf[i].dispatched_at) for i in range(n)]


def replay(ssn, decs, action, evicting=False):
    """Replays the new part of the cycle's decision log `decs` (the whole log
    of the cycle so far, as the library returns it) through the session in
    reference order: ssn.Allocate / ssn.Pipeline per decision, then
    ssn.dispatch for every task the decision's JobReady check bound
    (session.go:205-316)."""
    start = len(ssn.decisions)
    tasks = ssn.flat.task_objs
    names = ssn.flat.node_names
    bound_at = {}
    for t, _, _, disp in decs:
        if disp >= start:
            bound_at.setdefault(disp, []).append(tasks[t])
    for i in range(start, len(decs)):
        t, nd, kind, _ = decs[i]
        if kind == _abi.KIND_ALLOCATE:
            ssn.allocate(tasks[t], names[nd])
        elif evicting:
            ssn.pipeline_replay(tasks[t], names[nd])
        else:
            ssn.pipeline(tasks[t], names[nd])
        for bt in bound_at.pop(i, []):
            ssn.dispatch(bt)
    ssn.decisions = decs
    ssn.action_of.extend([action] * (len(decs) - start))


class _DeviceAction:
    _entry = None
    _evicting = False

    def initialize(self):
        pass

    def uninitialize(self):
        pass

    def execute(self, ssn):
        L = _abi.lib()
        cap = max(1, ssn.flat.pending_all)
        buf = (_abi.kbg_decision * cap)()
        n = ctypes.c_int32(0)
        code = getattr(L, self._entry)(ssn.handle, buf, cap, ctypes.byref(n))
        err = L.kbg_last_error().decode() if code != _abi.KBG_OK else ""
        if code not in (_abi.KBG_OK, _abi.KBG_E_REF_PANIC):
            _abi.check(code)
        decs = decision_list(buf, n.value)
        replay(ssn, decs, self.name(), self._evicting)
        result = ActionResult(decs, _abi.STATUS_NAMES[code], err)
        if code == _abi.KBG_E_REF_PANIC:
            raise _abi.KbgError(code, err)
        return result


class AllocateAction(_DeviceAction):
    _entry = "kbg_allocate"

    def name(self):
        return "allocate"


class BackfillAction(_DeviceAction):
    _entry = "kbg_backfill"

    def name(self):
        return "backfill"


class _EvictingAction(_DeviceAction):
    """reclaim / preempt: pipelines and committed evictions replay as statuses
    (framework.Session.pipeline_replay / evict); the committed evictions go
    through the cache's evictor (cache.Evict). Node Idle / Releasing (which a
    discarded statement also changes, statement.go:81-108) are then taken from
    the device session, so the actions after this one replay from them."""

    _evicting = True

    def execute(self, ssn):
        seen = len(ssn.evictions)
        try:
            return super().execute(ssn)
        finally:
            L = _abi.lib()
            n = ctypes.c_int32(0)
            _abi.check(L.kbg_evictions_get(ssn.handle, None, 0, ctypes.byref(n)))
            buf = (_abi.kbg_eviction * max(1, n.value))()
            _abi.check(L.kbg_evictions_get(ssn.handle, buf, n.value, ctypes.byref(n)))
            tasks = ssn.flat.task_objs
            for i in range(seen, n.value):
                ev = (tasks[buf[i].task], tasks[buf[i].by], _abi.ACTION_NAMES[buf[i].action])
                ssn.evictions.append(ev)
                ssn.evict(ev[0], ev[2])
            ssn.sync_node_resources()


class ReclaimAction(_EvictingAction):
    _entry = "kbg_reclaim"

    def name(self):
        return "reclaim"


class PreemptAction(_EvictingAction):
    _entry = "kbg_preempt"

    def name(self):
        return "preempt"


def new():
    return AllocateAction()


register_action(AllocateAction())
register_action(BackfillAction())
register_action(ReclaimAction())
register_action(PreemptAction())
