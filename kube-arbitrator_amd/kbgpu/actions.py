"""The allocate action (pkg/scheduler/actions/allocate/allocate.go:27-178).

`AllocateAction.execute(ssn)` runs allocateAction.Execute on the MI355X path
(kbg_allocate) and replays its decision log through the session in reference
order: ssn.Allocate / ssn.Pipeline per decision, then ssn.dispatch for every
task the decision's JobReady check bound (session.go:283-290).
"""
import ctypes

from . import _abi
from .framework import register_action


class AllocateResult:
    def __init__(self, decisions, status, error):
        self.decisions = decisions  # list of (task_index, node_index, kind, dispatched_at)
        self.status = status
        self.error = error


class AllocateAction:
    def name(self):
        return "allocate"

    def initialize(self):
        pass

    def uninitialize(self):
        pass

    def execute(self, ssn):
        L = _abi.lib()
        cap = max(1, ssn.flat.pending_count)
        buf = (_abi.kbg_decision * cap)()
        n = ctypes.c_int32(0)
        code = L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n))
        err = L.kbg_last_error().decode() if code != _abi.KBG_OK else ""
        if code not in (_abi.KBG_OK, _abi.KBG_E_REF_PANIC):
            _abi.check(code)
        decs = [(buf[i].task, buf[i].node, buf[i].kind, buf[i].dispatched_at) for i in range(n.value)]
        tasks = ssn.flat.task_objs
        names = ssn.flat.node_names
        bound_at = {}
        for i, (t, nd, kind, disp) in enumerate(decs):
            task = tasks[t]
            if kind == _abi.KIND_ALLOCATE:
                ssn.allocate(task, names[nd])
            else:
                ssn.pipeline(task, names[nd])
            if disp >= 0:
                bound_at.setdefault(disp, []).append(task)
            for bt in bound_at.pop(i, []):
                ssn.dispatch(bt)
        ssn.decisions = decs
        result = AllocateResult(decs, _abi.STATUS_NAMES[code], err)
        if code == _abi.KBG_E_REF_PANIC:
            raise _abi.KbgError(code, err)
        return result


def new():
    return AllocateAction()


register_action(AllocateAction())
