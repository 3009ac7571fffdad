"""ctypes binding of include/kbgpu.h (the C ABI of the MI355X allocate path).

The library is loaded from this package directory (built in-tree by
`make -C kube-arbitrator_amd`). Loading fails loudly: there is no CPU
fallback for the product path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# KBG_LIB_PATH: another build of the library (same-box A/B runs of two trees)
LIB_PATH = os.environ.get("KBG_LIB_PATH") or os.path.join(_HERE, "libkbgpu.so")

# kbg_status
KBG_OK = 0
KBG_E_INVALID = 1
KBG_E_UNSUPPORTED = 2
KBG_E_REF_PANIC = 3
KBG_E_HIP = 4
KBG_E_RCCL = 5
KBG_E_NOMEM = 6
KBG_E_CAPACITY = 7

STATUS_NAMES = {
    KBG_OK: "ok", KBG_E_INVALID: "invalid", KBG_E_UNSUPPORTED: "unsupported",
    KBG_E_REF_PANIC: "ref_panic", KBG_E_HIP: "hip", KBG_E_RCCL: "rccl",
    KBG_E_NOMEM: "nomem", KBG_E_CAPACITY: "capacity",
}

# plugin disable flags
DISABLE_JOB_ORDER = 1 << 0
DISABLE_JOB_READY = 1 << 1
DISABLE_TASK_ORDER = 1 << 2
DISABLE_PREEMPTABLE = 1 << 3
DISABLE_RECLAIMABLE = 1 << 4
DISABLE_QUEUE_ORDER = 1 << 5
DISABLE_PREDICATE = 1 << 6
PLUGIN_REGISTERED = 0x80000000  # kbg_plugin_option.flags, read when kbg_options.plugin_registry = 1

ABI_VERSION = 13
COMM_ID_BYTES = 128

KIND_ALLOCATE = 0
KIND_PIPELINE = 1

i32 = ctypes.c_int32
i64 = ctypes.c_int64
f64 = ctypes.c_double
P = ctypes.POINTER


class kbg_resource(ctypes.Structure):
    _fields_ = [("milli_cpu", f64), ("memory", f64), ("milli_gpu", f64)]


class kbg_node(ctypes.Structure):
    _fields_ = [("name", i32), ("has_node", i32), ("allocatable", kbg_resource), ("idle", kbg_resource),
                ("releasing", kbg_resource), ("max_task_num", i32), ("num_tasks", i32), ("unschedulable", i32),
                ("label_off", i32), ("label_len", i32), ("taint_off", i32), ("taint_len", i32),
                ("port_off", i32), ("port_len", i32), ("task_off", i32), ("task_len", i32),
                ("key_off", i32), ("key_len", i32)]


class kbg_node_pod(ctypes.Structure):
    _fields_ = [("resreq", kbg_resource), ("status", i32), ("port_len", i32)]


class kbg_host_port(ctypes.Structure):
    _fields_ = [("host_ip", i32), ("protocol", i32), ("host_port", i32)]


class kbg_taint(ctypes.Structure):
    _fields_ = [("key", i32), ("value", i32), ("effect", i32)]


class kbg_job(ctypes.Structure):
    _fields_ = [("uid", i32), ("queue", i32), ("min_available", i32), ("priority", i32), ("creation_ns", i64)]


class kbg_queue(ctypes.Structure):
    _fields_ = [("uid", i32), ("weight", i32)]


class kbg_task(ctypes.Structure):
    _fields_ = [("uid", i32), ("job", i32), ("status", i32), ("priority", i32), ("resreq", kbg_resource),
                ("spec", i32), ("node_name", i32), ("pod_key", i32), ("reserved", i32)]


class kbg_spec(ctypes.Structure):
    _fields_ = [("selector_off", i32), ("selector_len", i32), ("has_required_affinity", i32), ("term_off", i32),
                ("term_len", i32), ("toleration_off", i32), ("toleration_len", i32), ("has_host_ports", i32),
                ("has_pod_affinity", i32), ("port_off", i32), ("port_len", i32), ("ns", i32),
                ("pod_label_off", i32), ("pod_label_len", i32), ("aff_off", i32), ("aff_len", i32),
                ("anti_off", i32), ("anti_len", i32)]


class kbg_pod_term(ctypes.Structure):
    _fields_ = [("has_selector", i32), ("match_off", i32), ("match_len", i32), ("expr_off", i32), ("expr_len", i32),
                ("ns_off", i32), ("ns_len", i32), ("topology_key", i32)]


class kbg_term(ctypes.Structure):
    _fields_ = [("expr_off", i32), ("expr_len", i32), ("field_off", i32), ("field_len", i32)]


class kbg_requirement(ctypes.Structure):
    _fields_ = [("key", i32), ("op", i32), ("value_off", i32), ("value_len", i32)]


class kbg_toleration(ctypes.Structure):
    _fields_ = [("key", i32), ("op", i32), ("value", i32), ("effect", i32)]


class kbg_plugin_option(ctypes.Structure):
    _fields_ = [("name", i32), ("flags", ctypes.c_uint32)]


class kbg_snapshot(ctypes.Structure):
    _fields_ = [
        ("strings", P(ctypes.c_char_p)), ("n_strings", i32),
        ("nodes", P(kbg_node)), ("n_nodes", i32),
        ("jobs", P(kbg_job)), ("n_jobs", i32),
        ("queues", P(kbg_queue)), ("n_queues", i32),
        ("tasks", P(kbg_task)), ("n_tasks", i32),
        ("others", P(kbg_resource)), ("n_others", i32),
        ("specs", P(kbg_spec)), ("n_specs", i32),
        ("terms", P(kbg_term)), ("n_terms", i32),
        ("reqs", P(kbg_requirement)), ("n_reqs", i32),
        ("values", P(i32)), ("n_values", i32),
        ("tolerations", P(kbg_toleration)), ("n_tolerations", i32),
        ("labels", P(i32)), ("n_labels", i32),
        ("taints", P(kbg_taint)), ("n_taints", i32),
        ("selectors", P(i32)), ("n_selectors", i32),
        ("plugins", P(kbg_plugin_option)), ("n_plugins", i32),
        ("tier_sizes", P(i32)), ("n_tiers", i32),
        ("ports", P(kbg_host_port)), ("n_ports", i32),
        ("node_tasks", P(i32)), ("n_node_tasks", i32),
        ("pod_terms", P(kbg_pod_term)), ("n_pod_terms", i32),
        ("pod_labels", P(i32)), ("n_pod_labels", i32),
        ("node_pod_keys", P(i32)), ("n_node_pod_keys", i32),
        ("node_pods", P(kbg_node_pod)), ("n_node_pods", i32),
    ]


class kbg_options(ctypes.Structure):
    _fields_ = [("device", i32), ("heap_rule", i32), ("batch_tasks", i32), ("candidates", i32),
                ("full_scan", i32), ("shards", i32), ("plugin_registry", i32), ("reserved", i32 * 5)]


class kbg_decision(ctypes.Structure):
    _fields_ = [("task", i32), ("node", i32), ("kind", i32), ("dispatched_at", i32)]


class kbg_job_state(ctypes.Structure):
    _fields_ = [("ready_num", i32), ("ready", i32), ("drf_share", f64), ("drf_allocated", kbg_resource),
                ("fit_valid", i32), ("fit_nodes", i32), ("fit_cpu", i32), ("fit_memory", i32), ("fit_gpu", i32),
                ("reserved", i32 * 3)]


class kbg_queue_state(ctypes.Structure):
    _fields_ = [("share", f64), ("deserved", kbg_resource), ("allocated", kbg_resource), ("request", kbg_resource),
                ("overused", i32), ("has_attr", i32)]


class kbg_node_state(ctypes.Structure):
    _fields_ = [("idle", kbg_resource), ("releasing", kbg_resource), ("num_tasks", i32)]


class kbg_stats(ctypes.Structure):
    _fields_ = [("evaluations", i64), ("node_visits", i64), ("batches", i64), ("mispredictions", i64),
                ("truncations", i64), ("scan_launches", i64), ("scan_kernel_ms", f64), ("select_kernel_ms", f64),
                ("allocate_ms", f64), ("open_ms", f64), ("engine_ms", f64), ("resolve_ms", f64),
                ("device_ms", f64), ("delta_ms", f64), ("replayed", i64), ("n_classes", i32), ("shards", i32), ("shard_index", i32),
                ("int_scan", i32), ("exchange_ms", f64), ("backfill_ms", f64),
                ("reclaim_ms", f64), ("preempt_ms", f64), ("victim_scans", i64), ("victim_kernel_ms", f64),
                ("victim_tries", i64), ("victim_host_evals", i64), ("task_evaluations", i64),
                ("resolve_steps", i64), ("resolve_rechecks", i64), ("overlapped", i64),
                ("update_ms", f64), ("update_rebuilds", i64), ("owner_rounds", i64),
                ("reused_batches", i64), ("refresh_scans", i64)]


EV_POD_UPDATE = 1
EV_POD_DELETE = 2
EV_POD_ADD = 3
EV_NODE_UPDATE = 4
EV_NODE_SET = 5
EV_NODE_ADD = 6
EV_NODE_DELETE = 7
EV_JOB_ADD = 8
EV_JOB_DELETE = 9
EV_QUEUE_ADD = 10
EV_QUEUE_DELETE = 11
RENUM_TASKS, RENUM_NODES, RENUM_JOBS, RENUM_QUEUES = 0, 1, 2, 3


class kbg_node_spec(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("labels", ctypes.POINTER(ctypes.c_char_p)), ("n_labels", i32),
                ("n_taints", i32), ("taints", ctypes.POINTER(ctypes.c_char_p))]


class kbg_event(ctypes.Structure):
    _fields_ = [("kind", i32), ("task", i32), ("status", i32), ("node", i32), ("job", i32), ("spec", i32),
                ("priority", i32), ("max_task_num", i32), ("resource", kbg_resource), ("unschedulable", i32),
                ("reserved", i32), ("uid", ctypes.c_char_p), ("pod_key", ctypes.c_char_p),
                ("node_spec", ctypes.POINTER(kbg_node_spec)), ("node_name", ctypes.c_char_p),
                ("name", ctypes.c_char_p), ("creation_ns", ctypes.c_int64), ("queue", i32), ("min_available", i32),
                ("weight", i32), ("reserved2", i32)]


class kbg_eviction(ctypes.Structure):
    _fields_ = [("task", i32), ("by", i32), ("action", i32), ("reserved", i32)]


ACTION_NAMES = {0: "allocate", 1: "backfill", 2: "reclaim", 3: "preempt"}


# Every symbol include/kbgpu.h declares, with its ctypes signature.
SIGNATURES = {
    "kbg_abi_version": (i32, []),
    "kbg_last_error": (ctypes.c_char_p, []),
    "kbg_device_count": (i32, []),
    "kbg_session_open": (i32, [P(kbg_snapshot), P(kbg_options), P(ctypes.c_void_p)]),
    "kbg_session_open_sharded": (i32, [P(kbg_snapshot), P(kbg_options), ctypes.c_void_p, P(ctypes.c_void_p)]),
    "kbg_comm_unique_id": (i32, [P(ctypes.c_uint8)]),
    "kbg_comm_init": (i32, [P(ctypes.c_uint8), i32, i32, i32, P(ctypes.c_void_p)]),
    "kbg_comm_init_host": (i32, [ctypes.c_char_p, i32, i32, i32, P(ctypes.c_void_p)]),
    "kbg_comm_destroy": (None, [ctypes.c_void_p]),
    "kbg_comm_transport": (i32, [ctypes.c_void_p]),
    "kbg_comm_ranks": (i32, [ctypes.c_void_p, P(i32), P(i32)]),
    "kbg_allocate": (i32, [ctypes.c_void_p, P(kbg_decision), i32, P(i32)]),
    "kbg_backfill": (i32, [ctypes.c_void_p, P(kbg_decision), i32, P(i32)]),
    "kbg_reclaim": (i32, [ctypes.c_void_p, P(kbg_decision), i32, P(i32)]),
    "kbg_preempt": (i32, [ctypes.c_void_p, P(kbg_decision), i32, P(i32)]),
    "kbg_evictions_get": (i32, [ctypes.c_void_p, P(kbg_eviction), i32, P(i32)]),
    "kbg_decision_actions_get": (i32, [ctypes.c_void_p, P(i32), i32, P(i32)]),
    "kbg_session_reset": (i32, [ctypes.c_void_p]),
    "kbg_session_update": (i32, [ctypes.c_void_p, P(kbg_event), i32]),
    "kbg_session_renumbering": (i32, [ctypes.c_void_p, i32, P(i32), i32, P(i32)]),
    "kbg_select": (i32, [ctypes.c_void_p, P(i32), i32, i32, P(i32), P(i32), P(i32)]),
    "kbg_apply": (i32, [ctypes.c_void_p, i32, P(kbg_resource), i32]),
    "kbg_job_state_get": (i32, [ctypes.c_void_p, i32, P(kbg_job_state)]),
    "kbg_queue_state_get": (i32, [ctypes.c_void_p, i32, P(kbg_queue_state)]),
    "kbg_node_state_get": (i32, [ctypes.c_void_p, i32, P(kbg_node_state)]),
    "kbg_stats_get": (i32, [ctypes.c_void_p, P(kbg_stats)]),
    "kbg_session_close": (None, [ctypes.c_void_p]),
    "kbg_snapshot_encode": (i32, [P(kbg_snapshot), ctypes.c_void_p, i64, P(i64)]),
    "kbg_snapshot_decode": (i32, [ctypes.c_void_p, i64, P(ctypes.c_void_p)]),
    "kbg_snapshot_save": (i32, [P(kbg_snapshot), ctypes.c_char_p]),
    "kbg_snapshot_load": (i32, [ctypes.c_char_p, P(ctypes.c_void_p)]),
    "kbg_snapshot_blob_get": (P(kbg_snapshot), [ctypes.c_void_p]),
    "kbg_snapshot_blob_free": (None, [ctypes.c_void_p]),
}

_lib = None


class KbgError(RuntimeError):
    """A kbg_status other than KBG_OK, with kbg_last_error()."""

    def __init__(self, code, msg):
        super().__init__(f"kbgpu {STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code
        self.status = STATUS_NAMES.get(code, str(code))


def lib():
    """The loaded libkbgpu.so; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C kube-arbitrator_amd` "
                              "(the MI355X path has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.kbg_abi_version() != ABI_VERSION:
            raise ImportError("libkbgpu ABI version mismatch")
        _lib = L
    return _lib


def check(code):
    if code != KBG_OK:
        raise KbgError(code, lib().kbg_last_error().decode("utf-8", "replace"))
