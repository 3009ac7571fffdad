"""Session data model: the host-side mirror of pkg/scheduler/api.

Resource (resource_info.go:26-168), TaskInfo (job_info.go:36-107),
JobInfo (job_info.go:118-358), NodeInfo (node_info.go:26-187),
QueueInfo (queue_info.go:27-54), task statuses (types.go:20-104).
Objects carry the k8s object dicts they came from (pods, nodes) as `pod` /
`node`; those dicts use the fixture schema documented in DESIGN.md.
"""
import math
from fractions import Fraction

MIN_MILLI_CPU = 10.0
MIN_MILLI_GPU = 10.0
MIN_MEMORY = 10.0 * 1024 * 1024
GPU_RESOURCE_NAME = "nvidia.com/gpu"
GROUP_NAME_ANNOTATION_KEY = "scheduling.k8s.io/group-name"  # pkg/apis/scheduling/v1alpha1/labels.go:21


class RefPanic(RuntimeError):
    """The reference would panic at this point (e.g. Resource.Sub underflow)."""


# ---------------------------------------------------------------- status
PENDING, ALLOCATED, PIPELINED, BINDING, BOUND, RUNNING, RELEASING, SUCCEEDED, FAILED, UNKNOWN = (
    1 << i for i in range(10))
STATUS_NAMES = {PENDING: "Pending", ALLOCATED: "Allocated", PIPELINED: "Pipelined", BINDING: "Binding",
                BOUND: "Bound", RUNNING: "Running", RELEASING: "Releasing", SUCCEEDED: "Succeeded",
                FAILED: "Failed", UNKNOWN: "Unknown"}


def allocated_status(s):  # api/helpers.go:63-70
    return s in (BOUND, BINDING, RUNNING, ALLOCATED)


def get_task_status(pod):  # api/helpers.go:35-61
    phase = pod.get("phase", "Pending")
    deleting = bool(pod.get("deleting")) or pod.get("deletionTimestamp") is not None
    if phase == "Running":
        return RELEASING if deleting else RUNNING
    if phase == "Pending":
        if deleting:
            return RELEASING
        return PENDING if not pod.get("nodeName") else BOUND
    return {"Unknown": UNKNOWN, "Succeeded": SUCCEEDED, "Failed": FAILED}.get(phase, UNKNOWN)


# -------------------------------------------------------------- quantity
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}


def parse_quantity(q):
    """resource.Quantity as an exact Fraction (k8s quantity grammar)."""
    if isinstance(q, int):
        return Fraction(q)
    s = str(q)
    i = 0
    sign = 1
    if s[:1] in "+-":
        sign = -1 if s[0] == "-" else 1
        i = 1
    j = i
    while j < len(s) and (s[j].isdigit() or s[j] == "."):
        j += 1
    num = s[i:j]
    if not num or num == "." or num.count(".") > 1:
        raise ValueError(f"bad quantity {q!r}")
    val = Fraction(num)
    suf = s[j:]
    if suf in _DEC:
        val *= Fraction(10) ** _DEC[suf]
    elif suf in _BIN:
        val *= 2 ** _BIN[suf]
    elif suf[:1] in ("e", "E"):
        val *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"bad quantity suffix {q!r}")
    return sign * val


def milli_value(q):  # Quantity.MilliValue(): rounds up
    return math.ceil(parse_quantity(q) * 1000)


def value(q):  # Quantity.Value(): rounds up
    return math.ceil(parse_quantity(q))


# -------------------------------------------------------------- Resource
class Resource:
    __slots__ = ("milli_cpu", "memory", "milli_gpu", "max_task_num")

    def __init__(self, milli_cpu=0.0, memory=0.0, milli_gpu=0.0, max_task_num=0):
        self.milli_cpu = float(milli_cpu)
        self.memory = float(memory)
        self.milli_gpu = float(milli_gpu)
        self.max_task_num = int(max_task_num)

    @staticmethod
    def from_list(rl):  # NewResource (resource_info.go:58-73)
        r = Resource()
        for name, q in (rl or {}).items():
            if name == "cpu":
                r.milli_cpu += float(milli_value(q))
            elif name == "memory":
                r.memory += float(value(q))
            elif name == "pods":
                r.max_task_num += int(value(q))
            elif name == GPU_RESOURCE_NAME:
                r.milli_gpu += float(milli_value(q))
        return r

    def clone(self):
        return Resource(self.milli_cpu, self.memory, self.milli_gpu, self.max_task_num)

    def is_empty(self):
        return self.milli_cpu < MIN_MILLI_CPU and self.memory < MIN_MEMORY and self.milli_gpu < MIN_MILLI_GPU

    def add(self, rr):
        self.milli_cpu += rr.milli_cpu
        self.memory += rr.memory
        self.milli_gpu += rr.milli_gpu
        return self

    def sub(self, rr):
        if rr.less_equal(self):
            self.milli_cpu -= rr.milli_cpu
            self.memory -= rr.memory
            self.milli_gpu -= rr.milli_gpu
            return self
        raise RefPanic(f"Resource is not sufficient to do operation: <{self}> sub <{rr}>")

    def less_equal(self, rr):
        return ((self.milli_cpu < rr.milli_cpu or abs(rr.milli_cpu - self.milli_cpu) < MIN_MILLI_CPU)
                and (self.memory < rr.memory or abs(rr.memory - self.memory) < MIN_MEMORY)
                and (self.milli_gpu < rr.milli_gpu or abs(rr.milli_gpu - self.milli_gpu) < MIN_MILLI_GPU))

    def as_tuple(self):
        return (self.milli_cpu, self.memory, self.milli_gpu)

    def __eq__(self, o):
        return isinstance(o, Resource) and self.as_tuple() == o.as_tuple() and self.max_task_num == o.max_task_num

    def __repr__(self):
        return f"cpu {self.milli_cpu:.2f}, memory {self.memory:.2f}, GPU {self.milli_gpu:.2f}"


# ------------------------------------------------------------ TaskInfo
def pod_key(pod):  # api/helpers.go:27-33 (MetaNamespaceKeyFunc)
    ns = pod.get("namespace", "")
    return f"{ns}/{pod['name']}" if ns else pod["name"]


def get_job_id(pod):  # job_info.go:53-62
    gn = (pod.get("annotations") or {}).get(GROUP_NAME_ANNOTATION_KEY, "")
    if gn:
        return f"{pod.get('namespace', '')}/{gn}"
    return pod.get("controller", "")  # utils.GetController: controller ownerRef UID


class TaskInfo:
    __slots__ = ("uid", "job", "name", "namespace", "resreq", "node_name", "status", "priority", "pod")

    def __init__(self, pod):  # NewTaskInfo (job_info.go:64-89)
        req = Resource()
        for c in pod.get("containers", []):
            req.add(Resource.from_list(c.get("requests")))
        self.uid = pod["uid"]
        self.job = get_job_id(pod)
        self.name = pod["name"]
        self.namespace = pod.get("namespace", "")
        self.node_name = pod.get("nodeName", "") or ""
        self.status = get_task_status(pod)
        self.priority = pod["priority"] if pod.get("priority") is not None else 1
        self.pod = pod
        self.resreq = req

    def clone(self):
        t = TaskInfo.__new__(TaskInfo)
        for k in TaskInfo.__slots__:
            setattr(t, k, getattr(self, k))
        t.resreq = self.resreq.clone()
        return t


# ------------------------------------------------------------ NodeInfo
class NodeInfo:
    def __init__(self, node=None):  # NewNodeInfo (node_info.go:44-71)
        self.node = node
        self.name = node["name"] if node else ""
        self.releasing = Resource()
        self.used = Resource()
        if node:
            self.idle = Resource.from_list(node.get("allocatable"))
            self.allocatable = Resource.from_list(node.get("allocatable"))
            self.capability = Resource.from_list(node.get("capacity", node.get("allocatable")))
        else:
            self.idle = Resource()
            self.allocatable = Resource()
            self.capability = Resource()
        self.tasks = {}

    def clone(self):
        res = NodeInfo(self.node)
        for t in self.tasks.values():
            res.add_task(t)
        return res

    def set_node(self, node):  # node_info.go:84-99 (Releasing and Used are not reset: the reference's own quirk)
        self.name = node["name"]
        self.node = node
        self.allocatable = Resource.from_list(node.get("allocatable"))
        self.capability = Resource.from_list(node.get("capacity", node.get("allocatable")))
        self.idle = Resource.from_list(node.get("allocatable"))
        for t in self.tasks.values():
            if t.status == RELEASING:
                self.releasing.add(t.resreq)
            self.idle.sub(t.resreq)
            self.used.add(t.resreq)

    def add_task(self, task):  # node_info.go:101-129
        key = pod_key(task.pod)
        if key in self.tasks:
            return False
        ti = task.clone()
        if self.node is not None:
            if ti.status == RELEASING:
                self.releasing.add(ti.resreq)
                self.idle.sub(ti.resreq)
            elif ti.status == PIPELINED:
                self.releasing.sub(ti.resreq)
            else:
                self.idle.sub(ti.resreq)
            self.used.add(ti.resreq)
        self.tasks[key] = ti
        return True

    def remove_task(self, ti):  # node_info.go:131-157: by PodKey, the node's copy's status
        key = pod_key(ti.pod)
        task = self.tasks.get(key)
        if task is None:
            return False  # "failed to find task"
        if self.node is not None:
            if task.status == RELEASING:
                self.releasing.sub(task.resreq)
                self.idle.add(task.resreq)
            elif task.status == PIPELINED:
                self.releasing.add(task.resreq)
            else:
                self.idle.add(task.resreq)
            self.used.sub(task.resreq)
        del self.tasks[key]
        return True


# ------------------------------------------------------------- JobInfo
class JobInfo:
    def __init__(self, uid):  # NewJobInfo (job_info.go:147-160)
        self.uid = uid
        self.name = ""
        self.namespace = ""
        self.queue = ""
        self.priority = 0
        self.min_available = 0
        self.task_status_index = {}
        self.tasks = {}
        self.allocated = Resource()
        self.total_request = Resource()
        self.creation_timestamp = 0
        self.pod_group = None
        self.pdb = None

    def set_pod_group(self, pg, default_queue=""):  # job_info.go:166-186
        self.name = pg["name"]
        self.namespace = pg.get("namespace", "")
        self.min_available = int(pg.get("minMember", 0) or 0)
        if pg.get("queue"):
            self.queue = pg["queue"]
        elif default_queue:
            self.queue = default_queue
        else:
            self.queue = self.namespace
        self.creation_timestamp = int(pg.get("creationTimestamp", 0) or 0)
        self.pod_group = pg

    def set_pdb(self, pdb, default_queue=""):  # job_info.go:188-200
        self.name = pdb["name"]
        self.min_available = int(pdb.get("minAvailable", 0) or 0)
        self.namespace = pdb.get("namespace", "")
        self.queue = default_queue if default_queue else self.namespace
        self.creation_timestamp = int(pdb.get("creationTimestamp", 0) or 0)
        self.pdb = pdb

    def add_task_info(self, ti):  # job_info.go:228-237
        self.tasks[ti.uid] = ti
        self.task_status_index.setdefault(ti.status, {})[ti.uid] = ti
        self.total_request.add(ti.resreq)
        if allocated_status(ti.status):
            self.allocated.add(ti.resreq)

    def delete_task_info(self, ti):  # job_info.go:264-280
        task = self.tasks.get(ti.uid)
        if task is None:
            return False
        self.total_request.sub(task.resreq)
        if allocated_status(task.status):
            self.allocated.sub(task.resreq)
        del self.tasks[task.uid]
        idx = self.task_status_index.get(task.status)
        if idx is not None:
            idx.pop(task.uid, None)
            if not idx:
                del self.task_status_index[task.status]
        return True

    def update_task_status(self, task, status):  # job_info.go:239-252
        self.delete_task_info(task)
        task.status = status
        self.add_task_info(task)

    def clone(self):  # job_info.go:282-313
        info = JobInfo(self.uid)
        info.name, info.namespace, info.queue = self.name, self.namespace, self.queue
        info.min_available = self.min_available
        info.pdb, info.pod_group = self.pdb, self.pod_group
        info.creation_timestamp = self.creation_timestamp
        for t in self.tasks.values():
            info.add_task_info(t.clone())
        return info

    def ready_task_num(self):  # gang.go:44-55
        return sum(len(ts) for st, ts in self.task_status_index.items()
                   if allocated_status(st) or st in (SUCCEEDED, PIPELINED))


class QueueInfo:
    def __init__(self, name, weight):  # queue_info.go:35-45
        self.uid = name
        self.name = name
        self.weight = int(weight)

    def clone(self):
        return QueueInfo(self.name, self.weight)
