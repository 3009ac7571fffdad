/*
 * kbgpu.h — C ABI of the MI355X allocate path (kube-batch v0.4 semantics).
 *
 * The boundary sits at the allocate ACTION, not at the per-pair predicate:
 * the reference exposes `framework.Action{Name, Initialize, Execute(*Session),
 * UnInitialize}` (pkg/scheduler/framework/interface.go:20-32) and registers
 * `allocate` by name (pkg/scheduler/framework/plugins.go:53-58,
 * pkg/scheduler/factory.go:34-46). A per-pair `api.PredicateFn`
 * (pkg/scheduler/api/types.go:101) offload would pay one cgo call and one
 * kernel launch per (task,node), so the entry points below replace the whole
 * of allocateAction.Execute (pkg/scheduler/actions/allocate/allocate.go:41-176)
 * and report its decisions; the caller replays them through its own
 * ssn.Allocate / ssn.Pipeline (pkg/scheduler/framework/session.go:205-293) so
 * event handlers, gang dispatch and cache.Bind stay on the host.
 *
 * Conventions: plain C structs and pointers only; the library copies what it
 * needs during kbg_session_open and keeps no caller pointer after any call
 * returns (cgo-safe). One session = one thread = one HIP stream. Every
 * function returns a kbg_status; kbg_last_error() gives the message.
 * All strings (UIDs, names, label keys/values, operators, effects) travel as
 * indices into one string table; the empty string must be interned like any
 * other. String ordering is bytewise, as Go's `<` on strings.
 */
#ifndef KBGPU_H_
#define KBGPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KBG_ABI_VERSION 13

typedef enum kbg_status {
  KBG_OK = 0,
  KBG_E_INVALID = 1,     /* malformed snapshot / arguments */
  KBG_E_UNSUPPORTED = 2, /* a case the device path declines, named in
                            kbg_last_error: a statement discard of a pipeline
                            whose pod key the node holds for a pod placed this
                            cycle (or for a pod outside the session jobs when
                            the snapshot carried no node_pods), and the
                            session-update cases listed at kbg_session_update.
                            The caller runs the reference path. Never a silent
                            fallback. */
  KBG_E_REF_PANIC = 3,   /* the reference would panic here (Resource.Sub underflow
                            resource_info.go:100-110, proportion water-fill F9
                            proportion.go:119-140, nil-Node predicate
                            predicates.go:122-123). Decisions made before the
                            panic point are returned. */
  KBG_E_HIP = 4,         /* HIP runtime error (no device, launch failure, ...) */
  KBG_E_RCCL = 5,
  KBG_E_NOMEM = 6,
  KBG_E_CAPACITY = 7     /* caller's output buffer is too small */
} kbg_status;

/* api.TaskStatus bit values (pkg/scheduler/api/types.go:23-58) */
enum {
  KBG_PENDING = 1 << 0,
  KBG_ALLOCATED = 1 << 1,
  KBG_PIPELINED = 1 << 2,
  KBG_BINDING = 1 << 3,
  KBG_BOUND = 1 << 4,
  KBG_RUNNING = 1 << 5,
  KBG_RELEASING = 1 << 6,
  KBG_SUCCEEDED = 1 << 7,
  KBG_FAILED = 1 << 8,
  KBG_UNKNOWN = 1 << 9
};

/* conf.PluginOption disable flags (pkg/scheduler/conf/scheduler_conf.go:33-50) */
enum {
  KBG_DISABLE_JOB_ORDER = 1 << 0,
  KBG_DISABLE_JOB_READY = 1 << 1,
  KBG_DISABLE_TASK_ORDER = 1 << 2,
  KBG_DISABLE_PREEMPTABLE = 1 << 3,
  KBG_DISABLE_RECLAIMABLE = 1 << 4,
  KBG_DISABLE_QUEUE_ORDER = 1 << 5,
  KBG_DISABLE_PREDICATE = 1 << 6
};

enum { KBG_KIND_ALLOCATE = 0, KBG_KIND_PIPELINE = 1 };

/* api.Resource without MaxTaskNum (resource_info.go:26-33); fp64 throughout. */
typedef struct kbg_resource {
  double milli_cpu;
  double memory;
  double milli_gpu;
} kbg_resource;

/* One session node = api.NodeInfo after cache.Snapshot() (node_info.go:26-42). */
typedef struct kbg_node {
  int32_t name;            /* string id of NodeInfo.Name ("" for a nil Node) */
  int32_t has_node;        /* 0 => NodeInfo.Node == nil (node_info.go:44-56) */
  kbg_resource allocatable;
  kbg_resource idle;       /* NodeInfo.Idle */
  kbg_resource releasing;  /* NodeInfo.Releasing */
  int32_t max_task_num;    /* Allocatable.MaxTaskNum ("pods" allocatable) */
  int32_t num_tasks;       /* len(NodeInfo.Tasks) */
  int32_t unschedulable;   /* Node.Spec.Unschedulable */
  int32_t label_off, label_len; /* Node.Labels: pairs (key,value) at labels[2*i] */
  int32_t taint_off, taint_len; /* Node.Spec.Taints: taints[taint_off ..] */
  int32_t port_off, port_len;   /* NodeInfo.UsedPorts(): the container ports (hostPort > 0) of the
                                   pods on the node (node.Pods(), node_info.go:181-187 -> vendor
                                   cache/node_info.go:593-605), one entry per pod and port, so a
                                   port stays used while any pod on the node lists it (duplicates
                                   are one used port to the predicate), ports[port_off ..] */
  int32_t task_off, task_len;   /* the session-job tasks in NodeInfo.Tasks, in its (insertion) order:
                                   node_tasks[task_off ..] are indices into tasks. preempt/reclaim
                                   take victims in this order (preempt.go:199-206, reclaim.go:113-126) */
  int32_t key_off, key_len;     /* the keys of NodeInfo.Tasks (PodKey "<ns>/<name>", api/helpers.go:27-33)
                                   of EVERY pod on the node, session job or not: node_pod_keys[key_off ..],
                                   string ids; key_len == num_tasks. A placement whose pod key is already
                                   there is logged but leaves the node unchanged (AddTask's "already on
                                   node" error, node_info.go:101-106) */
} kbg_node;

/* The NodeInfo.Tasks copy behind one node_pod_keys entry, as NodeInfo.RemoveTask
 * reads it (node_info.go:131-157) when a pod key collision makes the session
 * remove it by key: a statement discard's unpipeline of a pipeline whose key
 * the node already held (statement.go:156-192), or an update that deletes a
 * session pod whose key another pod holds on its node (event_handlers.go:
 * 90-120 -> deleteTask). Optional (n_node_pods == 0): without it such a
 * removal of a pod outside the session jobs is refused (KBG_E_UNSUPPORTED). */
typedef struct kbg_node_pod {
  kbg_resource resreq; /* TaskInfo.Resreq */
  int32_t status;      /* TaskStatus of the copy: Releasing (Releasing -= req, Idle += req), Pipelined
                          (Releasing += req), anything else (Idle += req) */
  int32_t port_len;    /* how many of the node's ports[port_off ..] entries are this pod's (the entries
                          follow NodeInfo.Tasks order, as node_pod_keys does) */
} kbg_node_pod;

/* One v1.ContainerPort as HostPortInfo sees it (vendor cache/host_ports.go). */
typedef struct kbg_host_port {
  int32_t host_ip;   /* string id of HostIP ("" means 0.0.0.0) */
  int32_t protocol;  /* string id of Protocol ("" means TCP) */
  int32_t host_port; /* HostPort; <= 0 never conflicts and is never recorded */
} kbg_host_port;

typedef struct kbg_taint {
  int32_t key, value, effect; /* string ids */
} kbg_taint;

/* One api.JobInfo in ssn.Jobs order (job_info.go:118-145). */
typedef struct kbg_job {
  int32_t uid;           /* string id of JobID */
  int32_t queue;         /* index into queues (the snapshot keeps only jobs whose queue exists) */
  int32_t min_available; /* PodGroup.Spec.MinMember / PDB minAvailable */
  int32_t priority;      /* JobInfo.Priority (never set in v0.4: 0) */
  int64_t creation_ns;   /* CreationTimestamp, nanoseconds */
} kbg_job;

/* One api.QueueInfo in ssn.Queues order (queue_info.go:27-45). */
typedef struct kbg_queue {
  int32_t uid;    /* string id of QueueID */
  int32_t weight; /* Queue.Spec.Weight */
} kbg_queue;

/* One api.TaskInfo of a session job, any status (job_info.go:36-50). */
typedef struct kbg_task {
  int32_t uid;       /* string id of TaskID (pod UID) */
  int32_t job;       /* index into jobs */
  int32_t status;    /* KBG_PENDING, ... */
  int32_t priority;  /* TaskInfo.Priority (pod priority, default 1) */
  kbg_resource resreq;
  int32_t spec;      /* index into specs (the pod's predicate inputs) */
  int32_t node_name; /* string id of TaskInfo.NodeName */
  int32_t pod_key;   /* string id of PodKey(task.Pod) = "<namespace>/<name>" (the NodeInfo.Tasks key) */
  int32_t reserved;
} kbg_task;

/* Predicate-relevant part of a pod spec (predicates.go:121-201). */
typedef struct kbg_spec {
  int32_t selector_off, selector_len; /* Spec.NodeSelector pairs at selectors[2*i] */
  int32_t has_required_affinity;      /* Affinity.NodeAffinity.RequiredDuringScheduling... != nil */
  int32_t term_off, term_len;         /* its NodeSelectorTerms */
  int32_t toleration_off, toleration_len;
  int32_t has_host_ports;             /* some container port has hostPort > 0 */
  int32_t has_pod_affinity;           /* some required pod (anti)affinity term */
  int32_t port_off, port_len;         /* GetContainerPorts(pod): ports[port_off ..] */
  /* inter-pod (anti)affinity (vendor predicates.go:1155-1466): the pod's
     namespace and labels (what other pods' terms select) and its own
     RequiredDuringSchedulingIgnoredDuringExecution terms */
  int32_t ns;                         /* string id of the pod namespace */
  int32_t pod_label_off, pod_label_len; /* pod labels, pairs at pod_labels[2*i] */
  int32_t aff_off, aff_len;           /* PodAffinity terms: pod_terms[aff_off ..] */
  int32_t anti_off, anti_len;         /* PodAntiAffinity terms */
} kbg_spec;

/* v1.PodAffinityTerm */
typedef struct kbg_pod_term {
  int32_t has_selector;               /* LabelSelector != nil (nil selects nothing) */
  int32_t match_off, match_len;       /* MatchLabels pairs at selectors[2*i] */
  int32_t expr_off, expr_len;         /* MatchExpressions: reqs[expr_off ..] */
  int32_t ns_off, ns_len;             /* Namespaces: values[ns_off ..] string ids (empty: the pod's own) */
  int32_t topology_key;               /* string id */
} kbg_pod_term;

typedef struct kbg_term {
  int32_t expr_off, expr_len;   /* MatchExpressions: reqs[expr_off ..] */
  int32_t field_off, field_len; /* MatchFields: reqs[field_off ..] */
} kbg_term;

typedef struct kbg_requirement {
  int32_t key;                  /* string id */
  int32_t op;                   /* string id of the operator text ("In", "NotIn", ...) */
  int32_t value_off, value_len; /* values[value_off ..] string ids */
} kbg_requirement;

typedef struct kbg_toleration {
  int32_t key, op, value, effect; /* string ids */
} kbg_toleration;

typedef struct kbg_plugin_option {
  int32_t name;   /* string id of the plugin name (conf.PluginOption.Name) */
  uint32_t flags; /* KBG_DISABLE_*, and KBG_PLUGIN_REGISTERED (see kbg_options.plugin_registry) */
} kbg_plugin_option;

/* framework.OpenSession instantiates a tier entry only when the process has a
 * builder registered under its name (framework.go:30-35, RegisterPluginBuilder
 * plugins.go:28-33); a name without one is skipped. The caller reports its
 * registry with this flag on every entry when kbg_options.plugin_registry = 1:
 * an entry without the flag is skipped (even one of the five names this path
 * implements); an entry with it whose name is not one of priority, gang, drf,
 * predicates, proportion is a plugin this path cannot evaluate, and
 * kbg_session_open returns KBG_E_UNSUPPORTED (the caller runs the reference
 * path). With plugin_registry = 0 the five names are taken as registered and
 * every other name as unregistered. */
#define KBG_PLUGIN_REGISTERED 0x80000000u

typedef struct kbg_snapshot {
  const char* const* strings;
  int32_t n_strings;
  const kbg_node* nodes;           int32_t n_nodes;
  const kbg_job* jobs;             int32_t n_jobs;
  const kbg_queue* queues;         int32_t n_queues;
  const kbg_task* tasks;           int32_t n_tasks;
  const kbg_resource* others;      int32_t n_others;   /* Session.Others resreq, in order */
  const kbg_spec* specs;           int32_t n_specs;
  const kbg_term* terms;           int32_t n_terms;
  const kbg_requirement* reqs;     int32_t n_reqs;
  const int32_t* values;           int32_t n_values;
  const kbg_toleration* tolerations; int32_t n_tolerations;
  const int32_t* labels;           int32_t n_labels;    /* 2*n_labels ints */
  const kbg_taint* taints;         int32_t n_taints;
  const int32_t* selectors;        int32_t n_selectors; /* 2*n_selectors ints */
  const kbg_plugin_option* plugins; int32_t n_plugins;
  const int32_t* tier_sizes;       int32_t n_tiers;     /* plugins grouped by tier, in order */
  const kbg_host_port* ports;      int32_t n_ports;
  const int32_t* node_tasks;       int32_t n_node_tasks;
  const kbg_pod_term* pod_terms;   int32_t n_pod_terms;
  const int32_t* pod_labels;       int32_t n_pod_labels;  /* 2*n_pod_labels ints */
  const int32_t* node_pod_keys;    int32_t n_node_pod_keys;
  const kbg_node_pod* node_pods;   int32_t n_node_pods;   /* 0, or one per node_pod_keys entry */
} kbg_snapshot;

typedef struct kbg_options {
  int32_t device;       /* HIP device ordinal; -1 = current */
  int32_t heap_rule;    /* container/heap down() tie rule: 0 = Go 1.11 (default), 1 = Go >= 1.13 */
  int32_t batch_tasks;  /* speculative batch size K (0 = default) */
  int32_t candidates;   /* first-M feasible nodes kept per task (0 = default) */
  int32_t full_scan;    /* 1 = every task evaluation scans the full node table */
  int32_t shards;       /* node-axis shards (0/1 = unsharded). Without a communicator every
                           shard lives in this process (same layout and exchange buffer as the
                           multi-GPU path, for single-device parity runs); with one (see
                           kbg_session_open_sharded) it must equal the communicator size. */
  int32_t plugin_registry; /* 1 = kbg_plugin_option.flags carry KBG_PLUGIN_REGISTERED (framework.go:30-35) */
  int32_t reserved[5];
} kbg_options;

/* One placement decision, in reference order. */
typedef struct kbg_decision {
  int32_t task;          /* index into snapshot tasks */
  int32_t node;          /* index into snapshot nodes */
  int32_t kind;          /* KBG_KIND_ALLOCATE / KBG_KIND_PIPELINE */
  int32_t dispatched_at; /* index of the decision whose ssn.Allocate dispatched
                            (bound) this task (session.go:283-290), or -1 */
} kbg_decision;

typedef struct kbg_job_state {
  int32_t ready_num;     /* gang readyTaskNum (gang.go:44-55) */
  int32_t ready;         /* gang jobReady predicate: ready_num >= MinAvailable (gang.go:72-78),
                            reported whether or not the gang plugin is configured */
  double drf_share;      /* drf attr.share (drf.go:152-166); 0 if drf is off */
  kbg_resource drf_allocated;
  /* JobInfo.NodesFitDelta of the job's last evaluated task (allocate.go:116-144),
     summarised as JobInfo.FitError counts it (job_info.go:329-358); filled after
     kbg_allocate for jobs that are not ready (what gang.go:169-190 reports). */
  int32_t fit_valid;     /* 1 when the counts below were computed */
  int32_t fit_nodes;     /* len(NodesFitDelta) */
  int32_t fit_cpu, fit_memory, fit_gpu; /* entries with a negative cpu / memory / GPU delta */
  int32_t reserved[3];
} kbg_job_state;

typedef struct kbg_queue_state {
  double share;          /* proportion attr.share (proportion.go:225-237) */
  kbg_resource deserved, allocated, request;
  int32_t overused;
  int32_t has_attr;      /* 0 if the queue has no job in the session */
} kbg_queue_state;

typedef struct kbg_node_state {
  kbg_resource idle, releasing;
  int32_t num_tasks;
} kbg_node_state;

typedef struct kbg_stats {
  int64_t evaluations;     /* task evaluations scanned on the device */
  int64_t node_visits;     /* (task,node) pairs evaluated on the device */
  int64_t batches;
  int64_t mispredictions;  /* batches cut by an unpredicted failure */
  int64_t truncations;     /* rescans of a batch remainder after an exhausted candidate list */
  int64_t scan_launches;
  double scan_kernel_ms;   /* scan-kernel time: the fused kernel's HIP-event time of every 4th launch x
                              launches / timed launches (events lengthen a round trip by ≈ 7 µs) */
  double select_kernel_ms; /* summed HIP-event time of the candidate-select kernel */
  double allocate_ms;      /* wall time of the last kbg_allocate */
  double open_ms;          /* wall time of kbg_session_open */
  double engine_ms;        /* host: queue/job/task ordering (prediction + replay) */
  double resolve_ms;       /* host: in-order commit of the device candidates */
  double device_ms;        /* host wall time spent in scan round trips (H2D, kernels, D2H) */
  double delta_ms;         /* host wall time spent writing touched node rows back to HBM */
  int64_t replayed;        /* engine steps replayed from a batch checkpoint after a cut (sharded rank 0; the
                              single-rank allocate restarts from the committed outcomes' engine: 0) */
  int32_t n_classes;       /* static predicate classes on the device */
  int32_t shards;          /* node-axis shards of the session (1 = unsharded) */
  int32_t shard_index;     /* the shard this process holds; -1 = every shard is local */
  int32_t int_scan;        /* 1 = the scan compares exact-integer thresholds (every value an
                              integer <= 2^51); 0 = the reference's LessEqual expression */
  double exchange_ms;      /* sharded sessions: time in the per-batch RCCL collectives (the bitmap
                              all-gather, or the owner-resolve broadcast / min-reduces) */
  double backfill_ms;      /* wall time of the last kbg_backfill */
  double reclaim_ms;       /* wall time of the last kbg_reclaim */
  double preempt_ms;       /* wall time of the last kbg_preempt */
  int64_t victim_scans;    /* victim-scan kernel launches (one per preemptor / reclaimer tried) */
  double victim_kernel_ms; /* victim-scan kernel time: HIP-event time of every 16th launch x launches / timed */
  int64_t victim_tries;    /* reclaimer / preemptor tasks tried (a scan, or the kept stop maps) */
  int64_t victim_host_evals; /* nodes re-evaluated on the host after a change since the last scan */
  int64_t task_evaluations;  /* node-loop runs of the reference (allocate.go:105-171: every task popped,
                                placed or not) in the last kbg_allocate: SURVEY §8(d)'s unit */
  int64_t resolve_steps;     /* candidate-list entries the in-order commit examined */
  int64_t resolve_rechecks;  /* of those, nodes touched since their scan and re-checked on the host mirror */
  int64_t overlapped;        /* batches whose scan ran while the host resolved the previous batch */
  double update_ms;          /* wall time of the last kbg_session_update */
  int64_t update_rebuilds;   /* kbg_session_update calls that rebuilt the static masks / device tables */
  int64_t owner_rounds;      /* owner-resolve (sharded allocate): exchange rounds over all batches */
  int64_t reused_batches;    /* batches resolved against an earlier scan's candidate lists after a cut
                                (grouped mode: no device round trip) */
  int64_t refresh_scans;     /* contended allocate: scans of every live shape launched beside the in-order
                                commit once it had re-checked enough nodes touched since its lists' scan (ABI 11) */
} kbg_stats;

typedef struct kbg_session kbg_session;

/* Node-axis sharding across GPUs (the reference has no multi-GPU
 * counterpart: allocate.go:119-162 is one node loop). A communicator is the
 * clique of the shards, one rank per process. Shard r holds the node-table
 * rows of 64-node words [r*Wl, (r+1)*Wl), Wl = ceil(ceil(N/64)/R), so rank
 * order is node order and first-fit is the lowest rank with a fitting node.
 * kbg_allocate runs the scan service (up to 8 ranks): rank 0 runs the
 * single-GPU pipeline, each of its scans is a launch message (ncclBroadcast)
 * every rank answers over its own words, the ranks' candidate masks are joined
 * by one sum-reduce, and the other ranks replay rank 0's commits.
 * KBG_OWNER_RESOLVE=1 selects the round-4 owner-resolve protocol instead
 * (up to 32 ranks). The other actions all-gather the per-rank bitmaps /
 * all-reduce the victim-scan words and resolve on every rank. Every rank
 * returns the identical decision log. All ranks must call
 * kbg_session_open_sharded and the actions with the same snapshot and
 * options, in lockstep.
 *
 * Two transports carry the same collectives in the same order:
 *  - kbg_comm_init: an RCCL clique, one rank per GPU, created collectively
 *    from one unique id that the caller distributes (rank 0 calls
 *    kbg_comm_unique_id; any side channel carries the bytes); the collectives
 *    run on the session's stream over xGMI.
 *  - kbg_comm_init_host (ABI 13): the ranks are processes of one host that
 *    name the same segment (`name`: letters, digits, '.', '_', '-'; fresh for
 *    each clique, e.g. rank 0's pid and a random suffix) and may share one
 *    device; every collective is a device -> host copy, an exchange through
 *    POSIX shared memory and a host -> device copy. It runs the multi-rank
 *    protocols across real processes where RCCL cannot (RCCL refuses two
 *    ranks on one GPU). Blocks until all n_ranks ranks joined.
 * A rank that fails inside a protocol aborts the communicator; a rank waiting
 * on a collective polls the transport's error state, the peers' liveness
 * (host: a peer process that exited or destroyed its communicator) and
 * KBG_COMM_TIMEOUT_MS (default 300000), and then returns KBG_E_RCCL: a failing
 * rank cannot hang its peers. */
#define KBG_COMM_ID_BYTES 128
typedef struct kbg_comm kbg_comm;
kbg_status kbg_comm_unique_id(uint8_t out[KBG_COMM_ID_BYTES]);
kbg_status kbg_comm_init(const uint8_t id[KBG_COMM_ID_BYTES], int32_t n_ranks, int32_t rank, int32_t device,
                         kbg_comm** out);
kbg_status kbg_comm_init_host(const char* name, int32_t n_ranks, int32_t rank, int32_t device, kbg_comm** out);
void kbg_comm_destroy(kbg_comm* c);
/* The transport's own view of the clique (RCCL: ncclCommCount,
 * ncclCommUserRank; host: the ranks that joined the segment): how many ranks
 * it spans and this process's rank (ABI 11). A bench line reports it so a
 * multi-GPU figure names the ranks that actually took part. */
kbg_status kbg_comm_ranks(const kbg_comm* c, int32_t* n_ranks, int32_t* rank);
enum { KBG_COMM_RCCL = 0, KBG_COMM_HOST = 1 };
/* KBG_COMM_RCCL or KBG_COMM_HOST (ABI 13); -1 for a null communicator. */
int32_t kbg_comm_transport(const kbg_comm* c);

/* ABI version and the last error message of this thread. */
int32_t kbg_abi_version(void);
const char* kbg_last_error(void);
/* Number of visible HIP devices (0 when none); never fails. */
int32_t kbg_device_count(void);

/* framework.OpenSession (framework.go:26-46) for the allocate path: copies the
 * snapshot, runs the plugins' OnSessionOpen (drf.go:55-78, proportion.go:54-144,
 * gang.go:80-166, priority.go:36-77, predicates.go:112-202) on the host, uploads
 * the node table to HBM and builds the static predicate masks on the device. */
kbg_status kbg_session_open(const kbg_snapshot* snap, const kbg_options* opts, kbg_session** out);

/* kbg_session_open for rank `comm` of a node-axis sharded session: this
 * process holds shard kbg_comm rank of opts->shards (= the communicator size);
 * the session runs on the communicator's device. The communicator must
 * outlive the session. */
kbg_status kbg_session_open_sharded(const kbg_snapshot* snap, const kbg_options* opts, kbg_comm* comm,
                                    kbg_session** out);

/* allocateAction.Execute (allocate.go:41-176). Writes at most `cap` decisions.
 * Can be called once per opened or reset session. */
kbg_status kbg_allocate(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out);

/* backfillAction.Execute (backfill.go:40-71), run after kbg_allocate on the
 * same cycle (the reference's default conf runs "allocate, backfill",
 * util.go:30-40) or alone: every Pending task requesting nothing (BestEffort)
 * of every job, in ssn.Jobs and status-index order, goes to the first node
 * whose PredicateFn passes (static predicate + pod cap, no resource fit)
 * through ssn.Allocate — so it counts toward gang readiness and may dispatch
 * earlier Allocate decisions of its job. Writes the cycle's whole decision
 * log (allocate's decisions first, dispatched_at updated) to `out`. */
kbg_status kbg_backfill(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out);

/* reclaimAction.Execute (reclaim.go:41-188) and preemptAction.Execute
 * (preempt.go:43-253) on the same cycle, in the conf's action order (the
 * reference's full conf is "reclaim, allocate, backfill, preempt"). Every
 * node a reclaimer / preemptor is tried on is evaluated on the device in one
 * victim-scan launch: PredicateFn, the filtered Running tasks of the node in
 * NodeInfo.Tasks order, the victim fns of the deciding tier
 * (session_plugins.go:59-140: gang, drf / gang, proportion) and
 * validateVictims; the host then evicts on the first such node exactly as the
 * reference does and pipelines the task. Statements (preempt) commit or
 * discard as statement.go does, including the node-side quirk of unevict.
 * Both write the cycle's decision log (pipelines carry the action); the
 * evictions are read with kbg_evictions_get. Pod (anti)affinity and host
 * ports are re-derived per eviction / pipeline (kbg_affinity.cpp, the port
 * atoms); nodes with up to 1024 Running session tasks are scanned on the
 * device in 64-wide candidate chunks, larger ones on the host when a stop
 * search reaches them (same victims, same order). */
kbg_status kbg_reclaim(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out);
kbg_status kbg_preempt(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out);

/* One committed eviction (cache.Evict), in commit order. */
typedef struct kbg_eviction {
  int32_t task;   /* the evicted task (index into tasks) */
  int32_t by;     /* the reclaimer / preemptor task */
  int32_t action; /* KBG_ACTION_RECLAIM or KBG_ACTION_PREEMPT */
  int32_t reserved;
} kbg_eviction;
enum { KBG_ACTION_ALLOCATE = 0, KBG_ACTION_BACKFILL = 1, KBG_ACTION_RECLAIM = 2, KBG_ACTION_PREEMPT = 3 };
/* out == NULL with cap == 0 only reports the count in *n_out. */
kbg_status kbg_evictions_get(kbg_session* s, kbg_eviction* out, int32_t cap, int32_t* n_out);
/* The action that produced decision i of the cycle's log (KBG_ACTION_*). */
kbg_status kbg_decision_actions_get(kbg_session* s, int32_t* out, int32_t cap, int32_t* n_out);

/* Resident sessions: cache events between scheduling cycles
 * (pkg/scheduler/cache/event_handlers.go) applied to an opened session as
 * deltas, instead of re-opening it from the next cache.Snapshot()
 * (cache.go:549-597). The session afterwards is exactly the session
 * kbg_session_open would build from the snapshot of the updated cache (same
 * decisions, tested): a pod update is the cache's delete + add (the task moves
 * to the end of its job's and its node's insertion order), a pod on a node is
 * NodeInfo.AddTask / RemoveTask by PodKey (node_info.go:101-157, including the
 * "already on node" and "not found" errors and updateTask's early return on
 * the latter), a node update is SetNode's new Allocatable (a snapshot clone
 * recomputes Idle from it). The host mirror, plugin state, pending lists and
 * the changed node rows in HBM are refreshed; the static predicate and the
 * device tables are rebuilt only when an event needs a class the session has
 * not compiled, flips the ghost-pod rule or changes schedulability. */
enum {
  KBG_EV_POD_UPDATE = 1, /* cache.UpdatePod: `task` gets `status` and NodeName = node `node` (-1: none) */
  KBG_EV_POD_DELETE = 2, /* cache.DeletePod: `task` leaves its job and its node */
  KBG_EV_POD_ADD = 3,    /* cache.AddPod: a new pod of session job `job` (index = the session's task count) */
  KBG_EV_NODE_UPDATE = 4, /* cache.UpdateNode -> NodeInfo.SetNode: node `node` gets `resource` as Allocatable,
                             `max_task_num` pods and `unschedulable` (labels and taints unchanged) */
  KBG_EV_NODE_SET = 5,    /* cache.AddNode / UpdateNode -> NodeInfo.SetNode with the whole Node (event_handlers.go
                             232-259, node_info.go:84-99): node `node` gets `node_spec`'s name, labels and taints,
                             `resource`, `max_task_num` and `unschedulable` — also a node the cache only knew from
                             a pod (NewNodeInfo(nil), Name ""), which then takes the name its pods' NodeName held */
  /* Structural events (ABI 13): the session's sets of nodes, jobs and queues
   * change. Indices in a batch are those before the batch (new ones take the
   * next index of their kind, in event order); after the batch every kind is
   * renumbered — what left is dropped, the rest keeps its order, new ones
   * last — and kbg_session_renumbering gives the old -> new maps. */
  KBG_EV_NODE_ADD = 6,     /* cache.AddNode of a node new to the cache (event_handlers.go:232-240, NewNodeInfo):
                              `node_spec`, `resource`, `max_task_num`, `unschedulable`; it joins ssn.Nodes last */
  KBG_EV_NODE_DELETE = 7,  /* cache.DeleteNode (event_handlers.go:262-268): node `node` leaves sc.Nodes with the
                              pods on it; their tasks stay in their jobs, on no node (NodeName unchanged) */
  KBG_EV_JOB_ADD = 8,      /* cache.AddPodGroup of a new job (event_handlers.go:344-358, setPodGroup): JobID
                              `name`, queue index `queue`, `min_available`, `creation_ns`, `priority`; it joins
                              ssn.Jobs last, its pods follow as KBG_EV_POD_ADD */
  KBG_EV_JOB_DELETE = 9,   /* cache.DeletePodGroup (event_handlers.go:361-381, UnsetPodGroup): job `job` leaves
                              ssn.Jobs; its pods stay on their nodes as pods outside the session jobs and its
                              Running tasks join Session.Others (cache.go:570-582) */
  KBG_EV_QUEUE_ADD = 10,   /* cache.AddQueue (event_handlers.go:635-640): queue `name` with `weight` joins ssn.Queues
                              last */
  KBG_EV_QUEUE_DELETE = 11 /* cache.DeleteQueue (event_handlers.go:650-654): queue `queue` leaves ssn.Queues, and
                              every job of it leaves ssn.Jobs (cache.go:584-588; not into Others) */
};
/* The Node of a KBG_EV_NODE_SET event (strings are copied). */
typedef struct kbg_node_spec {
  const char* name;          /* Node.Name */
  const char* const* labels; /* Node.Labels: 2 * n_labels strings, key then value */
  int32_t n_labels;
  int32_t n_taints;
  const char* const* taints; /* Node.Spec.Taints: 3 * n_taints strings, key, value, effect */
} kbg_node_spec;
typedef struct kbg_event {
  int32_t kind;
  int32_t task;          /* POD_UPDATE / POD_DELETE */
  int32_t status;        /* POD_UPDATE / POD_ADD: TaskStatus (api/helpers.go:35-61) */
  int32_t node;          /* POD_UPDATE / POD_ADD: node index of NodeName or -1; NODE_UPDATE: the node */
  int32_t job;           /* POD_ADD */
  int32_t spec;          /* POD_ADD: index into the session's specs, -1 = none */
  int32_t priority;      /* POD_ADD: TaskInfo.Priority */
  int32_t max_task_num;  /* NODE_UPDATE */
  kbg_resource resource; /* POD_ADD: Resreq; NODE_UPDATE: Allocatable */
  int32_t unschedulable; /* NODE_UPDATE */
  int32_t reserved;
  const char* uid;       /* POD_ADD: pod UID */
  const char* pod_key;   /* POD_ADD: "<namespace>/<name>" */
  const kbg_node_spec* node_spec; /* NODE_SET */
  const char* node_name; /* POD_UPDATE / POD_ADD (ABI 13, optional): the pod's NodeName when `node` is a node
                            the cache knows only from pods (Node nil, Name ""); without it the session takes the
                            NodeName that node's session pods carry, and refuses one holding none */
  const char* name;      /* JOB_ADD: JobID "<namespace>/<podgroup>"; QUEUE_ADD: the queue's name */
  int64_t creation_ns;   /* JOB_ADD: CreationTimestamp */
  int32_t queue;         /* JOB_ADD: its queue; QUEUE_DELETE: the queue */
  int32_t min_available; /* JOB_ADD: PodGroup.Spec.MinMember */
  int32_t weight;        /* QUEUE_ADD: Queue.Spec.Weight */
  int32_t reserved2;
} kbg_event;
/* Applies events[0..n) in order; the cycle state is reset as by
 * kbg_session_reset (node table, class masks, plugin state back to the
 * updated snapshot, whatever actions ran since the last open / reset / update).
 * KBG_E_UNSUPPORTED and KBG_E_INVALID found before the first event is applied
 * leave the session unchanged: an event naming a deleted task or an index out
 * of range, a removed pod whose key is held on its node by a pod outside the
 * session jobs when the snapshot carried no node_pods (kbg_node_pod: with
 * them that pod leaves the node as RemoveTask takes it), a KBG_EV_NODE_UPDATE
 * of a node the cache only knows from a pod (send KBG_EV_NODE_SET: the Node's
 * name, labels and taints), a KBG_EV_NODE_SET of such a node holding a pod
 * outside the session jobs without node_pods. KBG_E_REF_PANIC (the cache itself would
 * panic: a Resource.Sub underflow in AddTask / RemoveTask / SetNode) is found
 * while the events are applied: the session is then unusable and every later
 * call on it but kbg_session_close returns KBG_E_INVALID (re-open it). */
kbg_status kbg_session_update(kbg_session* s, const kbg_event* events, int32_t n);
/* After an update with structural events: the map old index -> new index
 * (-1: it left the session) of tasks, nodes, jobs or queues (kind
 * KBG_RENUM_*), over the indices valid before the update plus the ones its
 * events created. *n_out = the map's length (0: the last update renumbered
 * nothing — every index kept). A structural update rebuilds the session from
 * its own updated snapshot (the cost of an open, without the caller's
 * snapshot); pods that predate their PodGroup or queue (already on a node
 * as pods outside the session jobs) are refused (KBG_E_UNSUPPORTED). */
enum { KBG_RENUM_TASKS = 0, KBG_RENUM_NODES = 1, KBG_RENUM_JOBS = 2, KBG_RENUM_QUEUES = 3 };
kbg_status kbg_session_renumbering(kbg_session* s, int32_t kind, int32_t* out, int32_t cap, int32_t* n_out);

/* Restores the state captured at kbg_session_open (device-side copy); used to
 * re-run a cycle on the same snapshot without re-uploading it. */
kbg_status kbg_session_reset(kbg_session* s);

/* Low-level node-loop offload (allocate.go:105-171 for ONE job pop): evaluates
 * tasks[0..n) in order against the current device table with first-fit, stops
 * after the first success when stop_at_first_success != 0, and commits every
 * success to the device table (NodeInfo.AddTask, node_info.go:101-129).
 * out_node[i] = -1 when task i fits nowhere. Returns the number evaluated. */
kbg_status kbg_select(kbg_session* s, const int32_t* tasks, int32_t n, int32_t stop_at_first_success,
                      int32_t* out_node, int32_t* out_kind, int32_t* n_evaluated);

/* Applies one placement to the device table as NodeInfo.AddTask does. */
kbg_status kbg_apply(kbg_session* s, int32_t node, const kbg_resource* req, int32_t kind);

kbg_status kbg_job_state_get(kbg_session* s, int32_t job, kbg_job_state* out);
kbg_status kbg_queue_state_get(kbg_session* s, int32_t queue, kbg_queue_state* out);
kbg_status kbg_node_state_get(kbg_session* s, int32_t node, kbg_node_state* out);
kbg_status kbg_stats_get(kbg_session* s, kbg_stats* out);

void kbg_session_close(kbg_session* s);

/* Snapshot wire format: the flat kbg_snapshot as one
 * little-endian byte string — the header "KBGS", format version, layout
 * word (a hash of every snapshot struct's size: blobs survive ABI bumps that
 * leave those structs unchanged), the 22 counts of kbg_snapshot in
 * declaration order, then every
 * string as (uint32 length, bytes) and every array as its raw struct bytes in
 * declaration order. A cache adapter builds it once per scheduling cycle (or a
 * recorder keeps it for replay); decoding rebuilds the arrays in library-owned
 * memory, validates them as kbg_session_open does, and the snapshot it hands
 * back opens sessions unchanged. Counts are checked against the input length
 * before anything is allocated, so a corrupt blob is KBG_E_INVALID.
 * kbg_snapshot_encode with out == NULL / cap == 0 stores the size in *n_out. */
typedef struct kbg_snapshot_blob kbg_snapshot_blob;
#define KBG_SNAPSHOT_FORMAT 3
kbg_status kbg_snapshot_encode(const kbg_snapshot* snap, uint8_t* out, int64_t cap, int64_t* n_out);
kbg_status kbg_snapshot_decode(const uint8_t* data, int64_t n, kbg_snapshot_blob** out);
kbg_status kbg_snapshot_save(const kbg_snapshot* snap, const char* path);
kbg_status kbg_snapshot_load(const char* path, kbg_snapshot_blob** out);
const kbg_snapshot* kbg_snapshot_blob_get(const kbg_snapshot_blob* b);
void kbg_snapshot_blob_free(kbg_snapshot_blob* b);

#ifdef __cplusplus
}
#endif

#endif /* KBGPU_H_ */
