// Host-side session state of the MI355X allocate path.
#pragma once
#include <stdint.h>

#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/kbgpu.h"
#include "kbg_device.hpp"

namespace kbg {

struct Res {
  double c = 0, m = 0, g = 0;
};

// string-keyed maps looked up by a caller's C string without building a std::string
struct StrHash {
  using is_transparent = void;
  size_t operator()(std::string_view v) const noexcept { return std::hash<std::string_view>{}(v); }
};

// String content -> canonical id, an open-addressing table of ids into the
// session's string vector: an entry is an id and its hash, so interning a new
// pod key or UID allocates nothing beyond the string itself (a node-based
// map allocated a node and a second copy of the key per entry).
struct StrIndex {
  std::vector<int32_t> ids;  // -1: empty
  std::vector<uint64_t> hs;
  size_t n = 0;
  static uint64_t hash(std::string_view v) { return std::hash<std::string_view>{}(v); }
  void clear() {
    ids.clear();
    hs.clear();
    n = 0;
  }
  void reserve(size_t want) {
    size_t cap = 64;
    while (cap < 2 * want) cap <<= 1;
    if (cap <= ids.size()) return;
    std::vector<int32_t> oi(cap, -1);
    std::vector<uint64_t> oh(cap, 0);
    oi.swap(ids);
    oh.swap(hs);
    for (size_t i = 0; i < oi.size(); ++i)
      if (oi[i] >= 0) {
        size_t k = oh[i] & (cap - 1);
        while (ids[k] >= 0) k = (k + 1) & (cap - 1);
        ids[k] = oi[i];
        hs[k] = oh[i];
      }
  }
  // the slot a content of hash h is looked up from (a prefetch ahead of insert_h)
  void prefetch(uint64_t h) const {
    if (ids.empty()) return;
    const size_t k = h & (ids.size() - 1);
    __builtin_prefetch(&ids[k]);
    __builtin_prefetch(&hs[k]);
  }
  int32_t find(const std::vector<std::string>& strs, std::string_view v) const { return find_h(strs, v, hash(v)); }
  int32_t find_h(const std::vector<std::string>& strs, std::string_view v, uint64_t h) const {
    if (ids.empty()) return -1;
    const size_t m = ids.size() - 1;
    for (size_t k = h & m;; k = (k + 1) & m) {
      const int32_t id = ids[k];
      if (id < 0) return -1;
      if (hs[k] == h && strs[id] == v) return id;
    }
  }
  // strs[id]'s canonical id: the first id holding the same content (id itself if new)
  int32_t insert(const std::vector<std::string>& strs, int32_t id) { return insert_h(strs, id, hash(strs[id])); }
  // the same with the content's hash already computed (h = hash(strs[id]))
  int32_t insert_h(const std::vector<std::string>& strs, int32_t id, uint64_t h) {
    if (2 * (n + 1) > ids.size()) reserve(n + 1);
    const std::string_view v = strs[id];
    const size_t m = ids.size() - 1;
    size_t k = h & m;
    for (; ids[k] >= 0; k = (k + 1) & m)
      if (hs[k] == h && strs[ids[k]] == v) return ids[k];
    ids[k] = id;
    hs[k] = h;
    ++n;
    return id;
  }
};

// resource_info.go:142-146
inline bool res_le(const Res& r, const Res& a) {
  return (r.c < a.c || __builtin_fabs(a.c - r.c) < kMinMilliCPU) &&
         (r.m < a.m || __builtin_fabs(a.m - r.m) < kMinMemory) &&
         (r.g < a.g || __builtin_fabs(a.g - r.g) < kMinMilliGPU);
}
inline void res_add(Res& r, const Res& b) {
  r.c += b.c;
  r.m += b.m;
  r.g += b.g;
}
// Resource.Sub: false when the reference would panic (resource_info.go:100-110)
inline bool res_sub(Res& r, const Res& b) {
  if (!res_le(b, r)) return false;
  r.c -= b.c;
  r.m -= b.m;
  r.g -= b.g;
  return true;
}
// resource_info.go:75-77
inline bool res_empty(const Res& r) { return r.c < kMinMilliCPU && r.m < kMinMemory && r.g < kMinMilliGPU; }

// (class, request) shape of a pending task: identical rows of a scan
struct ShapeKey {
  int32_t cls;
  double c, m, g;
  bool operator==(const ShapeKey& o) const {
    return cls == o.cls && std::memcmp(&c, &o.c, 8) == 0 && std::memcmp(&m, &o.m, 8) == 0 && std::memcmp(&g, &o.g, 8) == 0;
  }
};
struct ShapeHash {
  size_t operator()(const ShapeKey& k) const {
    uint64_t h = (uint64_t)k.cls * 0x9E3779B97F4A7C15ull;
    uint64_t v;
    std::memcpy(&v, &k.c, 8);
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    std::memcpy(&v, &k.m, 8);
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    std::memcpy(&v, &k.g, 8);
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    return (size_t)h;
  }
};

struct StaticHost {
  int32_t n_classes = 0;
  int32_t label_words = 1, taint_words = 1, n_numcols = 0;
  std::vector<uint64_t> label_bits, taint_bits, mask_pool, tol_pool;
  std::vector<int64_t> num_vals;
  std::vector<uint8_t> num_ok, node_flags;
  std::vector<int32_t> name_id;
  std::vector<ReqProg> reqs;
  std::vector<TermProg> terms;
  std::vector<ClassProg> classes;
};

enum JobOrderPlugin : int32_t { JO_PRIORITY = 1, JO_GANG = 2, JO_DRF = 3 };

// Session.JobOrderFn flattened into one 128-bit order-preserving integer
// (exactly equivalent for the configured tier order). One field per
// job-order plugin in tier order — priority: dense rank of -Priority (32
// bits); gang: ready ? 1 : 0 (1 bit); drf: the share's IEEE bits (63 bits,
// shares are >= +0 so the sign bit is always clear and the bits order like
// the values) — fields after gang zeroed for a non-ready job (gang.go:148-160
// decides non-ready pairs by creation/UID without consulting later plugins),
// then the fallback (CreationTimestamp, UID) of session_plugins.go:212-220 as
// one dense rank in the low 32 bits. 32 + 1 + 63 + 32 = 128: every chain fits.
typedef unsigned __int128 JobKey;
constexpr JobKey kJobKeySentinel = ~(JobKey)0;  // above every real key (frank < 2^32 - 1)
inline uint32_t job_key_frank(JobKey k) { return (uint32_t)(uint64_t)k; }

// Mutable state of the ordering engine (queue/job/task priority queues and
// the plugin state they read). Flat arrays so a batch checkpoint is a copy.
struct Engine {
  std::vector<int32_t> qheap;   // queue heap items (queue index), util.PriorityQueue; qheap[qlen] = sentinel
  int32_t qlen = 0;
  std::vector<JobKey> jheap;    // per-queue job heaps (4-ary, inline keys), flat at joff[q]; [jlen ..] = sentinels
  std::vector<int32_t> jlen;    // live length of each per-queue heap
  std::vector<int32_t> cursor;  // per job: next position in its sorted pending list
  int32_t cur_q = -1, cur_j = -1;
  bool in_job = false;
  std::vector<Res> jalloc;      // drf attr.allocated
  std::vector<double> jshare;   // drf attr.share
  std::vector<int32_t> jready;  // gang readyTaskNum
  std::vector<Res> qalloc;      // proportion attr.allocated
  std::vector<double> qshare;   // proportion attr.share
  std::vector<int32_t> qorder;  // queues sorted by QueueOrderFn
  std::vector<int32_t> qrank;   // position of each queue in qorder; qrank[n_queues] = INT32_MAX (sentinel id)
  uint64_t qrank_pk = 0;        // the same 4 bits per queue id when n_queues <= 15 (the sentinel's: 15), so a
                                // queue-heap compare reads its ranks from a register, not memory
};

// ---- inter-pod (anti)affinity (kbg_affinity.cpp)
struct AffSelReq { int32_t key; int32_t op; std::vector<int32_t> vals; };  // op: 0 In/=, 1 NotIn, 2 Exists, 3 DoesNotExist
struct AffSel { bool err = false, nothing = false, everything = false; std::vector<AffSelReq> reqs; };
struct AffTerm {
  AffSel sel;
  std::vector<int32_t> ns;  // canonical ids; empty = the owner's namespace
  int32_t key = -1;         // canonical id of the topology key
  bool key_empty = false;
};
struct AffSpec {
  int32_t ns = -1;
  std::vector<std::pair<int32_t, int32_t>> labels;  // sorted by key (labels.Set)
  std::vector<AffTerm> aff, anti;
  bool aff_err = false, anti_err = false;  // a term's selector fails to build
};
// Node signatures over a list of topology keys (the values of those keys;
// -1 where a key is missing), shared by every class with the same key list.
struct AffSigTable {
  std::vector<int32_t> keys;
  std::vector<int32_t> sig;                  // per node
  std::vector<std::vector<int32_t>> nodes;   // per signature
};
struct AffClass {  // per static class
  bool hasB = false, b_err = false, b_empty_key = false, b_self = false;
  int32_t b_tab = -1;   // signatures over the affinity terms' keys
  bool hasC = false, c_err = false;
  int32_t c_tab = -1;   // over the anti terms' keys before the first empty one
};
struct AffState {  // counts over the AllocatedStatus pods
  int32_t poison = 0;     // pods whose anti term fails to build its selector
  int32_t allocated = 0;  // all of them (the podLister is not empty)
  std::vector<int32_t> nB;
  std::vector<std::vector<std::pair<int32_t, int32_t>>> cntB, cntC;  // per class: (signature, count), sparse
  std::vector<std::vector<std::pair<int64_t, int32_t>>> cntA;  // per class: (pair, count), few entries
};
struct AffinityModel {
  std::vector<AffSpec> specs;                                  // per kbg_spec
  std::vector<AffClass> cls;                                   // per class
  std::vector<AffSigTable> sigtabs;
  std::vector<std::vector<std::vector<int32_t>>> anti_match;   // [spec][anti term] -> classes it selects
  std::vector<std::vector<int32_t>> matchB, matchC;            // [spec] -> classes whose terms select it
  std::vector<char> spec_poison;
  std::vector<char> spec_effect;                               // [spec]: its allocation changes some count
  std::vector<int32_t> c_err_classes;
  std::vector<std::vector<std::pair<int32_t, int32_t>>> node_labels;
  std::unordered_map<int64_t, std::vector<int32_t>> pair_nodes;  // (topology key, value) -> nodes
  std::vector<std::vector<int32_t>> class_shapes;
  std::vector<uint64_t> panic_words;  // nil-Node nodes (kept reachable in every mask)
  uint64_t prof_cycles = 0, prof_calls = 0, prof_recomputes = 0;  // KBG_PROFILE_AFF
  AffState st0, st;  // at open / now
};

// What a node's stop status depends on besides the session state: the
// scan's mode, the preemptor's job, pod-spec class, queue, request and (drf)
// its job's share with it placed.
struct VictimKey {
  int32_t mode = -1, job = -1, cls = -1, queue = -1;
  double req[3] = {0, 0, 0};
  double ls = 0;
  bool operator==(const VictimKey& o) const {
    return mode == o.mode && job == o.job && cls == o.cls && queue == o.queue && req[0] == o.req[0] &&
           req[1] == o.req[1] && req[2] == o.req[2] && ls == o.ls;
  }
};

// One in-flight device round trip of the batch driver: pinned host staging
// for the evaluation rows going up and the candidate lists coming down, the
// batch's row map, and the events that time and complete it. Two stages let
// the scan of the next batch run while the host resolves the current one.
struct Stage {
  char* h_up = nullptr;              // pinned: TaskRec[padded G] then capoff[G + 1]
  uint32_t* h_down = nullptr;        // pinned: count[G] then the candidates
  TaskRec* h_tasks = nullptr;        // = h_up
  uint32_t* h_capoff = nullptr;      // per-row candidate slot offsets (inside h_up)
  uint32_t* h_count = nullptr;       // = h_down
  uint32_t* h_cand = nullptr;        // = h_down + G
  std::vector<int32_t> row_of;       // batch entry -> evaluation row
  std::vector<int32_t> row_shape;    // evaluation row -> (class, request) shape
  std::vector<int32_t> row_ext;      // full-scan: the last (longest-list) row of the row's shape in this scan
  // fused path (kbg_firstfit_kernel): rows map to shapes (grouped: row g is
  // shape g); each shape's list comes back as the masks of the words it covers
  int32_t n_slots = 0;               // shapes of the launch
  std::vector<int32_t> row_slot;     // row -> its shape's slot
  uint32_t* h_rowshape = nullptr;    // full-scan: row -> slot | kRowWriter (inside h_up)
  TaskRec* h_shapes = nullptr;       // full-scan: the shape table (inside h_up; grouped: h_tasks)
  std::vector<uint16_t> slot_rows;   // full-scan: rows of each slot (the kernel's run-length rows, FirstFitArgs.runs)
  uint32_t* h_info = nullptr;        // per slot: words covered | kInfoAnyBit | kCountIncompleteBit
  int32_t splits = 1;                // word parts of the launch (one info word per slot and part)
  std::vector<uint32_t> info_comb;   // splits > 1: the parts' info words combined per slot
  MaskPair* h_mask = nullptr;        // per slot: mw word masks from word w_lo
  uint32_t* h_avail = nullptr;       // owner-resolve: per slot, the ranks with a fitting node (summed)
  int32_t mw = 0, w_lo = 0;
  int32_t G = 0;
  int32_t base = 0;                  // the scan saw every node delta of resolutions with stamp <= base
  bool inflight = false;             // launched, results not yet collected
  bool timed = true;                 // the fused launch carries start / stop events (ev[0], ev[1])
  bool fused = false;                // kbg_firstfit_kernel (no select kernel, no copies)
  hipEvent_t ev[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // scan, select,
                                     // exchange start/stop; [6] = results on the host
};

struct SvcLink;  // kbg_session.cpp: the scan service's transport

struct Session {
  // ---- copied snapshot
  std::vector<std::string> strs;
  std::vector<int32_t> canon;  // string id -> canonical id of its content
  int32_t str_empty = -1;      // the canonical id of "" once an event needed it (empty_str)
  int32_t n_nodes = 0, n_jobs = 0, n_queues = 0, n_tasks = 0;
  std::vector<kbg_node> nodes_in;
  std::vector<kbg_job> jobs_in;
  std::vector<kbg_queue> queues_in;
  std::vector<kbg_task> tasks_in;
  std::vector<kbg_spec> specs_in;
  std::vector<kbg_term> terms_in;
  std::vector<kbg_requirement> reqs_in;
  std::vector<int32_t> values_in, labels_in, selectors_in;
  std::vector<kbg_toleration> tols_in;
  std::vector<kbg_taint> taints_in;
  std::vector<kbg_host_port> ports_in;
  kbg_options opts{};

  // ---- plugin configuration (session_plugins.go tier walks, flattened)
  bool has_drf = false, has_prop = false, has_gang = false, has_prio = false;
  bool pred_active = false;         // some tier entry "predicates" without disablePredicate
  std::vector<int32_t> job_chain;   // JobOrderPlugin in tier order (disabled entries removed)
  bool job_chain_pgd = false;       // job_chain is exactly (priority, gang, drf): make_job_key's fast path
  bool queue_order_prop = false;
  bool task_order_prio = false;
  bool ready_gang = false;
  bool heap_go111 = true;

  // ---- derived, immutable after open
  std::vector<int32_t> job_rank, queue_rank;             // bytewise UID order
  // Tasks: bytewise UID order as gapped ranks (multiples of kRankGap at open),
  // so a task added by an update takes a rank between its neighbours' without
  // re-ranking its job; equal UIDs share a rank. Only compared within a job.
  std::vector<int64_t> task_rank;
  // first 16 UID bytes, big-endian, zero-padded: unequal keys order the UIDs
  // as their bytes do (equal keys: the strings decide)
  struct UidKey {
    uint64_t a = 0, b = 0;
    bool operator<(const UidKey& o) const { return a != o.a ? a < o.a : b < o.b; }
    bool operator==(const UidKey& o) const { return a == o.a && b == o.b; }
  };
  std::vector<UidKey> task_uid_key;
  std::vector<int32_t> job_frank;                       // (CreationTimestamp, UID) order
  std::vector<int32_t> job_by_frank;                     // inverse of job_frank
  std::vector<uint32_t> job_prank;                       // dense rank of -Priority
  std::vector<int32_t> job_queue;                        // job -> queue index
  std::vector<int32_t> task_job;                         // task -> job index
  std::vector<int32_t> joff, jcap;                       // per-queue job-heap segment (jcap + 3 slots)
  std::vector<int32_t> pend, pend_off, pend_len;         // per-job pending tasks in TaskOrderFn order (this cycle)
  std::vector<int32_t> pend_all, pend_off_all, pend_len_all;  // the same at open
  std::vector<int32_t> job_min;  // jobs_in[j].min_available, packed for the engine
  std::vector<char> pending_candidate;                   // task is Pending and not BestEffort
  std::vector<char> be_task;                             // task is Pending and BestEffort (backfill.go:48-50)
  std::vector<int32_t> task_class;
  std::vector<int32_t> class_spec;                       // spec of each static class (-1: none)
  std::vector<int32_t> task_shape;                       // (class, request) shape id of a pending task
  // an update's job-list moves, applied once after its events (finish_job_lists)
  std::vector<int64_t> jmove;                            // per task: 0, -1 (left its job), or the sequence of its last re-add
  std::vector<std::pair<int32_t, int64_t>> jmove_add;    // (task, sequence) of every re-add, in event order
  std::vector<int32_t> jmove_out, jmove_jobs;            // tasks that left, jobs whose list changed
  std::vector<uint8_t> jmove_dirty;
  std::vector<int32_t> jmove_cnt, jmove_pos, jmove_flat;  // per job (zero between updates) / scratch
  int64_t jmove_seq = 0;
  bool jmove_defer = false;                              // this update defers its moves (many events); else in place
  std::vector<Res> shape_req;                            // each shape's request (the engine reads it by task_shape)
  std::vector<int32_t> shape_task;                       // a candidate task of each shape (-1: none; may be
                                                         // stale: valid while task_shape[it] == the shape)
  std::unordered_map<ShapeKey, int32_t, ShapeHash> shape_ids;  // shape ids, kept across updates
  std::vector<int32_t> shape_of_task;                    // a task's shape once it was a candidate (-1: not yet)
  std::vector<int32_t> pend_dirty_jobs;                  // jobs an update's events touched (their pending lists)
  std::vector<int32_t> pend_new;                         // tasks an update's events made (or re-made) Pending
  // An update's derive recomputes the per-task state of the tasks its events
  // touched only; the aggregates over tasks below are kept as counts.
  std::vector<int32_t> upd_tasks;                        // tasks an update's events touched (added, updated, deleted)
  std::vector<uint16_t> tstat_in;                        // tasks_in[t].status, packed for the per-job sums
  std::vector<uint8_t> t_aff, t_ghost;                   // per task: its contribution to has_aff / ghost
  int64_t n_aff = 0, n_ghost = 0;
  std::vector<uint8_t> t_inexact;                        // per candidate: a request the integer scan cannot take
  int64_t n_inexact = 0;
  __int128 isum_c = 0, isum_m = 0, isum_g = 0;           // candidates' requests, exact when n_inexact == 0
  // proportion's per-queue sums (allocated; allocated + pending) as exact
  // integers: while every live task's request is a non-negative integer and
  // the sums stay within 2^53, the sequential fp64 sums equal them
  std::vector<uint8_t> t_pinexact;
  int64_t n_pinexact = 0;
  std::vector<__int128> qa_sum, qr_sum;                  // [queue * 3 + dim]
  bool prop_sums_ok = false;                             // the sums above are current
  bool jalloc_exact = false;  // init.jalloc came from exact integer sums (an update may apply deltas)
  int32_t n_shapes = 0;
  std::vector<Res> treq;
  Res drf_total, prop_total;
  std::vector<char> q_has_attr;
  std::vector<Res> q_deserved, q_request;
  std::vector<int32_t> job_ready0;
  bool ghost = false;
  Engine init;  // engine state at session open

  // ---- node state (host mirror of the device table)
  std::vector<Res> idle0, rel0, idle, rel;
  std::vector<int32_t> ntasks0, ntasks, maxtasks;
  std::vector<char> nil_node;
  bool any_nil = false;
  std::vector<char> panic_node;  // nil Node under an active predicates plugin (predicates.go:122-123)

  // ---- the cycle's actions (allocate, then backfill) on this snapshot
  Engine fin;                 // plugin/ordering state after the last action
  bool cycle_started = false; // an action ran since open / reset
  bool allocated = false, backfilled = false, reclaimed = false, preempted = false;
  std::vector<kbg_decision> dec;              // decision log of the cycle
  std::vector<int32_t> undisp_head, undisp_next;  // Allocate decisions not yet dispatched, per job
  std::vector<int32_t> jt_off, jt;            // tasks of each job in snapshot (status-index) order
  int32_t action = KBG_ACTION_ALLOCATE;       // the action whose decisions are being logged
  std::vector<int32_t> dec_action;            // KBG_ACTION_* of each decision
  std::vector<int32_t> tstat;                 // job-side status of each task in the cycle
  // ---- preempt / reclaim (preempt.go, reclaim.go, statement.go)
  std::vector<int32_t> nt_off, nt_task;       // victim candidates per node: session tasks Running there at
                                              // open, in NodeInfo.Tasks order
  std::vector<int32_t> nt_off_buf, nt_task_buf;  // the next derive's copy (an update rebuilds by swap)
  std::vector<int32_t> upd_nodes;             // nodes an update's events touched (kbg_session_update) ...
  bool upd_nodes_valid = false;               // ... set for the derive that follows them
  std::vector<uint8_t> t_detached;            // a statement discard's RemoveTask took the task's copy off its node
  // (node, task): an AllocatedStatus pod whose spec names the node but that is
  // missing from the node's pods (a detached holder); the podLister Filter
  // leaves it out of that node's own pod-affinity predicate (vendor
  // cache/node_info.go:692-702), every other node still counts it
  std::vector<std::pair<int32_t, int32_t>> aff_filtered;
  std::vector<uint8_t> trun;                  // node-side copy still Running (an eviction makes it Releasing
                                              // for good: unevict's AddTask fails, node_info.go:101-106)
  std::vector<int32_t> task_node;             // node index of a task's NodeName (-1: not a session node)
  std::vector<int32_t> task_cnode;            // the NodeInfo the cache's sc.Nodes[NodeName] is: task_node, or
                                              // a node known only from pods carrying that NodeName (-1: none)
  std::vector<int32_t> nil_name;              // per node: the NodeName its pods carry when its Node is nil (-1)
  std::unordered_map<int32_t, int32_t> pod_only_of;  // that NodeName (canonical id) -> the node
  std::vector<kbg_eviction> evictions;        // committed cache.Evict calls
  std::vector<int32_t> t_pos;                 // a task's position in the candidate lists (-1: none)
  // what the device victim tables hold of the live state (running flags per
  // candidate position, gang readiness, drf / proportion allocations): an
  // action's start sends only the entries that differ (StateDelta, read in
  // place from mapped memory) instead of re-uploading the arrays
  bool vt_sh_valid = false;
  std::vector<uint8_t> vt_sh_run;
  std::vector<int32_t> vt_sh_ready;
  std::vector<double> vt_sh_jalloc, vt_sh_qalloc;  // [3 x J], [3 x Q]
  uint8_t* c_run_pinned = nullptr;            // running flags in candidate order (pinned upload staging)
  size_t c_run_pinned_cap = 0;
  std::vector<uint32_t> sd_seen[4];           // victim_push: last-write dedup stamps per StateDelta kind
  uint32_t sd_gen = 0;
  std::vector<int32_t> tier_preempt, tier_reclaim;  // VictimPlugin bits per tier holding an enabled victim fn
  int32_t max_candidates = 0;
  kbg::VictimTables vt{};                     // device copies (allocated at the first victim action)
  bool vt_ready = false;
  uint32_t* d_vbits = nullptr;                // sharded: [2][W32] stop / panic words of this rank's nodes, and
  uint32_t* d_vbits_red = nullptr;            //   their OR over the ranks (element-wise max of disjoint words)
  uint32_t* h_vbits = nullptr;                // pinned, coherent, device-mapped [2][W32] stop / panic words
  uint32_t* h_vbits_dev = nullptr;
  int32_t W32 = 0;                            // 32-node words over all N nodes
  // Stop maps of the last victim scan, kept current on the host between
  // scans (kbg_session.cpp VictimCache): valid for one preemptor shape; a
  // node whose inputs changed since the scan is marked unknown and
  // re-evaluated on the host when a search reaches it.
  struct VictimCache {
    bool valid = false;
    VictimKey key;                            // the preemptor shape the maps are for
    int32_t fns = 0;                          // victim fns of the deciding tier
    std::vector<uint32_t> stop, panic, unk;   // [W32]
    int32_t lb = 0;                           // every word below lb has no stop and no unknown bit
    void dirty(int32_t n) {
      unk[n >> 5] |= 1u << (n & 31);
      if ((n >> 5) < lb) lb = n >> 5;
    }
  } vc;
  std::vector<int32_t> jn_off, jn_node;       // per job: the nodes holding its tasks Running at open
  kbg::StateDelta* h_sdeltas = nullptr;       // pinned, device-mapped (the prep kernel reads it in place)
  kbg::StateDelta* h_sdeltas_dev = nullptr;
  kbg::NodeDelta* h_deltas_dev = nullptr;     // device address of h_deltas
  bool vstage_busy = false;                   // a prep launch may still read the staging buffers
  double vk_timed_ms = 0;                     // sampled victim-scan kernel time (this cycle)
  int64_t vk_timed = 0;
  // fused first-fit launches: start / stop events on one launch in
  // kFfTimeEvery (each timed launch adds ≈ 7 µs to its round trip); the
  // sampled time scaled to every launch of the cycle is scan_kernel_ms
  double ff_timed_ms = 0;
  int64_t ff_timed = 0, ff_launch_seq = 0;
  std::vector<kbg::StateDelta> sdeltas;       // queued victim-table changes
  std::vector<int32_t> be_shape;              // per pod-spec class: grouping id of its BestEffort tasks
  std::vector<int32_t> committed_ready;
  struct FitCounts { int32_t valid = 0, nodes = 0, cpu = 0, mem = 0, gpu = 0; };
  std::vector<FitCounts> fit;               // per job (A17)
  char* fit_h = nullptr;                    // FitError inputs: pinned staging, device copy, mapped results
  char* fit_d = nullptr;
  int32_t* fit_out = nullptr;
  size_t fit_cap = 0, fit_out_cap = 0;
  std::vector<uint64_t> h_class_mask;       // host copy of the class masks the scan reads (static predicate,
                                            // and with host ports the dynamic port fit)
  // ---- host ports (vendor predicates.go:1031-1051). A node's used ports only
  // grow during a cycle, so a (class, node) pair only ever loses feasibility:
  // the port fit is folded into the class masks and kept current by clearing
  // bits as placements record ports (monotone, like the pod cap).
  bool untimed_launches = false;  // (developer tools) fused launches without start / stop events
  bool has_ports = false;
  int32_t PW = 0;                              // u64 words per port-atom set
  std::vector<uint64_t> node_ports, node_ports0;  // [N][PW] used (ip, protocol, port) atoms
  std::unordered_map<int64_t, int32_t> port_hold; // (node << 32 | atom) -> pods placed this cycle holding it
  std::unordered_map<int64_t, int32_t> port_open; // (node << 32 | atom) -> entries of the pods there at open
  std::unordered_map<int64_t, int32_t> port_gone; //   ... of pods a statement discard removed this cycle
  std::unordered_map<std::string, int32_t> atom_of;  // "ip|protocol|port" -> atom
  std::vector<uint64_t> cls_conf, cls_add;     // [class][PW] atoms a class conflicts with / records
  std::vector<std::vector<int32_t>> atom_cls;  // classes that conflict with each atom
  std::vector<uint64_t> h_class_mask0, h_class_mask_static;  // at open (ports applied) / static predicate only
  std::vector<uint32_t> mask_dirty;            // class-mask words changed since the last write-back
  std::vector<uint8_t> mask_dirty_flag;
  MaskDelta* h_mdeltas = nullptr;              // pinned, mapped staging (read in place)
  // ---- inter-pod (anti)affinity folded into the class masks (kbg_affinity.cpp)
  bool has_aff = false;                        // some task carries a required pod (anti)affinity term
  std::shared_ptr<AffinityModel> affm;
  std::vector<kbg_pod_term> pod_terms_in;
  std::vector<int32_t> pod_labels_in;
  std::vector<int32_t> mwmark;                 // per class-mask word: resolution stamp of the last bit it lost
  int32_t mstamp = 0;                          // the current resolution stamp
  std::vector<uint8_t> aff_gain_flag;          // per class: gained nodes since the last cut
  std::vector<int32_t> aff_gain_classes;

  // ---- resident session (kbg_session_update edits the inputs above)
  StrIndex canon_of;  // string content -> canonical id
  std::unordered_map<int32_t, int32_t> node_of;       // canonical node name -> node index
  std::vector<uint8_t> task_live;                     // 0: the pod was deleted (event_handlers.go deletePod)
  std::vector<std::vector<int32_t>> job_task_order;   // per job: its tasks in JobInfo.Tasks insertion order
  std::vector<std::vector<int32_t>> job_rank_order;   // per job: its ranked tasks in task_rank order
  std::vector<std::vector<UidKey>> job_rank_key;      // per job: their UID keys, in the same order (a
                                                      // new task's place is searched in contiguous keys)
  std::vector<std::vector<int32_t>> node_task_order;  // per node: the session tasks in NodeInfo.Tasks order
  std::vector<std::vector<int32_t>> node_key_order;   // per node: PodKey (canonical id) of every pod on it
  std::vector<kbg_resource> others_in;                // Session.Others resreq
  // (node << 32 | key) held by pods outside the session jobs, with the node's
  // copy as RemoveTask reads it (kbgpu.h kbg_node_pod; status 0: the snapshot
  // carried no node_pods, so a removal by key is refused)
  struct Outsider {
    kbg_resource req{};
    int32_t status = 0;
    std::vector<kbg_host_port> ports;
  };
  std::unordered_map<int64_t, Outsider> outsiders;
  std::unordered_set<int64_t> outsider_gone;          // removed by a statement discard this cycle
  std::string broken;                                 // non-empty: an update failed part-way, re-open
  // structural events (KBG_EV_NODE_ADD ... QUEUE_DELETE): what left during the
  // update (dropped when the session is rebuilt from its updated snapshot),
  // and the old -> new maps of the last update that rebuilt (kbgpu.h
  // kbg_session_renumbering; empty: nothing renumbered)
  bool adopt_strings = false;                         // ingest keeps strs / canon / canon_of (restructure)
  std::vector<uint8_t> node_dead, job_dead, queue_dead, job_to_others;
  std::vector<int32_t> renum[4];
  std::vector<kbg_plugin_option> plugins_in;          // the snapshot's tier entries, for the rebuild
  std::vector<int32_t> tier_sizes_in;
  bool task_ranks_stale = false;                      // tasks were added: re-rank their jobs' UIDs
  std::vector<int32_t> rank_dirty_jobs;
  std::vector<int32_t> spec_class;                    // per spec: its static class (-1: none compiled)
  int32_t nospec_class = -1;                          // class of a task without a spec
  StaticTables static_tab{};                          // device static predicate inputs (mask rebuilds)
  uint8_t* d_node_flags = nullptr;
  std::vector<uint8_t> node_flags;                    // host copy of the device node flags
  double update_ms = 0;
  int64_t updates = 0, rebuilds = 0;
  bool vt_stale = false;                              // the victim tables follow older inputs
  std::vector<void*> vt_allocs;                       // their HBM (freed when they are rebuilt)
  std::vector<int32_t> big_rows;                      // table rows of nodes with 129 .. kMaxNodeCandidates victim candidates
  std::vector<int32_t> huge_nodes;                    // nodes (global) with more: evaluated on the host (host_stop)
  uint8_t* h_vbig = nullptr;                          // mapped: the big-node kernel's verdict per big row
  uint8_t* h_vbig_dev = nullptr;
  size_t h_vbig_cap = 0;
  int32_t* d_big_rows = nullptr;

  // ---- NodeInfo.Tasks keys (node_info.go:101-106): AddTask of a PodKey the
  // node already holds returns an error and leaves the node unchanged, while
  // ssn.Allocate / ssn.Pipeline still log the decision and run the handlers
  // (session.go:205-293). Only keys that can collide are tracked.
  std::vector<int32_t> task_key;                      // canonical string id of each task's PodKey
  bool has_dupkeys = false;                           // some candidate task's key can meet itself on a node
  std::vector<uint8_t> key_hot;                       // per canonical string id: a colliding key
  std::vector<int32_t> kc_cand, kc_node;              // per canonical key: candidate tasks / node entries holding it
  int64_t n_hot = 0;                                  // keys with key_hot set
  std::vector<int32_t> upd_keys;                      // keys whose node entries an update's events changed
  std::unordered_set<int64_t> node_keys, node_keys0;  // (node << 32 | key) of hot keys on nodes (now / at open)
  std::unordered_map<int64_t, int32_t> key_holder;     // of those, the ones this cycle's placements took: task << 1 | pipelined
  std::vector<uint8_t> dec_dup;                       // per decision of the cycle: the node was left unchanged

  // ---- device
  int32_t device = 0;
  hipStream_t stream = nullptr;
  int32_t W = 0;            // u64 words per node bitmap row
  bool int_mode = false;    // scan rows carry integer thresholds (kbg_device.hpp TaskRec)
  // node-axis sharding: R shards of Wl words; this process holds
  // shard `shard` (comm != null) or every shard (shard = -1)
  int32_t R = 1, Wl = 0, shard = -1;
  bool owner = false;  // owner-resolve protocol (allocate_sharded): each rank resolves the rows it owns
  // scan service (allocate_svc_root / allocate_serve): rank 0 runs the
  // single-GPU pipeline; each of its scans is a launch message every rank
  // answers by scanning its own words, and the ranks' word masks are summed.
  // `svc`: the transport while an allocate of this rank runs the service.
  SvcLink* svc = nullptr;
  SvcLink* svc_own = nullptr;         // the library's RCCL link, made at the first allocate (free_device deletes it)
  std::vector<NodeDelta> svc_nodes;   // rank 0: node rows written back since the last message (every rank's)
  std::vector<MaskDelta> svc_masks;   // rank 0: class-mask words written since the last message
  std::vector<uint32_t> svc_out;      // rank 0: committed outcomes since the last message (task, node<<1|pipe / ~0)
  uint32_t* d_svc = nullptr;          // the launch's info words and word masks, summed over the ranks in place
  int32_t tab_lo = 0, tab_n = 0;  // global node range of the device node table
  kbg_comm* comm = nullptr;
  int32_t n_classes = 0;
  int32_t K = 0, M = 0;     // batch tasks, candidates per row (full-scan) / slack (grouped)
  int64_t cand_cap = 0;     // candidate slots allocated
  int32_t n_shapes_cap = 0; // upper bound on the shapes of one scan (cand_cap sizing)
  NodeSoA d_nodes{};
  NodeSoA d_nodes0{};       // pristine copy for kbg_session_reset
  uint64_t* d_class_mask = nullptr;
  uint64_t* d_bits = nullptr;     // feasibility bitmaps [slot][plane][quad][row][4] (ScanGeom)
  char* d_up = nullptr;           // rows + capoff of the batch being scanned (stream-ordered reuse)
  uint32_t* d_down = nullptr;     // counts + candidates of the batch being selected
  Stage stages[2];                // host staging of two batches in flight
  size_t up_cap = 0;              // bytes of one pinned row buffer (Stage::h_up)
  std::vector<char*> up_pool;     // spare pinned row buffers: the allocate builder's batches borrow them
  // the allocate predictor's batch objects, kept across cycles (vector
  // capacities; the type is private to kbg_session.cpp)
  std::vector<std::unique_ptr<void, void (*)(void*)>> batch_pool;
  std::vector<Res> dec_old_buf;   // allocate: the Idle / Releasing row before each decision
  int32_t res_stamp = 0;          // resolution stamps: monotone over the session (mark / mwmark compare)
  NodeDelta* h_deltas = nullptr; // pinned, mapped: the apply kernels read it in place
  bool uva = false;              // mapped host memory has the same address on the device
  hipEvent_t stage_ev = nullptr; // after the last enqueued reader of the pinned staging (stage_acquire)
  hipEvent_t comm_ev = nullptr;  // comm_sync: the stream's end, polled against RCCL errors and the timeout
  bool stage_pending = false;
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  std::vector<void*> d_allocs;

  kbg_stats stats{};
};

// A class-mask bit of (c, n) changed: the host-kept victim stop maps of that
// class no longer know node n (Session::VictimCache).
inline void vc_mask_changed(Session& S, int32_t c, int32_t n) {
  if (S.vc.valid && S.vc.key.cls == c) S.vc.dirty(n);
}

// sets this thread's kbg_last_error message and returns `code`
kbg_status fail_with(kbg_status code, const std::string& msg);
bool parse_go_int64(const std::string& s, int64_t* out);
bool label_key_valid(const std::string& k);    // IsQualifiedName (validation.go:42-70)
bool label_value_valid(const std::string& v);  // IsValidLabelValue (validation.go:97-106)
void compile_static_predicates(Session& S, StaticHost* out);
// kbg_affinity.cpp
void setup_affinity(Session& S);
void aff_place(Session& S, int32_t t, int32_t n, int32_t sign, AffState& st, bool update_bits);
bool aff_ok(const Session& S, const AffState& st, int32_t c, int32_t n);
// aff_ok of the session's live state with the podLister Filter of node n applied
bool aff_ok_node(Session& S, int32_t c, int32_t n);
// the pod-affinity bits of every class on node n (its filtered pods changed)
void aff_refresh_node(Session& S, int32_t n);

}  // namespace kbg

struct kbg_session {
  kbg::Session s;
};
