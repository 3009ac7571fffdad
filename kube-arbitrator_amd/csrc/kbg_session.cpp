// Session open, ordering engine, speculative batch driver and the C ABI of
// the MI355X allocate path.
//
// Split of work:
//   host   — the reference's control flow, exactly: util.PriorityQueue over
//            Go 1.11 container/heap (util/priority_queue.go:25-88) for queues,
//            per-queue jobs and per-job tasks; the session tier walks
//            (session_plugins.go:142-295); drf/proportion/gang/priority state
//            (drf.go, proportion.go, gang.go, priority.go). Cost: O(log J)
//            integer/fp64 compares per placement.
//   device — the O(N) part: every (task, node) feasibility test of the node
//            loop (allocate.go:119-162), as a batched scan kernel over the
//            HBM-resident node table, and the first-M candidate extraction.
//
// Why batching is exact: during allocate a node's Idle,
// Releasing and pod count only move in the "less feasible" direction, and the
// static predicate never changes, so a node infeasible for a task at batch
// start stays infeasible. The task ORDER depends only on whether earlier
// tasks were placed, never on where. So the host predicts the next K task
// evaluations (success unless a task of the same shape already failed), the
// device evaluates all of them against the batch-start table, and the host
// commits in order: a task takes its first candidate that no earlier commit
// in the batch touched, re-checking touched candidates against the host
// mirror. An unpredicted outcome or an exhausted candidate list cuts the
// batch; the engine is restored from a checkpoint and replayed to the cut.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <tuple>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "kbg_comm.hpp"
#include "kbg_session.hpp"

namespace kbg {
struct SvcLink {
  virtual ~SvcLink() = default;
  // rank 0: msg[0 .. msg[1]) to every rank (may return before it is sent)
  virtual kbg_status send(Session& S, const uint32_t* msg) = 0;
  // ranks != 0: the next message
  virtual kbg_status recv(Session& S, std::vector<uint32_t>& msg) = 0;
  // after this rank's launch: the info words [0, info) and mask words [0, masks) of d_svc
  // summed over the ranks; rank 0 then has them in sg->h_down (stream-ordered before its
  // next event)
  virtual kbg_status sum(Session& S, kbg::Stage* sg, size_t info, size_t masks) = 0;
  // host words summed over the ranks, in place (synchronous)
  virtual kbg_status sum_host(Session& S, uint32_t* buf, size_t n) = 0;
};
}  // namespace kbg
using kbg::SvcLink;

namespace {

thread_local std::string g_err;

kbg_status fail(kbg_status code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace

kbg_status kbg::fail_with(kbg_status code, const std::string& msg) { return fail(code, msg); }

namespace {

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(KBG_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

using kbg::Engine;
using kbg::Res;
using kbg::Session;

// ---------------------------------------------------------- communicator
// A rank that fails between the collectives of a protocol round (a HIP error,
// a failed copy) cannot leave its peers blocked in theirs: it aborts the
// communicator, and a rank waiting on a collective polls RCCL's asynchronous
// error state and gives up after KBG_COMM_TIMEOUT_MS (default 300 s) without
// progress, aborting too. Either way the call returns KBG_E_RCCL and the
// communicator is dead for every session on it (kbgpu.h kbg_comm_init).
void comm_abort(kbg_comm* c) {
  if (!c || !c->coll) return;
  bool was = false;
  if (c->aborted.compare_exchange_strong(was, true)) c->coll->abort();
}

kbg_status comm_alive(const Session& S) {
  if (S.comm && S.comm->aborted.load())
    return fail(KBG_E_RCCL, "the communicator was aborted after a failure on a rank: destroy it and the sessions on it, "
                            "and re-create them");
  return KBG_OK;
}

// Waits for `ev` (recorded after collectives on the session's stream).
kbg_status comm_wait(Session& S, hipEvent_t ev) {
  if (!S.comm || !S.comm->coll) {
    HIP_TRY(hipEventSynchronize(ev));
    return KBG_OK;
  }
  static const double limit_ms = [] {
    const char* e = getenv("KBG_COMM_TIMEOUT_MS");
    return e && atof(e) > 0 ? atof(e) : 300000.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return KBG_OK;
    if (q != hipErrorNotReady) {
      comm_abort(S.comm);
      return fail(KBG_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
    }
    if ((spin & 63) == 0)
      if (const kbg_status h = S.comm->coll->health(); h != KBG_OK) {
        comm_abort(S.comm);
        return fail(h, S.comm->coll->err);
      }
    if (S.comm->aborted.load()) return comm_alive(S);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > limit_ms) {
      comm_abort(S.comm);
      return fail(KBG_E_RCCL, "a collective made no progress for KBG_COMM_TIMEOUT_MS: a peer rank failed or stopped");
    }
    if (spin > 2000) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// A collective of the session's communicator; its failure becomes this thread's error.
kbg_status coll_rc(Session& S, kbg_status st) { return st == KBG_OK ? KBG_OK : fail(st, S.comm->coll->err); }

kbg_status comm_sync(Session& S) {
  if (!S.comm || !S.comm->coll) {
    HIP_TRY(hipStreamSynchronize(S.stream));
    return KBG_OK;
  }
  HIP_TRY(hipEventRecord(S.comm_ev, S.stream));
  return comm_wait(S, S.comm_ev);
}

inline Res to_res(const kbg_resource& r) { return Res{r.milli_cpu, r.memory, r.milli_gpu}; }
inline kbg_resource to_kres(const Res& r) { return kbg_resource{r.c, r.m, r.g}; }

bool allocated_status(int32_t s) {  // api/helpers.go:63-70
  return s == KBG_BOUND || s == KBG_BINDING || s == KBG_RUNNING || s == KBG_ALLOCATED;
}
bool ready_status(int32_t s) {  // gang.go:44-55
  return allocated_status(s) || s == KBG_SUCCEEDED || s == KBG_PIPELINED;
}

// drf.go:156-166 / proportion.go:225-237 with helpers.Share (helpers/helpers.go:35-48)
double share_of(const Res& a, const Res& tot) {
  auto sh = [](double l, double r) { return r == 0 ? (l == 0 ? 0.0 : 1.0) : l / r; };
  double res = 0;
  double s = sh(a.c, tot.c);
  if (s > res) res = s;
  s = sh(a.m, tot.m);
  if (s > res) res = s;
  s = sh(a.g, tot.g);
  if (s > res) res = s;
  return res;
}

// Go math.Min
double go_min(double x, double y) {
  if (std::isinf(x) && x < 0) return x;
  if (std::isinf(y) && y < 0) return y;
  if (std::isnan(x) || std::isnan(y)) return NAN;
  if (x == 0 && x == y) return std::signbit(x) ? x : y;
  return x < y ? x : y;
}

// ---------------------------------------------------------------- heaps
// Go container/heap: up/down exactly (j-1)/2 truncating, right-child rule
// selectable (Go <= 1.11 "!Less(j1,j2)", later "Less(j2,j1)").
template <class L>
inline void go_up(int32_t* h, int j, L less) {
  for (;;) {
    const int i = (j - 1) / 2;
    if (i == j || !less(h[j], h[i])) break;
    std::swap(h[i], h[j]);
    j = i;
  }
}
template <class L>
inline void go_down(int32_t* h, int i0, int n, L less, bool go111) {
  int i = i0;
  for (;;) {
    const int j1 = 2 * i + 1;
    if (j1 >= n || j1 < 0) break;
    int j = j1;
    const int j2 = j1 + 1;
    if (j2 < n && (go111 ? !less(h[j1], h[j2]) : less(h[j2], h[j1]))) j = j2;
    if (!less(h[j], h[i])) break;
    std::swap(h[i], h[j]);
    i = j;
  }
}

kbg::JobKey make_job_key(const Session& S, const Engine& E, int32_t j) {
  if (S.job_chain_pgd) {  // the default tiers' chain (priority, gang, drf), without the loop
    const bool ready = E.jready[j] >= S.job_min[j];
    uint64_t u;
    __builtin_memcpy(&u, &E.jshare[j], 8);
    const uint64_t lo = ready ? (u & ~(1ull << 63)) : 0;  // fields after a non-ready gang are zero
    kbg::JobKey k = ((kbg::JobKey)S.job_prank[j] << 1) | (ready ? 1u : 0u);
    k = (k << 63) | lo;
    return (k << 32) | (uint32_t)S.job_frank[j];
  }
  kbg::JobKey k = 0;
  bool zero = false;
  for (int32_t p : S.job_chain) {
    if (p == kbg::JO_PRIORITY) {  // priority.go:58-74 (higher first)
      k = (k << 32) | (zero ? 0u : S.job_prank[j]);
    } else if (p == kbg::JO_GANG) {  // gang.go:129-163 (non-ready first)
      const bool ready = E.jready[j] >= S.job_min[j];
      k = (k << 1) | (zero ? 0u : (ready ? 1u : 0u));
      if (!ready) zero = true;
    } else {  // drf.go:109-125 (lower share first)
      uint64_t u;
      __builtin_memcpy(&u, &E.jshare[j], 8);
      k = (k << 63) | (zero ? 0 : (u & ~(1ull << 63)));
    }
  }
  return (k << 32) | (uint32_t)S.job_frank[j];
}

// Min-heap sift of `x` from the root over h[0..n), four children per node
// (4i+1 .. 4i+4: half the levels of a binary heap, the siblings on one or two
// cache lines). h[n .. n+2] hold the sentinel, so the child probes need no
// bounds test (hole-based). The job heaps' keys are static and strictly
// ordered while they are in the heap, so the pop sequence is that of any
// valid heap (the reference's binary container/heap included).
inline void job_heap_down(kbg::JobKey* h, int n, kbg::JobKey x) {
  int i = 0;
  for (;;) {
    const int c = 4 * i + 1;
    if (c >= n) break;
    // a tournament of index selects (no data-dependent branches)
    const int a = c + (h[c + 1] < h[c] ? 1 : 0), b = c + 2 + (h[c + 3] < h[c + 2] ? 1 : 0);
    const int m = h[b] < h[a] ? b : a;
    const kbg::JobKey mk = h[m];
    if (!(mk < x)) break;
    h[i] = mk;
    i = m;
  }
  h[i] = x;
}
constexpr int32_t kJobHeapPad = 3;  // sentinel slots past a job heap's capacity

// container/heap on queue ids compared through a rank table (rk[q] = position
// of q in QueueOrderFn order). Hole-based sifting is the same algorithm as
// Go's swap-based up/down: the element being moved is one side of every
// compare, so swapping it step by step or writing it once at the end gives
// the same array.
// `rk(q)`: the rank of queue id q (a table, or nibbles of a register).
template <class RK>
inline void rank_heap_up(int32_t* h, int j, RK rk) {
  const int32_t x = h[j];
  const int32_t rx = rk(x);
  while (j > 0) {
    const int p = (j - 1) / 2;
    if (!(rx < rk(h[p]))) break;
    h[j] = h[p];
    j = p;
  }
  h[j] = x;
}
// h[n] holds the sentinel queue id (the largest rank): never chosen as a child.
template <class RK>
inline void rank_heap_down(int32_t* h, int n, RK rk, bool go111) {
  if (n <= 1) return;
  const int32_t x = h[0];
  const int32_t rx = rk(x);
  int i = 0;
  for (;;) {
    const int j1 = 2 * i + 1;
    if (j1 >= n) break;
    const int32_t r1 = rk(h[j1]), r2 = rk(h[j1 + 1]);
    // go1.11: right child when !Less(j1, j2) (r2 <= r1); later: when Less(j2, j1)
    const bool right = go111 ? (r2 <= r1) : (r2 < r1);
    const int j = j1 + (right ? 1 : 0);
    const int32_t rj = right ? r2 : r1;
    if (!(rj < rx)) break;
    h[i] = h[j];
    i = j;
  }
  h[i] = x;
}

// Opt-in cycle counters of the ordering engine (KBG_PROFILE_ENGINE=1).
struct EngineProfile {
  bool on = false;
  uint64_t qpop = 0, qpush = 0, jtop = 0, apply = 0, steps = 0;
};
inline uint64_t cycles() { return __builtin_readcyclecounter(); }

// The session state the engine reads on every step, copied once per engine
// thread: pointers to the arrays and the scalars. The Session object's own
// cache lines also hold fields the committer and logger threads write during
// a cycle (stamps, statistics, the decision log's vector), so reading the
// arrays through it would keep pulling those lines across cores.
struct EngineView {
  const int32_t *pend, *pend_off, *pend_len, *job_by_frank, *joff, *job_min, *job_queue, *queue_rank, *job_frank;
  const uint32_t* job_prank;
  const Res *treq, *q_deserved;
  const int32_t* tshape;   // the task's shape: the engine reads its request from the small shape table
  const Res* shape_req;
  const char* q_has_attr;
  const int32_t* job_chain;
  int32_t n_job_chain, n_queues;
  Res drf_total;
  bool has_drf, has_prop, queue_order_prop, heap_go111, job_chain_pgd;
  explicit EngineView(const Session& S)
      : pend(S.pend.data()), pend_off(S.pend_off.data()), pend_len(S.pend_len.data()),
        job_by_frank(S.job_by_frank.data()), joff(S.joff.data()), job_min(S.job_min.data()),
        job_queue(S.job_queue.data()), queue_rank(S.queue_rank.data()), job_frank(S.job_frank.data()),
        job_prank(S.job_prank.data()), treq(S.treq.data()), q_deserved(S.q_deserved.data()),
        tshape(S.task_shape.data()), shape_req(S.shape_req.data()),
        q_has_attr(S.q_has_attr.data()), job_chain(S.job_chain.data()), n_job_chain((int32_t)S.job_chain.size()),
        n_queues(S.n_queues), drf_total(S.drf_total), has_drf(S.has_drf), has_prop(S.has_prop),
        queue_order_prop(S.queue_order_prop), heap_go111(S.heap_go111), job_chain_pgd(S.job_chain_pgd) {}
};

struct Ops {
  const Session& S;
  Engine& E;
  EngineProfile* prof = nullptr;
  alignas(64) const EngineView V;
  Ops(const Session& s, Engine& e, EngineProfile* p = nullptr) : S(s), E(e), prof(p), V(s) {}

  bool job_ready(int32_t j) const { return E.jready[j] >= V.job_min[j]; }

  // Session.JobOrderFn (session_plugins.go:196-221) over the configured tiers
  // is the order of kbg_session.hpp JobKey keys, built by make_job_key (the
  // same key from the view here).
  kbg::JobKey job_key(int32_t j) const {
    if (V.job_chain_pgd) {  // the default tiers' chain (priority, gang, drf), without the loop
      const bool ready = E.jready[j] >= V.job_min[j];
      uint64_t u;
      __builtin_memcpy(&u, &E.jshare[j], 8);
      const uint64_t lo = ready ? (u & ~(1ull << 63)) : 0;  // fields after a non-ready gang are zero
      kbg::JobKey k = ((kbg::JobKey)V.job_prank[j] << 1) | (ready ? 1u : 0u);
      k = (k << 63) | lo;
      return (k << 32) | (uint32_t)V.job_frank[j];
    }
    return make_job_key(S, E, j);
  }
  // Session.QueueOrderFn (session_plugins.go:223-245; proportion.go:146-159):
  // share, then UID. With proportion on, E.qrank holds every queue's position
  // in that order (maintained by reorder_queue), so a compare is two loads.
  bool queue_less_slow(int32_t a, int32_t b) const {
    if (V.queue_order_prop) {
      const double sa = E.qshare[a], sb = E.qshare[b];
      if (sa != sb) return sa < sb;
    }
    return V.queue_rank[a] < V.queue_rank[b];
  }
  bool queue_less(int32_t a, int32_t b) const { return E.qrank[a] < E.qrank[b]; }
  static constexpr int32_t kPackedQueues = 15;  // qrank_pk holds ids 0..14 and the sentinel (nibble 15)
  void set_rank(int32_t q, int32_t pos) {
    E.qrank[q] = pos;
    if (V.n_queues <= kPackedQueues)
      E.qrank_pk = (E.qrank_pk & ~(15ull << (4 * q))) | ((uint64_t)pos << (4 * q));
  }
  void reorder_queue(int32_t q) {  // q's share changed: move it to its new position
    int32_t pos = E.qrank[q];
    const int32_t Q = (int32_t)E.qorder.size();
    while (pos + 1 < Q && queue_less_slow(E.qorder[pos + 1], q)) {
      E.qorder[pos] = E.qorder[pos + 1];
      set_rank(E.qorder[pos], pos);
      ++pos;
    }
    while (pos > 0 && queue_less_slow(q, E.qorder[pos - 1])) {
      E.qorder[pos] = E.qorder[pos - 1];
      set_rank(E.qorder[pos], pos);
      --pos;
    }
    E.qorder[pos] = q;
    set_rank(q, pos);
  }
  // proportion.go:188-193
  bool overused(int32_t q) const {
    if (!V.has_prop || !V.q_has_attr[q]) return false;
    return kbg::res_le(V.q_deserved[q], E.qalloc[q]);
  }
  // The queue heap is a literal container/heap: it holds one entry per job
  // and entries keep stale keys, so its layout decides the order.
  // Fixed capacity (one entry per job at most, allocate.go:48-59 pushes one
  // per job and every pop is followed by at most one push); qheap[qlen] is the
  // sentinel id n_queues.
  void qpush(int32_t q) {
    int32_t* h = E.qheap.data();
    const int n = E.qlen++;
    h[n] = q;
    h[n + 1] = V.n_queues;
    if (V.n_queues <= kPackedQueues) {
      const uint64_t pk = E.qrank_pk;
      rank_heap_up(h, n, [pk](int32_t x) { return (int32_t)((pk >> (4 * x)) & 15u); });
    } else {
      const int32_t* rk = E.qrank.data();
      rank_heap_up(h, n, [rk](int32_t x) { return rk[x]; });
    }
  }
  int32_t qpop() {  // Pop: swap(0, n-1), down(0, n-1), take h[n-1]
    int32_t* h = E.qheap.data();
    const int n = --E.qlen;
    const int32_t q = h[0];
    h[0] = h[n];
    h[n] = V.n_queues;
    if (V.n_queues <= kPackedQueues) {
      const uint64_t pk = E.qrank_pk;
      rank_heap_down(h, n, [pk](int32_t x) { return (int32_t)((pk >> (4 * x)) & 15u); }, V.heap_go111);
    } else {
      const int32_t* rk = E.qrank.data();
      rank_heap_down(h, n, [rk](int32_t x) { return rk[x]; }, V.heap_go111);
    }
    return q;
  }
  // Per-queue job heaps. A job's key changes only while it is popped (drf and
  // gang update the allocated job, drf.go:131-139, gang.go:44-55), so keys in
  // a heap are static, the order is strict (UID tie-break) and the pop
  // sequence does not depend on the heap layout. allocate.go pops
  // the job, runs its tasks and pushes it back; here the job stays at the
  // root meanwhile and is re-sifted (success) or removed (no task fitted).
  void jfix_top(int32_t q, kbg::JobKey x) { job_heap_down(E.jheap.data() + V.joff[q], E.jlen[q], x); }
  void jremove_top(int32_t q) {
    kbg::JobKey* h = E.jheap.data() + V.joff[q];
    const int n = --E.jlen[q];
    const kbg::JobKey x = h[n];
    h[n] = kbg::kJobKeySentinel;
    if (n > 0) job_heap_down(h, n, x);
  }

  // allocate.go:65-112: advance the control flow to the next task whose node
  // loop has to run; -1 when the queue heap is exhausted.
  int32_t next_task() {
    for (;;) {
      if (E.in_job) {
        const int32_t j = E.cur_j;
        if (E.cursor[j] < V.pend_len[j]) return V.pend[V.pend_off[j] + E.cursor[j]++];
        jremove_top(E.cur_q);  // no task of the job fitted: the job is not pushed back
        qpush(E.cur_q);        // allocate.go:173-174
        E.in_job = false;
        continue;
      }
      if (E.qlen == 0) return -1;
      uint64_t c0 = prof ? cycles() : 0;
      const int32_t q = qpop();
      if (prof) prof->qpop += cycles() - c0;
      if (overused(q)) continue;     // :71-74
      if (E.jlen[q] == 0) continue;  // :78-81
      E.cur_j = V.job_by_frank[kbg::job_key_frank(E.jheap[V.joff[q]])];  // :85 jobs.Pop()
      E.cur_q = q;
      E.in_job = true;
    }
  }
  // After next_task() returned a task of shape known to fit nowhere: the
  // job's following tasks whose shapes are known to fit nowhere fail too
  // (monotone: a shape that fit nowhere fits nowhere for the rest of the
  // action), and a failure changes no plugin state (allocate.go:163-170: the
  // loop moves to the job's next task). They are consumed here at once; the
  // count (0: none) is what skip() replays. The job's turn goes on with its
  // next task, or ends when none is left.
  int32_t skip_dead(const std::atomic<uint8_t>* failed, const int32_t* tshape) {
    const int32_t j = E.cur_j;
    const int32_t end = V.pend_len[j];
    const int32_t* p = V.pend + V.pend_off[j];
    int32_t& c = E.cursor[j];
    const int32_t c0 = c;
    while (c < end && failed[tshape[p[c]]].load(std::memory_order_relaxed)) ++c;
    return c - c0;
  }
  void skip(int32_t n) { E.cursor[E.cur_j] += n; }  // n failed tasks of the current job (skip_dead's count)
  // Outcome of the node loop for the task returned by next_task().
  // Success = ssn.Allocate / ssn.Pipeline: drf + proportion AllocateFunc
  // (drf.go:131-139, proportion.go:197-206), then jobs.Push / queues.Push.
  void apply(int32_t t, bool success) {
    if (!success) return;
    uint64_t c0 = prof ? cycles() : 0;
    const int32_t j = E.cur_j, q = E.cur_q;
    const Res& r = V.shape_req[V.tshape[t]];  // (= treq[t]; the task's shape line is warm: the predictor read it)
    if (V.has_drf) {
      kbg::res_add(E.jalloc[j], r);
      // with gang ahead of drf in the job order (job_chain_pgd) a job short
      // of MinAvailable keys without its share: computed once it is ready
      // (and for every job when the cycle ends, finalize_shares)
      if (!V.job_chain_pgd || E.jready[j] + 1 >= V.job_min[j]) E.jshare[j] = share_of(E.jalloc[j], V.drf_total);
    }
    if (V.has_prop) {
      const int32_t jq = V.job_queue[j];
      kbg::res_add(E.qalloc[jq], r);
      E.qshare[jq] = share_of(E.qalloc[jq], V.q_deserved[jq]);
      if (V.queue_order_prop) reorder_queue(jq);
    }
    E.jready[j]++;
    const kbg::JobKey key = job_key(j);
    uint64_t c1 = prof ? cycles() : 0;
    // :164-168 jobs.Push(job): the popped job is still the root here; an
    // unchanged key (e.g. a gang job short of MinAvailable) leaves the heap as is
    if (key != E.jheap[V.joff[q]]) jfix_top(q, key);
    uint64_t c2 = prof ? cycles() : 0;
    qpush(q);     // :174
    E.in_job = false;
    if (prof) {
      const uint64_t c3 = cycles();
      prof->apply += c1 - c0;
      prof->jtop += c2 - c1;
      prof->qpush += c3 - c2;
      prof->steps++;
    }
  }
};

// The drf shares the engine left stale (Ops::apply: a job short of
// MinAvailable under job_chain_pgd), from each job's allocation: exactly the
// share an eager update computes (a function of jalloc alone).
void finalize_shares(const Session& S, Engine& E) {
  if (!S.has_drf) return;
  for (int32_t j = 0; j < S.n_jobs; ++j) E.jshare[j] = share_of(E.jalloc[j], S.drf_total);
}

// allocate.go:45-59: one queue entry per job (queue heap) and every job in
// its queue's job heap, keyed from E's plugin state.
void build_heaps(const Session& S, Engine& E) {
  E.jheap.assign((size_t)S.n_jobs + (size_t)S.n_queues * kJobHeapPad, kbg::kJobKeySentinel);
  E.jlen.assign(S.n_queues, 0);
  E.qheap.assign((size_t)S.n_jobs + 1, S.n_queues);
  E.qlen = 0;
  Ops ops{S, E};
  E.qorder.resize(S.n_queues);
  std::iota(E.qorder.begin(), E.qorder.end(), 0);
  std::sort(E.qorder.begin(), E.qorder.end(), [&](int32_t a, int32_t b) { return ops.queue_less_slow(a, b); });
  E.qrank.assign(S.n_queues + 1, INT32_MAX);  // [n_queues]: the heap sentinel
  for (int32_t i = 0; i < S.n_queues; ++i) E.qrank[E.qorder[i]] = i;
  E.qrank_pk = 0;
  if (S.n_queues <= Ops::kPackedQueues) {
    for (int32_t q = 0; q < S.n_queues; ++q) E.qrank_pk |= (uint64_t)E.qrank[q] << (4 * q);
    E.qrank_pk |= 15ull << (4 * S.n_queues);  // the sentinel id's rank: above every queue's (< n_queues <= 15)
  }
  for (int32_t j = 0; j < S.n_jobs; ++j) {
    ops.qpush(S.job_queue[j]);
    const int32_t q = S.job_queue[j];
    E.jheap[S.joff[q] + E.jlen[q]++] = make_job_key(S, E, j);
  }
  for (int32_t q = 0; q < S.n_queues; ++q)  // a sorted array is a valid min-heap
    std::sort(E.jheap.begin() + S.joff[q], E.jheap.begin() + S.joff[q] + E.jlen[q]);
}



// ---------------------------------------------------------------- device
// Buffers a closed (or rebuilt) session returns are kept for the next open in
// the process — a scheduler re-opens or rebuilds sessions every few cycles,
// and pinned allocations and frees cost milliseconds (hipHostMalloc maps the
// pages; hipFree synchronizes the device). Per kind (pinned host / device),
// device and size (rounded up to 64 KiB); at most kPoolKeep bytes idle per
// kind, the rest freed. A buffer is returned only after its session's stream
// has drained (free_device), so no kernel still reads or writes it.
struct BufPool {
  struct Buf {
    size_t bytes;
    int device;
    bool host;
  };
  std::mutex mu;
  std::unordered_map<void*, Buf> out;                       // every buffer handed out
  std::multimap<std::tuple<bool, int, size_t>, void*> idle;  // returned ones
  size_t idle_bytes[2] = {0, 0};
  static constexpr size_t kPoolKeep = size_t(1) << 30;
};
BufPool& buf_pool() {
  static BufPool* p = new BufPool();  // (never destroyed: buffers may be returned during process exit)
  return *p;
}
kbg_status pool_get(bool host, size_t bytes, void** p) {
  bytes = (std::max<size_t>(bytes, 64) + 65535) & ~size_t(65535);
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  BufPool& P = buf_pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.idle.lower_bound({host, dev, bytes});
    if (it != P.idle.end() && std::get<0>(it->first) == host && std::get<1>(it->first) == dev &&
        std::get<2>(it->first) <= 2 * bytes) {
      *p = it->second;
      P.idle_bytes[host] -= std::get<2>(it->first);
      P.idle.erase(it);
      return KBG_OK;
    }
  }
  if (host) HIP_TRY(hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  else HIP_TRY(hipMalloc(p, bytes));
  std::lock_guard<std::mutex> lk(P.mu);
  P.out[*p] = BufPool::Buf{bytes, dev, host};
  return KBG_OK;
}
void pool_put(void* p) {
  if (!p) return;
  BufPool& P = buf_pool();
  std::unique_lock<std::mutex> lk(P.mu);
  auto it = P.out.find(p);
  if (it == P.out.end()) return;  // (not a pooled buffer: never happens)
  const BufPool::Buf b = it->second;
  if (P.idle_bytes[b.host] + b.bytes <= BufPool::kPoolKeep) {
    P.idle.emplace(std::make_tuple(b.host, b.device, b.bytes), p);
    P.idle_bytes[b.host] += b.bytes;
    return;
  }
  P.out.erase(it);
  lk.unlock();
  if (b.host) (void)hipHostFree(p);
  else (void)hipFree(p);
}

template <class T>
kbg_status dalloc(Session& S, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  if (kbg_status st = pool_get(false, count * sizeof(T), &q); st != KBG_OK) return st;
  S.d_allocs.push_back(q);
  *p = (T*)q;
  return KBG_OK;
}
template <class T>
kbg_status hupload(Session& S, T** p, const std::vector<T>& v) {
  kbg_status st = dalloc(S, p, v.size());
  if (st != KBG_OK) return st;
  if (!v.empty()) HIP_TRY(hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, S.stream));
  return KBG_OK;
}

// Several host arrays into ONE device block with one copy (session open's
// static tables, the victim tables): one transfer instead of a copy per array.
struct BulkUpload {
  struct Item {
    void** p;
    size_t off;
  };
  std::vector<Item> items;
  std::vector<char> host;
  void add_raw(void** p, const void* data, size_t bytes) {
    const size_t off = (host.size() + 255) & ~(size_t)255;
    host.resize(off + std::max<size_t>(bytes, 16), 0);
    if (data && bytes) std::memcpy(host.data() + off, data, bytes);
    items.push_back({p, off});
  }
  template <class T>
  void add(T** p, const std::vector<T>& v) {
    add_raw((void**)p, v.data(), v.size() * sizeof(T));
  }
  template <class T>
  void zeros(T** p, size_t count) {  // zero-filled on the device
    add_raw((void**)p, nullptr, count * sizeof(T));
  }
  // allocates the block, points every item into it, copies once and waits
  // (the host vectors the items came from may end after this)
  kbg_status commit(Session& S) {
    if (items.empty()) return KBG_OK;
    char* d = nullptr;
    if (kbg_status st = dalloc(S, &d, host.size()); st != KBG_OK) return st;
    for (const Item& it : items) *it.p = d + it.off;
    HIP_TRY(hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, S.stream));
    HIP_TRY(hipStreamSynchronize(S.stream));
    items.clear();
    host.clear();
    return KBG_OK;
  }
};

// The node table as ONE block (FirstFitArgs.nodes): idle c/m/g and rel c/m/g
// f64[stride], then ntasks and maxtasks i32[stride], stride = tab_n rounded
// up to 64 rows. A reset restores it with one copy.
int32_t soa_stride(const Session& S) { return std::max(64, (S.tab_n + 63) / 64 * 64); }

// Fused-path results in a stage's down buffer (u32 units): per slot the info
// word, then (16-B aligned) per slot `mw` word-mask pairs, then per slot the
// owner-resolve availability. mw = the words one launch covers (this rank's
// words when the session is sharded).
int32_t fused_mask_words(const Session& S) { return std::max(1, S.owner ? S.Wl : S.W); }
inline size_t fused_mask_off(int32_t K) { return ((size_t)K * kbg::kFfMaxSplits + 3) & ~(size_t)3; }
inline size_t fused_avail_off(int32_t K, int32_t mw) { return fused_mask_off(K) + (size_t)K * mw * 4; }
inline size_t fused_down_words(int32_t K, int32_t mw) { return fused_avail_off(K, mw) + (size_t)K; }
size_t soa_bytes(const Session& S) { return (size_t)soa_stride(S) * (6 * 8 + 2 * 4); }

kbg_status alloc_soa(Session& S, kbg::NodeSoA* soa) {
  const size_t L = (size_t)soa_stride(S);
  double* b = nullptr;
  kbg_status st = dalloc(S, (char**)&b, soa_bytes(S));
  if (st != KBG_OK) return st;
  *soa = kbg::NodeSoA{b, b + L, b + 2 * L, b + 3 * L, b + 4 * L, b + 5 * L, (int32_t*)(b + 6 * L),
                      (int32_t*)(b + 6 * L) + L};
  return KBG_OK;
}

kbg_status copy_soa(Session& S, const kbg::NodeSoA& dst, const kbg::NodeSoA& src) {
  if (S.tab_n == 0) return KBG_OK;
  // (a kernel of ours, not the runtime's blit: soa_bytes is a multiple of 16)
  HIP_TRY(kbg::launch_copy16(dst.idle_cpu, src.idle_cpu, soa_bytes(S) / 16, S.stream));
  return KBG_OK;
}

// Pinned host memory the kernels read and write in place (zero-copy: row
// uploads, candidate lists, node / mask deltas): mapped and fine-grained
// (coherent), so a kernel's stores are on the host when its completion event
// fires and the host's stores are seen by the next launch.
kbg_status host_alloc(void** p, size_t bytes) {
  return pool_get(true, bytes, p);  // (pool_put returns it)
}
// The device address of such memory (the host address itself under unified
// addressing, which build() checks once).
template <class T>
T* dev_ptr(const Session& S, T* h) {
  if (S.uva || !h) return h;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, (void*)h, 0) != hipSuccess) return nullptr;
  return (T*)d;
}

void free_device(Session& S) {
  if (S.stream) (void)hipStreamSynchronize(S.stream);  // every enqueued reader of the staging has run
  delete S.svc_own;
  S.svc_own = nullptr;
  for (kbg::Stage& g : S.stages) {
    if (g.inflight) (void)hipEventSynchronize(g.ev[6]);  // nothing may still write the staging
    pool_put(g.h_up);
    pool_put(g.h_down);
    for (auto& e : g.ev)
      if (e) {
        (void)hipEventDestroy(e);
        e = nullptr;
      }
    g = kbg::Stage{};
  }
  for (char* b : S.up_pool) pool_put(b);
  S.up_pool.clear();
  pool_put(S.h_deltas);
  pool_put(S.h_mdeltas);
  S.h_mdeltas = nullptr;
  pool_put(S.fit_h);
  pool_put(S.fit_out);
  if (S.fit_d) (void)hipFree(S.fit_d);
  S.fit_h = nullptr;
  S.fit_out = nullptr;
  S.fit_d = nullptr;
  S.fit_cap = S.fit_out_cap = 0;
  if (S.h_vbits) (void)hipHostFree(S.h_vbits);
  if (S.h_vbig) (void)hipHostFree(S.h_vbig);
  S.h_vbig = nullptr;
  S.h_vbig_dev = nullptr;
  S.h_vbig_cap = 0;
  if (S.h_sdeltas) (void)hipHostFree(S.h_sdeltas);
  if (S.c_run_pinned) (void)hipHostFree(S.c_run_pinned);
  S.c_run_pinned = nullptr;
  S.c_run_pinned_cap = 0;
  S.h_vbits = nullptr;
  S.h_sdeltas = nullptr;
  S.vt_ready = false;
  S.vt_sh_valid = false;
  S.vt_allocs.clear();
  S.h_deltas = nullptr;
  for (void* p : S.d_allocs) pool_put(p);
  S.d_allocs.clear();
  for (auto& e : S.ev)
    if (e) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
  if (S.stage_ev) (void)hipEventDestroy(S.stage_ev);
  S.stage_ev = nullptr;
  if (S.comm_ev) (void)hipEventDestroy(S.comm_ev);
  S.comm_ev = nullptr;
  S.stage_pending = false;
  if (S.stream) (void)hipStreamDestroy(S.stream);
  S.stream = nullptr;
}

// Node state as the device scans it: a nil Node under an active predicates
// plugin is "always feasible" so the first scan reaching it reports the
// reference's panic (predicates.go:122-123 SetNode(nil)).
void device_row(const Session& S, int32_t n, double* ic, double* im, double* ig, double* rc, double* rm, double* rg,
                int32_t* nt, int32_t* mt) {
  if (S.nil_node[n] && S.pred_active) {
    *ic = *im = *ig = INFINITY;
    *rc = *rm = *rg = 0;
    *nt = 0;
    *mt = INT32_MAX;
    return;
  }
  *ic = S.idle[n].c;
  *im = S.idle[n].m;
  *ig = S.idle[n].g;
  *rc = S.rel[n].c;
  *rm = S.rel[n].m;
  *rg = S.rel[n].g;
  *nt = S.ntasks[n];
  *mt = S.maxtasks[n];
}

// Uploads the node rows this process holds (global nodes [tab_lo, tab_lo + tab_n)).
kbg_status upload_nodes(Session& S) {
  const int32_t N = S.tab_n;
  if (N == 0) return KBG_OK;
  std::vector<double> ic(N), im(N), ig(N), rc(N), rm(N), rg(N);
  std::vector<int32_t> nt(N), mt(N);
  for (int32_t i = 0; i < N; ++i)
    device_row(S, S.tab_lo + i, &ic[i], &im[i], &ig[i], &rc[i], &rm[i], &rg[i], &nt[i], &mt[i]);
  auto up = [&](void* d, const void* h, size_t b) { return hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, S.stream); };
  HIP_TRY(up(S.d_nodes0.idle_cpu, ic.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.idle_mem, im.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.idle_gpu, ig.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.rel_cpu, rc.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.rel_mem, rm.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.rel_gpu, rg.data(), N * 8));
  HIP_TRY(up(S.d_nodes0.ntasks, nt.data(), N * 4));
  HIP_TRY(up(S.d_nodes0.maxtasks, mt.data(), N * 4));
  HIP_TRY(hipStreamSynchronize(S.stream));  // host vectors die here
  return copy_soa(S, S.d_nodes, S.d_nodes0);
}

// One device round trip for a batch: rows[0..G) of stage `sg` are the
// distinct evaluation rows (a task in full-scan mode, a (class, request) shape
// otherwise), each given cap_off[g+1]-cap_off[g] candidate slots. Everything
// is enqueued on the session stream; sg.ev[6] fires when the candidate lists
// are on the host. The device buffers are reused in stream order (the next
// upload runs after this batch's select has read them); only the host staging
// is per stage. `base`: the newest resolution whose node deltas are already
// enqueued, i.e. what this scan sees.
struct Trace;
thread_local Trace* t_trace = nullptr;  // the committer's KBG_TRACE timeline, if on
void trace_add(const char* what, int64_t v = 0);

constexpr int64_t kFfTimeEvery = 4;  // fused launches: one in this many carries start / stop events
// Full-scan mode (the roofline measurement, not the production number) times
// every launch: its launches alternate between batch scans and short
// rescans, and a one-in-four sample followed that pattern instead of the mix.
inline int64_t ff_time_every(const Session& S) { return S.opts.full_scan ? 1 : kFfTimeEvery; }
kbg_status svc_launch(Session& S, kbg::Stage& sg, kbg::FirstFitArgs& a, int32_t G, int32_t base);
kbg_status device_launch(Session& S, kbg::Stage& sg, int32_t G, int32_t base) {
  trace_add("l.begin", G);
  const int32_t Gp = kbg::kbg_pad_rows(G);  // Grouper::build padded the rows
  if (!S.comm || S.owner || S.svc) {
    // one launch: kbg_firstfit_kernel takes the shapes from its arguments
    // (or the stage's mapped buffer) and writes each shape's info word and
    // word masks straight into the other one; this process's words only
    // (owner-resolve), or every word
    thread_local kbg::FirstFitArgs a;  // (3 KB: the inline shape table)
    a = kbg::FirstFitArgs{};
    a.nodes = S.d_nodes.idle_cpu;
    a.stride = soa_stride(S);
    a.class_mask = S.d_class_mask;
    a.G = G;
    a.n_shapes = sg.n_slots;
    a.n_nodes = S.n_nodes;
    a.W = S.W;
    const bool own_words = S.owner || S.svc;
    a.w_lo = own_words ? std::min(S.W, S.shard * S.Wl) : 0;
    a.w_hi = own_words ? std::min(S.W, (S.shard + 1) * S.Wl) : S.W;
    a.mw = fused_mask_words(S);
    a.tab_lo = S.tab_lo;
    a.tab_n = S.tab_n;
    a.cap_check = S.pred_active ? 1 : 0;
    a.early_exit = S.opts.full_scan ? 0 : 1;  // full-scan evaluates every node for every row
    // A table of one round (<= 128 words) is walked whole anyway: every
    // word's masks go out, so no list is ever cut (no truncation rescans).
    // Then a short batch's walk is split into word parts, one workgroup
    // each, so its handful of row blocks spreads over the CUs instead of
    // walking 5 words per wave on 6 of them.
    const int32_t tw = a.w_hi - a.w_lo;
    a.complete = tw <= kbg::kFfRoundWords ? 1 : 0;
    a.splits = 1;
    // Production walks of larger tables (C4's 313 words) split too: each part
    // stops at the row's `want` within its own words, and the parts' lists
    // join in node order up to the first one that stopped early (device_wait)
    const kbg::FfGeometry geo = kbg::firstfit_geometry(G, !a.early_exit);
    a.rows = geo.rows;
    if ((a.complete || a.early_exit) && !S.comm) {
      const int32_t blocks = (G + geo.rows - 1) / geo.rows;
      a.splits = std::max(1, std::min({kbg::kFfMaxSplits, 256 / std::max(1, blocks), tw / 8}));
    }
    if (tw > 0) {
      a.split_words = (tw + a.splits - 1) / a.splits;
      a.splits = (tw + a.split_words - 1) / a.split_words;  // no empty part
    } else {  // no words (a session without nodes)
      a.splits = 1;
      a.split_words = 0;
    }
    a.info_stride = a.splits;
    a.part0 = 0;
    a.mask_w0 = a.w_lo;
    sg.splits = a.splits;
    if (sg.n_slots <= kbg::kInlineShapes) {
      std::copy(sg.h_shapes, sg.h_shapes + sg.n_slots, a.inl);
    } else if (!(a.shapes = dev_ptr(S, sg.h_shapes))) {
      return fail(KBG_E_HIP, "hipHostGetDevicePointer of a stage buffer failed");
    }
    // Full-scan rows of one slot are identical evaluations and only the
    // slot's writer row produces output, so with the shapes inline the launch
    // takes its rows slot by slot from the run lengths in its arguments (no
    // row -> shape map read over PCIe at the start of every workgroup)
    if (sg.h_rowshape && sg.n_slots <= kbg::kInlineShapes && (int32_t)sg.slot_rows.size() == sg.n_slots) {
      a.runs = 1;
      uint32_t end = 0;
      for (int32_t sl = 0; sl < sg.n_slots; ++sl) a.run_end[sl] = (uint16_t)(end += sg.slot_rows[sl]);
      if ((int32_t)end != G) return fail(KBG_E_INVALID, "internal: full-scan slot rows do not add up to the batch");
    } else if (sg.h_rowshape && !(a.row_shape = dev_ptr(S, sg.h_rowshape))) {
      return fail(KBG_E_HIP, "hipHostGetDevicePointer of a stage buffer failed");
    }
    if (S.svc) return svc_launch(S, sg, a, G, base);
    a.info = dev_ptr(S, sg.h_down);
    a.masks = reinterpret_cast<kbg::MaskPair*>(dev_ptr(S, sg.h_down + fused_mask_off(S.K)));
    if (!a.info || !a.masks) return fail(KBG_E_HIP, "hipHostGetDevicePointer of a stage buffer failed");
    const bool avail = S.owner && S.comm;
    if (avail) {  // owner-resolve: the shapes' availability over the ranks, summed in the same round trip
      a.avail = S.d_down;
      a.avail_bit = 1u << S.shard;
    }
    sg.timed = !S.untimed_launches && S.ff_launch_seq++ % ff_time_every(S) == 0;
    HIP_TRY(kbg::launch_firstfit(a, S.int_mode ? 1 : 0, S.stream, sg.timed ? sg.ev[0] : nullptr,
                                 sg.timed ? sg.ev[1] : nullptr));
    trace_add("l.firstfit");

    if (avail) {
      const int32_t ns = sg.n_slots;
      if (S.comm->coll)  // (a communicator without a transport — R sessions of one process, tools — sums on the host)
        if (kbg_status st = coll_rc(S, S.comm->coll->allreduce(S.d_down, S.d_down, (size_t)ns, kbg::kCollSum, S.stream));
            st != KBG_OK)
          return st;
      HIP_TRY(hipMemcpyAsync(sg.h_down + fused_avail_off(S.K, a.mw), S.d_down, (size_t)ns * 4, hipMemcpyDeviceToHost,
                             S.stream));
    }
    HIP_TRY(hipEventRecord(sg.ev[6], S.stream));
    trace_add("l.event");
    sg.fused = true;
    sg.G = G;
    sg.base = base;
    sg.inflight = true;
    return KBG_OK;
  }
  sg.fused = false;
  // replicated sharded sessions (pod affinity, backfill on a communicator):
  // every rank scans its slot, the slots are all-gathered, every rank selects
  const uint32_t total = sg.h_capoff[G];
  const size_t up_bytes = (size_t)Gp * sizeof(kbg::TaskRec) + (size_t)(G + 1) * 4;
  const kbg::TaskRec* d_tasks = (const kbg::TaskRec*)S.d_up;
  const uint32_t* d_capoff = (const uint32_t*)(S.d_up + (size_t)Gp * sizeof(kbg::TaskRec));
  HIP_TRY(hipMemcpyAsync(S.d_up, sg.h_up, up_bytes, hipMemcpyHostToDevice, S.stream));
  trace_add("l.h2d", (int64_t)up_bytes);
  const kbg::ScanGeom geo{S.n_nodes, S.W, S.Wl, S.shard * S.Wl, S.Wl, S.tab_lo};  // this rank's slot
  const size_t slot_words = (size_t)2 * G * kbg::kbg_slot_words(S.Wl);
  uint64_t* out = S.d_bits + (size_t)S.shard * slot_words;
  HIP_TRY(kbg::launch_scan(S.d_nodes, geo, S.d_class_mask, d_tasks, G, S.pred_active ? 1 : 0, S.int_mode ? 1 : 0, out,
                           S.stream, sg.ev[0], sg.ev[1]));
  trace_add("l.scan");
  // in-place all-gather: every rank receives every shard's slot, in rank (= node) order
  HIP_TRY(hipEventRecord(sg.ev[4], S.stream));
  if (kbg_status st = coll_rc(S, S.comm->coll->allgather(out, S.d_bits, slot_words * 8, S.stream)); st != KBG_OK)
    return st;
  HIP_TRY(hipEventRecord(sg.ev[5], S.stream));
  HIP_TRY(kbg::launch_select(S.d_bits, 0, S.W, S.Wl, G, d_capoff, S.d_down + G, S.d_down, S.stream, sg.ev[2],
                             sg.ev[3]));
  trace_add("l.select");
  const size_t down = (size_t)G + total;
  HIP_TRY(hipMemcpyAsync(sg.h_down, S.d_down, down * 4, hipMemcpyDeviceToHost, S.stream));
  trace_add("l.d2h", (int64_t)down * 4);
  HIP_TRY(hipEventRecord(sg.ev[6], S.stream));
  trace_add("l.event");
  sg.G = G;
  sg.base = base;
  sg.inflight = true;
  return KBG_OK;
}

kbg_status device_wait(Session& S, kbg::Stage& sg) {
  if (kbg_status st = comm_wait(S, sg.ev[6]); st != KBG_OK) return st;
  sg.inflight = false;
  const int32_t G = sg.G;
  if (sg.fused) {
    sg.h_info = sg.h_down;
    if (sg.splits > 1) {
      // the parts' lists in node order: the slot's list covers the words of
      // every part up to and including the first that stopped at the row's
      // want before its last word (a complete walk: every word); it fits
      // somewhere if any part found a node
      const int32_t P = sg.splits;
      sg.info_comb.resize(sg.n_slots);
      for (int32_t sl = 0; sl < sg.n_slots; ++sl) {
        uint32_t any = 0, covered = 0;
        bool cut = false;
        for (int32_t p = 0; p < P; ++p) {
          const uint32_t v = sg.h_down[(size_t)sl * P + p];
          any |= v & kbg::kInfoAnyBit;
          if (cut) continue;
          covered += v & kbg::kInfoWordsMask;
          cut = (v & kbg::kCountIncompleteBit) != 0;
        }
        sg.info_comb[sl] = covered | (cut ? kbg::kCountIncompleteBit : 0u) | any;
      }
      sg.h_info = sg.info_comb.data();
    }
    sg.h_mask = reinterpret_cast<kbg::MaskPair*>(sg.h_down + fused_mask_off(S.K));
    sg.mw = fused_mask_words(S);
    sg.w_lo = S.owner ? S.shard * S.Wl : 0;
    sg.h_avail = sg.h_down + fused_avail_off(S.K, sg.mw);
  } else {
    sg.h_count = sg.h_down;
    sg.h_cand = sg.h_down + G;
  }
  float ms = 0;
  if (!sg.fused) {
    HIP_TRY(hipEventElapsedTime(&ms, sg.ev[0], sg.ev[1]));
    S.stats.scan_kernel_ms += ms;
  } else if (sg.timed) {
    HIP_TRY(hipEventElapsedTime(&ms, sg.ev[0], sg.ev[1]));
    S.ff_timed_ms += ms;
    S.ff_timed++;
  }
  if (!sg.fused) {
    HIP_TRY(hipEventElapsedTime(&ms, sg.ev[2], sg.ev[3]));
    S.stats.select_kernel_ms += ms;
  }
  if (S.comm && !S.owner && !sg.fused) {
    HIP_TRY(hipEventElapsedTime(&ms, sg.ev[4], sg.ev[5]));
    S.stats.exchange_ms += ms;
  }
  S.stats.scan_launches++;
  if (sg.fused && S.ff_timed) S.stats.scan_kernel_ms = S.ff_timed_ms / S.ff_timed * (double)S.stats.scan_launches;
  S.stats.evaluations += G;
  S.stats.node_visits += (int64_t)G * (S.comm ? S.tab_n : S.n_nodes);
  return KBG_OK;
}

// Results of a launch that will not be used (its batch was predicted before a
// cut): wait for it so its staging can be rewritten, keep the kernel times.
kbg_status device_drop(Session& S, kbg::Stage& sg) {
  if (!sg.inflight) return KBG_OK;
  return device_wait(S, sg);
}

// One synchronous device round trip (backfill, kbg_select).
kbg_status device_scan(Session& S, kbg::Stage& sg, int32_t G, int32_t base) {
  kbg_status st = device_launch(S, sg, G, base);
  return st != KBG_OK ? st : device_wait(S, sg);
}

#include "kbg_svc_link.ipp"  // the scan service's transport (SvcLink), its messages and the device side of a served launch

#include "kbg_open.ipp"  // session open: ingest, the host derive and the device build

#include "kbg_allocate.ipp"  // the allocate cycle: predictor, committer, truth engine

#include "kbg_owner.ipp"  // sharded allocate over the owner-resolve protocol

#include "kbg_svc.ipp"  // the scan service: rank 0 and the serving ranks

#include "kbg_victims.ipp"  // preempt / reclaim and their victim scans

#include "kbg_update.ipp"  // resident session updates (kbg_session_update)

}  // namespace

// ================================================================== C ABI
namespace {
// A session whose update failed part-way answers nothing but close.
kbg_status usable(kbg_session* s) {
  if (!s) return fail(KBG_E_INVALID, "null session");
  if (!s->s.broken.empty())
    return fail(KBG_E_INVALID, "the session is unusable after a failed kbg_session_update (" + s->s.broken + "): re-open it");
  return comm_alive(s->s);
}
}  // namespace

extern "C" {

int32_t kbg_abi_version(void) { return KBG_ABI_VERSION; }

const char* kbg_last_error(void) { return g_err.c_str(); }

int32_t kbg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

static kbg_status session_open(const kbg_snapshot* snap, const kbg_options* opts, kbg_comm* comm, kbg_session** out) {
  if (!out) return fail(KBG_E_INVALID, "null out");
  *out = nullptr;
  kbg_session* s = new (std::nothrow) kbg_session();
  if (!s) return fail(KBG_E_NOMEM, "session");
  kbg_status st;
  try {
    st = open_session(s->s, snap, opts, comm);
  } catch (const std::bad_alloc&) {
    st = fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {  // a derive worker's error, rethrown after its join
    st = fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
  if (st != KBG_OK) {
    free_device(s->s);
    delete s;
    return st;
  }
  *out = s;
  return KBG_OK;
}

kbg_status kbg_session_open(const kbg_snapshot* snap, const kbg_options* opts, kbg_session** out) {
  return session_open(snap, opts, nullptr, out);
}

kbg_status kbg_session_open_sharded(const kbg_snapshot* snap, const kbg_options* opts, kbg_comm* comm,
                                    kbg_session** out) {
  if (!comm) return fail(KBG_E_INVALID, "null communicator");
  if (comm->aborted.load())
    return fail(KBG_E_RCCL, "the communicator was aborted after a failure on a rank: destroy it and re-create it");
  return session_open(snap, opts, comm, out);
}

kbg_status kbg_allocate(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  HIP_TRY(hipSetDevice(s->s.device));
  try {
    if (scan_service_ok(s->s)) {
      if (!s->s.svc_own) {  // pinned ring and device buffer, kept for the session's later cycles
        std::unique_ptr<CommSvc> link(new CommSvc(s->s));
        if (kbg_status st = link->init(); st != KBG_OK) {
          comm_abort(s->s.comm);  // the other ranks are about to wait on this rank's messages or sums
          return st;
        }
        s->s.svc_own = link.release();
      }
      SvcLink& link = *s->s.svc_own;
      return s->s.shard == 0 ? allocate_svc_root(s->s, link, out, cap, n_out)
                             : allocate_serve(s->s, link, out, cap, n_out);
    }
    if (owner_resolve_ok(s->s)) {
      RcclIO io(s->s);
      return allocate_sharded(s->s, io, out, cap, n_out);
    }
    return allocate_cycle(s->s, out, cap, n_out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
}

kbg_status kbg_backfill(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  HIP_TRY(hipSetDevice(s->s.device));
  try {
    return backfill_cycle(s->s, out, cap, n_out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
}

kbg_status kbg_reclaim(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  HIP_TRY(hipSetDevice(s->s.device));
  try {
    return reclaim_cycle(s->s, out, cap, n_out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
}

kbg_status kbg_preempt(kbg_session* s, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  HIP_TRY(hipSetDevice(s->s.device));
  try {
    return preempt_cycle(s->s, out, cap, n_out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
}

kbg_status kbg_evictions_get(kbg_session* s, kbg_eviction* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  const auto& ev = s->s.evictions;
  if (n_out) *n_out = (int32_t)ev.size();
  if (!out && cap == 0) return KBG_OK;  // size query
  if ((int32_t)ev.size() > cap || (!out && !ev.empty()))
    return fail(KBG_E_CAPACITY, "eviction buffer too small: need " + std::to_string(ev.size()));
  if (!ev.empty()) std::memcpy(out, ev.data(), ev.size() * sizeof(kbg_eviction));
  return KBG_OK;
}

kbg_status kbg_decision_actions_get(kbg_session* s, int32_t* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  const auto& a = s->s.dec_action;
  if (n_out) *n_out = (int32_t)a.size();
  if (!out && cap == 0) return KBG_OK;  // size query
  if ((int32_t)a.size() > cap || (!out && !a.empty()))
    return fail(KBG_E_CAPACITY, "action buffer too small: need " + std::to_string(a.size()));
  if (!a.empty()) std::memcpy(out, a.data(), a.size() * sizeof(int32_t));
  return KBG_OK;
}

namespace {
// kbg_session_reset's body (also the tools' repeated sharded cycles)
kbg_status session_reset(Session& S) {
  HIP_TRY(hipSetDevice(S.device));
  S.idle = S.idle0;
  S.rel = S.rel0;
  S.ntasks = S.ntasks0;
  S.allocated = S.backfilled = S.reclaimed = S.preempted = S.cycle_started = false;
  S.node_keys = S.node_keys0;
  S.port_hold.clear();
  S.port_gone.clear();
  S.outsider_gone.clear();
  S.key_holder.clear();
  if (S.has_ports || S.has_aff) {  // the class masks carry the port fit / affinity: back to the snapshot's
    S.node_ports = S.node_ports0;
    S.h_class_mask = S.h_class_mask0;
    S.mask_dirty.clear();
    std::fill(S.mask_dirty_flag.begin(), S.mask_dirty_flag.end(), 0);
    HIP_TRY(hipMemcpyAsync(S.d_class_mask, S.h_class_mask.data(), S.h_class_mask.size() * 8, hipMemcpyHostToDevice,
                           S.stream));
  }
  kbg_status st = copy_soa(S, S.d_nodes, S.d_nodes0);
  if (st != KBG_OK) return st;
  HIP_TRY(hipStreamSynchronize(S.stream));
  return KBG_OK;
}
}  // namespace

kbg_status kbg_session_reset(kbg_session* s) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  return session_reset(s->s);
}

kbg_status kbg_session_update(kbg_session* s, const kbg_event* events, int32_t n) {
  if (kbg_status st = usable(s); st != KBG_OK) return st;
  Session& S = s->s;
  HIP_TRY(hipSetDevice(S.device));
  if (n < 0 || (n > 0 && !events)) return fail(KBG_E_INVALID, "events");
  kbg_status st;
  try {
    st = update_precheck(S, events, n);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");  // before the first event: the session is unchanged
  }
  if (st != KBG_OK) return st;  // refused: nothing changed
  try {
    st = session_update(S, events, n);
  } catch (const std::bad_alloc&) {
    st = fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::exception& e) {  // a derive worker's error, rethrown after its join
    st = fail(KBG_E_INVALID, std::string("internal: ") + e.what());
  }
  if (st != KBG_OK) S.broken = g_err;  // events were applied part-way
  return st;
}

kbg_status kbg_session_renumbering(kbg_session* s, int32_t kind, int32_t* out, int32_t cap, int32_t* n_out) {
  if (kbg_status st = usable(s); st != KBG_OK) return st;
  if (kind < KBG_RENUM_TASKS || kind > KBG_RENUM_QUEUES) return fail(KBG_E_INVALID, "renumbering kind");
  const std::vector<int32_t>& r = s->s.renum[kind];
  if (n_out) *n_out = (int32_t)r.size();
  if (!out && cap == 0) return KBG_OK;  // size query
  if ((int32_t)r.size() > cap || (!out && !r.empty()))
    return fail(KBG_E_CAPACITY, "renumbering buffer too small: need " + std::to_string(r.size()));
  if (!r.empty()) std::memcpy(out, r.data(), r.size() * sizeof(int32_t));
  return KBG_OK;
}

kbg_status kbg_select(kbg_session* s, const int32_t* tasks, int32_t n, int32_t stop_at_first_success, int32_t* out_node,
                      int32_t* out_kind, int32_t* n_evaluated) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (n > 0 && (!tasks || !out_node)) return fail(KBG_E_INVALID, "null argument");
  Session& S = s->s;
  HIP_TRY(hipSetDevice(S.device));
  for (int32_t i = 0; i < n; ++i)
    if (tasks[i] < 0 || tasks[i] >= S.n_tasks || !S.pending_candidate[tasks[i]])
      return fail(KBG_E_INVALID, "task index (must be a Pending, non-BestEffort session task)");
  std::vector<int32_t> mark(S.n_nodes, -1), touched, bt;
  Grouper grouper(S);
  Resolver rs{S, mark};
  kbg::Stage& sg = S.stages[0];
  int32_t done = 0;
  bool stop = false;
  while (done < n && !stop) {
    const int32_t cnt = std::min(n - done, S.K);
    bt.assign(tasks + done, tasks + done + cnt);
    const int32_t G = grouper.build(sg, bt.data(), cnt);
    kbg_status st = device_scan(S, sg, G, S.res_stamp);  // every earlier commit is in the table
    if (st != KBG_OK) return st;
    touched.clear();
    rs.reset(sg);
    const int32_t rstamp = ++S.res_stamp;
    S.mstamp = rstamp;
    int32_t i = 0;
    for (; i < cnt; ++i) {
      int32_t node = -1, kind = 0;
      const int r = rs.resolve(sg.row_of[i], bt[i], &node, &kind);
      if (r == RES_TRUNC) break;  // rescan from this task with the updated table
      if (r == RES_PANIC) {
        if ((st = push_deltas(S, touched)) != KBG_OK) return st;
        HIP_TRY(hipStreamSynchronize(S.stream));
        if (n_evaluated) *n_evaluated = done + i;
        return fail(KBG_E_REF_PANIC, "node with nil Node reached (predicates.go:122-123)");
      }
      out_node[done + i] = node;
      if (out_kind) out_kind[done + i] = kind;
      if (node >= 0) {
        mirror_add(S, bt[i], node, kind);
        if (mark[node] != rstamp) {
          mark[node] = rstamp;
          touched.push_back(node);
        }
        if (stop_at_first_success) {
          ++i;
          stop = true;
          break;
        }
        if (!S.aff_gain_classes.empty()) {  // pod affinity gave a class nodes: rescan the rest
          for (int32_t c : S.aff_gain_classes) S.aff_gain_flag[c] = 0;
          S.aff_gain_classes.clear();
          ++i;
          break;
        }
      }
    }
    if ((st = push_deltas(S, touched)) != KBG_OK) return st;
    done += i;
  }
  HIP_TRY(hipStreamSynchronize(S.stream));
  if (n_evaluated) *n_evaluated = done;
  return KBG_OK;
}

kbg_status kbg_apply(kbg_session* s, int32_t node, const kbg_resource* req, int32_t kind) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (!req) return fail(KBG_E_INVALID, "null argument");
  Session& S = s->s;
  if (node < 0 || node >= S.n_nodes) return fail(KBG_E_INVALID, "node index");
  HIP_TRY(hipSetDevice(S.device));
  const Res r = to_res(*req);
  if (!S.nil_node[node]) {
    Res& target = kind == KBG_KIND_PIPELINE ? S.rel[node] : S.idle[node];
    if (!kbg::res_sub(target, r)) return fail(KBG_E_REF_PANIC, "Resource.Sub underflow (resource_info.go:100-110)");
  }
  S.ntasks[node]++;
  kbg_status st = push_deltas(S, std::vector<int32_t>{node});
  if (st != KBG_OK) return st;
  HIP_TRY(hipStreamSynchronize(S.stream));
  return KBG_OK;
}

kbg_status kbg_job_state_get(kbg_session* s, int32_t job, kbg_job_state* out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (!out) return fail(KBG_E_INVALID, "null argument");
  Session& S = s->s;
  if (job < 0 || job >= S.n_jobs) return fail(KBG_E_INVALID, "job index");
  const Engine& E = S.cycle_started ? S.fin : S.init;
  out->ready_num = S.cycle_started ? S.committed_ready[job] : S.job_ready0[job];
  out->ready = out->ready_num >= S.jobs_in[job].min_available ? 1 : 0;  // gang jobReady (gang.go:72-78)
  out->drf_share = S.has_drf ? E.jshare[job] : 0.0;
  out->drf_allocated = to_kres(E.jalloc[job]);
  out->fit_valid = out->fit_nodes = out->fit_cpu = out->fit_memory = out->fit_gpu = 0;
  // gang reports FitError for jobs not ready at session close (gang.go:169-190);
  // NodesFitDelta comes from allocate only (empty when it did not run)
  if (S.cycle_started && out->ready_num < S.jobs_in[job].min_available && (size_t)job < S.fit.size()) {
    out->fit_valid = 1;
    out->fit_nodes = S.fit[job].nodes;
    out->fit_cpu = S.fit[job].cpu;
    out->fit_memory = S.fit[job].mem;
    out->fit_gpu = S.fit[job].gpu;
  }
  return KBG_OK;
}

kbg_status kbg_queue_state_get(kbg_session* s, int32_t queue, kbg_queue_state* out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (!out) return fail(KBG_E_INVALID, "null argument");
  Session& S = s->s;
  if (queue < 0 || queue >= S.n_queues) return fail(KBG_E_INVALID, "queue index");
  const Engine& E = S.cycle_started ? S.fin : S.init;
  out->has_attr = S.has_prop && S.q_has_attr[queue];
  out->share = E.qshare[queue];
  out->deserved = to_kres(S.q_deserved[queue]);
  out->allocated = to_kres(E.qalloc[queue]);
  out->request = to_kres(S.q_request[queue]);
  out->overused = out->has_attr && kbg::res_le(S.q_deserved[queue], E.qalloc[queue]);
  return KBG_OK;
}

kbg_status kbg_node_state_get(kbg_session* s, int32_t node, kbg_node_state* out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (!out) return fail(KBG_E_INVALID, "null argument");
  Session& S = s->s;
  if (node < 0 || node >= S.n_nodes) return fail(KBG_E_INVALID, "node index");
  out->idle = to_kres(S.idle[node]);
  out->releasing = to_kres(S.rel[node]);
  out->num_tasks = S.ntasks[node];
  return KBG_OK;
}

kbg_status kbg_stats_get(kbg_session* s, kbg_stats* out) {
  if (kbg_status st_ = usable(s); st_ != KBG_OK) return st_;
  if (!out) return fail(KBG_E_INVALID, "null argument");
  *out = s->s.stats;
  return KBG_OK;
}

void kbg_session_close(kbg_session* s) {
  if (!s) return;
  (void)hipSetDevice(s->s.device);
  free_device(s->s);
  delete s;
}

}  // extern "C"

#include "kbg_wire.ipp"  // the snapshot wire format
