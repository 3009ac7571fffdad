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
template <class T>
kbg_status dalloc(Session& S, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  HIP_TRY(hipMalloc(&q, count * sizeof(T)));
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
  HIP_TRY(hipHostMalloc(p, std::max<size_t>(bytes, 64), hipHostMallocMapped | hipHostMallocCoherent));  // never 0 B
  return KBG_OK;
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
    if (g.h_up) (void)hipHostFree(g.h_up);
    if (g.h_down) (void)hipHostFree(g.h_down);
    for (auto& e : g.ev)
      if (e) {
        (void)hipEventDestroy(e);
        e = nullptr;
      }
    g = kbg::Stage{};
  }
  for (char* b : S.up_pool) (void)hipHostFree(b);
  S.up_pool.clear();
  if (S.h_deltas) (void)hipHostFree(S.h_deltas);
  if (S.h_mdeltas) (void)hipHostFree(S.h_mdeltas);
  S.h_mdeltas = nullptr;
  if (S.fit_h) (void)hipHostFree(S.fit_h);
  if (S.fit_out) (void)hipHostFree(S.fit_out);
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
  for (void* p : S.d_allocs) (void)hipFree(p);
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

// ============================================ the scan service: transport
// Sharded allocate as ONE committer: rank 0 runs the single-GPU
// pipeline (ordering engine, in-order commit, overlapped and reused scans)
// and every scan it launches is a message to the other ranks: the launch's
// arguments, the node rows and class-mask words its commits wrote since the
// last message (every rank writes the rows it holds), and the committed
// outcomes (each rank replays them into its mirror, decision log and engine,
// beside its scans). Every rank runs the fused kernel over its own words into
// a zeroed (slot, rank) info array and a [slot][W] mask array; one summing
// all-reduce over the ranks (disjoint words: the sum is the union) gives rank
// 0 the whole table's lists, joined in node order like a split launch's
// parts. Rank 0's collectives are enqueued on its stream (no host wait); the
// other ranks wait for each message.

enum : uint32_t { kSvcLaunch = 0, kSvcEnd = 1, kSvcAbort = 2, kSvcState = 3 };
constexpr size_t kSvcHead = 16;          // header words: kind, words, nodes, masks, outcomes, args, shapes, rowshape,
                                         // status, G, slots
constexpr size_t kSvcMaxWords = 1u << 19;  // one message (2 MB); a longer state goes out in kSvcState chunks
constexpr size_t kSvcNodeWords = sizeof(kbg::NodeDelta) / 4, kSvcMaskWords = sizeof(kbg::MaskDelta) / 4;
constexpr size_t kSvcStreamWords = 2 * 2048;  // rank 0 streams its commits once this many words wait
static_assert(sizeof(kbg::NodeDelta) % 4 == 0 && sizeof(kbg::MaskDelta) % 4 == 0, "message words");

inline void svc_put(std::vector<uint32_t>& m, const void* p, size_t bytes) {
  const size_t o = m.size();
  m.resize(o + (bytes + 3) / 4, 0u);
  if (bytes) std::memcpy(&m[o], p, bytes);
}

// Rank 0: the pending state (rows, mask words, outcomes) in messages of kind
// `kind` (kSvcState chunks first when it does not fit into one message with
// `reserve` more words); leaves the last part for the caller when `keep` is set.
kbg_status svc_flush_state(Session& S, std::vector<uint32_t>& m, size_t reserve, bool keep, uint32_t kind,
                           uint32_t status) {
  size_t ni = 0, mi = 0, oi = 0;
  for (;;) {
    const size_t room = kSvcMaxWords - kSvcHead - reserve;
    const size_t nn = std::min(S.svc_nodes.size() - ni, room / kSvcNodeWords);
    const size_t nm = std::min(S.svc_masks.size() - mi, (room - nn * kSvcNodeWords) / kSvcMaskWords);
    const size_t no = std::min((S.svc_out.size() - oi) / 2,
                               (room - nn * kSvcNodeWords - nm * kSvcMaskWords) / 2);
    const bool last = ni + nn == S.svc_nodes.size() && mi + nm == S.svc_masks.size() && oi + 2 * no == S.svc_out.size();
    m.assign(kSvcHead, 0u);
    m[0] = last ? kind : kSvcState;
    m[2] = (uint32_t)nn;
    m[3] = (uint32_t)nm;
    m[4] = (uint32_t)no;
    m[8] = status;
    svc_put(m, S.svc_nodes.data() + ni, nn * sizeof(kbg::NodeDelta));
    svc_put(m, S.svc_masks.data() + mi, nm * sizeof(kbg::MaskDelta));
    svc_put(m, S.svc_out.data() + oi, no * 8);
    ni += nn;
    mi += nm;
    oi += 2 * no;
    if (last && keep) break;  // the caller appends its part and sends
    m[1] = (uint32_t)m.size();
    if (kbg_status st = S.svc->send(S, m.data()); st != KBG_OK) return st;
    if (last) break;
  }
  S.svc_nodes.clear();
  S.svc_masks.clear();
  S.svc_out.clear();
  return KBG_OK;
}

// Rank 0's part of a scan: the launch message, its own words, the sum.
kbg_status svc_launch(Session& S, kbg::Stage& sg, kbg::FirstFitArgs& a, int32_t G, int32_t base) {
  const int32_t ns = sg.n_slots;
  // the arguments go out before this rank's words are set in them (each rank sets its own)
  const size_t args_w = (sizeof(kbg::FirstFitArgs) + 3) / 4;
  const size_t shapes_w = a.shapes ? ((size_t)ns * sizeof(kbg::TaskRec) + 3) / 4 : 0;
  const size_t rows_w = a.row_shape ? (size_t)G : 0;
  thread_local std::vector<uint32_t> m;
  if (kbg_status st = svc_flush_state(S, m, args_w + shapes_w + rows_w, true, kSvcLaunch, 0); st != KBG_OK) return st;
  m[5] = (uint32_t)args_w;
  m[6] = (uint32_t)shapes_w;
  m[7] = (uint32_t)rows_w;
  m[9] = (uint32_t)G;
  m[10] = (uint32_t)ns;
  // payload order: args, shapes, rows, then the state svc_flush_state put
  std::vector<uint32_t> state(m.begin() + kSvcHead, m.end());
  m.resize(kSvcHead);
  svc_put(m, &a, sizeof(kbg::FirstFitArgs));
  if (shapes_w) svc_put(m, sg.h_shapes, (size_t)ns * sizeof(kbg::TaskRec));
  if (rows_w) svc_put(m, sg.h_rowshape, (size_t)G * 4);
  m.insert(m.end(), state.begin(), state.end());
  m[1] = (uint32_t)m.size();
  if (kbg_status st = S.svc->send(S, m.data()); st != KBG_OK) return st;
  // this rank's words, every rank's info column and the whole mask width
  a.w_lo = std::min(S.W, S.shard * S.Wl);
  a.w_hi = std::min(S.W, (S.shard + 1) * S.Wl);
  a.splits = 1;
  a.split_words = a.w_hi - a.w_lo;
  a.info_stride = S.R;
  a.part0 = S.shard;
  a.mask_w0 = 0;
  a.mw = S.W;
  a.complete = a.w_hi - a.w_lo <= kbg::kFfRoundWords ? 1 : 0;
  a.avail = nullptr;
  a.info = S.d_svc;
  a.masks = reinterpret_cast<kbg::MaskPair*>(S.d_svc + fused_mask_off(S.K));
  const size_t info_w = (size_t)ns * S.R, mask_w = (size_t)ns * S.W * 4;
  HIP_TRY(hipMemsetAsync(S.d_svc, 0, info_w * 4, S.stream));
  HIP_TRY(hipMemsetAsync(a.masks, 0, mask_w * 4, S.stream));
  sg.timed = !S.untimed_launches && S.ff_launch_seq++ % ff_time_every(S) == 0;
  HIP_TRY(kbg::launch_firstfit(a, S.int_mode ? 1 : 0, S.stream, sg.timed ? sg.ev[0] : nullptr,
                               sg.timed ? sg.ev[1] : nullptr));
  trace_add("l.firstfit");
  if (kbg_status st = S.svc->sum(S, &sg, info_w, mask_w); st != KBG_OK) return st;
  HIP_TRY(hipEventRecord(sg.ev[6], S.stream));
  sg.splits = S.R;  // device_wait joins the ranks' parts in node order
  sg.fused = true;
  sg.G = G;
  sg.base = base;
  sg.inflight = true;
  return KBG_OK;
}

kbg_status svc_sum_counts(Session& S, int32_t* counts, size_t n) {
  return S.svc->sum_host(S, reinterpret_cast<uint32_t*>(counts), n);
}

// Writes the rows of the nodes touched by the last commits back to HBM (only
// the rows this process holds; every shard's host mirror saw every commit).
// The pinned staging buffers (h_deltas, h_mdeltas, h_sdeltas) are read by
// the stream when a copy or kernel executes, not when it is enqueued, and the
// stream may still be behind (a scan enqueued earlier runs first): a writer
// waits for the last reader (stage_acquire) and every enqueued reader marks
// the stream (stage_release).
kbg_status stage_acquire(Session& S) {
  if (S.stage_pending) {
    HIP_TRY(hipEventSynchronize(S.stage_ev));
    S.stage_pending = false;
  }
  return KBG_OK;
}
kbg_status stage_release(Session& S) {
  HIP_TRY(hipEventRecord(S.stage_ev, S.stream));
  S.stage_pending = true;
  return KBG_OK;
}

// Class-mask words changed on the host (host ports, pod affinity) into HBM;
// every shard holds the whole mask.
kbg_status push_mask_deltas(Session& S) {
  for (size_t m = 0; m < S.mask_dirty.size();) {
    kbg_status st = stage_acquire(S);
    if (st != KBG_OK) return st;
    const int32_t cnt = (int32_t)std::min<size_t>(S.mask_dirty.size() - m, (size_t)kbg::kMaskDeltaCap);
    for (int32_t k = 0; k < cnt; ++k) {
      const uint32_t idx = S.mask_dirty[m + k];
      S.h_mdeltas[k] = kbg::MaskDelta{idx, 0u, S.h_class_mask[idx]};
      S.mask_dirty_flag[idx] = 0;
    }
    if (S.svc) S.svc_masks.insert(S.svc_masks.end(), S.h_mdeltas, S.h_mdeltas + cnt);  // for every rank's table
    const kbg::MaskDelta* md = dev_ptr(S, S.h_mdeltas);
    if (!md) return fail(KBG_E_HIP, "hipHostGetDevicePointer of the mask-delta buffer failed");
    HIP_TRY(kbg::launch_mask_apply(S.d_class_mask, md, cnt, S.stream));  // read in place
    if ((st = stage_release(S)) != KBG_OK) return st;
    m += cnt;
  }
  S.mask_dirty.clear();
  return KBG_OK;
}

kbg_status push_deltas(Session& S, const std::vector<int32_t>& touched) {
  kbg_status st = push_mask_deltas(S);
  if (st != KBG_OK) return st;
  if (S.svc)  // the scan service: every rank's rows go out with the next message (each rank writes its own)
    for (const int32_t n : touched) {
      kbg::NodeDelta d{};
      d.node = n;
      device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
      S.svc_nodes.push_back(d);
    }
  size_t i = 0;
  while (i < touched.size()) {
    if ((st = stage_acquire(S)) != KBG_OK) return st;
    int32_t cnt = 0;
    for (; i < touched.size() && cnt < S.K; ++i) {
      const int32_t n = touched[i];
      if (n < S.tab_lo || n >= S.tab_lo + S.tab_n) continue;
      kbg::NodeDelta& d = S.h_deltas[cnt++];
      d.node = n - S.tab_lo;
      device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
    }
    if (cnt == 0) break;
    HIP_TRY(kbg::launch_apply(S.d_nodes, S.h_deltas_dev, cnt, S.stream));  // read in place
    if ((st = stage_release(S)) != KBG_OK) return st;
  }
  return KBG_OK;
}

// Groups the tasks of a batch into device rows and sizes their candidate
// lists. Full-scan mode: one row per task (every evaluation scans the whole
// table — the SURVEY §8(d) roofline rule) with M + r slots, r = the number of
// earlier rows of the same (class, request) shape in this scan: each earlier
// commit can exhaust at most one node of the list, so a row rarely runs out
// before the table does. Grouped mode: one row per distinct shape with (tasks
// of the shape + slack) slots; tasks of a shape share the row and a cursor.
constexpr int32_t kGroupSlack = 512;     // extra candidate slots per shape row (grouped mode)
constexpr int32_t kContendedSlack = 4096;  // the same in a rescan of the contended part of a cycle
constexpr int32_t kFullScanGrow = 1024;  // cap on a full-scan row's extra slots
constexpr int32_t kFullScanK = 8192;     // default batch of the full-scan mode

// Bytes of one stage's row buffer for batches of K tasks: the rows
// (TaskRec, padded) and their candidate offsets, then (fused full-scan path)
// each row's shape slot and the shape table.
inline size_t up_bytes_for(int32_t K) {
  const size_t rows = (size_t)kbg::kbg_pad_rows(K) * sizeof(kbg::TaskRec) + ((size_t)K + 1) * 4;
  return ((rows + 15) & ~(size_t)15) + (((size_t)K * 4 + 15) & ~(size_t)15) + (size_t)K * sizeof(kbg::TaskRec);
}

// A row whose scan found no fitting node in a complete walk of the table.
inline bool row_fits_nowhere(const kbg::Stage& g, int32_t r) {
  if (g.fused) return (g.h_info[g.row_slot[r]] & (kbg::kInfoAnyBit | kbg::kCountIncompleteBit)) == 0;
  return g.h_count[r] == 0;
}
// A row with some fitting node in the words its scan covered (listed or not).
inline bool row_fits_somewhere(const kbg::Stage& g, int32_t r) {
  if (g.fused) return (g.h_info[g.row_slot[r]] & kbg::kInfoAnyBit) != 0;
  return g.h_count[r] != 0;
}

struct Grouper {
  Session& S;
  std::vector<int32_t> shape_row, shape_stamp, count, ext_slot;
  int32_t stamp = 0;
  explicit Grouper(Session& s) : S(s), shape_row(s.n_shapes, -1), shape_stamp(s.n_shapes, -1) {}
  // `slack`: grouped mode's extra candidate slots per shape row (the
  // contended part of a cycle asks for long lists: few nodes still fit a
  // shape there, and a list that holds all of them needs no rescan to
  // learn that the shape fits nowhere)
  int32_t build(kbg::Stage& sg, const int32_t* bt, int32_t n, int32_t slack = kGroupSlack) {
    sg.h_tasks = (kbg::TaskRec*)sg.h_up;
    ++stamp;
    sg.row_of.resize(n);
    sg.row_shape.clear();
    count.clear();
    int32_t G = 0;
    for (int32_t i = 0; i < n; ++i) {
      const int32_t t = bt[i];
      int32_t g;
      const int32_t sh = S.task_shape[t];
      const bool seen = shape_stamp[sh] == stamp;
      if (!S.opts.full_scan && seen) {
        g = shape_row[sh];
      } else {
        g = G++;
        // full-scan: count[g] = earlier rows of this shape in the scan (the list grows with them)
        count.push_back(S.opts.full_scan && seen ? count[shape_row[sh]] + 1 : 0);
        shape_stamp[sh] = stamp;
        shape_row[sh] = g;
        sg.row_shape.push_back(sh);
        kbg::TaskRec& r = sg.h_tasks[g];
        const Res& q = S.treq[t];
        if (S.be_task[t]) {  // backfill: PredicateFn only — every node fits (a > -inf in both modes)
          r.req[0] = r.req[1] = r.req[2] = -INFINITY;
        } else if (S.int_mode) {  // thresholds: LessEqual(q, a) == (a > q - min), exact (kbg_device.hpp)
          r.req[0] = q.c - kbg::kMinMilliCPU;
          r.req[1] = q.m - kbg::kMinMemory;
          r.req[2] = q.g - kbg::kMinMilliGPU;
        } else {
          r.req[0] = q.c;
          r.req[1] = q.m;
          r.req[2] = q.g;
        }
        r.cls = S.task_class[t];
        r.flags = (S.be_task[t] || kbg::res_le(q, Res{})) ? kbg::kRowRelZeroFits : 0;
      }
      sg.row_of[i] = g;
      if (!S.opts.full_scan) count[g]++;
    }
    const int32_t Gp = kbg::kbg_pad_rows(G);
    for (int32_t g = G; g < Gp; ++g) sg.h_tasks[g] = sg.h_tasks[0];  // padding rows: scanned, never stored
    sg.h_capoff = (uint32_t*)(sg.h_up + (size_t)Gp * sizeof(kbg::TaskRec));
    sg.h_capoff[0] = 0;
    // full-scan: rows of one shape in one scan evaluate identical inputs
    // against the same table, so their lists are one sequence. Every row is
    // evaluated against the whole table on the device; the list is written
    // once, for the shape's last row (a long list: every commit before it can
    // exhaust one node), and the shape's other rows read it (Resolver).
    if (S.opts.full_scan) {
      sg.row_ext.resize(G);
      for (int32_t g = 0; g < G; ++g) sg.row_ext[g] = shape_row[sg.row_shape[g]];
    }
    int32_t grow_cap = kFullScanGrow;
    if (S.opts.full_scan) {  // more shapes than the buffers were sized for: shorter long lists
      int64_t longs = 0;
      for (int32_t g = 0; g < G; ++g) longs += sg.row_ext[g] == g;
      const int64_t spare = S.cand_cap - (int64_t)G * S.M;
      if (longs * kFullScanGrow > spare) grow_cap = (int32_t)std::max<int64_t>(0, spare / std::max<int64_t>(1, longs));
    }
    if (!S.opts.full_scan && slack > kGroupSlack) {  // within the candidate buffer (sized for K x (kGroupSlack + 1))
      const int64_t room = (S.cand_cap - n) / std::max(1, G);
      slack = (int32_t)std::max<int64_t>(kGroupSlack, std::min<int64_t>(slack, room));
    }
    const int32_t cap_want = std::max(4096, slack);
    for (int32_t g = 0; g < G; ++g) {
      uint32_t want;
      if (!S.opts.full_scan) want = (uint32_t)std::min(count[g] + slack, cap_want);
      else if (sg.row_ext[g] != g) want = 0;  // its list is the shape's long one (Resolver: alias rows)
      else want = (uint32_t)(S.M + std::min(2 * count[g] + (g >> 3) + 64, grow_cap));
      sg.h_capoff[g + 1] = sg.h_capoff[g] + want;
      // the fused kernel reads the row's want from its flags (kbg_device.hpp FirstFitArgs)
      sg.h_tasks[g].flags = (sg.h_tasks[g].flags & kbg::kRowRelZeroFits) | (int32_t)(want << kbg::kRowWantShift);
    }
    // Fused path: grouped rows are their own shapes; full-scan rows name the
    // slot of their shape (the shape's last row, which writes the list; the
    // shape table holds that row's record, so no launch reads all G records)
    sg.row_slot.resize(G);
    if (S.opts.full_scan) {
      const size_t rows_b = ((size_t)Gp * sizeof(kbg::TaskRec) + ((size_t)G + 1) * 4 + 15) & ~(size_t)15;
      sg.h_rowshape = (uint32_t*)(sg.h_up + rows_b);
      sg.h_shapes = (kbg::TaskRec*)(sg.h_up + rows_b + (((size_t)G * 4 + 15) & ~(size_t)15));
      ext_slot.resize(G);
      int32_t ns = 0;
      for (int32_t g = 0; g < G; ++g)
        if (sg.row_ext[g] == g) {
          ext_slot[g] = ns;
          sg.h_shapes[ns++] = sg.h_tasks[g];
        }
      sg.slot_rows.assign(ns, 0);
      for (int32_t g = 0; g < G; ++g) {
        const int32_t sl = ext_slot[sg.row_ext[g]];
        sg.row_slot[g] = sl;
        sg.h_rowshape[g] = (uint32_t)sl | (sg.row_ext[g] == g ? kbg::kRowWriter : 0u);
        sg.slot_rows[sl]++;
      }
      sg.n_slots = ns;
    } else {
      for (int32_t g = 0; g < G; ++g) sg.row_slot[g] = g;
      sg.h_rowshape = nullptr;
      sg.h_shapes = sg.h_tasks;
      sg.n_slots = G;
      sg.slot_rows.clear();
    }
    return G;
  }
};

// In-order commit against the candidate lists of one scan. A node the list
// names is taken as it is unless a resolution newer than the scan touched it
// (mark > base: resources, pod count, or a class-mask bit it lost); those are
// re-checked on the host mirror. A row's cursor only moves forward: a
// candidate found infeasible for a (class, request) shape stays infeasible
// for every later task of that shape (monotonicity). In full-scan mode every
// task has its own row, and rows of one shape in one scan hold the same list
// (same inputs, same table): the prefix an earlier row of the shape rejected
// is skipped instead of re-checked (`shape_skip`).
enum { RES_OK = 0, RES_TRUNC = 1, RES_PANIC = 2 };
// The in-order commit's view of one node, in one cache line: what a
// re-check of a candidate touched since its scan reads (Idle, Releasing, pod
// count and cap, the stamp of the node's last commit, the nil-Node panic
// flag), instead of five separate arrays. The allocate committer keeps it
// current with every commit (mirror_row).
struct alignas(64) MirrorRow {
  double ic, im, ig, rc, rm, rg;
  int32_t nt, mt;
  int32_t mark;
  int32_t panic;
};
static_assert(sizeof(MirrorRow) == 64, "one cache line per node");
inline void mirror_row(const Session& S, MirrorRow& q, int32_t nd) {
  q.ic = S.idle[nd].c;
  q.im = S.idle[nd].m;
  q.ig = S.idle[nd].g;
  q.rc = S.rel[nd].c;
  q.rm = S.rel[nd].m;
  q.rg = S.rel[nd].g;
  q.nt = S.ntasks[nd];
}
struct Resolver {
  Session& S;
  std::vector<int32_t>& mark;
  const kbg::Stage* sg = nullptr;
  int32_t base = 0;
  std::vector<int32_t> cursor;
  std::vector<int32_t> shape_skip, skip_stamp;
  int32_t skip_gen = 0;
  // per shape, the first node not yet found infeasible this action (nullptr:
  // off). Nodes only lose room while an allocate runs (a pod-affinity gain
  // resets its class's shapes), so what a shape rejected under one scan
  // stays rejected under every later scan: a fresh stage's cursor starts
  // there instead of re-checking the nodes the earlier batches filled.
  int32_t* floor = nullptr;
  // the committer's packed mirror (nullptr: the separate arrays and `mark`)
  const MirrorRow* rows = nullptr;
  void reset(const kbg::Stage& stage) {
    sg = &stage;
    base = stage.base;
    cursor.assign(stage.G, 0);
    if (S.opts.full_scan) {
      if (shape_skip.size() < (size_t)S.n_shapes) {
        shape_skip.assign(S.n_shapes, 0);
        skip_stamp.assign(S.n_shapes, -1);
      }
      ++skip_gen;
    }
  }
  bool dirty(int32_t t, int32_t nd) const {
    return mark[nd] > base || (S.has_aff && S.mwmark[(size_t)S.task_class[t] * S.W + (nd >> 6)] > base);
  }
  // the host mirror's verdict on node nd for task t, for a candidate touched
  // since the scan: 1 Allocate, 2 Pipeline, 0 it no longer fits
  int recheck(int32_t t, int32_t nd, const Res& r) const {
    if (S.pred_active && S.ntasks[nd] >= S.maxtasks[nd]) return 0;
    if ((S.has_ports || S.has_aff) &&
        !((S.h_class_mask[(size_t)S.task_class[t] * S.W + (nd >> 6)] >> (nd & 63)) & 1ull))
      return 0;
    if (S.be_task[t]) return 1;  // backfill: PredicateFn only, always ssn.Allocate
    if (kbg::res_le(r, S.idle[nd])) return 1;
    if (kbg::res_le(r, S.rel[nd])) return 2;
    return 0;
  }
  // Fused stages: the row's shape list as word masks (kbg_device.hpp
  // FirstFitArgs); the cursor is the next node to look at, in node order.
  int resolve_mask(int32_t g, int32_t t, int32_t* node, int32_t* kind) {
    const int32_t sl = sg->row_slot[g];
    const uint32_t info = sg->h_info[sl];
    const int32_t wl = sg->w_lo;
    const kbg::MaskPair* m = sg->h_mask + (size_t)sl * sg->mw - wl;  // indexed by global word
    const int32_t end = (wl + (int32_t)(info & kbg::kInfoWordsMask)) * 64;
    const Res& r = S.treq[t];
    int32_t sh = -1;
    int32_t& k = cursor[g];
    if (k < wl * 64) k = wl * 64;
    if (S.opts.full_scan) {
      sh = sg->row_shape[g];
      if (skip_stamp[sh] == skip_gen) k = std::max(k, shape_skip[sh]);  // what earlier rows of the shape rejected
    }
    int32_t* const fl = floor ? floor + S.task_shape[t] : nullptr;
    if (fl && k < *fl) k = *fl;
    int res = -1;
    int64_t steps = 0, rechecks = 0;
    // A word's candidates are taken lowest first by clearing bits (a short
    // dependency chain: the checks of successive candidates overlap), the
    // mirror's rows through pointers held in registers. In contended
    // cycles most candidates are nodes touched since the scan that no
    // longer fit, so this loop is the in-order commit's hot spot.
    const char* panic = S.panic_node.data();
    const int32_t* mk = mark.data();
    const int32_t* nt = S.ntasks.data();
    const int32_t* mt = S.maxtasks.data();
    const Res* idle = S.idle.data();
    const Res* rel = S.rel.data();
    const bool cap = S.pred_active, masked = S.has_ports || S.has_aff, aff = S.has_aff, be = S.be_task[t];
    const uint64_t* cmask = S.h_class_mask.data() + (size_t)S.task_class[t] * S.W;
    const int32_t bs = base;
    if (rows) {  // the same walk over one cache line per candidate
      const int32_t* awm = aff ? S.mwmark.data() + (size_t)S.task_class[t] * S.W : nullptr;
      const double rc_ = r.c, rm_ = r.m, rg_ = r.g;
      auto fits = [&](double a0, double a1, double a2) {  // Resource.LessEqual (resource_info.go:142-146)
        return (rc_ < a0 || __builtin_fabs(a0 - rc_) < kbg::kMinMilliCPU) &&
               (rm_ < a1 || __builtin_fabs(a1 - rm_) < kbg::kMinMemory) &&
               (rg_ < a2 || __builtin_fabs(a2 - rg_) < kbg::kMinMilliGPU);
      };
      while (k < end && res < 0) {
        const int32_t w = k >> 6;
        uint64_t bits = m[w].f & (~0ull << (k & 63));
        const bool wdirty = aff && awm[w] > bs;
        while (bits) {
          const int32_t nd = (w << 6) | __builtin_ctzll(bits);
          bits &= bits - 1;
          if (bits) __builtin_prefetch(rows + ((w << 6) | __builtin_ctzll(bits)));
          const MirrorRow& q = rows[nd];
          ++steps;
          if (q.panic) {
            k = nd;
            res = RES_PANIC;
            break;
          }
          if (!(q.mark > bs || wdirty)) {
            k = nd;
            *node = nd;
            *kind = ((m[w].i >> (nd & 63)) & 1ull) ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
            res = RES_OK;
            break;
          }
          ++rechecks;  // touched since the scan: re-check on the host mirror
          if (cap && q.nt >= q.mt) continue;
          if (masked && !((cmask[w] >> (nd & 63)) & 1ull)) continue;
          const int v = be ? 1 : fits(q.ic, q.im, q.ig) ? 1 : fits(q.rc, q.rm, q.rg) ? 2 : 0;
          if (v) {
            k = nd;
            *node = nd;
            *kind = v == 1 ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
            res = RES_OK;
            break;
          }
        }
        if (res < 0) k = (w + 1) << 6;
      }
    }
    while (k < end && res < 0) {
      const int32_t w = k >> 6;
      uint64_t bits = m[w].f & (~0ull << (k & 63));
      while (bits) {
        const int32_t nd = (w << 6) | __builtin_ctzll(bits);
        bits &= bits - 1;
        ++steps;
        if (panic[nd]) {
          k = nd;
          res = RES_PANIC;
          break;
        }
        if (!(mk[nd] > bs || (aff && S.mwmark[(size_t)S.task_class[t] * S.W + w] > bs))) {
          k = nd;
          *node = nd;
          *kind = ((m[w].i >> (nd & 63)) & 1ull) ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
          res = RES_OK;
          break;
        }
        ++rechecks;  // touched since the scan: re-check on the host mirror (recheck())
        if (cap && nt[nd] >= mt[nd]) continue;
        if (masked && !((cmask[w] >> (nd & 63)) & 1ull)) continue;
        const int v = be ? 1 : kbg::res_le(r, idle[nd]) ? 1 : kbg::res_le(r, rel[nd]) ? 2 : 0;
        if (v) {
          k = nd;
          *node = nd;
          *kind = v == 1 ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
          res = RES_OK;
          break;
        }
      }
      if (res < 0) k = (w + 1) << 6;
    }
    S.stats.resolve_steps += steps;
    S.stats.resolve_rechecks += rechecks;
    if (sh >= 0 && res != RES_PANIC) {  // nodes before k are infeasible for the shape from now on
      shape_skip[sh] = k;
      skip_stamp[sh] = skip_gen;
    }
    if (fl && res != RES_PANIC) *fl = k;
    if (res >= 0) return res;
    if (info & kbg::kCountIncompleteBit) return RES_TRUNC;
    *node = -1;
    return RES_OK;
  }
  int resolve(int32_t g, int32_t t, int32_t* node, int32_t* kind) {
    if (sg->fused) return resolve_mask(g, t, node, kind);
    if (S.opts.full_scan && sg->h_capoff[g + 1] == sg->h_capoff[g])
      g = sg->row_ext[g];  // an alias row: its shape's long list (Grouper::build), this row's cursor
    const uint32_t cnt = sg->h_count[g];
    const int32_t n = (int32_t)(cnt & kbg::kCountMask);
    const uint32_t* c = sg->h_cand + sg->h_capoff[g];
    const Res& r = S.treq[t];
    int32_t sh = -1;
    if (S.opts.full_scan) {
      sh = sg->row_shape[g];
      // the skip may pass this row's own M entries: the loop moves to the long list
      if (skip_stamp[sh] == skip_gen) cursor[g] = std::max(cursor[g], shape_skip[sh]);
    }
    int res = -1;
    int32_t& k = cursor[g];
    const int32_t k0 = k;
    int64_t rechecks = 0;
    int32_t n_end = n;
    uint32_t cnt_end = cnt;
    for (;; ++k) {
      if (k >= n_end) {  // full-scan: continue in the shape's longest list of this scan
        if (sh < 0 || !(cnt_end & kbg::kCountIncompleteBit)) break;
        const int32_t g2 = sg->row_ext[g];
        const uint32_t cnt2 = sg->h_count[g2];
        if (g2 == g || (int32_t)(cnt2 & kbg::kCountMask) <= n_end) break;
        c = sg->h_cand + sg->h_capoff[g2];
        n_end = (int32_t)(cnt2 & kbg::kCountMask);
        cnt_end = cnt2;
        if (k >= n_end) break;
      }
      const int32_t nd = (int32_t)(c[k] & ~kbg::kCandPipelineBit);
      if (S.panic_node[nd]) {
        res = RES_PANIC;
        break;
      }
      if (!dirty(t, nd)) {
        *node = nd;
        *kind = (c[k] & kbg::kCandPipelineBit) ? KBG_KIND_PIPELINE : KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      // touched since the scan: re-check on the host mirror
      ++rechecks;
      if (S.pred_active && S.ntasks[nd] >= S.maxtasks[nd]) continue;
      if ((S.has_ports || S.has_aff) &&
          !((S.h_class_mask[(size_t)S.task_class[t] * S.W + (nd >> 6)] >> (nd & 63)) & 1ull))
        continue;
      if (S.be_task[t]) {  // backfill: PredicateFn only, always ssn.Allocate
        *node = nd;
        *kind = KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      if (kbg::res_le(r, S.idle[nd])) {
        *node = nd;
        *kind = KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      if (kbg::res_le(r, S.rel[nd])) {
        *node = nd;
        *kind = KBG_KIND_PIPELINE;
        res = RES_OK;
        break;
      }
    }
    S.stats.resolve_steps += k - k0 + (k < n_end ? 1 : 0);
    S.stats.resolve_rechecks += rechecks;
    if (sh >= 0 && res != RES_PANIC) {  // entries before k are infeasible for the shape from now on
      shape_skip[sh] = k;
      skip_stamp[sh] = skip_gen;
    }
    if (res >= 0) return res;
    if (cnt_end & kbg::kCountIncompleteBit) return RES_TRUNC;
    *node = -1;
    return RES_OK;
  }
};

// NodeInfo.AddTask on the host mirror (node_info.go:101-129): Allocated ->
// Idle -= req; Pipelined -> Releasing -= req; both add a task.
void clear_mask_bit(Session& S, int32_t c, int32_t nd) {
  const uint32_t idx = (uint32_t)((size_t)c * S.W + (nd >> 6));
  const uint64_t bit = 1ull << (nd & 63);
  if (!(S.h_class_mask[idx] & bit)) return;
  S.h_class_mask[idx] &= ~bit;
  vc_mask_changed(S, c, nd);
  if (!S.mask_dirty_flag[idx]) {
    S.mask_dirty_flag[idx] = 1;
    S.mask_dirty.push_back(idx);
  }
}

// The bit of (c, n) from the static predicate, the port fit and the pod
// affinity counts (a nil-Node node stays reachable: SetNode panics first).
void refresh_mask_bit(Session& S, int32_t c, int32_t n) {
  const uint32_t idx = (uint32_t)((size_t)c * S.W + (n >> 6));
  const uint64_t bit = 1ull << (n & 63);
  bool v = (S.h_class_mask_static[idx] & bit) != 0;
  if (v && !S.panic_node[n]) {
    for (int32_t w = 0; w < S.PW && v; ++w)
      v = (S.node_ports[(size_t)n * S.PW + w] & S.cls_conf[(size_t)c * S.PW + w]) == 0;
    if (v && S.has_aff) v = kbg::aff_ok_node(S, c, n);
  }
  if (v == ((S.h_class_mask[idx] & bit) != 0)) return;
  S.h_class_mask[idx] ^= bit;
  vc_mask_changed(S, c, n);
  if (!S.mask_dirty_flag[idx]) {
    S.mask_dirty_flag[idx] = 1;
    S.mask_dirty.push_back(idx);
  }
}

// The pod joins node.Pods(), so its ports join the node's HostPortInfo
// (vendor cache/node_info.go:593-605): every class that conflicts with a newly
// used (ip, protocol, port) loses the node.
void add_ports(Session& S, int32_t c, int32_t nd) {
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  const uint64_t* add = &S.cls_add[(size_t)c * S.PW];
  for (int32_t w = 0; w < S.PW; ++w) {
    for (uint64_t b = add[w]; b; b &= b - 1)  // holders, for a statement discard (remove_ports)
      S.port_hold[((int64_t)nd << 32) | (uint32_t)(w * 64 + __builtin_ctzll(b))]++;
    uint64_t nb = add[w] & ~np[w];
    np[w] |= nb;
    while (nb) {
      const int32_t a = w * 64 + __builtin_ctzll(nb);
      nb &= nb - 1;
      for (int32_t c2 : S.atom_cls[a]) clear_mask_bit(S, c2, nd);
    }
  }
}

// The pod leaves node.Pods() (statement.go:156-192 unpipeline ->
// NodeInfo.RemoveTask): an atom no other pod holds — and that no pod held at
// open — is free again, and the classes it blocked get the node back where
// nothing else forbids it.
int32_t open_ports_left(const Session& S, int32_t nd, int32_t a) {  // entries of open pods still on the node
  const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
  auto o = S.port_open.find(k);
  if (o == S.port_open.end()) return 0;
  auto g = S.port_gone.find(k);
  return o->second - (g == S.port_gone.end() ? 0 : g->second);
}
void remove_ports(Session& S, int32_t c, int32_t nd) {
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  const uint64_t* add = &S.cls_add[(size_t)c * S.PW];
  for (int32_t w = 0; w < S.PW; ++w)
    for (uint64_t b = add[w]; b; b &= b - 1) {
      const int32_t a = w * 64 + __builtin_ctzll(b);
      auto it = S.port_hold.find(((int64_t)nd << 32) | (uint32_t)a);
      if (it == S.port_hold.end() || --it->second > 0) continue;
      S.port_hold.erase(it);
      const uint64_t bit = 1ull << (a & 63);
      if (open_ports_left(S, nd, a) > 0) continue;  // a pod on the node at open still holds it
      np[w] &= ~bit;
      for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
    }
}

// The port atom of one of a pod's host-port entries (-1: no atom; every port
// a pod on a node uses is one).
int32_t port_atom(const Session& S, const kbg_host_port& hp) {
  if (hp.host_port <= 0) return -1;
  const std::string ip = S.strs[hp.host_ip].empty() ? std::string("0.0.0.0") : S.strs[hp.host_ip];
  const std::string pr = S.strs[hp.protocol].empty() ? std::string("TCP") : S.strs[hp.protocol];
  auto ai = S.atom_of.find(ip + "|" + pr + "|" + std::to_string(hp.host_port));
  return ai == S.atom_of.end() ? -1 : ai->second;
}

// A pod that was on the node at open leaves node.Pods() (a statement
// discard's RemoveTask by key of the pod holding the key): each of its port
// entries goes; an atom no pod holds any more is free again.
void release_open_ports(Session& S, int32_t nd, const kbg_host_port* ports, int32_t n) {
  if (!S.has_ports) return;
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  for (int32_t i = 0; i < n; ++i) {
    const int32_t a = port_atom(S, ports[i]);
    if (a < 0) continue;
    const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
    S.port_gone[k]++;
    if (open_ports_left(S, nd, a) > 0 || S.port_hold.count(k)) continue;
    const uint64_t bit = 1ull << (a & 63);
    if (!(np[a / 64] & bit)) continue;
    np[a / 64] &= ~bit;
    for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
  }
}

// The reverse: a discarded statement's unevict adds that pod back to the node
// (statement.go:81-108 node.AddTask), so it is in node.Pods() again and its
// port entries are used again (vendor cache/node_info.go:593-605): every class
// one of them conflicts with loses the node.
void restore_open_ports(Session& S, int32_t nd, const kbg_host_port* ports, int32_t n) {
  if (!S.has_ports) return;
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  for (int32_t i = 0; i < n; ++i) {
    const int32_t a = port_atom(S, ports[i]);
    if (a < 0) continue;
    const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
    auto g = S.port_gone.find(k);
    if (g != S.port_gone.end() && --g->second <= 0) S.port_gone.erase(g);
    const uint64_t bit = 1ull << (a & 63);
    if (np[a / 64] & bit) continue;
    np[a / 64] |= bit;
    for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
  }
}

// NodeInfo.Tasks already holds the task's PodKey (node_info.go:101-106)
inline int64_t node_key_of(const Session& S, int32_t t, int32_t nd) {
  return ((int64_t)nd << 32) | (uint32_t)S.task_key[t];
}
bool node_has_key(const Session& S, int32_t t, int32_t nd) {
  return S.has_dupkeys && S.key_hot[S.task_key[t]] && S.node_keys.count(node_key_of(S, t, nd)) != 0;
}

// Returns true when the node already held the task's pod key: the decision
// stands, the node is unchanged (AddTask's error), the pod is not among
// node.Pods() (ports), but it is an Allocated pod of its job (the podLister).
bool mirror_add(Session& S, int32_t t, int32_t nd, int32_t kind) {
  const bool dup = node_has_key(S, t, nd);
  if (!dup) {
    if (!S.nil_node[nd]) {
      if (kind == KBG_KIND_ALLOCATE) kbg::res_sub(S.idle[nd], S.treq[t]);
      else kbg::res_sub(S.rel[nd], S.treq[t]);
    }
    S.ntasks[nd]++;
    if (S.has_ports) add_ports(S, S.task_class[t], nd);
    if (S.has_dupkeys && S.key_hot[S.task_key[t]]) {
      S.node_keys.insert(node_key_of(S, t, nd));
      S.key_holder[node_key_of(S, t, nd)] = t << 1 | (kind != KBG_KIND_ALLOCATE);
    }
  }
  // an Allocated pod joins the podLister (api/helpers.go:63-70); Pipelined does not
  if (S.has_aff && kind == KBG_KIND_ALLOCATE) {
    static const bool prof = getenv("KBG_PROFILE_AFF") != nullptr;
    const uint64_t c0 = prof ? __builtin_readcyclecounter() : 0;
    kbg::aff_place(S, t, nd, +1, S.affm->st, true);
    if (prof) {
      S.affm->prof_cycles += __builtin_readcyclecounter() - c0;
      S.affm->prof_calls++;
    }
  }
  return dup;
}

// Which pod keys can collide: a candidate task's key that another candidate
// shares or that some node already holds (a StatefulSet pod recreated while
// its predecessor is still on a node). Usually none: then nothing is tracked.
// Kept as counts per canonical key — candidate (Pending) tasks holding it,
// node entries holding it — so an update adjusts the keys its events and
// touched tasks changed instead of rescanning every task and node.
void pod_key_refresh(Session& S, int32_t k) {
  const bool hot = S.kc_cand[k] >= 2 || (S.kc_cand[k] >= 1 && S.kc_node[k] >= 1);
  if (hot != (S.key_hot[k] != 0)) {
    S.n_hot += hot ? 1 : -1;
    S.key_hot[k] = hot ? 1 : 0;
  }
}
void setup_pod_keys(Session& S, bool incr = false, const std::vector<int32_t>* touched = nullptr,
                    const std::vector<uint8_t>* was = nullptr) {
  const size_t NS = S.strs.size();
  S.task_key.resize(S.n_tasks);
  if (!incr || S.kc_cand.empty()) {
    for (int32_t t = 0; t < S.n_tasks; ++t) S.task_key[t] = S.canon[S.tasks_in[t].pod_key];
    S.kc_cand.assign(NS, 0);
    S.kc_node.assign(NS, 0);
    S.key_hot.assign(NS, 0);
    S.n_hot = 0;
    for (int32_t t = 0; t < S.n_tasks; ++t)
      if (S.pending_candidate[t] || S.be_task[t]) S.kc_cand[S.task_key[t]]++;  // (false for removed tasks)
    for (int32_t n = 0; n < S.n_nodes; ++n)
      for (int32_t k : S.node_key_order[n]) S.kc_node[k]++;
    for (size_t k = 0; k < NS; ++k) pod_key_refresh(S, (int32_t)k);
  } else {
    S.kc_cand.resize(NS, 0);
    if (S.kc_node.size() < NS) S.kc_node.resize(NS, 0);
    S.key_hot.resize(NS, 0);
    for (size_t i = 0; i < touched->size(); ++i) {
      const int32_t t = (*touched)[i];
      const int32_t k = S.task_key[t] = S.canon[S.tasks_in[t].pod_key];
      const bool was_c = ((*was)[i] & 3) != 0, now_c = S.pending_candidate[t] || S.be_task[t];
      if (was_c == now_c) continue;
      S.kc_cand[k] += now_c ? 1 : -1;
      pod_key_refresh(S, k);
    }
    for (int32_t k : S.upd_keys) pod_key_refresh(S, k);  // node entries added / removed by the events
  }
  S.upd_keys.clear();
  S.has_dupkeys = S.n_hot > 0;
  S.node_keys.clear();
  if (S.has_dupkeys)
    for (int32_t n = 0; n < S.n_nodes; ++n)
      for (int32_t k : S.node_key_order[n])
        if (S.key_hot[k]) S.node_keys.insert(((int64_t)n << 32) | (uint32_t)k);
  S.node_keys0 = S.node_keys;
}

// Builds the port-atom dictionary (distinct sanitized (ip, protocol, port)
// with port > 0 over the nodes' used ports and the candidate classes' wanted
// ports), each class's conflict set (host_ports.go CheckConflict: same
// protocol and port, and either side 0.0.0.0 or the same ip) and folds the
// nodes' current conflicts into the class masks.
void setup_host_ports(Session& S) {
  S.has_ports = false;
  if (!S.pred_active) return;
  const int32_t C = (int32_t)S.class_spec.size();
  auto ip_of = [&](int32_t id) { return S.strs[id].empty() ? std::string("0.0.0.0") : S.strs[id]; };
  auto proto_of = [&](int32_t id) { return S.strs[id].empty() ? std::string("TCP") : S.strs[id]; };
  typedef std::tuple<std::string, std::string, int32_t> Atom;
  std::map<Atom, int32_t> atoms;
  std::vector<Atom> atom_list;
  auto atom = [&](const kbg_host_port& hp) {
    Atom a{ip_of(hp.host_ip), proto_of(hp.protocol), hp.host_port};
    auto it = atoms.find(a);
    if (it != atoms.end()) return it->second;
    const int32_t id = (int32_t)atom_list.size();
    atoms.emplace(a, id);
    atom_list.push_back(a);
    return id;
  };
  std::vector<std::vector<int32_t>> want(C);
  bool any = false;
  // only classes some candidate task uses (a resident session keeps classes
  // whose tasks have left; they must not switch the port machinery on)
  std::vector<uint8_t> in_use(C, 0);
  for (int32_t t = 0; t < S.n_tasks; ++t)
    if (S.pending_candidate[t] || S.be_task[t]) in_use[S.task_class[t]] = 1;
  for (int32_t c = 0; c < C; ++c) {
    const int32_t sp = S.class_spec[c];
    if (sp < 0 || !in_use[c]) continue;
    const kbg_spec& spec = S.specs_in[sp];
    for (int32_t i = 0; i < spec.port_len; ++i) {
      const kbg_host_port& hp = S.ports_in[spec.port_off + i];
      if (hp.host_port <= 0) continue;
      want[c].push_back(atom(hp));
      any = true;
    }
  }
  if (!any) return;
  std::vector<std::vector<int32_t>> used(S.n_nodes);
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    const kbg_node& nd = S.nodes_in[n];
    for (int32_t i = 0; i < nd.port_len; ++i) {
      const kbg_host_port& hp = S.ports_in[nd.port_off + i];
      if (hp.host_port > 0) used[n].push_back(atom(hp));
    }
  }
  S.has_ports = true;
  const int32_t A = (int32_t)atom_list.size();
  S.PW = (A + 63) / 64;
  S.cls_conf.assign((size_t)C * S.PW, 0);
  S.cls_add.assign((size_t)C * S.PW, 0);
  S.atom_cls.assign(A, {});
  for (int32_t c = 0; c < C; ++c)
    for (int32_t w : want[c]) {
      S.cls_add[(size_t)c * S.PW + w / 64] |= 1ull << (w % 64);
      const Atom& wa = atom_list[w];
      for (int32_t a = 0; a < A; ++a) {
        const Atom& ea = atom_list[a];
        if (std::get<1>(ea) != std::get<1>(wa) || std::get<2>(ea) != std::get<2>(wa)) continue;
        if (std::get<0>(wa) == "0.0.0.0" || std::get<0>(ea) == "0.0.0.0" || std::get<0>(ea) == std::get<0>(wa))
          S.cls_conf[(size_t)c * S.PW + a / 64] |= 1ull << (a % 64);
      }
    }
  for (int32_t c = 0; c < C; ++c)
    for (int32_t a = 0; a < A; ++a)
      if ((S.cls_conf[(size_t)c * S.PW + a / 64] >> (a % 64)) & 1ull) S.atom_cls[a].push_back(c);
  S.atom_of.clear();
  for (int32_t a = 0; a < A; ++a)
    S.atom_of[std::get<0>(atom_list[a]) + "|" + std::get<1>(atom_list[a]) + "|" + std::to_string(std::get<2>(atom_list[a]))] = a;
  S.port_open.clear();  // one entry per pod and port: how many pods at open use each atom
  for (int32_t n = 0; n < S.n_nodes; ++n)
    for (int32_t a : used[n]) S.port_open[((int64_t)n << 32) | (uint32_t)a]++;
  S.node_ports.assign((size_t)S.n_nodes * S.PW, 0);
  S.mask_dirty_flag.assign(S.h_class_mask.size(), 0);
  S.mask_dirty.clear();
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    for (int32_t a : used[n]) S.node_ports[(size_t)n * S.PW + a / 64] |= 1ull << (a % 64);
    if (S.panic_node[n]) continue;  // SetNode(nil) panics before any check: keep the node reachable
    for (int32_t c = 0; c < C; ++c) {
      bool conflict = false;
      for (int32_t w = 0; w < S.PW && !conflict; ++w)
        conflict = (S.node_ports[(size_t)n * S.PW + w] & S.cls_conf[(size_t)c * S.PW + w]) != 0;
      if (conflict) S.h_class_mask[(size_t)c * S.W + (n >> 6)] &= ~(1ull << (n & 63));
    }
  }
  S.node_ports0 = S.node_ports;
}
kbg_status validate(const kbg_snapshot* s) {
  if (!s) return fail(KBG_E_INVALID, "null snapshot");
  auto in = [](int32_t v, int32_t n) { return v >= 0 && v < n; };
  auto range = [](int32_t off, int32_t len, int32_t n) { return off >= 0 && len >= 0 && (int64_t)off + len <= n; };
  if (s->n_strings < 0 || (s->n_strings > 0 && !s->strings)) return fail(KBG_E_INVALID, "strings");
  {  // every count non-negative, every non-empty array present (encode must never emit an unreadable blob)
    const std::pair<const void*, int32_t> arrays[] = {
        {s->nodes, s->n_nodes},         {s->jobs, s->n_jobs},           {s->queues, s->n_queues},
        {s->tasks, s->n_tasks},         {s->others, s->n_others},       {s->specs, s->n_specs},
        {s->terms, s->n_terms},         {s->reqs, s->n_reqs},           {s->values, s->n_values},
        {s->tolerations, s->n_tolerations}, {s->labels, s->n_labels},   {s->taints, s->n_taints},
        {s->selectors, s->n_selectors}, {s->plugins, s->n_plugins},     {s->tier_sizes, s->n_tiers},
        {s->ports, s->n_ports},         {s->node_tasks, s->n_node_tasks}, {s->pod_terms, s->n_pod_terms},
        {s->pod_labels, s->n_pod_labels}, {s->node_pod_keys, s->n_node_pod_keys}, {s->node_pods, s->n_node_pods}};
    for (const auto& a : arrays)
      if (a.second < 0 || (a.second > 0 && !a.first)) return fail(KBG_E_INVALID, "negative count or null array");
  }
  for (int32_t i = 0; i < s->n_strings; ++i)
    if (!s->strings[i]) return fail(KBG_E_INVALID, "null string " + std::to_string(i));
  const int32_t NS = s->n_strings;
  for (int32_t i = 0; i < s->n_nodes; ++i) {
    const kbg_node& n = s->nodes[i];
    if (!in(n.name, NS) || !range(n.label_off, n.label_len, s->n_labels) || !range(n.taint_off, n.taint_len, s->n_taints) ||
        !range(n.port_off, n.port_len, s->n_ports))
      return fail(KBG_E_INVALID, "node " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_labels * 2; ++i)
    if (!in(s->labels[i], NS)) return fail(KBG_E_INVALID, "label string");
  for (int32_t i = 0; i < s->n_selectors * 2; ++i)
    if (!in(s->selectors[i], NS)) return fail(KBG_E_INVALID, "selector string");
  for (int32_t i = 0; i < s->n_taints; ++i) {
    const kbg_taint& t = s->taints[i];
    if (!in(t.key, NS) || !in(t.value, NS) || !in(t.effect, NS)) return fail(KBG_E_INVALID, "taint");
  }
  for (int32_t i = 0; i < s->n_queues; ++i)
    if (!in(s->queues[i].uid, NS)) return fail(KBG_E_INVALID, "queue");
  for (int32_t i = 0; i < s->n_jobs; ++i)
    if (!in(s->jobs[i].uid, NS) || !in(s->jobs[i].queue, s->n_queues)) return fail(KBG_E_INVALID, "job " + std::to_string(i));
  for (int32_t i = 0; i < s->n_tasks; ++i) {
    const kbg_task& t = s->tasks[i];
    if (!in(t.uid, NS) || !in(t.job, s->n_jobs) || !(t.spec == -1 || in(t.spec, s->n_specs)) || !in(t.node_name, NS) ||
        !in(t.pod_key, NS))
      return fail(KBG_E_INVALID, "task " + std::to_string(i));
    if (t.status <= 0 || t.status > KBG_UNKNOWN || (t.status & (t.status - 1))) return fail(KBG_E_INVALID, "task status");
  }
  if (s->n_pod_terms < 0 || (s->n_pod_terms > 0 && !s->pod_terms)) return fail(KBG_E_INVALID, "pod_terms");
  if (s->n_pod_labels < 0 || (s->n_pod_labels > 0 && !s->pod_labels)) return fail(KBG_E_INVALID, "pod_labels");
  for (int32_t i = 0; i < s->n_specs; ++i) {
    const kbg_spec& p = s->specs[i];
    if (!range(p.selector_off, p.selector_len, s->n_selectors) || !range(p.term_off, p.term_len, s->n_terms) ||
        !range(p.toleration_off, p.toleration_len, s->n_tolerations) || !range(p.port_off, p.port_len, s->n_ports) ||
        !in(p.ns, NS) || !range(p.pod_label_off, p.pod_label_len, s->n_pod_labels) ||
        !range(p.aff_off, p.aff_len, s->n_pod_terms) || !range(p.anti_off, p.anti_len, s->n_pod_terms))
      return fail(KBG_E_INVALID, "spec " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_pod_labels * 2; ++i)
    if (!in(s->pod_labels[i], NS)) return fail(KBG_E_INVALID, "pod label string");
  for (int32_t i = 0; i < s->n_pod_terms; ++i) {
    const kbg_pod_term& t = s->pod_terms[i];
    if (!range(t.match_off, t.match_len, s->n_selectors) || !range(t.expr_off, t.expr_len, s->n_reqs) ||
        !range(t.ns_off, t.ns_len, s->n_values) || !in(t.topology_key, NS))
      return fail(KBG_E_INVALID, "pod term " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_terms; ++i) {
    const kbg_term& t = s->terms[i];
    if (!range(t.expr_off, t.expr_len, s->n_reqs) || !range(t.field_off, t.field_len, s->n_reqs))
      return fail(KBG_E_INVALID, "term");
  }
  for (int32_t i = 0; i < s->n_reqs; ++i) {
    const kbg_requirement& r = s->reqs[i];
    if (!in(r.key, NS) || !in(r.op, NS) || !range(r.value_off, r.value_len, s->n_values)) return fail(KBG_E_INVALID, "req");
  }
  for (int32_t i = 0; i < s->n_values; ++i)
    if (!in(s->values[i], NS)) return fail(KBG_E_INVALID, "value");
  if (s->n_ports < 0 || (s->n_ports > 0 && !s->ports)) return fail(KBG_E_INVALID, "ports");
  if (s->n_node_tasks < 0 || (s->n_node_tasks > 0 && !s->node_tasks)) return fail(KBG_E_INVALID, "node_tasks");
  for (int32_t i = 0; i < s->n_nodes; ++i)
    if (!range(s->nodes[i].task_off, s->nodes[i].task_len, s->n_node_tasks))
      return fail(KBG_E_INVALID, "node task list " + std::to_string(i));
  for (int32_t i = 0; i < s->n_node_tasks; ++i)
    if (!in(s->node_tasks[i], s->n_tasks)) return fail(KBG_E_INVALID, "node task index");
  for (int32_t i = 0; i < s->n_nodes; ++i) {  // NodeInfo.Tasks keys: one per pod on the node
    const kbg_node& n = s->nodes[i];
    if (!range(n.key_off, n.key_len, s->n_node_pod_keys) || n.key_len != n.num_tasks)
      return fail(KBG_E_INVALID, "node pod keys " + std::to_string(i) + " (key_len must equal num_tasks)");
  }
  for (int32_t i = 0; i < s->n_node_pod_keys; ++i)
    if (!in(s->node_pod_keys[i], NS)) return fail(KBG_E_INVALID, "node pod key string");
  if (s->n_node_pods != 0 && s->n_node_pods != s->n_node_pod_keys)
    return fail(KBG_E_INVALID, "node_pods: none or one per node_pod_keys entry");
  for (int32_t i = 0; i < s->n_nodes && s->n_node_pods; ++i) {  // each pod's ports: the node's, in order
    const kbg_node& n = s->nodes[i];
    int64_t pl = 0;
    for (int32_t k = 0; k < n.key_len; ++k) {
      const kbg_node_pod& q = s->node_pods[n.key_off + k];
      if (q.port_len < 0 || q.status <= 0 || q.status > KBG_UNKNOWN || (q.status & (q.status - 1)))
        return fail(KBG_E_INVALID, "node pod " + std::to_string(n.key_off + k));
      pl += q.port_len;
    }
    if (pl != n.port_len) return fail(KBG_E_INVALID, "node " + std::to_string(i) + ": node_pods port_len sum != port_len");
  }
  for (int32_t i = 0; i < s->n_ports; ++i)
    if (!in(s->ports[i].host_ip, NS) || !in(s->ports[i].protocol, NS)) return fail(KBG_E_INVALID, "port");
  for (int32_t i = 0; i < s->n_tolerations; ++i) {
    const kbg_toleration& t = s->tolerations[i];
    if (!in(t.key, NS) || !in(t.op, NS) || !in(t.value, NS) || !in(t.effect, NS)) return fail(KBG_E_INVALID, "toleration");
  }
  int32_t np = 0;
  for (int32_t i = 0; i < s->n_tiers; ++i) {
    if (s->tier_sizes[i] < 0) return fail(KBG_E_INVALID, "tier size");
    np += s->tier_sizes[i];
  }
  if (np != s->n_plugins) return fail(KBG_E_INVALID, "tier sizes do not sum to n_plugins");
  for (int32_t i = 0; i < s->n_plugins; ++i)
    if (!in(s->plugins[i].name, NS)) return fail(KBG_E_INVALID, "plugin name");
  return KBG_OK;
}

template <class T>
std::vector<T> copy_arr(const T* p, int32_t n) {
  return (p && n > 0) ? std::vector<T>(p, p + n) : std::vector<T>();
}

constexpr int64_t kRankGap = int64_t(1) << 20;  // task_rank spacing at open (kbg_session.hpp)

std::vector<int32_t> ranks_of(const Session& S, const std::vector<int32_t>& ids) {
  std::vector<int32_t> idx(ids.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return S.strs[ids[a]] < S.strs[ids[b]]; });
  std::vector<int32_t> rank(ids.size());
  int32_t r = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    if (i > 0 && S.strs[ids[idx[i]]] != S.strs[ids[idx[i - 1]]]) ++r;
    rank[idx[i]] = r;
  }
  return rank;
}

// ---------------------------------------------------------------- open
// A session is built in two steps: ingest() copies the snapshot into the
// session's own mutable inputs (the resident snapshot that kbg_session_update
// edits), build() derives every host structure and the device tables from
// those inputs. derive_host() is the host part of build() that an update
// re-runs without recompiling the static predicate or reallocating HBM.

// String id of `v` for an event: an existing content's canonical id, or a new entry.
int32_t intern_h(Session& S, std::string_view key, uint64_t h) {  // h = StrIndex::hash(key)
  const int32_t known = S.canon_of.find_h(S.strs, key, h);
  if (known >= 0) return known;  // a canonical id is its own canonical id
  const int32_t id = (int32_t)S.strs.size();
  S.strs.emplace_back(key);
  S.canon.push_back(id);
  S.canon_of.insert_h(S.strs, id, h);
  return id;
}
int32_t intern(Session& S, const char* v) {
  const std::string_view key(v ? v : "");
  return intern_h(S, key, kbg::StrIndex::hash(key));
}

// The canonical id of "" (an event's NodeName of a pod on no node).
int32_t empty_str(Session& S) {
  if (S.str_empty < 0 || S.str_empty >= (int32_t)S.strs.size() || !S.strs[S.str_empty].empty())
    S.str_empty = intern(S, "");
  return S.str_empty;
}

// A string only ever read as text (a task UID: TaskOrderFn's fallback compares
// UIDs as strings, nothing looks it up by content): appended without the
// content map, as its own canonical id.
int32_t append_str(Session& S, const char* v) {
  const int32_t id = (int32_t)S.strs.size();
  S.strs.emplace_back(v ? v : "");
  S.canon.push_back(id);
  return id;
}

kbg_status ingest(Session& S, const kbg_snapshot* snap, const kbg_options* o) {
  static const bool prof = getenv("KBG_PROFILE_OPEN") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[kbg ingest] %-20s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - tl).count());
    tl = now;
  };
  kbg_status st = validate(snap);
  if (st != KBG_OK) return st;
  phase("validate");
  if (o) S.opts = *o;
  S.heap_go111 = S.opts.heap_rule == 0;
  S.K = S.opts.batch_tasks > 0 ? S.opts.batch_tasks : (S.opts.full_scan ? kFullScanK : 8192);
  S.M = S.opts.candidates > 0 ? S.opts.candidates : 32;
  if (S.M > 4096) return fail(KBG_E_INVALID, "candidates > 4096");
  // full-scan: K rows x (M + rank) slots; grouped: sum over shapes of min(n_s + slack, 4096)


  // headroom for pods added by session updates (no reallocation per event batch)
  const size_t more = (size_t)std::max(0, snap->n_tasks) / 4 + 1024;
  // The strings are copied and hashed by a few workers (each its own range),
  // then entered into the content index in id order (the first id of a
  // content is its canonical id), each slot requested a few strings ahead.
  const size_t NS = (size_t)std::max(0, snap->n_strings);
  // a session rebuilt from its own updated snapshot (restructure) adopts its
  // string table and content index: the snapshot's strings are that table
  const bool adopted = S.adopt_strings && S.strs.size() == NS && S.canon.size() == NS;
  S.adopt_strings = false;
  std::vector<uint64_t> sh(adopted ? 0 : NS);
  if (!adopted) {
  S.strs.clear();
  S.strs.reserve(NS + 2 * more);
  S.strs.resize(NS);
  {
    const size_t P = NS < 65536 ? 1 : std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency()));
    auto copy_range = [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        S.strs[i].assign(snap->strings[i]);
        sh[i] = kbg::StrIndex::hash(S.strs[i]);
      }
    };
    std::vector<std::thread> th;
    const size_t chunk = (NS + P - 1) / P;
    size_t done_to = chunk;  // a range no worker took is copied here
    try {
      for (size_t p = 1; p < P; ++p) {
        th.emplace_back(copy_range, std::min(NS, p * chunk), std::min(NS, (p + 1) * chunk));
        done_to = (p + 1) * chunk;
      }
    } catch (const std::system_error&) {
    }
    copy_range(0, std::min(NS, chunk));
    copy_range(std::min(NS, done_to), NS);
    for (std::thread& t : th) t.join();
  }
  phase("strings copy");
  S.canon_of.clear();
  S.canon_of.reserve(NS);
  S.canon.reserve(NS + 2 * more);
  S.canon.resize(NS);
  constexpr size_t kStrAhead = 16;
  for (size_t i = 0; i < NS; ++i) {
    if (i + kStrAhead < NS) S.canon_of.prefetch(sh[i + kStrAhead]);
    S.canon[i] = S.canon_of.insert_h(S.strs, (int32_t)i, sh[i]);
  }
  }
  phase("strings");
  S.n_nodes = snap->n_nodes;
  S.n_jobs = snap->n_jobs;
  S.n_queues = snap->n_queues;
  S.n_tasks = snap->n_tasks;
  S.nodes_in = copy_arr(snap->nodes, snap->n_nodes);
  S.jobs_in = copy_arr(snap->jobs, snap->n_jobs);
  S.queues_in = copy_arr(snap->queues, snap->n_queues);
  S.tasks_in.clear();
  S.tasks_in.reserve((size_t)std::max(0, snap->n_tasks) + more);
  if (snap->tasks && snap->n_tasks > 0) S.tasks_in.assign(snap->tasks, snap->tasks + snap->n_tasks);
  S.specs_in = copy_arr(snap->specs, snap->n_specs);
  S.terms_in = copy_arr(snap->terms, snap->n_terms);
  S.reqs_in = copy_arr(snap->reqs, snap->n_reqs);
  S.values_in = copy_arr(snap->values, snap->n_values);
  S.labels_in = copy_arr(snap->labels, 2 * snap->n_labels);
  S.selectors_in = copy_arr(snap->selectors, 2 * snap->n_selectors);
  S.tols_in = copy_arr(snap->tolerations, snap->n_tolerations);
  S.taints_in = copy_arr(snap->taints, snap->n_taints);
  S.ports_in = copy_arr(snap->ports, snap->n_ports);
  S.pod_terms_in = copy_arr(snap->pod_terms, snap->n_pod_terms);
  S.pod_labels_in = copy_arr(snap->pod_labels, 2 * snap->n_pod_labels);
  S.others_in = copy_arr(snap->others, snap->n_others);
  S.plugins_in = copy_arr(snap->plugins, snap->n_plugins);
  S.tier_sizes_in = copy_arr(snap->tier_sizes, snap->n_tiers);
  S.task_live.clear();
  S.task_live.reserve(S.n_tasks + more);
  S.task_live.assign(S.n_tasks, 1);
  phase("arrays");
  // JobInfo.Tasks / NodeInfo.Tasks insertion orders, kept as lists
  // an update reorders the way the cache's delete + add does
  S.job_task_order.assign(S.n_jobs, {});
  for (int32_t t = 0; t < S.n_tasks; ++t) S.job_task_order[S.tasks_in[t].job].push_back(t);
  S.node_task_order.assign(S.n_nodes, {});
  S.node_key_order.assign(S.n_nodes, {});
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    const kbg_node& nd = S.nodes_in[n];
    S.node_task_order[n].assign(snap->node_tasks + nd.task_off, snap->node_tasks + nd.task_off + nd.task_len);
    for (int32_t i = 0; i < nd.key_len; ++i) S.node_key_order[n].push_back(S.canon[snap->node_pod_keys[nd.key_off + i]]);
  }
  // keys held on a node by pods outside the session jobs, with their node
  // copies when the snapshot carries them (kbg_node_pod): no event ever adds
  // such a pod, only a removal by key takes one off (in_node_remove)
  S.outsiders.clear();
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    if (S.node_key_order[n].size() == S.node_task_order[n].size()) continue;  // every entry is a session task's
    const kbg_node& nd = S.nodes_in[n];
    std::unordered_set<int32_t> mine;
    for (int32_t t : S.node_task_order[n]) mine.insert(S.canon[S.tasks_in[t].pod_key]);
    int32_t po = nd.port_off;  // the entry's own ports follow NodeInfo.Tasks order
    for (int32_t i = 0; i < (int32_t)S.node_key_order[n].size(); ++i) {
      const kbg_node_pod* q = snap->n_node_pods ? &snap->node_pods[nd.key_off + i] : nullptr;
      const int32_t k = S.node_key_order[n][i];
      if (!mine.count(k)) {
        Session::Outsider& o = S.outsiders[((int64_t)n << 32) | (uint32_t)k];
        if (q) {
          o.req = q->resreq;
          o.status = q->status;
          o.ports.assign(S.ports_in.begin() + po, S.ports_in.begin() + po + q->port_len);
        }
      }
      if (q) po += q->port_len;
    }
  }
  S.broken.clear();
  S.node_of.clear();
  for (int32_t n = 0; n < S.n_nodes; ++n)
    if (S.nodes_in[n].has_node) S.node_of[S.canon[S.nodes_in[n].name]] = n;
  // sc.Nodes[NodeName] of a node the cache knows only from its pods
  // (NewNodeInfo(nil), event_handlers.go:49-53): its Name is "", so the
  // NodeName its pods carry is the only name it has; pod events naming it
  // (kbg_event.node = its index) take that name
  S.nil_name.assign(S.n_nodes, -1);
  S.pod_only_of.clear();
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    if (S.nodes_in[n].has_node) continue;
    for (const int32_t t : S.node_task_order[n]) {
      const int32_t nm = S.canon[S.tasks_in[t].node_name];
      if (S.strs[nm].empty()) continue;
      if (S.nil_name[n] < 0) S.nil_name[n] = nm;
      S.pod_only_of.emplace(nm, n);
    }
  }
  phase("orders");

  // ---- plugins (framework.go:26-46): a tier entry counts only when the
  // caller's process has a builder under its name (GetPluginBuilder); one of
  // its own builders this path cannot evaluate refuses the session
  std::vector<char> active(snap->n_plugins, 1);
  {
    static const char* const kImplemented[] = {"priority", "gang", "drf", "predicates", "proportion"};
    for (int32_t p = 0; p < snap->n_plugins; ++p) {
      const std::string& name = S.strs[snap->plugins[p].name];
      const bool known = std::find(std::begin(kImplemented), std::end(kImplemented), name) != std::end(kImplemented);
      const bool registered = S.opts.plugin_registry ? (snap->plugins[p].flags & KBG_PLUGIN_REGISTERED) != 0 : known;
      if (registered && !known)
        return fail(KBG_E_UNSUPPORTED, "plugin \"" + name + "\" is registered in the caller's process but the device "
                                       "path does not implement it (framework.go:30-35): run the reference path");
      active[p] = registered;
    }
  }
  {
    int32_t p = 0;
    bool seen_prio = false, seen_gang = false, seen_drf = false;
    for (int32_t ti = 0; ti < snap->n_tiers; ++ti)
      for (int32_t k = 0; k < snap->tier_sizes[ti]; ++k, ++p) {
        if (!active[p]) continue;
        const kbg_plugin_option& po = snap->plugins[p];
        const std::string& name = S.strs[po.name];
        const uint32_t f = po.flags;
        if (name == "priority") {
          S.has_prio = true;
          if (!(f & KBG_DISABLE_TASK_ORDER)) S.task_order_prio = true;
          if (!(f & KBG_DISABLE_JOB_ORDER) && !seen_prio) { S.job_chain.push_back(kbg::JO_PRIORITY); seen_prio = true; }
        } else if (name == "gang") {
          S.has_gang = true;
          if (!(f & KBG_DISABLE_JOB_READY)) S.ready_gang = true;
          if (!(f & KBG_DISABLE_JOB_ORDER) && !seen_gang) { S.job_chain.push_back(kbg::JO_GANG); seen_gang = true; }
        } else if (name == "drf") {
          S.has_drf = true;
          if (!(f & KBG_DISABLE_JOB_ORDER) && !seen_drf) { S.job_chain.push_back(kbg::JO_DRF); seen_drf = true; }
        } else if (name == "proportion") {
          S.has_prop = true;
          if (!(f & KBG_DISABLE_QUEUE_ORDER)) S.queue_order_prop = true;
        } else if (name == "predicates") {
          if (!(f & KBG_DISABLE_PREDICATE)) S.pred_active = true;
        }
      }
    // victim fns per tier (session_plugins.go:59-140): gang and drf register
    // preemptable fns, gang and proportion reclaimable ones (gang.go:104-127,
    // drf.go:80-107, proportion.go:161-186)
    p = 0;
    for (int32_t ti = 0; ti < snap->n_tiers; ++ti) {
      int32_t pre = 0, rec = 0;
      for (int32_t k = 0; k < snap->tier_sizes[ti]; ++k, ++p) {
        if (!active[p]) continue;
        const std::string& name = S.strs[snap->plugins[p].name];
        const uint32_t f = snap->plugins[p].flags;
        if (name == "gang" && !(f & KBG_DISABLE_PREEMPTABLE)) pre |= kbg::VP_GANG;
        if (name == "drf" && !(f & KBG_DISABLE_PREEMPTABLE)) pre |= kbg::VP_DRF;
        if (name == "gang" && !(f & KBG_DISABLE_RECLAIMABLE)) rec |= kbg::VP_GANG;
        if (name == "proportion" && !(f & KBG_DISABLE_RECLAIMABLE)) rec |= kbg::VP_PROP;
      }
      // `init` outlives the tier loop (session_plugins.go:60-61, 115-131):
      // once a tier has run a fn, later tiers intersect with its result, so
      // an empty result stays empty and the first tier with a fn decides alone
      if (pre && S.tier_preempt.empty()) S.tier_preempt.push_back(pre);
      if (rec && S.tier_reclaim.empty()) S.tier_reclaim.push_back(rec);
    }
  }

  // ---- job / queue ranks (jobs and queues do not change over a resident session)
  {
    std::vector<int32_t> ids(S.n_jobs);
    for (int32_t j = 0; j < S.n_jobs; ++j) ids[j] = S.jobs_in[j].uid;
    S.job_rank = ranks_of(S, ids);
    ids.resize(S.n_queues);
    for (int32_t q = 0; q < S.n_queues; ++q) ids[q] = S.queues_in[q].uid;
    S.queue_rank = ranks_of(S, ids);
  }
  {
    std::vector<int32_t> order(S.n_jobs);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
      if (S.jobs_in[a].creation_ns != S.jobs_in[b].creation_ns) return S.jobs_in[a].creation_ns < S.jobs_in[b].creation_ns;
      return S.job_rank[a] < S.job_rank[b];
    });
    S.job_frank.assign(S.n_jobs, 0);
    for (int32_t i = 0; i < S.n_jobs; ++i) S.job_frank[order[i]] = i;
    S.job_by_frank = order;
    std::vector<int32_t> prios(S.n_jobs);
    for (int32_t j = 0; j < S.n_jobs; ++j) prios[j] = S.jobs_in[j].priority;
    std::sort(prios.begin(), prios.end(), std::greater<int32_t>());
    prios.erase(std::unique(prios.begin(), prios.end()), prios.end());
    S.job_prank.resize(S.n_jobs);
    for (int32_t j = 0; j < S.n_jobs; ++j)
      S.job_prank[j] = (uint32_t)(std::lower_bound(prios.begin(), prios.end(), S.jobs_in[j].priority,
                                                   std::greater<int32_t>()) - prios.begin());
    S.job_queue.resize(S.n_jobs);
    for (int32_t j = 0; j < S.n_jobs; ++j) S.job_queue[j] = S.jobs_in[j].queue;
  }
  S.task_rank.clear();  // computed by derive_host
  phase("plugins+rest");
  return KBG_OK;
}

// S.task_uid_key[from, n_tasks): each UID's first 16 bytes, big-endian and
// zero-padded, so unequal keys order the UIDs as their bytes do
void fill_uid_keys(Session& S, int32_t from) {
  S.task_uid_key.resize(S.n_tasks);
  for (int32_t t = from; t < S.n_tasks; ++t) {
    const std::string& u = S.strs[S.tasks_in[t].uid];
    uint64_t a = 0, b = 0;
    for (size_t i = 0; i < 8; ++i) a = a << 8 | (i < u.size() ? (uint8_t)u[i] : 0);
    for (size_t i = 8; i < 16; ++i) b = b << 8 | (i < u.size() ? (uint8_t)u[i] : 0);
    S.task_uid_key[t] = Session::UidKey{a, b};
  }
}

enum { DERIVE_OK = 0, DERIVE_REBUILD = 1 };  // REBUILD: the static classes / masks must be recompiled

// Every host structure that follows from the inputs. `sh` non-null: compile
// the static predicate classes (build); null: keep the session's classes and
// map each candidate task to its spec's class (update), or ask for a rebuild
// when a candidate needs a class the session does not have.
void pin_near(int cpu, int nth);

// Sorted, duplicate-free ids in [0, n): a flag sweep when the list is a
// sizeable share of the range (a bind update touches every placed task: a
// comparison sort of 500k ids was a third of its derive), else a sort.
void sort_unique_ids(std::vector<int32_t>& v, int32_t n) {
  if (v.size() > 64 && (int64_t)v.size() * 16 > (int64_t)n) {
    std::vector<uint8_t> flag((size_t)std::max(n, 1), 0);
    for (const int32_t x : v) flag[x] = 1;
    v.clear();
    for (int32_t x = 0; x < n; ++x)
      if (flag[x]) v.push_back(x);
    return;
  }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

kbg_status derive_host(Session& S, kbg::StaticHost* sh, int* outcome) {
  *outcome = DERIVE_OK;
  S.job_chain_pgd = S.job_chain == std::vector<int32_t>{kbg::JO_PRIORITY, kbg::JO_GANG, kbg::JO_DRF};
  const int32_t N = S.n_nodes, T = S.n_tasks;
  static const bool prof = getenv("KBG_PROFILE_OPEN") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[kbg derive] %-20s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - tl).count());
    tl = now;
  };
  // bytewise UID order: TaskOrderFn's fallback compares tasks of one job only
  // (session_plugins.go:266-276), so a job that gained tasks is re-ranked alone
  // a full derive (open, or a rebuild after an update) recomputes everything;
  // an update's derive keeps what its events cannot have changed
  const bool full = sh != nullptr;
  // The ranks are computed on a worker of their own, beside this thread on
  // its last-level cache, while the phases up to the pending lists run (none
  // of them reads a rank or writes what the ranks are computed from: UIDs,
  // job task lists); joined before the pending lists sort by rank. The
  // victim lists below take a second worker.
  // A worker's exception (std::bad_alloc, std::length_error from a resize,
  // anything the KBG_CHECK_DERIVE comparison throws) is kept and rethrown on
  // this thread after the join, where derive_host's callers catch it.
  struct Worker {
    std::thread th;
    std::exception_ptr err;
    void join() {
      if (th.joinable()) th.join();
    }
    void rethrow() {
      if (err) std::rethrow_exception(err);
    }
    ~Worker() { join(); }
  };
  const int hcpu = sched_getcpu();
  // a worker that cannot be started runs inline
  auto start = [](Worker& w, auto&& fn) {
    try {
      w.th = std::thread(fn);
    } catch (const std::system_error&) {
      fn();
    }
  };
  Worker rwork;
  start(rwork, [&S, T, hcpu, &rwork] {
    pin_near(hcpu, 1);
    try {
  if (S.task_rank.empty() && T > 0) {
    // ranks are only ever compared between tasks of one job (the pending
    // lists, a job's re-rank after an update): each job's UIDs are ranked
    // alone, by their 16-byte keys and, on a tie, the strings
    fill_uid_keys(S, 0);
    S.task_rank.resize(T);
    S.job_rank_order.assign(S.n_jobs, {});
    S.job_rank_key.assign(S.n_jobs, {});
    const Session::UidKey* key = S.task_uid_key.data();
    const auto uid = [&](int32_t t) -> const std::string& { return S.strs[S.tasks_in[t].uid]; };
    const auto same = [&](int32_t a, int32_t b) { return key[a] == key[b] && uid(a) == uid(b); };
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      std::vector<int32_t>& ro = S.job_rank_order[j];
      ro = S.job_task_order[j];
      std::stable_sort(ro.begin(), ro.end(), [&](int32_t a, int32_t b) {
        return !(key[a] == key[b]) ? key[a] < key[b] : uid(a) < uid(b);
      });
      std::vector<Session::UidKey>& rk = S.job_rank_key[j];
      rk.resize(ro.size());
      int64_t r = 0;
      for (size_t i = 0; i < ro.size(); ++i) {
        if (i > 0 && !same(ro[i - 1], ro[i])) ++r;  // equal UIDs share a rank
        S.task_rank[ro[i]] = r * kRankGap;
        rk[i] = key[ro[i]];
      }
    }
  } else if (S.task_ranks_stale) {
    // a job that gained tasks: each new UID takes a rank between the ranked
    // tasks around it (the same rank as an equal UID); a job whose gap ran out
    // is renumbered first
    const int32_t T_old = (int32_t)S.task_rank.size();
    if (S.task_rank.capacity() < (size_t)T) S.task_rank.reserve((size_t)T + T / 4 + 1024);
    S.task_rank.resize(T, 0);
    if (S.task_uid_key.size() != (size_t)T_old) fill_uid_keys(S, 0);  // keys follow the ranks
    if (S.task_uid_key.capacity() < (size_t)T) S.task_uid_key.reserve((size_t)T + T / 4 + 1024);
    fill_uid_keys(S, T_old);
    std::sort(S.rank_dirty_jobs.begin(), S.rank_dirty_jobs.end());
    S.rank_dirty_jobs.erase(std::unique(S.rank_dirty_jobs.begin(), S.rank_dirty_jobs.end()), S.rank_dirty_jobs.end());
    const auto uid = [&](int32_t t) -> const std::string& { return S.strs[S.tasks_in[t].uid]; };
    // bytewise UID order: the 16-byte keys decide unless they tie
    const Session::UidKey* key = S.task_uid_key.data();
    const auto uid_less = [&](int32_t a, int32_t b) { return !(key[a] == key[b]) ? key[a] < key[b] : uid(a) < uid(b); };
    std::vector<int32_t> news;
    // a job's ranked tasks and their keys sit in two contiguous arrays; the
    // next jobs' arrays are requested a few jobs ahead (scattered rows:
    // latency, not work)
    const std::vector<int32_t>& dj = S.rank_dirty_jobs;
    auto ahead = [&](const void* p, size_t bytes) {
      const char* c = static_cast<const char*>(p);
      for (size_t o = 0; o < std::min<size_t>(bytes, 1024); o += 64) __builtin_prefetch(c + o);
    };
    for (size_t k = 0; k < dj.size(); ++k) {
      const int32_t j = dj[k];
      if (k + 4 < dj.size()) {
        __builtin_prefetch(&S.job_task_order[dj[k + 4]]);
        __builtin_prefetch(&S.job_rank_order[dj[k + 4]]);
        __builtin_prefetch(&S.job_rank_key[dj[k + 4]]);
      }
      if (k + 2 < dj.size()) {
        const std::vector<int32_t>& t2 = S.job_task_order[dj[k + 2]];
        const std::vector<Session::UidKey>& k2 = S.job_rank_key[dj[k + 2]];
        ahead(t2.data(), t2.size() * 4);
        ahead(k2.data(), k2.size() * sizeof(Session::UidKey));
        ahead(S.job_rank_order[dj[k + 2]].data(), S.job_rank_order[dj[k + 2]].size() * 4);
      }
      news.clear();
      for (int32_t t : S.job_task_order[j])
        if (t >= T_old) news.push_back(t);
      if (news.size() > 1) std::stable_sort(news.begin(), news.end(), uid_less);
      std::vector<int32_t>& ro = S.job_rank_order[j];
      std::vector<Session::UidKey>& rk = S.job_rank_key[j];
      if (rk.size() != ro.size()) {  // (never expected: kept beside ro)
        rk.resize(ro.size());
        for (size_t i = 0; i < ro.size(); ++i) rk[i] = key[ro[i]];
      }
      for (int32_t nt : news) {
        // upper_bound by (key, then UID string) over the contiguous keys
        const Session::UidKey kn = key[nt];
        size_t lo_i = 0, hi_i = ro.size();
        while (lo_i < hi_i) {
          const size_t mid = (lo_i + hi_i) / 2;
          const bool before = !(kn == rk[mid]) ? kn < rk[mid] : uid(nt) < uid(ro[mid]);
          if (before) hi_i = mid;
          else lo_i = mid + 1;
        }
        const size_t pos = lo_i;
        if (pos > 0 && rk[pos - 1] == kn && uid(ro[pos - 1]) == uid(nt)) {
          S.task_rank[nt] = S.task_rank[ro[pos - 1]];
        } else {
          auto bounds = [&](int64_t* lo, int64_t* hi) {
            *lo = pos > 0 ? S.task_rank[ro[pos - 1]] : (ro.empty() ? 0 : S.task_rank[ro[0]] - 2 * kRankGap);
            *hi = pos < ro.size() ? S.task_rank[ro[pos]] : (ro.empty() ? 2 * kRankGap : S.task_rank[ro.back()] + 2 * kRankGap);
          };
          int64_t lo, hi;
          bounds(&lo, &hi);
          if (hi - lo < 2) {  // no rank left between the neighbours: renumber the job (equal ranks stay equal)
            int64_t r = 0, prev = 0;
            for (size_t k2 = 0; k2 < ro.size(); ++k2) {
              const int64_t old = S.task_rank[ro[k2]];
              if (k2 > 0 && old != prev) ++r;
              prev = old;
              S.task_rank[ro[k2]] = r * kRankGap;
            }
            bounds(&lo, &hi);
          }
          S.task_rank[nt] = lo + (hi - lo) / 2;
        }
        ro.insert(ro.begin() + pos, nt);
        rk.insert(rk.begin() + pos, kn);
      }
    }
  }
  S.task_ranks_stale = false;
  S.rank_dirty_jobs.clear();
    } catch (...) {
      rwork.err = std::current_exception();
    }
  });
  // per-task vectors grow with every update's new pods: keep headroom so an
  // update does not reallocate (and copy) them
  auto headroom = [](auto& v, size_t n) {
    if (v.capacity() < n) v.reserve(n + n / 4 + 1024);
  };
  headroom(S.treq, T);
  headroom(S.task_node, T);
  headroom(S.task_cnode, T);
  headroom(S.task_job, T);
  headroom(S.tstat_in, T);
  headroom(S.pending_candidate, T);
  headroom(S.be_task, T);
  headroom(S.t_aff, T);
  headroom(S.t_ghost, T);
  headroom(S.t_inexact, T);
  headroom(S.t_pinexact, T);
  headroom(S.task_class, T);
  headroom(S.task_shape, T);
  headroom(S.shape_of_task, T);
  headroom(S.task_key, T);
  headroom(S.kc_cand, S.strs.size());
  headroom(S.kc_node, S.strs.size());
  headroom(S.key_hot, S.strs.size());
  // An update recomputes the tasks its events touched; their old candidate
  // state is kept aside for the counts below (`was`: bit 0 candidate, 1 BE).
  const bool incr = !full && (int32_t)S.pending_candidate.size() <= T && !S.t_aff.empty();
  sort_unique_ids(S.upd_tasks, T);
  std::vector<uint8_t> was;
  std::vector<uint16_t> was_stat;  // the touched tasks' statuses at the last derive
  const int32_t T_prev = (int32_t)S.tstat_in.size();
  auto task_row = [&](int32_t t) {
    S.treq[t] = to_res(S.tasks_in[t].resreq);
    S.task_job[t] = S.tasks_in[t].job;
    S.tstat_in[t] = (uint16_t)S.tasks_in[t].status;
    S.pending_candidate[t] = 0;
    S.be_task[t] = 0;
    if (!S.task_live[t]) return;
    // allocate.go:88-96: only Pending, non-BestEffort tasks enter the node loop
    S.pending_candidate[t] = S.tasks_in[t].status == KBG_PENDING && !kbg::res_empty(S.treq[t]);
    S.be_task[t] = S.tasks_in[t].status == KBG_PENDING && kbg::res_empty(S.treq[t]);
  };
  S.treq.resize(T);
  S.task_job.resize(T);
  S.tstat_in.resize(T);
  if (incr) {
    S.pending_candidate.resize(T, 0);
    S.be_task.resize(T, 0);
    was.resize(S.upd_tasks.size());
    was_stat.resize(S.upd_tasks.size());
    for (size_t i = 0; i < S.upd_tasks.size(); ++i) {
      const int32_t t = S.upd_tasks[i];
      was[i] = (S.pending_candidate[t] ? 1 : 0) | (S.be_task[t] ? 2 : 0);
      was_stat[i] = t < T_prev ? S.tstat_in[t] : 0;
      task_row(t);
    }
  } else {
    S.pending_candidate.assign(T, 0);
    S.be_task.assign(T, 0);
    for (int32_t t = 0; t < T; ++t) task_row(t);
  }

  phase("tasks");
  // ---- nodes
  S.idle.resize(N);
  S.rel.resize(N);
  S.ntasks.resize(N);
  S.maxtasks.resize(N);
  S.nil_node.resize(N);
  for (int32_t n = 0; n < N; ++n) {
    S.idle[n] = to_res(S.nodes_in[n].idle);
    S.rel[n] = to_res(S.nodes_in[n].releasing);
    S.ntasks[n] = S.nodes_in[n].num_tasks;
    S.maxtasks[n] = S.nodes_in[n].max_task_num;
    S.nil_node[n] = S.nodes_in[n].has_node ? 0 : 1;
  }
  S.any_nil = std::find(S.nil_node.begin(), S.nil_node.end(), 1) != S.nil_node.end();
  S.panic_node.assign(N, 0);
  if (S.pred_active)
    for (int32_t n = 0; n < N; ++n) S.panic_node[n] = S.nil_node[n];
  S.idle0 = S.idle;
  S.rel0 = S.rel;
  S.ntasks0 = S.ntasks;
  phase("nodes");
  // victim candidates (preempt/reclaim): session tasks Running on each node,
  // in NodeInfo.Tasks order; a task's node by NodeName (ssn.NodeIndex)
  if (full || (int32_t)S.task_node.size() != T || (int32_t)S.task_cnode.size() != T) {
    // (an update's events keep both current, apply_event)
    S.task_node.assign(T, -1);
    S.task_cnode.assign(T, -1);
    for (int32_t t = 0; t < T; ++t) {
      const int32_t nm = S.canon[S.tasks_in[t].node_name];
      if (S.strs[nm].empty()) continue;  // no NodeName: no lookup (event_handlers.go:45-48)
      auto it = S.node_of.find(nm);
      if (it != S.node_of.end()) {
        S.task_node[t] = S.task_cnode[t] = it->second;
      } else if (auto po = S.pod_only_of.find(nm); po != S.pod_only_of.end()) {
        S.task_cnode[t] = po->second;
      }
    }
  }
  // An update's events change a node's list only through its NodeInfo
  // (in_node_add / in_node_remove mark the node) and a task's status only by
  // moving it off and onto its node: the lists of the other nodes are copied
  // from the last derive, the marked ones (and the updated tasks' nodes) are
  // rebuilt.
  const bool vincr = incr && S.upd_nodes_valid && (int32_t)S.nt_off.size() == N + 1;
  std::vector<int32_t>& off = vincr ? S.nt_off_buf : S.nt_off;
  std::vector<int32_t>& vt = vincr ? S.nt_task_buf : S.nt_task;
  std::vector<uint8_t> vdirty;
  if (vincr) {
    vdirty.assign(N, 0);
    for (int32_t n : S.upd_nodes) vdirty[n] = 1;
    for (int32_t t : S.upd_tasks)
      if (S.task_node[t] >= 0 && S.task_node[t] < N) vdirty[S.task_node[t]] = 1;
    vt.reserve(S.nt_task.size() + S.upd_tasks.size());
  }
  S.upd_nodes_valid = false;
  // The lists are built on a thread of their own while the phases below run
  // (none of them reads the lists or writes what the lists are built from:
  // node_task_order, tstat_in, task_node); joined before derive_host returns.
  const bool check = !full && getenv("KBG_CHECK_DERIVE") != nullptr;
  bool vbad = false;
  Worker vwork;
  auto victims = [&S, &off, &vt, &vbad, &vwork, N, vincr, check, hcpu, vdirty = std::move(vdirty)] {
    pin_near(hcpu, 2);  // beside this thread, on its last-level cache (the lists are warm there)
    try {
    off.assign(N + 1, 0);
    vt.clear();
    int32_t mc = 0;
    for (int32_t n = 0; n < N; ++n) {
      if (vincr && !vdirty[n]) {
        vt.insert(vt.end(), S.nt_task.begin() + S.nt_off[n], S.nt_task.begin() + S.nt_off[n + 1]);
      } else {
        for (int32_t t : S.node_task_order[n])
          if (S.tstat_in[t] == KBG_RUNNING) vt.push_back(t);
      }
      off[n + 1] = (int32_t)vt.size();
      mc = std::max(mc, off[n + 1] - off[n]);
    }
    S.max_candidates = mc;
    if (vincr) {
      S.nt_off.swap(S.nt_off_buf);
      S.nt_task.swap(S.nt_task_buf);
    }
    // KBG_CHECK_DERIVE=1 (tests): an update's incremental results against the
    // full recomputation, bit for bit
    if (check) {
      std::vector<int32_t> o2(N + 1, 0), t2;
      for (int32_t n = 0; n < N; ++n) {
        for (int32_t t : S.node_task_order[n])
          if (S.tstat_in[t] == KBG_RUNNING) t2.push_back(t);
        o2[n + 1] = (int32_t)t2.size();
      }
      vbad = o2 != S.nt_off || t2 != S.nt_task;
    }
    } catch (...) {
      vwork.err = std::current_exception();
    }
  };
  start(vwork, victims);
  phase("victims");
  setup_pod_keys(S, incr, &S.upd_tasks, &was);

  phase("pod keys");
  // ---- engine initial state
  Engine& E = S.init;
  // an update recomputes the ready counts and drf allocations of the jobs its
  // events touched (each from its own tasks, in order: the same sums)
  const bool jincr = incr && (int32_t)E.jalloc.size() == S.n_jobs && (int32_t)S.job_ready0.size() == S.n_jobs;
  std::vector<Res> prev_jalloc;
  std::vector<int32_t> prev_jready;
  std::vector<char> jtouch;
  if (jincr) {
    prev_jalloc = std::move(E.jalloc);
    prev_jready = std::move(S.job_ready0);
    jtouch.assign(S.n_jobs, 0);
    for (int32_t j : S.pend_dirty_jobs) jtouch[j] = 1;
  }
  E = Engine{};
  E.jalloc.assign(S.n_jobs, Res{});
  E.jshare.assign(S.n_jobs, 0.0);
  E.jready.assign(S.n_jobs, 0);
  E.qalloc.assign(S.n_queues, Res{});
  E.qshare.assign(S.n_queues, 0.0);
  E.cursor.assign(S.n_jobs, 0);
  S.q_has_attr.assign(S.n_queues, 0);
  S.q_deserved.assign(S.n_queues, Res{});
  S.q_request.assign(S.n_queues, Res{});
  S.jt_off.assign(S.n_jobs + 1, 0);
  S.jt.clear();
  for (int32_t j = 0; j < S.n_jobs; ++j) {
    S.jt.insert(S.jt.end(), S.job_task_order[j].begin(), S.job_task_order[j].end());
    S.jt_off[j + 1] = (int32_t)S.jt.size();
  }
  auto job_tasks = [&](int32_t j) { return std::make_pair(S.jt.begin() + S.jt_off[j], S.jt.begin() + S.jt_off[j + 1]); };
  phase("job lists");
  if (jincr) {
    // counts: the updated tasks' old statuses out, their new ones in (a task
    // below T_prev was live, in its job's list, at the last derive)
    E.jready = std::move(prev_jready);
    for (size_t i = 0; i < S.upd_tasks.size(); ++i) {
      const int32_t t = S.upd_tasks[i];
      const int32_t j = S.task_job[t];
      if (t < T_prev && ready_status(was_stat[i])) E.jready[j]--;
      if (S.task_live[t] && ready_status(S.tstat_in[t])) E.jready[j]++;
    }
  } else {
    for (int32_t j = 0; j < S.n_jobs; ++j)
      for (auto [b, e] = job_tasks(j); b != e; ++b)
        if (ready_status(S.tstat_in[*b])) E.jready[j]++;
  }
  S.job_ready0 = E.jready;

  phase("ready counts");
  S.drf_total = Res{};
  S.prop_total = Res{};
  bool prop_exact = false;  // every queue sum below is an exact integer sum (proportion block)
  // drf.go:55-78, after the proportion sums (they say whether the job sums
  // are exact): an update's job allocations follow from its tasks' old and
  // new statuses when every request is an integer and every sum stays below
  // 2^53 (any summation order then gives the same doubles), else each
  // touched job is summed again in task order
  auto drf_block = [&]() {
    if (!S.has_drf) return;
    for (int32_t n = 0; n < N; ++n) kbg::res_add(S.drf_total, to_res(S.nodes_in[n].allocatable));
    const bool dexact = jincr && prop_exact && S.jalloc_exact;
    if (dexact) {
      E.jalloc = std::move(prev_jalloc);
      for (size_t i = 0; i < S.upd_tasks.size(); ++i) {  // out first: the partial sums stay below the final
        const int32_t t = S.upd_tasks[i];
        if (t < T_prev && allocated_status(was_stat[i])) {
          Res& a = E.jalloc[S.task_job[t]];
          const Res& r = S.treq[t];
          a = Res{a.c - r.c, a.m - r.m, a.g - r.g};
        }
      }
      for (int32_t t : S.upd_tasks)
        if (S.task_live[t] && allocated_status(S.tstat_in[t])) kbg::res_add(E.jalloc[S.task_job[t]], S.treq[t]);
    }
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      if (!dexact) {
        if (jincr && !jtouch[j]) {
          E.jalloc[j] = prev_jalloc[j];
        } else {
          for (auto [b, e] = job_tasks(j); b != e; ++b)
            if (allocated_status(S.tstat_in[*b])) kbg::res_add(E.jalloc[j], S.treq[*b]);
        }
      }
      E.jshare[j] = share_of(E.jalloc[j], S.drf_total);  // the total may have changed (SetNode)
    }
  };
  // proportion.go:54-144 (queue attrs in order of first job)
  if (S.has_prop) {
    for (int32_t n = 0; n < N; ++n) kbg::res_add(S.prop_total, to_res(S.nodes_in[n].allocatable));
    for (const kbg_resource& o : S.others_in)
      if (!kbg::res_sub(S.prop_total, to_res(o)))
        return fail(KBG_E_REF_PANIC, "proportion: Others exceed the cluster total (proportion.go:61-63)");
    std::vector<int32_t> qorder;
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      const int32_t q = S.job_queue[j];
      if (!S.q_has_attr[q]) {
        S.q_has_attr[q] = 1;
        qorder.push_back(q);
      }
    }
    // a task's part of its queue's sums: allocated -> both, Pending -> request
    constexpr double kExact = 9007199254740992.0;  // 2^53
    auto pexact = [&](const Res& r) {
      auto ok = [&](double v) { return v >= 0 && v <= kExact && v == (double)(int64_t)v; };
      return ok(r.c) && ok(r.m) && ok(r.g);
    };
    auto psum = [&](int32_t t, int32_t st, int sign) {
      if (S.t_pinexact[t]) {
        S.n_pinexact += sign;
        return;
      }
      const bool a = allocated_status(st);
      if (!a && st != KBG_PENDING) return;
      const int32_t q = S.job_queue[S.task_job[t]];
      const Res& r = S.treq[t];
      const __int128 v[3] = {(__int128)(int64_t)r.c, (__int128)(int64_t)r.m, (__int128)(int64_t)r.g};
      for (int d = 0; d < 3; ++d) {
        if (a) S.qa_sum[3 * (size_t)q + d] += sign * v[d];
        S.qr_sum[3 * (size_t)q + d] += sign * v[d];
      }
    };
    bool exact_sums = false;
    if (incr && S.prop_sums_ok && (int32_t)S.qa_sum.size() == 3 * S.n_queues) {
      S.t_pinexact.resize(T, 0);
      for (size_t i = 0; i < S.upd_tasks.size(); ++i) {
        const int32_t t = S.upd_tasks[i];
        if (t < T_prev) psum(t, was_stat[i], -1);  // live at the last derive (events only touch live tasks)
        if (t >= T_prev) S.t_pinexact[t] = !pexact(S.treq[t]);
        if (S.task_live[t]) psum(t, S.tstat_in[t], +1);
      }
      exact_sums = S.n_pinexact == 0;
    } else {  // (re)build the sums from every live task
      S.t_pinexact.assign(T, 0);
      S.n_pinexact = 0;
      S.qa_sum.assign(3 * (size_t)S.n_queues, 0);
      S.qr_sum.assign(3 * (size_t)S.n_queues, 0);
      for (int32_t j = 0; j < S.n_jobs; ++j)
        for (auto [b, e] = job_tasks(j); b != e; ++b) {
          S.t_pinexact[*b] = !pexact(S.treq[*b]);
          psum(*b, S.tstat_in[*b], +1);
        }
      S.prop_sums_ok = true;
      exact_sums = S.n_pinexact == 0;
    }
    for (int32_t q = 0; q < S.n_queues && exact_sums; ++q)
      for (int d = 0; d < 3; ++d)
        if (S.qr_sum[3 * (size_t)q + d] > (__int128)kExact) exact_sums = false;
    prop_exact = exact_sums;
    if (exact_sums) {
      for (int32_t q = 0; q < S.n_queues; ++q) {
        E.qalloc[q] = Res{(double)(int64_t)S.qa_sum[3 * (size_t)q], (double)(int64_t)S.qa_sum[3 * (size_t)q + 1],
                          (double)(int64_t)S.qa_sum[3 * (size_t)q + 2]};
        S.q_request[q] = Res{(double)(int64_t)S.qr_sum[3 * (size_t)q], (double)(int64_t)S.qr_sum[3 * (size_t)q + 1],
                             (double)(int64_t)S.qr_sum[3 * (size_t)q + 2]};
      }
    } else {  // the reference's sequential fp64 sums, job by job, task by task
      for (int32_t j = 0; j < S.n_jobs; ++j) {
        const int32_t q = S.job_queue[j];
        for (auto [b, e] = job_tasks(j); b != e; ++b) {
          const int32_t s = S.tstat_in[*b];
          if (allocated_status(s)) {
            kbg::res_add(E.qalloc[q], S.treq[*b]);
            kbg::res_add(S.q_request[q], S.treq[*b]);
          } else if (s == KBG_PENDING) {
            kbg::res_add(S.q_request[q], S.treq[*b]);
          }
        }
      }
    }
    Res remaining = S.prop_total;
    std::vector<char> meet(S.n_queues, 0);
    for (;;) {
      int32_t total_w = 0;
      for (int32_t q : qorder)
        if (!meet[q]) total_w += S.queues_in[q].weight;
      if (total_w == 0) break;
      Res deserved;
      for (int32_t q : qorder) {
        if (meet[q]) continue;
        const double ratio = (double)S.queues_in[q].weight / (double)total_w;
        Res part{remaining.c * ratio, remaining.m * ratio, remaining.g * ratio};
        kbg::res_add(S.q_deserved[q], part);
        if (!kbg::res_le(S.q_deserved[q], S.q_request[q])) {
          const Res d = S.q_deserved[q], r = S.q_request[q];
          S.q_deserved[q] = Res{go_min(d.c, r.c), go_min(d.m, r.m), go_min(d.g, r.g)};
          meet[q] = 1;
        }
        E.qshare[q] = share_of(E.qalloc[q], S.q_deserved[q]);
        kbg::res_add(deserved, S.q_deserved[q]);
      }
      if (!kbg::res_sub(remaining, deserved))
        return fail(KBG_E_REF_PANIC, "proportion water-fill: remaining.Sub(deserved) underflow (proportion.go:140, SURVEY F9)");
      if (kbg::res_empty(remaining)) break;
    }
  }

  phase("proportion");
  drf_block();
  S.jalloc_exact = prop_exact;
  if (check) {
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      int32_t r = 0;
      Res a{};
      for (auto [b, e] = job_tasks(j); b != e; ++b) {
        if (ready_status(S.tstat_in[*b])) ++r;
        if (allocated_status(S.tstat_in[*b])) kbg::res_add(a, S.treq[*b]);
      }
      if (r != E.jready[j]) return fail(KBG_E_INVALID, "internal: incremental ready count differs");
      if (S.has_drf && std::memcmp(&a, &E.jalloc[j], sizeof(Res)) != 0)
        return fail(KBG_E_INVALID, "internal: incremental drf allocation differs");
    }
  }
  phase("drf");
  // ---- predicates preconditions
  const bool had_ghost = S.ghost;
  {
    // per task: a pod (anti)affinity spec (kbg_affinity.cpp) and the ghost
    // rule (an allocated task whose node is outside the session), counted
    auto flags = [&](int32_t t) {
      S.n_aff -= S.t_aff[t];
      S.n_ghost -= S.t_ghost[t];
      S.t_aff[t] = S.t_ghost[t] = 0;
      if (!S.task_live[t]) return;
      const kbg_task& tk = S.tasks_in[t];
      const kbg_spec* sp = tk.spec >= 0 ? &S.specs_in[tk.spec] : nullptr;
      S.t_aff[t] = sp && (sp->aff_len > 0 || sp->anti_len > 0);
      S.t_ghost[t] = allocated_status(tk.status) && S.task_node[t] < 0;
      S.n_aff += S.t_aff[t];
      S.n_ghost += S.t_ghost[t];
    };
    if (incr) {
      S.t_aff.resize(T, 0);
      S.t_ghost.resize(T, 0);
      for (int32_t t : S.upd_tasks) flags(t);
    } else {
      S.t_aff.assign(T, 0);
      S.t_ghost.assign(T, 0);
      S.n_aff = S.n_ghost = 0;
      for (int32_t t = 0; t < T; ++t) flags(t);
    }
    S.has_aff = S.pred_active && S.n_aff > 0;
    S.ghost = S.pred_active && S.n_ghost > 0;
  }

  phase("preconditions");
  rwork.join();
  phase("ranks join");
  rwork.rethrow();
  // ---- pending task lists in TaskOrderFn order (session_plugins.go:266-276)
  // an update's derive copies the lists of the jobs no event touched
  const bool keep_lists = !full && (int32_t)S.pend_off_all.size() == S.n_jobs;
  std::vector<char> jdirty, listed;
  std::vector<int32_t> fresh_off, fresh;  // per dirty job: its tasks that entered Pending through an event
  std::vector<int32_t> merge_tmp;
  auto task_before = [&](int32_t a, int32_t c) {
    if (S.task_order_prio && S.tasks_in[a].priority != S.tasks_in[c].priority)
      return S.tasks_in[a].priority > S.tasks_in[c].priority;
    return S.task_rank[a] < S.task_rank[c];
  };
  if (keep_lists) {
    listed.assign(T, 0);
    jdirty.assign(S.n_jobs, 0);
    for (int32_t j : S.pend_dirty_jobs) jdirty[j] = 1;
    std::sort(S.pend_new.begin(), S.pend_new.end());
    S.pend_new.erase(std::unique(S.pend_new.begin(), S.pend_new.end()), S.pend_new.end());
    fresh_off.assign(S.n_jobs + 1, 0);
    for (int32_t t : S.pend_new)
      if (t < T && S.pending_candidate[t]) fresh_off[S.task_job[t] + 1]++;
    for (int32_t j = 0; j < S.n_jobs; ++j) fresh_off[j + 1] += fresh_off[j];
    fresh.assign(fresh_off[S.n_jobs], 0);
    std::vector<int32_t> at(fresh_off.begin(), fresh_off.end() - 1);
    for (int32_t t : S.pend_new)
      if (t < T && S.pending_candidate[t]) fresh[at[S.task_job[t]]++] = t;
  }
  S.pend_dirty_jobs.clear();
  S.pend_new.clear();
  S.pend_off.assign(S.n_jobs, 0);
  S.pend_len.assign(S.n_jobs, 0);
  S.pend.clear();
  S.pend.reserve(keep_lists ? S.pend_all.size() + 1024 : 0);
  for (int32_t j = 0; j < S.n_jobs; ++j) {
    S.pend_off[j] = (int32_t)S.pend.size();
    if (keep_lists) {
      const auto b0 = S.pend_all.begin() + S.pend_off_all[j];
      if (!jdirty[j]) {
        S.pend.insert(S.pend.end(), b0, b0 + S.pend_len_all[j]);
        S.pend_len[j] = S.pend_len_all[j];
        continue;
      }
      // the old list minus the tasks that left Pending (order kept), merged
      // with the tasks that entered it
      for (auto b = b0; b != b0 + S.pend_len_all[j]; ++b)
        if (*b < T && S.pending_candidate[*b]) {
          S.pend.push_back(*b);
          listed[*b] = 1;
        }
      auto f0 = fresh.begin() + fresh_off[j], f1 = fresh.begin() + fresh_off[j + 1];
      f1 = std::remove_if(f0, f1, [&](int32_t t) { return listed[t] != 0; });  // already Pending before the event
      for (auto b = S.pend.begin() + S.pend_off[j]; b != S.pend.end(); ++b) listed[*b] = 0;
      if (f0 != f1) {  // a stable merge (old tasks first among equals) through one reused buffer
        std::sort(f0, f1, task_before);
        const size_t o = S.pend_off[j], mid = S.pend.size();
        merge_tmp.assign(S.pend.begin() + o, S.pend.begin() + mid);
        S.pend.resize(mid + (f1 - f0));
        std::merge(merge_tmp.begin(), merge_tmp.end(), f0, f1, S.pend.begin() + o, task_before);
      }
      S.pend_len[j] = (int32_t)S.pend.size() - S.pend_off[j];
      continue;
    }
    for (auto [b, e] = job_tasks(j); b != e; ++b)
      if (S.pending_candidate[*b]) S.pend.push_back(*b);
    std::sort(S.pend.begin() + S.pend_off[j], S.pend.end(), task_before);
    S.pend_len[j] = (int32_t)S.pend.size() - S.pend_off[j];
  }

  phase("pend lists");
  // ---- per-queue job heaps (allocate.go:45-59)
  S.joff.assign(S.n_queues, 0);
  S.jcap.assign(S.n_queues, 0);
  for (int32_t j = 0; j < S.n_jobs; ++j) S.jcap[S.job_queue[j]]++;
  for (int32_t q = 1; q < S.n_queues; ++q) S.joff[q] = S.joff[q - 1] + S.jcap[q - 1] + kJobHeapPad;
  S.pend_all = S.pend;
  S.pend_off_all = S.pend_off;
  S.pend_len_all = S.pend_len;
  S.job_min.resize(S.n_jobs);
  for (int32_t j = 0; j < S.n_jobs; ++j) S.job_min[j] = S.jobs_in[j].min_available;
  build_heaps(S, E);

  phase("heaps");
  // ---- static predicate classes
  if (sh) {
    compile_static_predicates(S, sh);
    S.n_classes = sh->n_classes;
  } else {
    if (S.ghost != had_ghost) {  // the ghost rule fails every node (NF_DEAD): the masks change
      *outcome = DERIVE_REBUILD;
      return KBG_OK;
    }
    auto cls = [&](int32_t t) {  // false: a pod spec no candidate had at open (compile its class)
      S.task_class[t] = 0;
      if (!S.pred_active || (!S.pending_candidate[t] && !S.be_task[t])) return true;
      const int32_t sp = S.tasks_in[t].spec;
      const int32_t c = sp >= 0 ? S.spec_class[sp] : S.nospec_class;
      if (c < 0) return false;
      S.task_class[t] = c;
      return true;
    };
    bool ok = true;
    if (incr) {
      S.task_class.resize(T, 0);
      for (int32_t t : S.upd_tasks) ok = ok && cls(t);
    } else {
      S.task_class.assign(T, 0);
      for (int32_t t = 0; t < T && ok; ++t) ok = cls(t);
    }
    if (!ok) {
      *outcome = DERIVE_REBUILD;
      return KBG_OK;
    }
  }
  phase("classes");
  S.W = (N + 63) / 64;
  // ---- integer scan mode (kbg_device.hpp TaskRec): every value the scan
  // compares is an exact integer and stays one through the cycle
  {
    constexpr double kLim = 2251799813685248.0;  // 2^51
    auto exact = [&](double v) { return std::fabs(v) <= kLim && v == (double)(int64_t)v; };  // (NaN fails the bound)
    bool ok = true;
    for (int32_t n = 0; n < N && ok; ++n)
      ok = exact(S.idle[n].c) && exact(S.idle[n].m) && exact(S.idle[n].g) && exact(S.rel[n].c) &&
           exact(S.rel[n].m) && exact(S.rel[n].g);
    // every candidate's request an exact non-negative integer, and their sum
    // (exact as an integer; the doubles summed in any order agree on the bound)
    // within 2^51: counts of the candidates, kept per task across updates
    auto contrib = [&](int32_t t, int sign) {
      if (S.t_inexact[t]) {
        S.n_inexact += sign;
        return;
      }
      const Res& q = S.treq[t];
      S.isum_c += sign * (__int128)(int64_t)q.c;
      S.isum_m += sign * (__int128)(int64_t)q.m;
      S.isum_g += sign * (__int128)(int64_t)q.g;
    };
    auto enter = [&](int32_t t) {  // t is a candidate now
      const Res& q = S.treq[t];
      S.t_inexact[t] = !(exact(q.c) && exact(q.m) && exact(q.g) && q.c >= 0 && q.m >= 0 && q.g >= 0);
      contrib(t, +1);
    };
    if (incr) {
      S.t_inexact.resize(T, 0);
      for (size_t i = 0; i < S.upd_tasks.size(); ++i) {
        const int32_t t = S.upd_tasks[i];
        if (was[i] & 1) contrib(t, -1);  // the old candidate leaves (its request never changes)
        if (S.pending_candidate[t]) enter(t);
      }
    } else {
      S.t_inexact.assign(T, 0);
      S.n_inexact = 0;
      S.isum_c = S.isum_m = S.isum_g = 0;
      for (int32_t t = 0; t < T; ++t)
        if (S.pending_candidate[t]) enter(t);
    }
    const __int128 lim = (__int128)kLim;
    ok = ok && S.n_inexact == 0 && S.isum_c <= lim && S.isum_m <= lim && S.isum_g <= lim;
    S.int_mode = ok && getenv("KBG_FORCE_GENERAL_SCAN") == nullptr;
  }
  phase("int mode");
  // ---- (class, request) shapes of the candidates
  // Shape ids persist across updates (a task's class and request never
  // change): an update looks up only the tasks that are new candidates.
  {
    if (full) {
      S.shape_ids.clear();
      S.shape_task.clear();
      S.shape_of_task.assign(T, -1);
      S.be_shape.assign(std::max(1, S.n_classes), -1);
      S.n_shapes = 0;
    } else {
      S.shape_of_task.resize(T, -1);
      if ((int32_t)S.be_shape.size() < std::max(1, S.n_classes)) S.be_shape.resize(std::max(1, S.n_classes), -1);
    }
    auto cand_shape = [&](int32_t t) {
      if (!S.pending_candidate[t]) return;
      int32_t& sh_t = S.shape_of_task[t];
      if (sh_t < 0) {
        auto it = S.shape_ids.emplace(kbg::ShapeKey{S.task_class[t], S.treq[t].c, S.treq[t].m, S.treq[t].g}, S.n_shapes);
        if (it.second) S.n_shapes++;
        sh_t = it.first->second;
      }
      S.task_shape[t] = sh_t;
      if ((int32_t)S.shape_task.size() <= sh_t) S.shape_task.resize((size_t)sh_t + 1, -1);
      int32_t& rep = S.shape_task[sh_t];
      if (rep < 0 || rep >= T || S.task_shape[rep] != sh_t) rep = t;
    };
    // backfill rows: one grouping id per class (the request does not matter)
    auto be_shape = [&](int32_t t) {
      if (!S.be_task[t]) return;
      int32_t& b = S.be_shape[S.task_class[t]];
      if (b < 0) b = S.n_shapes++;
      S.task_shape[t] = b;
    };
    if (incr) {
      S.task_shape.resize(T, -1);
      for (int32_t t : S.upd_tasks) {
        S.task_shape[t] = -1;
        cand_shape(t);
      }
      for (int32_t t : S.upd_tasks) be_shape(t);
    } else {
      S.task_shape.assign(T, -1);
      for (int32_t t = 0; t < T; ++t) cand_shape(t);
      for (int32_t t = 0; t < T; ++t) be_shape(t);
    }
  }
  S.upd_tasks.clear();
  // each shape's request (a shape is one (class, request) value; a task's
  // request never changes, so any task that had the shape gives it)
  S.shape_req.assign(std::max(1, S.n_shapes), Res{});
  for (int32_t sh = 0; sh < (int32_t)S.shape_task.size() && sh < S.n_shapes; ++sh) {
    const int32_t rep = S.shape_task[sh];
    if (rep >= 0 && rep < T) S.shape_req[sh] = S.treq[rep];
  }
  phase("shapes");
  vwork.join();
  phase("victims join");
  vwork.rethrow();
  if (vbad) return fail(KBG_E_INVALID, "internal: incremental victim lists differ");
  return KBG_OK;
}

// Derived state, device tables and static masks from the session's inputs.
kbg_status build(Session& S, kbg_comm* comm, const std::function<void(const char*)>& phase) {
  kbg_status st;
  kbg::StaticHost sh;
  int outcome;
  if ((st = derive_host(S, &sh, &outcome)) != KBG_OK) return st;
  phase("plugins+ranks+engine+static");
  const int32_t N = S.n_nodes;
  // ---- node-axis shards: contiguous 64-node word ranges, so
  // rank order is node order and first-fit survives the split
  S.comm = comm;
  S.R = std::max(1, S.opts.shards);
  if (comm) {
    if (S.opts.shards > 0 && S.opts.shards != comm->n_ranks)
      return fail(KBG_E_INVALID, "options.shards differs from the communicator size");
    S.R = comm->n_ranks;
    S.shard = comm->rank;
  }
  if (S.R > 1024) return fail(KBG_E_INVALID, "shards > 1024");
  S.Wl = std::max(1, (S.W + S.R - 1) / S.R);
  if (S.comm) {
    S.tab_lo = std::min(N, S.shard * S.Wl * 64);
    S.tab_n = std::min(N, (S.shard + 1) * S.Wl * 64) - S.tab_lo;
  } else {
    S.tab_lo = 0;
    S.tab_n = N;
  }

  // candidate slots: grouped, sum over shapes of min(n_s + slack, 4096) <= K (slack + 1);
  // full-scan, K rows x M plus the long list of each shape's last row (sessions
  // that gain shapes in an update share what is left: Grouper::build)
  S.n_shapes_cap = std::max(S.n_shapes, 64);
  S.cand_cap = S.opts.full_scan
                   ? (int64_t)S.K * S.M + (int64_t)std::min(S.K, S.n_shapes_cap) * (kFullScanGrow + S.M)
                   : (int64_t)S.K * (kGroupSlack + 1);
  // ---- device
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(KBG_E_HIP, "no HIP device visible");
  S.device = S.opts.device >= 0 ? S.opts.device : 0;
  if (S.opts.device < 0) HIP_TRY(hipGetDevice(&S.device));
  if (comm) S.device = comm->device;
  HIP_TRY(hipSetDevice(S.device));
  HIP_TRY(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
  for (auto& e : S.ev) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipEventCreateWithFlags(&S.stage_ev, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&S.comm_ev, hipEventDisableTiming));
  S.stage_pending = false;
  if ((st = alloc_soa(S, &S.d_nodes)) || (st = alloc_soa(S, &S.d_nodes0))) return st;
  const size_t up_cap = up_bytes_for(S.K);
  S.up_cap = up_cap;
  // Host side (pinned, per stage; u32 units): per-slot info, the slots' word
  // masks and availability (fused path), and on a communicator also counts
  // and candidates (replicated path). Device side: the replicated path's
  // select output or the owner-resolve availability (K words, summed over
  // RCCL) — only a communicator needs either; the fused kernel writes its
  // results straight into the pinned buffer.
  const size_t repl_cap = 2 * (size_t)S.K + (size_t)S.cand_cap;
  const size_t fused_cap = fused_down_words(S.K, fused_mask_words(S));
  const size_t down_cap = S.comm ? std::max(repl_cap, fused_cap) : fused_cap;
  const size_t d_down_cap = S.comm ? std::max(repl_cap, (size_t)S.K) : 1;
  if ((st = dalloc(S, &S.d_class_mask, (size_t)S.n_classes * S.W)) ||
      (st = dalloc(S, &S.d_up, S.comm ? up_cap : 1)) ||
      (st = dalloc(S, &S.d_bits, S.comm ? (size_t)S.R * 2 * S.K * kbg::kbg_slot_words(S.Wl) : 1)) ||
      (st = dalloc(S, &S.d_down, d_down_cap)) ||
      (st = dalloc(S, &S.d_svc, S.comm ? fused_cap : 1)))  // the scan service's summed launch results
    return st;
  for (kbg::Stage& g : S.stages) {
    if ((st = host_alloc((void**)&g.h_up, up_cap)) || (st = host_alloc((void**)&g.h_down, down_cap * 4))) return st;
    for (int e = 0; e < 6; ++e) HIP_TRY(hipEventCreate(&g.ev[e]));
    HIP_TRY(hipEventCreateWithFlags(&g.ev[6], hipEventDisableTiming));
  }
  {  // unified addressing: a mapped host buffer has the same address on the device
    void* d = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&d, S.stages[0].h_up, 0));
    S.uva = d == (void*)S.stages[0].h_up;
  }
  if ((st = host_alloc((void**)&S.h_deltas, (size_t)S.K * sizeof(kbg::NodeDelta)))) return st;
  S.h_deltas_dev = dev_ptr(S, S.h_deltas);
  if (!S.h_deltas_dev) return fail(KBG_E_HIP, "hipHostGetDevicePointer of the node-delta buffer failed");
  if ((st = upload_nodes(S))) return st;
  phase("device alloc+nodes");

  {
    kbg::StaticTables& t = S.static_tab;
    t = kbg::StaticTables{};
    uint64_t *lb, *tb, *mp, *tp;
    int64_t* nv;
    uint8_t *nok, *nf;
    int32_t* nid;
    kbg::ReqProg* rq;
    kbg::TermProg* tm;
    kbg::ClassProg* cl;
    BulkUpload bu;  // the static predicate tables in one block, one copy
    bu.add(&lb, sh.label_bits);
    bu.add(&tb, sh.taint_bits);
    bu.add(&mp, sh.mask_pool);
    bu.add(&tp, sh.tol_pool);
    bu.add(&nv, sh.num_vals);
    bu.add(&nok, sh.num_ok);
    bu.add(&nf, sh.node_flags);
    bu.add(&nid, sh.name_id);
    bu.add(&rq, sh.reqs);
    bu.add(&tm, sh.terms);
    bu.add(&cl, sh.classes);
    if ((st = bu.commit(S))) return st;
    t.n_nodes = N;
    t.label_words = sh.label_words;
    t.taint_words = sh.taint_words;
    t.n_numcols = sh.n_numcols;
    t.label_bits = lb;
    t.taint_bits = tb;
    t.num_vals = nv;
    t.num_ok = nok;
    t.name_id = nid;
    t.node_flags = nf;
    t.mask_pool = mp;
    t.tol_pool = tp;
    t.reqs = rq;
    t.terms = tm;
    t.classes = cl;
    S.d_node_flags = nf;
    S.node_flags = sh.node_flags;
    HIP_TRY(kbg::launch_build_class_mask(t, S.n_classes, S.W, S.d_class_mask, S.stream));
    S.h_class_mask.resize((size_t)S.n_classes * S.W);
    HIP_TRY(hipMemcpyAsync(S.h_class_mask.data(), S.d_class_mask, S.h_class_mask.size() * 8, hipMemcpyDeviceToHost,
                           S.stream));
    HIP_TRY(hipStreamSynchronize(S.stream));  // sh's host vectors end with this scope
  }
  phase("class-mask kernel");
  // host ports: the port fit is folded into the class masks (setup_host_ports)
  S.h_class_mask_static = S.h_class_mask;
  setup_host_ports(S);
  setup_affinity(S);  // inter-pod (anti)affinity: folded in the same way (kbg_affinity.cpp)
  if ((st = host_alloc((void**)&S.h_mdeltas, (size_t)kbg::kMaskDeltaCap * sizeof(kbg::MaskDelta)))) return st;
  if (S.has_ports || S.has_aff)
    HIP_TRY(hipMemcpy(S.d_class_mask, S.h_class_mask.data(), S.h_class_mask.size() * 8, hipMemcpyHostToDevice));
  S.h_class_mask0 = S.h_class_mask;
  phase("ports+affinity");
  S.stats.n_classes = S.n_classes;
  S.stats.shards = S.R;
  S.stats.shard_index = S.comm ? S.shard : -1;
  S.stats.int_scan = S.int_mode ? 1 : 0;
  return KBG_OK;
}

kbg_status open_session(Session& S, const kbg_snapshot* snap, const kbg_options* o, kbg_comm* comm) {
  const auto t_open = std::chrono::steady_clock::now();
  // opt-in phase timing of the session open (KBG_PROFILE_OPEN=1)
  const bool prof = getenv("KBG_PROFILE_OPEN") != nullptr;
  auto t_last = t_open;
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[kbg open] %-24s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - t_last).count());
    t_last = now;
  };
  kbg_status st = ingest(S, snap, o);
  if (st != KBG_OK) return st;
  phase("validate+copy+strings");
  if ((st = build(S, comm, phase)) != KBG_OK) return st;
  S.stats.open_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_open).count();
  return KBG_OK;
}

// The host side of one allocate cycle runs on two threads:
//   predictor (std::thread) — the ordering engine: predicts batches of K task
//                             evaluations ahead, each with a checkpoint of the
//                             engine state it started from;
//   committer (caller)      — per batch: device scan, in-order commit against
//                             the candidates, node-row write-back.
// When a batch is cut (an unpredicted outcome or an exhausted candidate list)
// the committer bumps the epoch and hands the predictor the batch's
// checkpoint plus the actual outcomes up to the cut; the predictor restores,
// replays them and continues; batches of an older epoch are dropped.
// Opt-in timeline of an allocate cycle (KBG_TRACE=1): per thread, (µs since
// the cycle start, event, value), printed to stderr when the cycle ends.
struct Trace {
  using clk = std::chrono::steady_clock;
  bool on = false;
  clk::time_point t0;
  std::vector<std::tuple<double, const char*, int64_t>> ev;
  void start(clk::time_point t) {
    on = getenv("KBG_TRACE") != nullptr;
    t0 = t;
    if (on) ev.reserve(4096);
  }
  void add(const char* what, int64_t v = 0) {
    if (on) ev.emplace_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count(), what, v);
  }
};
void trace_add(const char* what, int64_t v) {
  if (t_trace) t_trace->add(what, v);
}
void print_traces(const Trace& a, const Trace& b) {
  if (!a.on) return;
  std::vector<std::tuple<double, const char*, int64_t, char>> all;
  for (auto& [t, w, v] : a.ev) all.emplace_back(t, w, v, 'C');
  for (auto& [t, w, v] : b.ev) all.emplace_back(t, w, v, 'P');
  std::sort(all.begin(), all.end(), [](const auto& x, const auto& y) { return std::get<0>(x) < std::get<0>(y); });
  for (auto& [t, w, v, who] : all) fprintf(stderr, "[kbg trace] %9.1f %c %-10s %lld\n", t, who, w, (long long)v);
}

// A condition variable whose waiters spin briefly before they block: the
// hand-offs of an allocate cycle (predictor -> committer batches, rollbacks,
// the truth engine) are tens of microseconds apart, less than a futex wake-up
// takes to come back. Every state change a waiter can see is followed by
// notify_all(), which bumps `gen`; a waiter re-checks its predicate under the
// lock whenever gen moves, for about 50 us, then sleeps on the real
// condition variable.
struct SpinCV {
  std::condition_variable cv;
  std::atomic<uint64_t> gen{0};
  void notify_all() {
    gen.fetch_add(1, std::memory_order_release);
    cv.notify_all();
  }
  template <class Pred>
  void wait(std::unique_lock<std::mutex>& lk, Pred pred) {
    if (pred()) return;
    constexpr int kSpins = 4096;
    for (int i = 0; i < kSpins;) {
      const uint64_t g = gen.load(std::memory_order_acquire);
      lk.unlock();
      while (gen.load(std::memory_order_acquire) == g && ++i < kSpins) __builtin_ia32_pause();
      lk.lock();
      if (pred()) return;
    }
    cv.wait(lk, pred);
  }
};

// A shape is known to fit nowhere (the committer's side of the flags the
// predictor reads every step): store only when the flag is still clear, so
// the line stays shared in the predictor's cache instead of being
// invalidated by every failed task.
inline void mark_failed(std::atomic<uint8_t>* f, int32_t sh) {
  if (!f[sh].load(std::memory_order_relaxed)) f[sh].store(1, std::memory_order_relaxed);
}

struct Batch {
  std::vector<int32_t> bt;
  std::vector<char> bpred;
  // per entry: the tasks of its job right after it, of shapes known to fit
  // nowhere, consumed with it as failures (Ops::skip_dead); 0 for most
  std::vector<int32_t> brun;
  Engine ckpt;
  int64_t epoch = 0;
  // rows built ahead by the builder thread (G >= 0) into a pinned buffer
  // (st.h_up) that launch swaps with the stage's: no copy, and the buffer the
  // stage gives back has been read by its last upload (the stage was waited)
  kbg::Stage st;
  int32_t G = -1;
};

struct Pipe {
  std::mutex mu;
  SpinCV cv;
  std::deque<Batch*> ready;    // predicted, waiting for the committer
  std::vector<Batch*> free;    // recycled buffers
  int64_t epoch = 0;           // current epoch (committer-owned, read by predictor under mu)
  bool rollback = false;       // predictor must restore `rb_ckpt` and replay (or copy *rb_truth)
  Engine rb_ckpt;
  const Engine* rb_truth = nullptr;  // the committed outcomes' engine, idle until the next batch
  std::vector<int32_t> rb_tasks;
  std::vector<char> rb_actual;
  std::vector<int32_t> rb_runs;
  bool stop = false;
  std::atomic<bool> hungry{false};  // the committer is blocked on an empty queue: emit what is predicted
  std::atomic<int64_t> epoch_now{0};  // = epoch, read without the lock: a batch of an older epoch is abandoned
  std::deque<Batch*> raw;      // predicted, waiting for the builder (allocate_cycle)
  bool building = false;       // the builder holds a batch
  static constexpr size_t kDepth = 3;
  // how far the predictor may run ahead: batches queued and tasks per batch.
  // Past the first cut (the contended part of a cycle) every prediction
  // beyond the next cut is work thrown away, so the committer narrows both
  std::atomic<int32_t> depth{(int32_t)kDepth};
  std::atomic<int32_t> kmax{INT32_MAX};
};
// Smallest batch the predictor hands over early to a waiting committer (the
// first batch of an epoch, and near the end of the cycle); KBG_MIN_EMIT overrides.
int32_t min_emit() {
  static const int32_t v = [] {
    const char* e = getenv("KBG_MIN_EMIT");
    return e ? std::max(1, atoi(e)) : 512;
  }();
  return v;
}

// The predictor and the committer exchange batches, the failed-shape flags
// and the engine checkpoints: keep the predictor on another physical core of
// the committer's last-level cache (sysfs topology), never on its SMT
// sibling. KBG_NO_PIN=1 leaves placement to the OS.
void pin_near(int cpu, int nth = 1) {
  static const bool off = getenv("KBG_NO_PIN") != nullptr;
  if (off || cpu < 0) return;
  auto read_list = [](const std::string& path) {
    std::vector<int> out;
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return out;
    char buf[4096];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    buf[n] = 0;
    for (char* p = buf; *p;) {  // "0-7,128-135"
      char* e;
      const long a = std::strtol(p, &e, 10);
      if (e == p) break;
      long b = a;
      if (*e == '-') b = std::strtol(e + 1, &e, 10);
      for (long c = a; c <= b; ++c) out.push_back((int)c);
      p = (*e == ',') ? e + 1 : e;
      if (*p == '\n') break;
    }
    return out;
  };
  // the topology of a cpu is read from sysfs once per process (every cycle
  // starts its helper threads here)
  static std::mutex topo_mu;
  static std::unordered_map<int, std::pair<std::vector<int>, std::vector<int>>> topo;
  std::vector<int> llc, smt;
  {
    std::lock_guard<std::mutex> lk(topo_mu);
    auto it = topo.find(cpu);
    if (it == topo.end()) {
      const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(cpu);
      it = topo.emplace(cpu, std::make_pair(read_list(base + "/cache/index3/shared_cpu_list"),
                                            read_list(base + "/topology/thread_siblings_list"))).first;
    }
    llc = it->second.first;
    smt = it->second.second;
  }
  cpu_set_t allowed;
  if (llc.empty() || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  const size_t at = std::find(llc.begin(), llc.end(), cpu) - llc.begin();
  int seen = 0;
  for (size_t k = 1; k <= llc.size(); ++k) {  // the nth usable core after the committer's
    const int c = llc[(at + k) % llc.size()];
    if (std::find(smt.begin(), smt.end(), c) != smt.end() || !CPU_ISSET(c, &allowed)) continue;
    if (++seen < nth) continue;
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(c, &one);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
    return;
  }
}

// Last node-loop run of a job: the task, how many decisions preceded it and
// where it ended (node -1 = fitted nowhere).
struct LastEval {
  int32_t task = -1, before = 0, node = -1, kind = 0;
};

// JobInfo.NodesFitDelta of each not-ready job's last evaluated task
// (allocate.go:116-144; reset per task, so only the last one survives), as
// the counts JobInfo.FitError prints (job_info.go:329-358). The node states
// at each job's evaluation point are rebuilt by undoing the decision log
// backwards from the final mirror (exact: the pre-commit values are logged).
// The same counts on the device (kbg_fitdelta_kernel): one workgroup per job
// over the final node table with each node's decisions after the job's point
// undone, for sessions whose predicate at an evaluation point is the static
// mask plus the pod cap (no host ports, no pod affinity, no nil Node) and
// whose whole node table is local.
kbg_status svc_sum_counts(Session& S, int32_t* counts, size_t n);
kbg_status fit_deltas_device(Session& S, const std::vector<kbg_decision>& dec, const std::vector<Res>& dec_old,
                             const std::vector<LastEval>& last, const std::vector<int32_t>& jobs) {
  std::vector<int32_t> qj;
  int32_t kmin = (int32_t)dec.size();
  for (int32_t j : jobs) {
    Session::FitCounts& fc = S.fit[j];
    fc.valid = 1;
    if (last[j].task < 0) continue;  // never evaluated: empty map, "0 nodes are available"
    qj.push_back(j);
    kmin = std::min(kmin, last[j].before);
  }
  if (qj.empty()) return KBG_OK;
  const int32_t N = S.n_nodes, Q = (int32_t)qj.size();
  std::vector<int32_t> cnt(N + 1, 0);
  for (int32_t k = kmin; k < (int32_t)dec.size(); ++k)
    if (!S.dec_dup[k]) cnt[dec[k].node + 1]++;
  for (int32_t n = 0; n < N; ++n) cnt[n + 1] += cnt[n];
  const int32_t E = cnt[N];
  // one block: hoff[N+1] | hk[E] | na[E] | pad | hold[E][3] | queries[Q]; results [Q][4] mapped
  const size_t o_hk = (size_t)(N + 1) * 4, o_na = o_hk + (size_t)E * 4, o_hold = (o_na + (size_t)E * 4 + 15) / 16 * 16,
               o_q = o_hold + (size_t)E * 24, bytes = o_q + (size_t)Q * sizeof(kbg::FitQuery),
               out_bytes = (size_t)Q * 16;
  if (bytes > S.fit_cap) {
    if (S.fit_h) (void)hipHostFree(S.fit_h);
    if (S.fit_d) (void)hipFree(S.fit_d);
    S.fit_h = nullptr;
    S.fit_d = nullptr;
    S.fit_cap = 0;
    if (host_alloc((void**)&S.fit_h, bytes) != KBG_OK) return fail(KBG_E_HIP, "FitError staging");
    HIP_TRY(hipMalloc((void**)&S.fit_d, bytes));
    S.fit_cap = bytes;
  }
  if (out_bytes > S.fit_out_cap) {
    if (S.fit_out) (void)hipHostFree(S.fit_out);
    S.fit_out = nullptr;
    S.fit_out_cap = 0;
    if (host_alloc((void**)&S.fit_out, out_bytes) != KBG_OK) return fail(KBG_E_HIP, "FitError results");
    S.fit_out_cap = out_bytes;
  }
  int32_t* hoff = (int32_t*)S.fit_h;
  int32_t* hk = (int32_t*)(S.fit_h + o_hk);
  double* hold = (double*)(S.fit_h + o_hold);
  kbg::FitQuery* fq = (kbg::FitQuery*)(S.fit_h + o_q);
  std::copy(cnt.begin(), cnt.end(), hoff);
  for (int32_t k = kmin; k < (int32_t)dec.size(); ++k) {
    if (S.dec_dup[k]) continue;
    const int32_t e = cnt[dec[k].node]++;
    hk[e] = k | (dec[k].kind == KBG_KIND_PIPELINE ? (int32_t)0x80000000 : 0);
    hold[3 * (size_t)e] = dec_old[k].c;
    hold[3 * (size_t)e + 1] = dec_old[k].m;
    hold[3 * (size_t)e + 2] = dec_old[k].g;
  }
  int32_t* na = (int32_t*)(S.fit_h + o_na);  // each decision's first Allocate at or after it on its node
  for (int32_t n = 0; n < N; ++n) {
    int32_t next = -1;
    for (int32_t e = hoff[n + 1] - 1; e >= hoff[n]; --e) {
      if (!(hk[e] & (int32_t)0x80000000)) next = e;
      na[e] = next;
    }
  }
  for (int32_t i = 0; i < Q; ++i) {
    const LastEval& le = last[qj[i]];
    const Res& r = S.treq[le.task];
    fq[i] = kbg::FitQuery{S.task_class[le.task], le.node < 0 ? N : le.node + (le.kind == KBG_KIND_PIPELINE ? 1 : 0),
                          le.before, le.node, {r.c, r.m, r.g}};
  }
  int32_t* fit_out = dev_ptr(S, S.fit_out);
  if (!fit_out) return fail(KBG_E_HIP, "hipHostGetDevicePointer of the FitError buffer failed");
  HIP_TRY(hipMemcpyAsync(S.fit_d, S.fit_h, bytes, hipMemcpyHostToDevice, S.stream));
  kbg::FitArgs a{S.d_nodes.idle_cpu, soa_stride(S), S.W, S.d_class_mask, (const int32_t*)S.fit_d,
                 (const int32_t*)(S.fit_d + o_hk), (const double*)(S.fit_d + o_hold), (const int32_t*)(S.fit_d + o_na),
                 (const kbg::FitQuery*)(S.fit_d + o_q), Q, S.pred_active ? 1 : 0, fit_out, S.tab_lo, S.tab_n};
  HIP_TRY(kbg::launch_fitdelta(a, S.stream));
  HIP_TRY(hipStreamSynchronize(S.stream));
  if (S.svc)  // each rank counted its own nodes
    if (kbg_status st = svc_sum_counts(S, S.fit_out, (size_t)Q * 4); st != KBG_OK) return st;
  for (int32_t i = 0; i < Q; ++i) {
    Session::FitCounts& fc = S.fit[qj[i]];
    fc.nodes = S.fit_out[4 * i];
    fc.cpu = S.fit_out[4 * i + 1];
    fc.mem = S.fit_out[4 * i + 2];
    fc.gpu = S.fit_out[4 * i + 3];
  }
  return KBG_OK;
}

kbg_status compute_fit_deltas(Session& S, const std::vector<kbg_decision>& dec, const std::vector<Res>& dec_old,
                              const std::vector<uint64_t>& dec_oldp, const std::vector<LastEval>& last) {
  S.fit.assign(S.n_jobs, Session::FitCounts{});
  std::vector<int32_t> jobs;
  for (int32_t j = 0; j < S.n_jobs; ++j)
    if (S.committed_ready[j] < S.jobs_in[j].min_available) jobs.push_back(j);
  if (jobs.empty()) return KBG_OK;
  const bool host_only = getenv("KBG_HOST_FITDELTA") != nullptr;  // read per cycle (A/B parity tests)
  if (S.stream && (!S.comm || S.svc) && !S.has_ports && !S.has_aff && !S.any_nil && !host_only)
    return fit_deltas_device(S, dec, dec_old, last, jobs);
  std::sort(jobs.begin(), jobs.end(), [&](int32_t a, int32_t b) { return last[a].before > last[b].before; });
  std::vector<Res> idle = S.idle, rel = S.rel;
  std::vector<int32_t> ntasks = S.ntasks;
  std::vector<uint64_t> ports = S.node_ports;  // host ports: [N][PW]
  const int32_t PW = S.PW;
  kbg::AffState aff;  // pod affinity counts, rewound with the decisions
  if (S.has_aff) aff = S.affm->st;
  int32_t k = (int32_t)dec.size();
  for (int32_t j : jobs) {
    Session::FitCounts& fc = S.fit[j];
    fc.valid = 1;
    const LastEval& le = last[j];
    if (le.task < 0) continue;  // never evaluated: empty map, "0 nodes are available"
    while (k > le.before) {
      --k;
      const int32_t n = dec[k].node;
      if (!S.dec_dup[k]) {  // a decision whose pod key the node held left the node unchanged
        if (!S.nil_node[n]) (dec[k].kind == KBG_KIND_ALLOCATE ? idle[n] : rel[n]) = dec_old[k];
        ntasks[n]--;
        if (S.has_ports)
          std::copy(dec_oldp.begin() + (size_t)k * PW, dec_oldp.begin() + (size_t)(k + 1) * PW,
                    ports.begin() + (size_t)n * PW);
      }
      if (S.has_aff && dec[k].kind == KBG_KIND_ALLOCATE) kbg::aff_place(S, dec[k].task, n, -1, aff, false);
    }
    const int32_t t = le.task;
    const Res& r = S.treq[t];
    const uint64_t* cm = S.h_class_mask_static.data() + (size_t)S.task_class[t] * S.W;
    const uint64_t* conf = S.has_ports ? S.cls_conf.data() + (size_t)S.task_class[t] * PW : nullptr;
    const int32_t end = le.node < 0 ? S.n_nodes : le.node + (le.kind == KBG_KIND_PIPELINE ? 1 : 0);
    bool nil_seen = false;
    Res nil_delta{};
    for (int32_t n = 0; n < end; ++n) {
      if (!((cm[n >> 6] >> (n & 63)) & 1ull)) continue;                 // static predicate
      if (S.pred_active && ntasks[n] >= S.maxtasks[n]) continue;       // pod cap
      if (conf && !S.panic_node[n]) {                                  // host ports
        bool clash = false;
        for (int32_t w = 0; w < PW && !clash; ++w) clash = (ports[(size_t)n * PW + w] & conf[w]) != 0;
        if (clash) continue;
      }
      if (S.has_aff && !S.panic_node[n] && !kbg::aff_ok(S, aff, S.task_class[t], n)) continue;  // pod affinity
      if (n != le.node && kbg::res_le(r, idle[n])) continue;           // would have been chosen
      Res d = idle[n];                                                 // Resource.FitDelta
      if (r.c > 0) d.c -= r.c + kbg::kMinMilliCPU;
      if (r.m > 0) d.m -= r.m + kbg::kMinMemory;
      if (r.g > 0) d.g -= r.g + kbg::kMinMilliGPU;
      if (S.nil_node[n]) {  // every nil Node is named "": one map entry, the last one wins
        nil_seen = true;
        nil_delta = d;
        continue;
      }
      fc.nodes++;
      fc.cpu += d.c < 0;
      fc.mem += d.m < 0;
      fc.gpu += d.g < 0;
    }
    if (nil_seen) {
      fc.nodes++;
      fc.cpu += nil_delta.c < 0;
      fc.mem += nil_delta.m < 0;
      fc.gpu += nil_delta.g < 0;
    }
  }
  return KBG_OK;
}

// State of a cycle's first action: the decision log, gang dispatch lists,
// committed readiness and the plugin state start from the session snapshot.
void begin_cycle(Session& S) {
  S.dec.clear();
  S.dec.reserve(S.pend.size());
  S.undisp_head.assign(S.n_jobs, -1);
  S.undisp_next.clear();
  S.undisp_next.reserve(S.pend.size());
  S.committed_ready = S.job_ready0;
  S.fin = S.init;
  S.fit.assign(S.n_jobs, Session::FitCounts{});
  const kbg_stats prev = S.stats;
  S.stats = kbg_stats{};
  S.vk_timed_ms = 0;
  S.vk_timed = 0;
  S.ff_timed_ms = 0;
  S.ff_timed = 0;
  S.stats.n_classes = prev.n_classes;
  S.stats.shards = prev.shards;
  S.stats.shard_index = prev.shard_index;
  S.stats.int_scan = prev.int_scan;
  S.stats.open_ms = prev.open_ms;
  S.dec_action.clear();
  S.dec_dup.clear();
  S.node_keys = S.node_keys0;
  S.port_hold.clear();
  S.port_gone.clear();
  S.outsider_gone.clear();
  S.key_holder.clear();
  S.evictions.clear();
  if ((int32_t)S.tstat_in.size() == S.n_tasks) {
    S.tstat.assign(S.tstat_in.begin(), S.tstat_in.end());  // tasks_in[t].status, packed by derive_host
  } else {  // an update that failed part-way
    S.tstat.resize(S.n_tasks);
    for (int32_t t = 0; t < S.n_tasks; ++t) S.tstat[t] = S.tasks_in[t].status;
  }
  S.trun.assign(S.n_tasks, 0);
  for (int32_t t : S.nt_task) S.trun[t] = 1;
  if (S.has_dupkeys) S.t_detached.assign(S.n_tasks, 0);
  else S.t_detached.clear();
  S.aff_filtered.clear();
  S.pend = S.pend_all;
  S.pend_off = S.pend_off_all;
  S.pend_len = S.pend_len_all;
  if (S.has_aff) {
    S.affm->st = S.affm->st0;
    std::fill(S.aff_gain_flag.begin(), S.aff_gain_flag.end(), 0);
    S.aff_gain_classes.clear();
  }
  S.cycle_started = true;
}

// The allocate engine's starting state when an earlier action of the cycle
// (reclaim) changed the session: plugin state and readiness as they are now,
// the pending lists without the tasks that left Pending, fresh heaps.
Engine live_engine(Session& S) {
  Engine E;
  E.jalloc = S.fin.jalloc;
  E.jshare = S.fin.jshare;
  E.jready = S.committed_ready;
  E.qalloc = S.fin.qalloc;
  E.qshare = S.fin.qshare;
  E.cursor.assign(S.n_jobs, 0);
  S.pend.clear();
  for (int32_t j = 0; j < S.n_jobs; ++j) {
    S.pend_off[j] = (int32_t)S.pend.size();
    for (int32_t k = 0; k < S.pend_len_all[j]; ++k) {
      const int32_t t = S.pend_all[S.pend_off_all[j] + k];
      if (S.tstat[t] == KBG_PENDING) S.pend.push_back(t);
    }
    S.pend_len[j] = (int32_t)S.pend.size() - S.pend_off[j];
  }
  build_heaps(S, E);
  return E;
}

// Appends a decision to the cycle's log (no gang bookkeeping). `dup`: the
// node already held the pod key and was left unchanged.
void append_log(Session& S, int32_t t, int32_t node, int32_t kind, bool dup = false) {
  S.dec.push_back(kbg_decision{t, node, kind, -1});
  S.undisp_next.push_back(-1);
  S.dec_action.push_back(S.action);
  S.dec_dup.push_back(dup ? 1 : 0);
}

// Appends one committed decision to the log and runs the gang part of
// ssn.Allocate (session.go:283-290): every Allocated task of the job is
// dispatched when this decision makes the job ready. Pipelined tasks count
// toward readiness (gang.go:44-55) but never dispatch.
void record_decision(Session& S, int32_t t, int32_t node, int32_t kind, bool dup) {
  const int32_t j = S.task_job[t];
  const int32_t di = (int32_t)S.dec.size();
  append_log(S, t, node, kind, dup);
  S.committed_ready[j]++;
  S.tstat[t] = kind == KBG_KIND_ALLOCATE ? KBG_ALLOCATED : KBG_PIPELINED;
  if (kind == KBG_KIND_ALLOCATE) {
    S.undisp_next[di] = S.undisp_head[j];
    S.undisp_head[j] = di;
    if (!S.ready_gang || S.committed_ready[j] >= S.jobs_in[j].min_available) {
      for (int32_t d = S.undisp_head[j]; d >= 0; d = S.undisp_next[d]) {
        S.dec[d].dispatched_at = di;
        S.tstat[S.dec[d].task] = KBG_BINDING;  // dispatch (session.go:295-316)
      }
      S.undisp_head[j] = -1;
    }
  }
}

kbg_status copy_log(Session& S, kbg_decision* out, int32_t cap, int32_t* n_out, kbg_status result) {
  if (n_out) *n_out = (int32_t)S.dec.size();
  if ((int32_t)S.dec.size() > cap || (!out && !S.dec.empty())) {
    if (result == KBG_OK) result = fail(KBG_E_CAPACITY, "decision buffer too small: need " + std::to_string(S.dec.size()));
    return result;
  }
  if (!S.dec.empty()) std::memcpy(out, S.dec.data(), S.dec.size() * sizeof(kbg_decision));
  return result;
}

// The committed outcomes replayed into an engine copy on a thread of its own.
// Ranks other than 0 of a sharded allocate do not predict: this is their
// engine (the plugin state later actions and the state queries read). In the
// single-rank allocate it is the engine's "truth" a few tasks behind the
// committer: at a cut the predictor takes its state instead of restoring a
// checkpoint and replaying the batch's prefix.
// One committed outcome for an engine replay: task, placed or not, and the
// failed tasks of its job consumed with it (Batch::brun).
struct Outcome {
  int32_t t, run;
  char ok;
};
struct Replayer {
  Session& S;
  Engine& E;
  std::thread th;
  std::mutex mu;
  SpinCV cv;
  std::deque<std::vector<Outcome>> q;
  bool done = false, busy = false;
  std::string error;
  // committer_cpu >= 0: on its own core of the committer's last-level cache
  // (after the predictor, logger and builder), never time-sharing the predictor's
  Replayer(Session& s, Engine& e, int committer_cpu = -1) : S(s), E(e) {
    th = std::thread([this, committer_cpu]() {
      pin_near(committer_cpu, 4);
      run();
    });
  }
  ~Replayer() { join(); }
  void push(std::vector<Outcome>&& v) {
    std::lock_guard<std::mutex> lk(mu);
    q.push_back(std::move(v));
    cv.notify_all();
  }
  void push(const std::vector<std::pair<int32_t, char>>& v) {
    std::vector<Outcome> o(v.size());
    for (size_t k = 0; k < v.size(); ++k) o[k] = Outcome{v[k].first, 0, v[k].second};
    push(std::move(o));
  }
  void join() {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
      cv.notify_all();
    }
    if (th.joinable()) th.join();
  }
  // the outcomes not applied yet are dropped (the caller has the same state
  // elsewhere) and the thread ends after its current chunk
  void abandon() {
    {
      std::lock_guard<std::mutex> lk(mu);
      q.clear();
      done = true;
      cv.notify_all();
    }
    if (th.joinable()) th.join();
  }
  // blocks until every pushed outcome is applied: E is then the engine state
  // after the last of them
  void wait_idle() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return q.empty() && !busy; });
  }
  void run() {
    Ops ops{S, E, nullptr};
    for (;;) {
      std::vector<Outcome> v;
      {
        std::unique_lock<std::mutex> lk(mu);
        busy = false;
        cv.notify_all();
        cv.wait(lk, [&] { return done || !q.empty(); });
        if (q.empty()) return;
        v = std::move(q.front());
        q.pop_front();
        busy = true;
      }
      for (const Outcome& o : v) {
        if (!error.empty()) break;
        if (ops.next_task() != o.t) {
          error = "internal: engine replay diverged from the committed outcomes";
          break;
        }
        ops.apply(o.t, o.ok);
        if (o.run) ops.skip(o.run);
      }
    }
  }
};

// The predictor thread of an allocate cycle (the ordering engine) and its
// hand-off with the committer: predicted batches, recycled buffers, rollbacks.
struct Predictor {
  using clk = std::chrono::steady_clock;
  Session& S;
  Engine& E;                      // the engine state the predictor advances
  std::atomic<uint8_t>* failed;   // shapes known to fit nowhere (monotone), set by the committer
  Pipe P;
  double engine_ms = 0;
  int64_t replayed = 0;
  std::string error;
  EngineProfile prof;
  Trace tr;
  std::thread th, bth;
  bool builder = false;       // a builder thread turns predicted batches into device rows (allocate_cycle)
  bool truth_mode = false;    // rollbacks copy a truth engine (rollback_truth): no batch checkpoints
  bool runs = false;          // consume a job's tasks of shapes known to fit nowhere as one entry (Batch::brun)
  std::vector<Batch*> all;    // every batch of this predictor (freed by finish)
  Predictor(Session& s, Engine& e, std::atomic<uint8_t>* f) : S(s), E(e), failed(f) {
    prof.on = getenv("KBG_PROFILE_ENGINE") != nullptr;
  }
  void start(int committer_cpu, bool with_builder = false) {
    builder = with_builder;
    th = std::thread([this, committer_cpu]() { run(committer_cpu); });
    if (builder) bth = std::thread([this, committer_cpu]() { build_run(committer_cpu); });
  }
  // Builder: Grouper::build of each predicted batch into the batch's own
  // pinned row buffer, so the committer only swaps buffers at launch.
  void build_run(int committer_cpu) {
    pin_near(committer_cpu, 3);
    Grouper g(S);
    for (;;) {
      Batch* b;
      {
        std::unique_lock<std::mutex> lk(P.mu);
        P.cv.wait(lk, [&] { return P.stop || !P.raw.empty(); });
        if (P.stop) return;
        b = P.raw.front();
        P.raw.pop_front();
        P.building = true;
      }
      b->G = 0;
      if (!b->bt.empty()) {
        if (!b->st.h_up) {
          if (!S.up_pool.empty()) {  // only this thread takes from the pool during a cycle
            b->st.h_up = S.up_pool.back();
            S.up_pool.pop_back();
          } else if (host_alloc((void**)&b->st.h_up, S.up_cap) != KBG_OK) {
            b->st.h_up = nullptr;
            std::lock_guard<std::mutex> lk(P.mu);
            error = "hipHostMalloc of a batch row buffer failed";
            P.stop = true;
            P.building = false;
            P.ready.push_back(nullptr);
            P.cv.notify_all();
            return;
          }
        }
        b->G = g.build(b->st, b->bt.data(), (int32_t)b->bt.size());
      }
      std::lock_guard<std::mutex> lk(P.mu);
      P.building = false;
      P.ready.push_back(b);
      P.cv.notify_all();
    }
  }
  void run(int committer_cpu) {
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    pin_near(committer_cpu);
    Ops ops{S, E, prof.on ? &prof : nullptr};
    const int32_t* const tshape = S.task_shape.data();  // (not through the Session's lines, EngineView)
    bool exhausted = false, restarted = false;
    for (;;) {
      Batch* b = nullptr;
      int64_t my_epoch;
      {
        std::unique_lock<std::mutex> lk(P.mu);
        P.cv.wait(lk, [&] {
          return P.stop || P.rollback ||
                 (!exhausted && P.ready.size() + P.raw.size() < (size_t)P.depth.load(std::memory_order_relaxed));
        });
        if (P.stop) return;
        if (P.rollback && P.rb_truth) {  // the engine state at the cut, kept by the truth replayer
          const auto tp = clk::now();
          E = *P.rb_truth;
          P.rb_truth = nullptr;
          engine_ms += ms_since(tp);
          P.rollback = false;
          exhausted = false;
          restarted = true;
        } else if (P.rollback) {
          const auto tp = clk::now();
          E = P.rb_ckpt;
          for (size_t k = 0; k < P.rb_tasks.size(); ++k) {
            const int32_t t = ops.next_task();
            if (t != P.rb_tasks[k]) {
              error = "internal: replay diverged";
              P.stop = true;
              P.ready.push_back(nullptr);
              P.cv.notify_all();
              return;
            }
            ops.apply(t, P.rb_actual[k]);
            if (k < P.rb_runs.size() && P.rb_runs[k]) ops.skip(P.rb_runs[k]);
          }
          replayed += (int64_t)P.rb_tasks.size();
          engine_ms += ms_since(tp);
          P.rollback = false;
          exhausted = false;
        }
        my_epoch = P.epoch;
        if (!P.free.empty()) {
          b = P.free.back();
          P.free.pop_back();
        }
      }
      if (!b) {
        std::lock_guard<std::mutex> lk(P.mu);
        if (!S.batch_pool.empty()) {  // an earlier cycle's batch: its vectors keep their capacity
          b = static_cast<Batch*>(S.batch_pool.back().release());
          S.batch_pool.pop_back();
        } else {
          b = new Batch();
        }
        all.push_back(b);
      }
      const auto tp = clk::now();
      if (!truth_mode) {
        tr.add("ckpt.begin");
        b->ckpt = E;
        tr.add("ckpt");
      }
      b->epoch = my_epoch;
      b->bt.clear();
      b->bpred.clear();
      b->brun.clear();
      // right after a cut the committer waits with nothing to scan: hand it
      // the first 64 tasks (the next cut is often a few tasks away)
      const size_t emit_at = restarted ? 64 : (size_t)min_emit();
      restarted = false;
      bool abandoned = false;
      const int32_t kcap = std::min(S.K, P.kmax.load(std::memory_order_relaxed));
      while ((int32_t)b->bt.size() < kcap) {
        const int32_t t = ops.next_task();
        if (t < 0) break;
        const bool p = !failed[tshape[t]].load(std::memory_order_relaxed);
        b->bt.push_back(t);
        b->bpred.push_back(p);
        ops.apply(t, p);
        b->brun.push_back(!p && runs ? ops.skip_dead(failed, tshape) : 0);
        if ((b->bt.size() & 63) == 0) {
          // the committer cut an earlier batch: this one follows a wrong
          // prediction, stop here and roll back
          if (P.epoch_now.load(std::memory_order_relaxed) != my_epoch) {
            abandoned = true;
            break;
          }
          // a committer with nothing to do takes a short batch now
          if (b->bt.size() >= emit_at && P.hungry.load(std::memory_order_relaxed)) {
            P.hungry.store(false, std::memory_order_relaxed);  // one early batch per wait
            break;
          }
        }
      }
      engine_ms += ms_since(tp);
      if (abandoned) {
        std::lock_guard<std::mutex> lk(P.mu);
        P.free.push_back(b);
        continue;
      }
      tr.add("emit", (int64_t)b->bt.size());
      if (b->bt.empty()) exhausted = true;  // the empty batch marks the end of this epoch
      std::lock_guard<std::mutex> lk(P.mu);
      (builder ? P.raw : P.ready).push_back(b);
      P.cv.notify_all();
    }
  }
  // a predicted batch; nullptr when the predictor failed. Non-blocking: also
  // nullptr (with *none = true) when no batch is ready yet.
  Batch* take(bool block, bool* none) {
    std::unique_lock<std::mutex> lk(P.mu);
    if (!block && P.ready.empty()) {
      *none = true;
      return nullptr;
    }
    *none = false;
    if (P.ready.empty()) {
      // nothing predicted on its way: the predictor hands over what it has
      if (P.raw.empty() && !P.building) P.hungry.store(true, std::memory_order_relaxed);
      P.cv.wait(lk, [&] { return !P.ready.empty(); });
      P.hungry.store(false, std::memory_order_relaxed);
    }
    Batch* b = P.ready.front();
    P.ready.pop_front();
    P.cv.notify_all();
    return b;
  }
  void recycle(Batch* b) {
    if (!b) return;
    std::lock_guard<std::mutex> lk(P.mu);
    P.free.push_back(b);
  }
  // a new epoch: the predictor restores `cur`'s checkpoint and replays the
  // actual outcomes of its first `cut` tasks; `cur` and `nxt` are recycled
  void rollback(int64_t epoch, Batch* cur, int32_t cut, const std::vector<char>& actual, Batch* nxt) {
    P.epoch_now.store(epoch, std::memory_order_relaxed);
    std::lock_guard<std::mutex> lk(P.mu);
    P.epoch = epoch;
    P.rollback = true;
    P.rb_ckpt = cur->ckpt;
    P.rb_tasks.assign(cur->bt.begin(), cur->bt.begin() + cut);
    P.rb_actual.assign(actual.begin(), actual.begin() + cut);
    P.rb_runs.assign(cur->brun.begin(), cur->brun.begin() + std::min<size_t>(cut, cur->brun.size()));
    P.free.push_back(cur);
    if (nxt) P.free.push_back(nxt);
    P.cv.notify_all();
  }
  // a new epoch from the engine state `truth` holds (the committed outcomes
  // up to and including the cut, applied); `cur` and `nxt` are recycled
  void rollback_truth(int64_t epoch, const Engine* truth, Batch* cur, Batch* nxt) {
    P.epoch_now.store(epoch, std::memory_order_relaxed);
    std::lock_guard<std::mutex> lk(P.mu);
    P.epoch = epoch;
    P.rollback = true;
    P.rb_truth = truth;
    P.free.push_back(cur);
    if (nxt) P.free.push_back(nxt);
    P.cv.notify_all();
  }
  ~Predictor() { finish(); }
  void finish() {
    {
      std::lock_guard<std::mutex> lk(P.mu);
      P.stop = true;
      P.cv.notify_all();
    }
    if (th.joinable()) th.join();
    if (bth.joinable()) bth.join();
    std::lock_guard<std::mutex> lk(P.mu);
    for (Batch* b : all) {  // row buffers go back to the session's pool, the batch to its batch pool
      if (b->st.h_up) S.up_pool.push_back(b->st.h_up);
      b->st.h_up = nullptr;
      b->G = -1;
      S.batch_pool.emplace_back(b, [](void* q) { delete static_cast<Batch*>(q); });
    }
    all.clear();
    P.ready.clear();
    P.raw.clear();
    P.free.clear();
  }
};

// One committed outcome of a resolve walk (single-rank or owner-resolve), for the log side.
struct LogItem {
  int32_t t, node, kind;
  bool ok, own, dup;
  Res old;  // own commit: the Idle / Releasing row before it
};

// The log side of a resolve walk on a thread of its own: batches of committed
// outcomes in commit order.
struct Logger {
  std::function<void(const LogItem&)> fn;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::vector<LogItem>> q;
  bool done = false;
  explicit Logger(std::function<void(const LogItem&)> f, int committer_cpu) : fn(std::move(f)) {
    th = std::thread([this, committer_cpu]() {
      pin_near(committer_cpu, 2);  // not the predictor's core (the builder takes the third)
      run();
    });
  }
  ~Logger() { join(); }
  void push(std::vector<LogItem>&& v) {
    std::lock_guard<std::mutex> lk(mu);
    q.push_back(std::move(v));
    cv.notify_all();
  }
  void join() {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
      cv.notify_all();
    }
    if (th.joinable()) th.join();
  }
  void run() {
    for (;;) {
      std::vector<LogItem> v;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done || !q.empty(); });
        if (q.empty()) return;
        v = std::move(q.front());
        q.pop_front();
      }
      for (const LogItem& it : v) fn(it);
    }
  }
};

// Two engine states hold the same plugin state (KBG_CHECK_TRUTH): what a
// cycle's final engine hands on (S.fin: drf / proportion allocations and
// shares, gang readiness; live_engine rebuilds the heaps and cursors, which
// differ — the predictor ran its queues dry past the last outcome).
bool engines_equal(const Engine& a, const Engine& b) {
  auto res_eq = [](const std::vector<Res>& x, const std::vector<Res>& y) {
    return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), x.size() * sizeof(Res)) == 0);
  };
  auto dbl_eq = [](const std::vector<double>& x, const std::vector<double>& y) {
    return x.size() == y.size() && (x.empty() || std::memcmp(x.data(), y.data(), x.size() * sizeof(double)) == 0);
  };
  return res_eq(a.jalloc, b.jalloc) && dbl_eq(a.jshare, b.jshare) && a.jready == b.jready &&
         res_eq(a.qalloc, b.qalloc) && dbl_eq(a.qshare, b.qshare);
}

// allocate_cycle under the scan service: the FitError inputs it leaves for
// allocate_svc_root (same thread), which counts after the end message
struct SvcFit {
  std::vector<uint64_t> dec_oldp;
  std::vector<LastEval> last;
};
thread_local SvcFit g_svc_fit;

kbg_status allocate_cycle(Session& S, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.allocated || S.backfilled || S.preempted)
    return fail(KBG_E_INVALID, "allocate runs once per cycle, before backfill and preempt; call kbg_session_reset");
  const bool first = !S.cycle_started;  // else reclaim ran first: start from the live state
  if (first) begin_cycle(S);
  S.action = KBG_ACTION_ALLOCATE;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  const auto t0 = clk::now();

  std::vector<kbg_decision>& dec = S.dec;
  // the Idle (Allocate) or Releasing (Pipeline) row before each decision
  // (indexed by decision; earlier actions' decisions are never undone)
  std::vector<Res>& dec_old = S.dec_old_buf;  // a session buffer: its pages stay mapped across cycles
  dec_old.assign(dec.size(), Res{});
  dec_old.reserve(dec.size() + S.pend.size());
  std::vector<uint64_t> dec_oldp(dec.size() * (size_t)S.PW);  // host ports: used-port atoms before each decision
  std::vector<LastEval> last(S.n_jobs);
  // shapes known to fit nowhere (monotone): written by the committer, read by the predictor
  std::unique_ptr<std::atomic<uint8_t>[]> failed(new std::atomic<uint8_t>[std::max(1, S.n_shapes)]);
  for (int32_t i = 0; i < S.n_shapes; ++i) failed[i].store(0, std::memory_order_relaxed);
  std::vector<int32_t> mark(S.n_nodes, -1), touched;
  std::vector<char> bactual;
  kbg_status result = KBG_OK;
  Grouper grouper(S);
  Resolver rs{S, mark};
  static const bool use_floor = [] {
    const char* e = getenv("KBG_SHAPE_FLOOR");
    return !e || std::atoi(e) != 0;
  }();
  std::vector<int32_t> shape_floor;
  if (use_floor) {
    shape_floor.assign(std::max(1, S.n_shapes), 0);
    rs.floor = shape_floor.data();
  }
  constexpr bool packed = true;
  std::vector<MirrorRow> mrow;
  if (packed) {
    mrow.resize(S.n_nodes);
    for (int32_t n = 0; n < S.n_nodes; ++n) {
      mirror_row(S, mrow[n], n);
      mrow[n].mt = S.maxtasks[n];
      mrow[n].mark = -1;
      mrow[n].panic = S.panic_node[n];
    }
    rs.rows = mrow.data();
  }
  // The log side of the walk (decision log, gang dispatch, FitError
  // bookkeeping) on a thread of its own, unless host ports or colliding pod
  // keys need the pre-commit port rows (then inline, below).
  auto log_one = [&](const LogItem& it) {
    last[S.task_job[it.t]] = LastEval{it.t, (int32_t)dec.size(), it.node, it.kind};
    if (!it.ok) return;
    dec_old.push_back(it.old);
    record_decision(S, it.t, it.node, it.kind, it.dup);
  };
  static const bool no_logger = getenv("KBG_NO_LOGGER") != nullptr;
  std::unique_ptr<Logger> lg;
  if (!S.has_ports && !S.has_dupkeys && !no_logger) lg.reset(new Logger(log_one, sched_getcpu()));
  std::vector<LogItem> items;

  // ------------------------------------------------------------ predictor
  Engine E = first ? S.init : live_engine(S);
  Engine E_truth = E;  // the committed outcomes only (Replayer), the state a cut restarts from
  Replayer truth(S, E_truth, sched_getcpu());
  Predictor pr(S, E, failed.get());
  pr.truth_mode = true;
  // a job's run of tasks of shapes known to fit nowhere is one batch entry
  // (Batch::brun); not in full-scan mode, where every task evaluation scans
  // the table. KBG_NO_RUNS=1 (A/B) turns it off.
  static const bool no_runs = getenv("KBG_NO_RUNS") != nullptr;
  pr.runs = !S.opts.full_scan && !no_runs;
  EngineProfile& eprof = pr.prof;
  Trace ctr;
  ctr.start(t0);
  pr.tr.start(t0);
  struct TraceHook {  // cleared on every return path
    explicit TraceHook(Trace* t) { t_trace = t; }
    ~TraceHook() { t_trace = nullptr; }
  } trace_hook(ctr.on ? &ctr : nullptr);
  static const bool no_builder = getenv("KBG_NO_BUILDER") != nullptr;
  ctr.add("setup");
  pr.start(sched_getcpu(), !no_builder);
  ctr.add("started");
  auto take = [&](bool block, bool* none) { return pr.take(block, none); };
  auto recycle = [&](Batch* b) { pr.recycle(b); };
  auto finish = [&]() {
    pr.finish();
    truth.join();
  };
  // committed outcomes of the current batch not yet handed to the truth engine
  int32_t truth_from = 0;
  // KBG_NO_TRUTH=1 (experiment, cut-free cycles only): no truth engine; the
  // predictor's own engine is the cycle's final state
  static const bool no_truth = getenv("KBG_NO_TRUTH") != nullptr;
  auto to_truth = [&](const Batch* b, int32_t end) {
    if (no_truth) {
      truth_from = end;
      return;
    }
    if (end <= truth_from) return;
    std::vector<Outcome> v(end - truth_from);
    for (int32_t k = truth_from; k < end; ++k) v[k - truth_from] = Outcome{b->bt[k], b->brun[k], bactual[k]};
    truth.push(std::move(v));
    truth_from = end;
  };

  // ------------------------------------------------------------ committer
  // Two stages in flight: while the host resolves batch b (stage `si`), the
  // device scans batch b+1 (stage si^1) against the table without b's commits;
  // b+1's resolve re-checks every node b touched (mark > that scan's base).
  int64_t cur_epoch = 0;
  int32_t pushed = S.res_stamp;  // newest resolution whose node deltas are enqueued
  int32_t rstamp = S.res_stamp;  // the stamp of the commits being made (mark[] of their nodes)
  // The rows the commits since the last write-back touched reach HBM right
  // before a scan is launched (or the cycle ends), not after every batch: a
  // batch resolved against earlier lists (contended cycles) needs no
  // write-back, and a scan launched mid-batch sees the batch's commits so
  // far. Commits after the write-back take a new stamp, above the scan's base.
  auto flush = [&]() -> kbg_status {
    if (touched.empty() && S.mask_dirty.empty()) return KBG_OK;
    const auto t0 = clk::now();
    const kbg_status st = push_deltas(S, touched);
    touched.clear();
    pushed = rstamp;
    rstamp = ++S.res_stamp;
    S.mstamp = rstamp;
    S.stats.delta_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    return st;
  };
  bool pred_failed = false;
  // the next batch of the current epoch (stale ones are recycled); nullptr:
  // none ready (non-blocking) or the predictor failed (pred_failed)
  auto next_batch = [&](bool block) -> Batch* {
    for (;;) {
      bool none = false;
      Batch* b = take(block, &none);
      if (none) return nullptr;
      if (!b) {
        pred_failed = true;
        return nullptr;
      }
      if (b->epoch != cur_epoch) {
        recycle(b);
        continue;
      }
      return b;
    }
  };
  auto launch = [&](kbg::Stage& sg, Batch* b) -> kbg_status {
    if (kbg_status fs = flush(); fs != KBG_OK) return fs;
    int32_t G;
    if (b->G >= 0) {  // built by the builder thread: take its row buffer and row maps
      std::swap(sg.h_up, b->st.h_up);
      sg.h_tasks = (kbg::TaskRec*)sg.h_up;
      sg.h_capoff = b->st.h_capoff;  // inside the buffer sg now holds
      sg.h_rowshape = b->st.h_rowshape;
      sg.h_shapes = b->st.h_shapes;
      sg.n_slots = b->st.n_slots;
      sg.row_of.swap(b->st.row_of);
      sg.row_shape.swap(b->st.row_shape);
      sg.row_ext.swap(b->st.row_ext);
      sg.row_slot.swap(b->st.row_slot);
      sg.slot_rows.swap(b->st.slot_rows);
      G = b->G;
      b->G = -1;
    } else {
      G = grouper.build(sg, b->bt.data(), (int32_t)b->bt.size());
    }
    const kbg_status st = device_launch(S, sg, G, pushed);
    ctr.add("launch", G);
    return st;
  };
  auto abort = [&](kbg_status st) {
    for (kbg::Stage& g : S.stages) (void)device_drop(S, g);
    finish();
    return st;
  };
  // A row whose scan found no node at all: its (class, request) shape fits
  // nowhere in that table, so (monotone) nowhere for the rest of the cycle.
  // The predictor predicts its later tasks as failures from now on instead of
  // each first failure cutting a batch (predictions only: the committer still
  // decides every task).
  auto learn_failed = [&](const kbg::Stage& g) {
    for (int32_t r = 0; r < g.G; ++r)
      if (row_fits_nowhere(g, r)) mark_failed(failed.get(), g.row_shape[r]);
  };
  // opt-in cycle counters of the in-order commit (KBG_PROFILE_RESOLVE=1):
  // candidate walk, host mirror, decision log, whole loop
  const bool rprof = getenv("KBG_PROFILE_RESOLVE") != nullptr;
  uint64_t rcyc[4] = {0, 0, 0, 0};
  int64_t rk_phase[3] = {0, 0, 0};  // re-checks before the first cut, after it on fresh scans, on reused lists
  // Grouped mode, after a cut: the stage's candidate lists still hold for the
  // committed table (a list is every fitting node in order at scan time, up
  // to its length; feasibility only shrinks during allocate, and a node
  // touched since the scan is re-checked on the host mirror), so the
  // re-predicted tasks resolve against them with no device round trip — by
  // shape, the same (class, request) row any task of the shape used. A task
  // whose shape has no row there, or a list that runs out before the table
  // did, rescans the rest of its batch. Full-scan mode rescans (every task
  // evaluation scans the table); pod affinity (gains cut) and
  // sharded sessions too.
  const bool no_reuse = getenv("KBG_NO_CUT_REUSE") != nullptr;  // read per cycle (A/B parity tests)
  const bool rescan_all = [] {  // KBG_RESCAN_ALL=0: a contended rescan lists the shapes seen so far only
    const char* e = getenv("KBG_RESCAN_ALL");
    return !(e && e[0] == '0');
  }();
  const bool reuse_ok = !S.opts.full_scan && (!S.comm || S.svc) && !S.has_aff && !no_reuse;
  // the predictor's run-ahead past the first cut (Pipe::depth / kmax; 0 = unchanged)
  static const int32_t cont_depth = [] {
    const char* e = getenv("KBG_CONT_DEPTH");
    return e ? atoi(e) : 0;
  }();
  static const int32_t cont_batch = [] {
    const char* e = getenv("KBG_CONT_BATCH");
    return e ? atoi(e) : 0;
  }();
  bool reuse = false;
  // From the first cut on (the contended part of the cycle) every batch
  // resolves against the latest stage, and a rescan covers the rest of the
  // batch plus one row for every shape seen this cycle that is not known to
  // fit nowhere, so a later batch's shapes mostly have rows already.
  bool contended = false;
  std::vector<int32_t> shape_rep(reuse_ok ? std::max(1, S.n_shapes) : 0, -1), seen_shapes, scan_list, shape_in;
  int32_t shape_in_stamp = 0;
  if (reuse_ok) shape_in.assign(std::max(1, S.n_shapes), 0);
  std::vector<int32_t> shape_row_of(reuse_ok ? std::max(1, S.n_shapes) : 0, -1), shapes_set, row_rep;
  // the stage's row of each shape, and a task of each row (the batch entries
  // [seg0, ...) of `b` built the stage's rows)
  auto map_shapes = [&](const kbg::Stage& g, const std::vector<int32_t>& b, int32_t seg0) {
    for (int32_t sh : shapes_set) shape_row_of[sh] = -1;
    shapes_set.clear();
    row_rep.assign(g.G, -1);
    for (size_t i = seg0; i < b.size(); ++i) {
      const int32_t r = g.row_of[i - seg0];
      if (row_rep[r] < 0) row_rep[r] = b[i];
    }
    for (int32_t r = 0; r < g.G; ++r) {
      const int32_t sh = g.row_shape[r];
      if (shape_row_of[sh] < 0) {
        shape_row_of[sh] = r;
        shapes_set.push_back(sh);
      }
    }
  };
  // A shape whose list holds no fitting node any more (complete, and every
  // entry from its cursor infeasible on the host mirror) fits nowhere for the
  // rest of the cycle: the predictor learns it before it predicts again, so
  // the shape's next task does not cut a batch. The walk only moves cursors
  // past infeasible entries, as a resolve of a task of the shape would.
  auto probe_failed = [&](const kbg::Stage& g) {
    for (int32_t r = 0; r < g.G; ++r) {
      const int32_t sh = g.row_shape[r];
      if (row_rep[r] < 0 || failed[sh].load(std::memory_order_relaxed)) continue;
      int32_t node = -1, kind = 0;
      if (rs.resolve(r, row_rep[r], &node, &kind) == RES_OK && node < 0)
        mark_failed(failed.get(), sh);
    }
  };
  // Refresh scans (the contended part, batches resolving against an earlier
  // stage's lists): every node a commit touched since that scan is
  // re-checked on the host mirror by every shape whose list holds it, so the
  // re-checks grow with (live shapes) x (nodes filled since the scan). Once
  // the commit has re-checked KBG_REFRESH_RECHECKS nodes against the current
  // lists, the touched rows are written back and a scan of every live shape
  // is launched into the other stage beside the resolve; when it has landed
  // (polled, never waited for) the commit switches to its lists, whose base
  // is the write-back: the filled nodes are no longer in them, and only nodes
  // touched after the write-back are re-checked. Lists stay exact under the
  // switch for the reason any stage's do (feasibility only shrinks during
  // allocate; a node touched after the scan is re-checked).
  static const int64_t refresh_rechecks = [] {
    const char* e = getenv("KBG_REFRESH_RECHECKS");
    return e ? atoll(e) : (int64_t)16384;
  }();
  bool refresh_inflight = false;
  std::vector<int32_t> refresh_list;
  int64_t rechecks_at_scan = 0;
  int si = 0;
  kbg::Stage* sg = &S.stages[0];
  kbg::Stage* oth = &S.stages[1];
  // one task of every shape seen this cycle or kept by derive_host that is
  // not known to fit nowhere (at most K)
  auto live_list = [&](std::vector<int32_t>& out) {
    out.clear();
    ++shape_in_stamp;
    for (int32_t sh : seen_shapes) {
      if ((int32_t)out.size() >= S.K) break;
      if (shape_in[sh] == shape_in_stamp || failed[sh].load(std::memory_order_relaxed)) continue;
      shape_in[sh] = shape_in_stamp;
      out.push_back(shape_rep[sh]);
    }
    for (int32_t sh = 0; sh < (int32_t)S.shape_task.size() && sh < (int32_t)shape_in.size(); ++sh) {
      if ((int32_t)out.size() >= S.K) break;
      const int32_t rep = S.shape_task[sh];
      if (rep < 0 || rep >= S.n_tasks || S.task_shape[rep] != sh || shape_in[sh] == shape_in_stamp ||
          failed[sh].load(std::memory_order_relaxed))
        continue;
      shape_in[sh] = shape_in_stamp;
      out.push_back(rep);
    }
  };
  auto refresh_start = [&]() -> kbg_status {
    if (kbg_status fs = flush(); fs != KBG_OK) return fs;
    live_list(refresh_list);
    if (refresh_list.empty()) return KBG_OK;
    const int32_t G = grouper.build(*oth, refresh_list.data(), (int32_t)refresh_list.size(), kContendedSlack);
    if (kbg_status st = device_launch(S, *oth, G, pushed); st != KBG_OK) return st;
    refresh_inflight = true;
    S.stats.refresh_scans++;
    rechecks_at_scan = S.stats.resolve_rechecks;  // (no second refresh while this one is out)
    ctr.add("refresh", G);
    return KBG_OK;
  };
  // the refresh has landed: its lists become the ones the commit reads,
  // unless a synchronous rescan since then left fresher ones
  auto refresh_install = [&]() -> kbg_status {
    refresh_inflight = false;
    if (kbg_status st = device_wait(S, *oth); st != KBG_OK) return st;
    learn_failed(*oth);
    if (oth->base < sg->base) return KBG_OK;
    rs.reset(*oth);
    map_shapes(*oth, refresh_list, 0);
    si ^= 1;
    std::swap(sg, oth);
    rechecks_at_scan = S.stats.resolve_rechecks;
    ctr.add("installed");
    return KBG_OK;
  };
  auto refresh_poll = [&]() -> kbg_status {
    if (!reuse || refresh_rechecks <= 0) return KBG_OK;
    if (refresh_inflight) return hipEventQuery(oth->ev[6]) == hipSuccess ? refresh_install() : KBG_OK;
    if (S.stats.resolve_rechecks - rechecks_at_scan >= refresh_rechecks) return refresh_start();
    return KBG_OK;
  };
  ctr.add("take");
  Batch* cur = next_batch(true);
  ctr.add("took");
  if (!cur) {
    finish();
    return fail(KBG_E_INVALID, pr.error);
  }
  if (!cur->bt.empty()) {
    auto tp = clk::now();
    kbg_status st = launch(S.stages[si], cur);
    S.stats.device_ms += ms_since(tp);
    if (st != KBG_OK) return abort(st);
  }
  while (cur && !cur->bt.empty()) {
    const std::vector<int32_t>& bt = cur->bt;
    sg = &S.stages[si];
    oth = &S.stages[si ^ 1];
    kbg::Stage& other = *oth;
    S.stats.batches++;
    auto tp = clk::now();
    kbg_status st = KBG_OK;
    Batch* nxt = nullptr;
    if (!reuse) {
      ctr.add("wait");
      st = device_wait(S, *sg);
      ctr.add("waited");
      if (st != KBG_OK) return abort(st);
      learn_failed(*sg);
      // the next batch's scan overlaps this batch's resolve when it is ready
      nxt = next_batch(false);
      if (pred_failed) return abort(fail(KBG_E_INVALID, pr.error));
      if (nxt && !nxt->bt.empty()) {
        if ((st = launch(other, nxt)) != KBG_OK) return abort(st);
        S.stats.overlapped++;
      }
    } else {
      ctr.add("reuse", (int64_t)bt.size());
    }
    S.stats.device_ms += ms_since(tp);
    // commit in order
    tp = clk::now();
    if (!reuse) rs.reset(*sg);  // reuse: the stage's cursors carry on
    rstamp = ++S.res_stamp;  // this resolution's commits (touched keeps the rows not yet written back)
    S.mstamp = rstamp;
    bactual.assign(bt.size(), 0);
    int32_t cut = -1;
    bool aff_cut = false;  // a pod-affinity gain: the lists miss the gained nodes
    int32_t seg = 0;  // first batch entry covered by the current scan of this stage
    bool panic = false;
    const uint64_t cl0 = rprof ? cycles() : 0;
    const int32_t nb = (int32_t)bt.size();
    ctr.add("resolve", nb);
    truth_from = 0;
    for (int32_t i = 0; i < nb; ++i) {
      const int32_t t = bt[i];
      if ((i & 511) == 511) to_truth(cur, i);  // keep the truth engine a few hundred tasks behind
      if ((i & 127) == 127 && reuse) {  // contended: a refresh scan to start or to switch to
        if ((st = refresh_poll()) != KBG_OK) return abort(st);
      }
      if ((i & 255) == 255 && !nxt && !pred_failed && !reuse) {
        // the predictor's next batch, if it is ready now, scans while this one resolves
        nxt = next_batch(false);
        if (nxt && !nxt->bt.empty()) {
          if ((st = launch(other, nxt)) != KBG_OK) return abort(st);
          S.stats.overlapped++;
        }
      }
      if (i + 8 < nb) {  // task-indexed rows of the tasks ahead (batch order is not index order)
        const int32_t t8 = bt[i + 8];
        __builtin_prefetch(&S.treq[t8]);
        __builtin_prefetch(&S.task_job[t8]);
        __builtin_prefetch(&last[S.task_job[bt[i + 4]]]);
      }
      int32_t node = -1, kind = 0;
      const uint64_t c0 = rprof ? cycles() : 0;
      const int64_t rk0 = S.stats.resolve_rechecks;
      int r;
      if (reuse) {
        const int32_t row = shape_row_of[S.task_shape[t]];
        r = row >= 0 ? rs.resolve(row, t, &node, &kind) : RES_TRUNC;  // no row for the shape: rescan
      } else {
        r = rs.resolve(sg->row_of[i - seg], t, &node, &kind);
      }
      if (rprof) {
        rcyc[0] += cycles() - c0;
        rk_phase[reuse ? 2 : contended ? 1 : 0] += S.stats.resolve_rechecks - rk0;
      }
      if (r == RES_TRUNC) {
        if (reuse) ctr.add("reuse.rescan", i);
        const bool keep_reuse = contended;  // the rescan's rows by shape (else by batch entry)
        reuse = false;
        // A candidate list ran out before the table did. The predictions
        // still hold (no outcome differed), so instead of cutting the batch
        // and replaying the engine, write the commits so far back to HBM and
        // rescan the rest of the batch against the updated table.
        S.stats.resolve_ms += ms_since(tp);
        tp = clk::now();
        S.stats.truncations++;
        st = flush();
        if (st == KBG_OK) {
          const int32_t* list = bt.data() + i;
          int32_t len = nb - i;
          if (keep_reuse) {
            // one task per shape (rows are looked up by shape from here on):
            // this task, the other shapes of the rest of the batch, then the
            // live shapes it lacks (at most K entries)
            scan_list.clear();
            ++shape_in_stamp;
            for (int32_t k = i; k < nb && (int32_t)scan_list.size() < S.K; ++k) {
              const int32_t sh = S.task_shape[bt[k]];
              if (shape_in[sh] == shape_in_stamp) continue;
              shape_in[sh] = shape_in_stamp;
              scan_list.push_back(bt[k]);
            }
            for (int32_t sh : seen_shapes) {
              if ((int32_t)scan_list.size() >= S.K) break;
              if (shape_in[sh] == shape_in_stamp || failed[sh].load(std::memory_order_relaxed)) continue;
              shape_in[sh] = shape_in_stamp;
              scan_list.push_back(shape_rep[sh]);
            }
            // and every other candidate shape not known to fit nowhere (a
            // task of it, kept by derive_host): a shape that first appears in
            // a later batch finds a row instead of cutting for a rescan
            if (rescan_all)
              for (int32_t sh = 0; sh < (int32_t)S.shape_task.size() && sh < (int32_t)shape_in.size(); ++sh) {
                if ((int32_t)scan_list.size() >= S.K) break;
                const int32_t rep = S.shape_task[sh];
                if (rep < 0 || rep >= S.n_tasks || S.task_shape[rep] != sh || shape_in[sh] == shape_in_stamp ||
                    failed[sh].load(std::memory_order_relaxed))
                  continue;
                shape_in[sh] = shape_in_stamp;
                scan_list.push_back(rep);
              }
            list = scan_list.data();
            len = (int32_t)scan_list.size();
          }
          const int32_t G = grouper.build(*sg, list, len, keep_reuse ? kContendedSlack : kGroupSlack);
          st = device_launch(S, *sg, G, pushed);
        }
        if (st == KBG_OK) st = device_wait(S, *sg);
        if (st != KBG_OK) return abort(st);
        learn_failed(*sg);
        S.stats.device_ms += ms_since(tp);
        tp = clk::now();
        seg = i;
        rs.reset(*sg);  // (flush gave the commits after the rescan a new stamp)
        if (keep_reuse) {
          map_shapes(*sg, scan_list, 0);
          reuse = true;
          rechecks_at_scan = S.stats.resolve_rechecks;
        }
        r = rs.resolve(sg->row_of[0], t, &node, &kind);  // a fresh list always decides its first task
      }
      if (r == RES_PANIC) {
        panic = true;
        break;
      }
      const bool ok = node >= 0;
      bactual[i] = ok;
      S.stats.task_evaluations++;
      // the failed tasks of the job the predictor consumed with this one
      // (their shapes fit nowhere: the committer marked them so itself)
      const int32_t run = cur->brun[i];
      int32_t t_last = t;
      if (run && ok) return abort(fail(KBG_E_INVALID, "internal: a task of a shape known to fit nowhere was placed"));
      if (run) {
        const int32_t j = S.task_job[t];
        const int32_t* jp = S.pend.data() + S.pend_off[j];
        const int32_t pos = (int32_t)(std::find(jp, jp + S.pend_len[j], t) - jp);  // t's place in its job's order
        t_last = jp[pos + run];
        S.stats.task_evaluations += run;
        if (S.svc) {  // every rank replays them one by one
          S.svc_out.push_back((uint32_t)t);
          S.svc_out.push_back(~0u);
          for (int32_t k = 1; k < run; ++k) {
            S.svc_out.push_back((uint32_t)jp[pos + k]);
            S.svc_out.push_back(~0u);
          }
        }
      }
      if (reuse_ok) {
        const int32_t sh = S.task_shape[t];
        if (shape_rep[sh] < 0) {
          shape_rep[sh] = t;
          seen_shapes.push_back(sh);
        }
      }
      if (S.svc) {  // the scan service: every rank replays the committed outcomes
        S.svc_out.push_back((uint32_t)t_last);
        S.svc_out.push_back(ok ? ((uint32_t)node << 1 | (kind == KBG_KIND_PIPELINE ? 1u : 0u)) : ~0u);
      }
      if (ok) {
        const Res old = kind == KBG_KIND_ALLOCATE ? S.idle[node] : S.rel[node];
        if (S.has_ports)
          dec_oldp.insert(dec_oldp.end(), S.node_ports.begin() + (size_t)node * S.PW,
                          S.node_ports.begin() + (size_t)(node + 1) * S.PW);
        const uint64_t c1 = rprof ? cycles() : 0;
        const bool dup = mirror_add(S, t, node, kind);
        if (mark[node] != rstamp) {
          mark[node] = rstamp;
          touched.push_back(node);
        }
        if (packed) {
          mirror_row(S, mrow[node], node);
          mrow[node].mark = rstamp;
        }
        const uint64_t c2 = rprof ? cycles() : 0;
        const LogItem it{t, node, kind, true, true, dup, old};
        if (lg) items.push_back(it);
        else log_one(it);
        if (rprof) {
          rcyc[1] += c2 - c1;
          rcyc[2] += cycles() - c2;
        }
      } else {
        mark_failed(failed.get(), S.task_shape[t]);
        const LogItem it{t_last, -1, 0, false, true, false, Res{}};  // the job's last evaluated task (FitError)
        if (lg) items.push_back(it);
        else log_one(it);
      }
      if (ok != (bool)cur->bpred[i]) {
        cut = i + 1;
        S.stats.mispredictions++;
        break;
      }
      if (!S.aff_gain_classes.empty()) {
        // pod affinity: a class gained nodes (kbg_affinity.cpp). The rest of
        // the batch was scanned against the old masks and shapes of the class
        // marked failed may fit again: cut here, the predictor replays to this
        // point and the next batch is scanned against the new masks.
        for (int32_t c : S.aff_gain_classes) {
          S.aff_gain_flag[c] = 0;
          for (int32_t sh : S.affm->class_shapes[c]) {
            failed[sh].store(0, std::memory_order_relaxed);
            if (rs.floor) rs.floor[sh] = 0;  // the class's nodes may fit again
          }
        }
        S.aff_gain_classes.clear();
        cut = i + 1;
        aff_cut = true;
        S.stats.mispredictions++;
        break;
      }
    }
    if (rprof) rcyc[3] += cycles() - cl0;
    if (lg && !items.empty()) {
      lg->push(std::move(items));
      items = std::vector<LogItem>();
      items.reserve(bt.size());
    }
    ctr.add("resolved");
    if (S.svc && S.svc_out.size() >= kSvcStreamWords) {
      // the scan service: batches resolved against reused lists send no launch; stream their
      // commits so the other ranks replay beside this one instead of after the end message
      thread_local std::vector<uint32_t> sm;
      if ((st = svc_flush_state(S, sm, 0, false, kSvcState, 0)) != KBG_OK) return abort(st);
    }
    if (pred_failed) return abort(fail(KBG_E_INVALID, pr.error));  // seen by the look-ahead above
    S.stats.resolve_ms += ms_since(tp);
    tp = clk::now();
    if (panic) {
      recycle(cur);
      recycle(nxt);
      cur = nullptr;
      result = fail(KBG_E_REF_PANIC, "allocate reached a node whose NodeInfo.Node is nil with the predicates plugin on "
                                     "(predicates.go:122-123)");
      break;
    }
    if (cut >= 0) {  // restart the predictor from the engine state at the cut
      // a refresh scan in flight holds lists as valid as any: switch to them;
      // anything else in flight was predicted before the cut
      if (refresh_inflight) st = refresh_install();
      else st = device_drop(S, *oth);
      if (st != KBG_OK) return abort(st);
      const bool will_reuse = reuse_ok && !aff_cut;
      contended = will_reuse;
      if (cont_depth > 0) pr.P.depth.store(cont_depth, std::memory_order_relaxed);
      if (cont_batch > 0) pr.P.kmax.store(cont_batch, std::memory_order_relaxed);
      if (will_reuse) {  // before the predictor restarts: it reads the failed shapes
        // a batch that resolved against an earlier batch's stage keeps that
        // stage's map (its own entries built no rows); otherwise the stage's
        // rows are this batch's entries from `seg` on
        if (!reuse) {
          map_shapes(*sg, bt, seg);
          rechecks_at_scan = S.stats.resolve_rechecks;
        }
        probe_failed(*sg);
      }
      to_truth(cur, cut);
      ctr.add("cut", cut);
      truth.wait_idle();
      ctr.add("truth", cut);
      if (!truth.error.empty()) return abort(fail(KBG_E_INVALID, truth.error));
      pr.rollback_truth(++cur_epoch, &E_truth, cur, nxt);
      cur = next_batch(true);
      ctr.add("took");
      if (!cur) return abort(fail(KBG_E_INVALID, pr.error));
      if (will_reuse && !cur->bt.empty()) {  // resolve against this stage's lists
        reuse = true;
        S.stats.reused_batches++;
        continue;
      }
      reuse = false;
      if (!cur->bt.empty()) {
        tp = clk::now();
        if ((st = launch(S.stages[si], cur)) != KBG_OK) return abort(st);
        S.stats.device_ms += ms_since(tp);
      }
      continue;
    }
    to_truth(cur, nb);
    recycle(cur);
    if (reuse) {  // the next batch resolves against the same lists while they last
      if ((st = refresh_poll()) != KBG_OK) return abort(st);
      probe_failed(*sg);
      ctr.add("take");
      cur = next_batch(true);
      ctr.add("took");
      if (!cur) return abort(fail(KBG_E_INVALID, pr.error));
      if (!cur->bt.empty()) S.stats.reused_batches++;
      continue;
    }
    if (!nxt) {  // the predictor was behind: take its next batch now and scan it
      ctr.add("take");
      nxt = next_batch(true);
      ctr.add("took");
      if (!nxt) return abort(fail(KBG_E_INVALID, pr.error));
      if (!nxt->bt.empty()) {
        tp = clk::now();
        if ((st = launch(other, nxt)) != KBG_OK) return abort(st);
        S.stats.device_ms += ms_since(tp);
      }
    }
    cur = nxt;
    si ^= 1;
  }
  if (cur) recycle(cur);  // the epoch's end marker
  for (kbg::Stage& g : S.stages) {
    kbg_status st = device_drop(S, g);  // a scan launched before a panic
    if (st != KBG_OK) {
      finish();
      return st;
    }
  }
  // A cycle that ran to its end had no cut in its last epoch: the predictor's
  // engine then holds exactly the committed outcomes, the truth engine's
  // state-to-be. Its backlog is dropped instead of waited for (a truth engine
  // that fell behind on a shared core held the whole cycle's end).
  // KBG_CHECK_TRUTH=1 (tests) waits for it and compares the two.
  const bool check_truth = getenv("KBG_CHECK_TRUTH") != nullptr;  // (per cycle: the tests switch it)
  const bool predictor_final = result == KBG_OK && !no_truth;
  if (predictor_final && !check_truth) truth.abandon();
  finish();
  if (predictor_final) {
    if (check_truth && !engines_equal(E, E_truth))
      return fail(KBG_E_INVALID, "internal: KBG_CHECK_TRUTH: the predictor's final engine differs from the truth engine");
    E_truth = E;
  }
  ctr.add("joined");
  if (!truth.error.empty()) return fail(KBG_E_INVALID, truth.error);
  if (lg) lg->join();  // the decision log and FitError records are complete
  ctr.add("logged");
  if (kbg_status st = flush(); st != KBG_OK) return st;  // the cycle's last write-back
  HIP_TRY(hipStreamSynchronize(S.stream));
  if (S.svc) {  // the scan service: every rank counts its nodes after the end message (allocate_svc_root)
    g_svc_fit.dec_oldp = std::move(dec_oldp);
    g_svc_fit.last = std::move(last);
  } else if (kbg_status st = compute_fit_deltas(S, dec, dec_old, dec_oldp, last); st != KBG_OK) {
    return st;
  }
  ctr.add("fit");
  if (S.has_aff && getenv("KBG_PROFILE_AFF"))
    fprintf(stderr, "[kbg aff] aff_place %llu calls, %.1f cycles/call, %llu bit recomputes, mask words dirty %zu\n",
            (unsigned long long)S.affm->prof_calls,
            S.affm->prof_calls ? (double)S.affm->prof_cycles / S.affm->prof_calls : 0.0,
            (unsigned long long)S.affm->prof_recomputes, S.mask_dirty.size());
  if (no_truth) {
    if (S.stats.mispredictions) return fail(KBG_E_INVALID, "KBG_NO_TRUTH: a cycle with a misprediction");
    E_truth = E;  // (the predictor has finished)
  }
  finalize_shares(S, E_truth);
  S.fin = E_truth;
  S.stats.engine_ms = pr.engine_ms;
  S.stats.replayed = pr.replayed;
  if (rprof)
    fprintf(stderr, "[kbg resolve] %lld tasks, cycles/task: walk %.1f mirror %.1f log %.1f loop %.1f (incl. rescans)\n",
            (long long)S.stats.task_evaluations, (double)rcyc[0] / std::max<int64_t>(1, S.stats.task_evaluations),
            (double)rcyc[1] / std::max<int64_t>(1, S.stats.task_evaluations),
            (double)rcyc[2] / std::max<int64_t>(1, S.stats.task_evaluations),
            (double)rcyc[3] / std::max<int64_t>(1, S.stats.task_evaluations));
  if (rprof)
    fprintf(stderr, "[kbg resolve] re-checks: uncontended %lld, contended on fresh scans %lld, on reused lists %lld; "
                    "refresh scans %lld, overlapped batches %lld, batches %lld\n",
            (long long)rk_phase[0], (long long)rk_phase[1], (long long)rk_phase[2], (long long)S.stats.refresh_scans,
            (long long)S.stats.overlapped, (long long)S.stats.batches);
  if (eprof.on && eprof.steps)
    fprintf(stderr, "[kbg engine] steps %llu cycles/step: qpop %.1f apply %.1f jfix %.1f qpush %.1f (engine %.3f ms)\n",
            (unsigned long long)eprof.steps, (double)eprof.qpop / eprof.steps, (double)eprof.apply / eprof.steps,
            (double)eprof.jtop / eprof.steps, (double)eprof.qpush / eprof.steps, pr.engine_ms);
  S.allocated = true;
  S.stats.allocate_ms = ms_since(t0);
  ctr.add("end");
  print_traces(ctr, pr.tr);
  return copy_log(S, out, cap, n_out, result);
}

// ============================================== sharded allocate: owner-resolve
// SURVEY §8(e). Rank r holds the node rows [tab_lo, tab_lo + tab_n); first-fit
// over the whole cluster is the lowest rank that has a fitting node, then that
// rank's first fitting node. Per batch:
//   1. rank 0 runs the ordering engine (Predictor) and broadcasts the batch's
//      task list with the predicted outcomes;
//   2. every rank scans its own rows on its device and selects its own
//      candidates (kbg_select_kernel over its words);
//   3. a sum-reduce of one bit per rank and row says which ranks have any
//      fitting node for each row (`avail`);
//   4. rounds: each rank resolves, in batch order, exactly the tasks it owns —
//      the lowest rank in `avail` that has not failed the row at or before the
//      task — against its host mirror of its own rows; one min-reduce per round
//      publishes the packed winners (node << 1 | kind) and each rank's first
//      failure per row. A failure hands the row's later tasks to the next rank
//      (a rank never fits a row again once it failed it: Idle, Releasing and
//      the pod cap only shrink during allocate), which rolls its own commits
//      back to the first task it gained and resolves again. No new failure:
//      every owned task has its node;
//   5. every rank walks the outcomes in order exactly as the single-rank
//      committer does (decision log, gang dispatch, mirror of the other ranks'
//      rows, cut at the first misprediction), rolls its own commits past the
//      cut back and writes its touched rows to HBM.
// The collectives go through ShardIO: RCCL over xGMI in the library, a host
// transport in the CPU tests (tools/engine_bench.cpp).
struct ShardIO {
  virtual ~ShardIO() = default;
  virtual kbg_status bcast(uint32_t* buf, size_t n) = 0;                   // rank 0's words to every rank
  virtual kbg_status scan(Session& S, kbg::Stage& sg, int32_t G, int32_t base) = 0;  // this rank's candidates
  virtual kbg_status allreduce(uint32_t* buf, size_t n, bool sum) = 0;      // element-wise min (sum), in place
  // the scan plus the rows' availability over the ranks (bit r: rank r has a candidate)
  virtual kbg_status scan_avail(Session& S, kbg::Stage& sg, int32_t G, int32_t base, uint32_t* avail) {
    kbg_status st = scan(S, sg, G, base);
    if (st != KBG_OK) return st;
    for (int32_t g = 0; g < G; ++g) avail[g] = row_fits_somewhere(sg, g) ? (1u << S.shard) : 0u;  // any node (listed or not)
    return allreduce(avail, G, true);
  }
  // this rank's committed rows (and class-mask words) to the table its scans read
  virtual kbg_status push(Session& S, const std::vector<int32_t>& touched) { return push_deltas(S, touched); }
  virtual kbg_status sync(Session& S) { return comm_sync(S); }
  double ms = 0;                                                            // time in collectives
};

// The library's transport: the session's stream, a device exchange buffer
// and the communicator.
struct RcclIO final : ShardIO {
  Session& S;
  uint32_t* d = nullptr;  // device exchange buffer
  uint32_t* h = nullptr;  // pinned staging
  size_t cap = 0;
  explicit RcclIO(Session& s) : S(s) {}
  ~RcclIO() override {
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
  }
  kbg_status reserve(size_t n) {
    if (n <= cap) return KBG_OK;
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
    d = nullptr;
    h = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc((void**)&d, std::max<size_t>((size_t)n * 4, 64)));
    HIP_TRY(hipHostMalloc((void**)&h, std::max<size_t>((size_t)n * 4, 64), hipHostMallocDefault));
    cap = n;
    return KBG_OK;
  }
  kbg_status bcast(uint32_t* buf, size_t n) override {
    const auto t0 = std::chrono::steady_clock::now();
    kbg_status st = reserve(n);
    if (st != KBG_OK) return st;
    if (S.shard == 0) {
      std::memcpy(h, buf, n * 4);
      HIP_TRY(hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, S.stream));
    }
    if (kbg_status st2 = coll_rc(S, S.comm->coll->bcast(d, n, S.stream)); st2 != KBG_OK) return st2;
    HIP_TRY(hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, S.stream));
    if (kbg_status st2 = comm_sync(S); st2 != KBG_OK) return st2;
    std::memcpy(buf, h, n * 4);
    ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return KBG_OK;
  }
  kbg_status scan(Session& S2, kbg::Stage& sg, int32_t G, int32_t base) override {
    return device_scan(S2, sg, G, base);
  }
  // one round trip: scan, select, availability bits and their sum-reduce
  kbg_status scan_avail(Session& S2, kbg::Stage& sg, int32_t G, int32_t base, uint32_t* avail) override {
    kbg_status st = device_scan(S2, sg, G, base);
    if (st != KBG_OK) return st;
    for (int32_t g = 0; g < G; ++g) avail[g] = sg.h_avail[sg.row_slot[g]];  // summed per shape slot
    return KBG_OK;
  }
  kbg_status allreduce(uint32_t* buf, size_t n, bool sum) override {
    const auto t0 = std::chrono::steady_clock::now();
    kbg_status st = reserve(n);
    if (st != KBG_OK) return st;
    std::memcpy(h, buf, n * 4);
    HIP_TRY(hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, S.stream));
    if (kbg_status st2 = coll_rc(S, S.comm->coll->allreduce(d, d, n, sum ? kbg::kCollSum : kbg::kCollMin, S.stream));
        st2 != KBG_OK)
      return st2;
    HIP_TRY(hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, S.stream));
    if (kbg_status st2 = comm_sync(S); st2 != KBG_OK) return st2;
    std::memcpy(buf, h, n * 4);
    ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return KBG_OK;
  }
};

// Sessions whose allocate runs the owner-resolve protocol: sharded over a
// communicator of at most 32 ranks (one availability bit each), without pod
// affinity (its counts couple nodes of different ranks through a topology
// domain; those sessions all-gather the bitmaps and resolve on every rank).
// KBG_OWNER_RESOLVE=1 also runs it on a one-rank communicator (the RCCL
// transport and the own-word select on a one-GPU box).
bool owner_resolve_ok(const Session& S) {
  static const bool off = getenv("KBG_REPLICATED_RESOLVE") != nullptr;
  const char* force = getenv("KBG_OWNER_RESOLVE");
  const bool ranks = S.R > 1 || (force && force[0] == '1');
  return S.comm && ranks && S.shard >= 0 && S.R <= 32 && !S.has_aff && !off;
}

kbg_status allocate_sharded(Session& S, ShardIO& io, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.allocated || S.backfilled || S.preempted)
    return fail(KBG_E_INVALID, "allocate runs once per cycle, before backfill and preempt; call kbg_session_reset");
  const bool first = !S.cycle_started;
  if (first) begin_cycle(S);
  S.action = KBG_ACTION_ALLOCATE;
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  const auto t0 = clk::now();
  const int32_t R = S.R, me = S.shard;
  constexpr uint32_t kNone = 0xffffffffu;
  std::vector<kbg_decision>& dec = S.dec;
  std::vector<Res> dec_old(dec.size());
  std::vector<uint64_t> dec_oldp(dec.size() * (size_t)S.PW);
  std::vector<LastEval> last(S.n_jobs);
  std::unique_ptr<std::atomic<uint8_t>[]> failed(new std::atomic<uint8_t>[std::max(1, S.n_shapes)]);
  for (int32_t i = 0; i < S.n_shapes; ++i) failed[i].store(0, std::memory_order_relaxed);
  std::vector<int32_t> mark(S.n_nodes, -1), touched;
  Grouper grouper(S);
  Resolver rs{S, mark};
  kbg::Stage& sg = S.stages[0];
  kbg_status result = KBG_OK;

  // rank 0: the ordering engine; every rank replays the committed outcomes
  // (rank 0 into a truth engine a cut restarts its predictor from, as the
  // single-rank committer does: no checkpoint copies, no replay of a batch
  // prefix)
  Engine E = first ? S.init : live_engine(S);
  Engine E_truth;
  std::unique_ptr<Predictor> pr;
  std::unique_ptr<Replayer> rp;
  if (me == 0) {
    E_truth = E;
    pr.reset(new Predictor(S, E, failed.get()));
    pr->truth_mode = true;
    rp.reset(new Replayer(S, E_truth, sched_getcpu()));
    pr->start(sched_getcpu());
  } else {
    rp.reset(new Replayer(S, E));
  }
  int64_t cur_epoch = 0;
  auto next_batch = [&]() -> Batch* {  // rank 0: the next batch of the current epoch (nullptr: predictor failed)
    for (;;) {
      bool none = false;
      Batch* b = pr->take(true, &none);
      if (!b) return nullptr;
      if (b->epoch != cur_epoch) {
        pr->recycle(b);
        continue;
      }
      return b;
    }
  };
  // batch message: [kind, n, task ids..., predicted outcomes...]; kind 0 =
  // batch, 1 = end of the cycle, 2 = the predictor failed
  std::vector<uint32_t> msg(2 + 2 * (size_t)S.K);
  std::vector<int32_t> bt;
  std::vector<char> bpred, bactual;
  // own commits of the current segment, in batch order (rolled back past a cut)
  struct Undo {
    int32_t pos, node, kind;
    bool dup;
    Res old;
  };
  std::vector<Undo> undo;
  auto rollback_from = [&](int32_t pos) {
    while (!undo.empty() && undo.back().pos >= pos) {
      const Undo& u = undo.back();
      const int32_t t = bt[u.pos];
      if (!u.dup) {
        if (!S.nil_node[u.node]) (u.kind == KBG_KIND_ALLOCATE ? S.idle[u.node] : S.rel[u.node]) = u.old;
        S.ntasks[u.node]--;
        if (S.has_ports) remove_ports(S, S.task_class[t], u.node);
        if (S.has_dupkeys && S.key_hot[S.task_key[t]]) {
          S.node_keys.erase(node_key_of(S, t, u.node));
          S.key_holder.erase(node_key_of(S, t, u.node));
        }
      }
      undo.pop_back();
    }
  };
  std::vector<uint64_t> pos_oldp;  // host ports before each own commit (decision log order needs them)
  Batch* cur = nullptr;
  int32_t seg = 0;  // rank 0: first entry of `cur` in the current segment
  int32_t stamp = S.res_stamp;
  std::unique_ptr<Logger>* lg_ref = nullptr;  // set once the logger exists (below)
  auto finish = [&]() {
    if (pr) {
      if (cur) pr->recycle(cur);
      cur = nullptr;
      pr->finish();
    }
    if (rp) rp->join();
    if (lg_ref && *lg_ref) (*lg_ref)->join();
  };
  auto abort = [&](kbg_status st) {
    // a failure of this rank alone (the batch messages and the reduced
    // results are the same on every rank): the peers are, or will be,
    // blocked in a collective this rank never joins
    if (st == KBG_E_HIP || st == KBG_E_RCCL || st == KBG_E_NOMEM) comm_abort(S.comm);
    finish();
    S.owner = false;
    return st;
  };
  // The log side of a committed outcome: decision log and gang dispatch
  // (record_decision), FitError bookkeeping, and — for another rank's row —
  // this rank's mirror of it. `oldp`: host ports before an own commit.
  int64_t logged = 0;  // task evaluations: counted apart from S.stats (the committer updates that line)
  auto log_one = [&](const LogItem& it, const uint64_t* oldp) {
    ++logged;
    last[S.task_job[it.t]] = LastEval{it.t, (int32_t)dec.size(), it.node, it.kind};
    if (!it.ok) return;
    bool dup = it.dup;
    if (it.own) {  // committed during the resolve
      dec_old.push_back(it.old);
      if (S.has_ports) dec_oldp.insert(dec_oldp.end(), oldp, oldp + S.PW);
    } else {  // another rank's row: this rank's mirror follows
      dec_old.push_back(it.kind == KBG_KIND_ALLOCATE ? S.idle[it.node] : S.rel[it.node]);
      if (S.has_ports)
        dec_oldp.insert(dec_oldp.end(), S.node_ports.begin() + (size_t)it.node * S.PW,
                        S.node_ports.begin() + (size_t)(it.node + 1) * S.PW);
      dup = mirror_add(S, it.t, it.node, it.kind);
    }
    record_decision(S, it.t, it.node, it.kind, dup);
  };
  // On a thread of its own unless host ports or colliding pod keys make the
  // mirror share state across nodes (used-port holders, the pod-key set).
  std::unique_ptr<Logger> lg;
  if (!S.has_ports && !S.has_dupkeys)
    lg.reset(new Logger([&](const LogItem& it) { log_one(it, nullptr); }, sched_getcpu()));
  lg_ref = &lg;
  S.owner = true;  // device_launch: own words, no all-gather
  for (;;) {
    // ---- 1. the segment's tasks from rank 0
    auto tp = clk::now();
    if (me == 0) {
      if (!cur) {
        cur = next_batch();
        seg = 0;
      }
      if (!cur) {
        msg[0] = 2;
        msg[1] = 0;
      } else {
        const int32_t n = (int32_t)cur->bt.size() - seg;
        msg[0] = n > 0 ? 0 : 1;
        msg[1] = (uint32_t)n;
        for (int32_t i = 0; i < n; ++i) {
          msg[2 + i] = (uint32_t)cur->bt[seg + i];
          msg[2 + S.K + i] = (uint32_t)cur->bpred[seg + i];
        }
      }
    }
    kbg_status st = io.bcast(msg.data(), msg.size());
    if (st != KBG_OK) return abort(st);
    if (msg[0] == 2) return abort(fail(KBG_E_INVALID, pr ? pr->error : std::string("the ordering engine failed on rank 0")));
    if (msg[0] == 1) break;
    const int32_t n = (int32_t)msg[1];
    if (n <= 0 || n > S.K) return abort(fail(KBG_E_INVALID, "internal: bad batch message"));
    bt.assign(n, 0);
    bpred.assign(n, 0);
    for (int32_t i = 0; i < n; ++i) {
      bt[i] = (int32_t)msg[2 + i];
      bpred[i] = (char)msg[2 + S.K + i];
      if (bt[i] < 0 || bt[i] >= S.n_tasks) return abort(fail(KBG_E_INVALID, "internal: bad task in batch message"));
    }
    S.stats.batches++;
    // ---- 2. own candidates against the table with every earlier commit
    const int32_t G = grouper.build(sg, bt.data(), n);
    // ---- 3. which ranks fit each row at all
    std::vector<uint32_t> avail(G);
    if ((st = io.scan_avail(S, sg, G, stamp, avail.data())) != KBG_OK) return abort(st);
    S.stats.device_ms += ms_since(tp);
    // ---- 4. owner rounds
    tp = clk::now();
    std::vector<uint32_t> fail_at((size_t)G * R, kNone);  // first failing task of (row, rank), global
    auto owner_of = [&](int32_t g, int32_t i) -> int32_t {
      for (uint32_t m = avail[g]; m; m &= m - 1) {
        const int32_t r = __builtin_ctz(m);
        if (fail_at[(size_t)g * R + r] > (uint32_t)i) return r;
      }
      return -1;
    };
    std::vector<uint32_t> xbuf((size_t)n + (size_t)G * R + 2);
    std::vector<uint32_t> win(n, kNone);
    std::vector<uint32_t> my_fail(G, kNone);
    std::vector<Res> pos_old(n);
    std::vector<char> pos_dup(n, 0);
    pos_oldp.assign((size_t)n * S.PW, 0);
    undo.clear();
    const int32_t stamp0 = ++S.res_stamp;  // commits of this segment
    S.mstamp = stamp0;
    touched.clear();
    int32_t from = 0, end = n;
    uint32_t my_trunc = kNone, my_panic = kNone;
    for (;;) {
      S.stats.owner_rounds++;
      // resolve the own tasks from `from` on (earlier ones keep their commits)
      rollback_from(from);
      for (int32_t i = from; i < n; ++i) win[i] = kNone;
      for (int32_t g = 0; g < G; ++g)
        if (my_fail[g] != kNone && my_fail[g] >= (uint32_t)from) my_fail[g] = kNone;
      if (my_trunc >= (uint32_t)from) my_trunc = kNone;
      if (my_panic >= (uint32_t)from) my_panic = kNone;
      rs.reset(sg);  // rolled-back commits may make skipped candidates fit again
      for (int32_t i = from; i < n; ++i) {
        const int32_t g = sg.row_of[i];
        if (my_fail[g] != kNone || owner_of(g, i) != me) continue;
        const int32_t t = bt[i];
        int32_t node = -1, kind = 0;
        const int r = rs.resolve(g, t, &node, &kind);
        if (r == RES_TRUNC) {  // the list ran out before the rows did: rescan from here
          my_trunc = (uint32_t)i;
          break;
        }
        if (r == RES_PANIC) {
          my_panic = (uint32_t)i;
          break;
        }
        if (node < 0) {
          my_fail[g] = (uint32_t)i;  // the row's later tasks go to the next rank
          continue;
        }
        pos_old[i] = kind == KBG_KIND_ALLOCATE ? S.idle[node] : S.rel[node];
        if (S.has_ports)
          std::copy(S.node_ports.begin() + (size_t)node * S.PW, S.node_ports.begin() + (size_t)(node + 1) * S.PW,
                    pos_oldp.begin() + (size_t)i * S.PW);
        const bool dup = mirror_add(S, t, node, kind);
        pos_dup[i] = dup;
        undo.push_back(Undo{i, node, kind, dup, pos_old[i]});
        if (mark[node] != stamp0) {
          mark[node] = stamp0;
          touched.push_back(node);
        }
        win[i] = ((uint32_t)node << 1) | (kind == KBG_KIND_PIPELINE ? 1u : 0u);
      }
      // publish: winners, this rank's first failure per row, truncation and panic points
      std::copy(win.begin(), win.end(), xbuf.begin());
      std::fill(xbuf.begin() + n, xbuf.end(), kNone);
      for (int32_t g = 0; g < G; ++g) xbuf[(size_t)n + (size_t)g * R + me] = my_fail[g];
      xbuf[(size_t)n + (size_t)G * R] = my_trunc;
      xbuf[(size_t)n + (size_t)G * R + 1] = my_panic;
      if ((st = io.allreduce(xbuf.data(), xbuf.size(), false)) != KBG_OK) return abort(st);
      end = (int32_t)std::min<uint32_t>((uint32_t)n, std::min(xbuf[(size_t)n + (size_t)G * R], xbuf[(size_t)n + (size_t)G * R + 1]));
      // new failures before `end` move ownership; the first task a rank gains is where it resolves again
      int32_t my_from = n;
      bool changed = false;
      for (int32_t g = 0; g < G; ++g)
        for (int32_t r = 0; r < R; ++r) {
          const uint32_t f = xbuf[(size_t)n + (size_t)g * R + r];
          uint32_t& cur_f = fail_at[(size_t)g * R + r];
          if (f == cur_f || f >= (uint32_t)end) continue;
          cur_f = std::min(cur_f, f);
          changed = true;
        }
      if (!changed) {
        for (int32_t i = 0; i < end; ++i) win[i] = xbuf[i];
        break;
      }
      // the earliest task whose owner is now this rank but was not a task it resolved
      for (int32_t i = 0; i < end && my_from == n; ++i) {
        const int32_t g = sg.row_of[i];
        if (owner_of(g, i) == me && xbuf[i] == kNone) my_from = i;
      }
      from = my_from;
    }
    S.stats.resolve_ms += ms_since(tp);
    // ---- 5. outcomes in order (every rank), cut at the first misprediction;
    // the log side (decision log, gang dispatch, the other ranks' rows in
    // this rank's mirror) goes to the logger thread when it can run beside
    // the next batch's resolve
    int32_t cut = end;  // entries [0, cut) are final
    bool mispred = false;
    bactual.assign(n, 0);
    std::vector<LogItem> items;
    if (lg) items.reserve(end);
    for (int32_t i = 0; i < end; ++i) {
      const int32_t t = bt[i];
      const int32_t g = sg.row_of[i];
      const int32_t own = owner_of(g, i);
      const bool ok = own >= 0;
      if (ok && win[i] == kNone) return abort(fail(KBG_E_INVALID, "internal: owner-resolve left a task without a node"));
      LogItem it{t, ok ? (int32_t)(win[i] >> 1) : -1, ok && (win[i] & 1u) ? KBG_KIND_PIPELINE : KBG_KIND_ALLOCATE,
                 ok, own == me, own == me && pos_dup[i], own == me ? pos_old[i] : Res{}};
      bactual[i] = ok;
      if (!ok) mark_failed(failed.get(), S.task_shape[t]);
      if (lg) items.push_back(it);
      else log_one(it, pos_oldp.data() + (size_t)i * S.PW);
      if (ok != (bool)bpred[i]) {
        cut = i + 1;
        mispred = true;
        S.stats.mispredictions++;
        break;
      }
    }
    if (lg) lg->push(std::move(items));
    // Shapes that fit nowhere from now on, learned from the exchange every
    // rank already holds (the predictor predicts their later tasks failed
    // instead of each first failure cutting a batch): no rank fits the row
    // (availability 0), or every rank that did failed it at a task before
    // the cut (a rank fails a row only on a complete list; commits past the
    // cut are rolled back, so later failures do not count). Monotone: Idle,
    // Releasing and the pod cap only shrink during allocate.
    for (int32_t g = 0; g < G; ++g) {
      const int32_t sh = sg.row_shape[g];
      bool nowhere = avail[g] == 0;
      if (!nowhere) {
        nowhere = true;
        for (uint32_t m = avail[g]; m && nowhere; m &= m - 1) {
          const uint32_t f = fail_at[(size_t)g * R + __builtin_ctz(m)];
          nowhere = f != kNone && f < (uint32_t)cut;
        }
      }
      if (nowhere) mark_failed(failed.get(), sh);
    }
    rollback_from(cut);
    if (rp) {
      std::vector<std::pair<int32_t, char>> v(cut);
      for (int32_t i = 0; i < cut; ++i) v[i] = {bt[i], bactual[i]};
      rp->push(std::move(v));
    }
    tp = clk::now();
    // test hook (tests/test_shard_gpu.py): a failure of this rank alone
    // between two protocol rounds
    if (const char* f = getenv("KBG_TEST_FAULT"); f && !strcmp(f, "push"))
      return abort(fail(KBG_E_HIP, "injected fault before the delta push (KBG_TEST_FAULT=push)"));
    if ((st = io.push(S, touched)) != KBG_OK) return abort(st);
    stamp = S.res_stamp;
    S.stats.delta_ms += ms_since(tp);
    const uint32_t panic_at = xbuf[(size_t)n + (size_t)G * R + 1];
    if (!mispred && panic_at != kNone && (int32_t)panic_at == end) {
      result = fail(KBG_E_REF_PANIC, "allocate reached a node whose NodeInfo.Node is nil with the predicates plugin on "
                                     "(predicates.go:122-123)");
      break;
    }
    const bool trunc = !mispred && end < n;
    if (trunc) S.stats.truncations++;
    if (me == 0) {
      if (mispred) {
        rp->wait_idle();  // the truth engine holds every outcome up to the cut
        if (!rp->error.empty()) return abort(fail(KBG_E_INVALID, rp->error));
        pr->rollback_truth(++cur_epoch, &E_truth, cur, nullptr);
        cur = nullptr;
      } else if (trunc) {
        seg += end;  // the rest of the batch, rescanned against the commits so far
      } else {
        pr->recycle(cur);
        cur = nullptr;
      }
    }
  }
  finish();
  S.owner = false;
  if (kbg_status st = io.sync(S); st != KBG_OK) return st;
  if (kbg_status st = compute_fit_deltas(S, dec, dec_old, dec_oldp, last); st != KBG_OK) return st;
  S.stats.task_evaluations += logged;
  if (rp && !rp->error.empty()) return fail(KBG_E_INVALID, rp->error);
  S.fin = me == 0 ? E_truth : E;  // the committed outcomes' engine state
  finalize_shares(S, S.fin);
  if (pr) {
    S.stats.engine_ms = pr->engine_ms;
    S.stats.replayed = pr->replayed;
  }
  S.stats.exchange_ms = io.ms;
  S.allocated = true;
  S.stats.allocate_ms = ms_since(t0);
  return copy_log(S, out, cap, n_out, result);
}

// ============================================ the scan service: rank 0 and the other ranks
// The library's transport: the communicator's collectives (RCCL on the
// session's stream, or the host transport's shared memory). Rank 0 stages a
// message in a pinned ring slot and enqueues its copy and the broadcasts
// (header, then payload); the other ranks wait for the header to learn the
// payload's length.
struct CommSvc final : SvcLink {
  Session& S;
  static constexpr int kRing = 4;
  uint32_t* d_msg = nullptr;
  uint32_t* h_ring[kRing] = {};
  hipEvent_t ev_ring[kRing] = {};
  bool used[kRing] = {};
  int slot = 0;
  uint32_t* h_recv = nullptr;
  explicit CommSvc(Session& s) : S(s) {}
  ~CommSvc() override {
    if (S.stream) (void)hipStreamSynchronize(S.stream);  // no enqueued copy still reads a ring slot
    if (d_msg) (void)hipFree(d_msg);
    for (int i = 0; i < kRing; ++i) {
      if (h_ring[i]) (void)hipHostFree(h_ring[i]);
      if (ev_ring[i]) (void)hipEventDestroy(ev_ring[i]);
    }
    if (h_recv) (void)hipHostFree(h_recv);
  }
  kbg_status init() {
    HIP_TRY(hipMalloc((void**)&d_msg, kSvcMaxWords * 4));
    if (S.shard == 0) {
      for (int i = 0; i < kRing; ++i) {
        HIP_TRY(hipHostMalloc((void**)&h_ring[i], kSvcMaxWords * 4, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&ev_ring[i], hipEventDisableTiming));
      }
    } else {
      HIP_TRY(hipHostMalloc((void**)&h_recv, kSvcMaxWords * 4, hipHostMallocDefault));
    }
    return KBG_OK;
  }
  kbg_status bcast(uint32_t* d, size_t n) {
    return coll_rc(S, S.comm->coll->bcast(d, n, S.stream));
  }
  kbg_status send(Session&, const uint32_t* msg) override {
    const size_t n = msg[1];
    if (n < kSvcHead || n > kSvcMaxWords) return fail(KBG_E_INVALID, "internal: scan service message size");
    const int i = slot;
    slot = (slot + 1) % kRing;
    if (used[i]) HIP_TRY(hipEventSynchronize(ev_ring[i]));  // its last copy has been read
    std::memcpy(h_ring[i], msg, n * 4);
    HIP_TRY(hipMemcpyAsync(d_msg, h_ring[i], n * 4, hipMemcpyHostToDevice, S.stream));
    HIP_TRY(hipEventRecord(ev_ring[i], S.stream));
    used[i] = true;
    if (kbg_status st = bcast(d_msg, kSvcHead); st != KBG_OK) return st;
    if (n > kSvcHead) return bcast(d_msg + kSvcHead, n - kSvcHead);
    return KBG_OK;
  }
  kbg_status recv(Session&, std::vector<uint32_t>& msg) override {
    if (kbg_status st = bcast(d_msg, kSvcHead); st != KBG_OK) return st;
    HIP_TRY(hipMemcpyAsync(h_recv, d_msg, kSvcHead * 4, hipMemcpyDeviceToHost, S.stream));
    if (kbg_status st = comm_sync(S); st != KBG_OK) return st;
    const size_t n = h_recv[1];
    if (n < kSvcHead || n > kSvcMaxWords) return fail(KBG_E_INVALID, "internal: scan service message size");
    if (n > kSvcHead) {
      if (kbg_status st = bcast(d_msg + kSvcHead, n - kSvcHead); st != KBG_OK) return st;
      HIP_TRY(hipMemcpyAsync(h_recv + kSvcHead, d_msg + kSvcHead, (n - kSvcHead) * 4, hipMemcpyDeviceToHost, S.stream));
      if (kbg_status st = comm_sync(S); st != KBG_OK) return st;
    }
    msg.assign(h_recv, h_recv + n);
    return KBG_OK;
  }
  kbg_status sum(Session&, kbg::Stage* sg, size_t info, size_t masks) override {
    uint32_t* dm = S.d_svc + fused_mask_off(S.K);
    kbg::Coll& c = *S.comm->coll;
    c.group_start();
    kbg_status st = c.allreduce(S.d_svc, S.d_svc, info, kbg::kCollSum, S.stream);
    const kbg_status st2 = c.allreduce(dm, dm, masks, kbg::kCollSum, S.stream);
    const kbg_status st3 = c.group_end();
    if (st == KBG_OK) st = st2 != KBG_OK ? st2 : st3;
    if (st != KBG_OK) return coll_rc(S, st);
    if (sg) {
      HIP_TRY(hipMemcpyAsync(sg->h_down, S.d_svc, info * 4, hipMemcpyDeviceToHost, S.stream));
      HIP_TRY(hipMemcpyAsync(sg->h_down + fused_mask_off(S.K), dm, masks * 4, hipMemcpyDeviceToHost, S.stream));
    }
    return KBG_OK;
  }
  kbg_status sum_host(Session&, uint32_t* buf, size_t n) override {
    for (size_t o = 0; o < n; o += kSvcMaxWords) {  // through the message buffer
      const size_t c = std::min(n - o, kSvcMaxWords);
      uint32_t* h = S.shard == 0 ? h_ring[0] : h_recv;
      if (S.shard == 0 && used[0]) HIP_TRY(hipEventSynchronize(ev_ring[0]));
      std::memcpy(h, buf + o, c * 4);
      HIP_TRY(hipMemcpyAsync(d_msg, h, c * 4, hipMemcpyHostToDevice, S.stream));
      if (kbg_status st = coll_rc(S, S.comm->coll->allreduce(d_msg, d_msg, c, kbg::kCollSum, S.stream)); st != KBG_OK)
        return st;
      HIP_TRY(hipMemcpyAsync(h, d_msg, c * 4, hipMemcpyDeviceToHost, S.stream));
      if (kbg_status st = comm_sync(S); st != KBG_OK) return st;
      std::memcpy(buf + o, h, c * 4);
    }
    return KBG_OK;
  }
};

// The sessions whose allocate runs the scan service: sharded over a
// communicator (at most kFfMaxSplits ranks: one info word per (slot, rank)
// in the staging). KBG_OWNER_RESOLVE=1 selects the owner-resolve protocol
// instead; KBG_SCAN_SERVICE=1 runs the service on a one-rank communicator
// (its RCCL path on a one-GPU box).
bool scan_service_ok(const Session& S) {
  const char* oe = getenv("KBG_OWNER_RESOLVE");  // (read per call: the tests switch it)
  const char* fe = getenv("KBG_SCAN_SERVICE");
  const bool owner = oe && oe[0] == '1', force = fe && fe[0] == '1';
  return S.comm && S.shard >= 0 && !owner && (S.R > 1 || force) && S.R <= kbg::kFfMaxSplits;
}

// Rank 0: the single-GPU allocate with every scan served by all ranks, then
// the end message (the rest of the state and the cycle's status).
kbg_status allocate_svc_root(Session& S, SvcLink& link, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.allocated || S.backfilled || S.preempted)  // (every rank returns this without a message)
    return fail(KBG_E_INVALID, "allocate runs once per cycle, before backfill and preempt; call kbg_session_reset");
  S.svc = &link;
  S.svc_nodes.clear();
  S.svc_masks.clear();
  S.svc_out.clear();
  const kbg_status st = allocate_cycle(S, out, cap, n_out);
  const std::string err = g_err;
  kbg_status st2 = KBG_OK;
  if (st == KBG_E_HIP || st == KBG_E_RCCL || st == KBG_E_NOMEM) {
    comm_abort(S.comm);  // the other ranks are in a collective this rank may never join
  } else {
    thread_local std::vector<uint32_t> m;
    static const bool prof = getenv("KBG_PROFILE_SVC") != nullptr;
    const auto c0 = std::chrono::steady_clock::now();
    st2 = svc_flush_state(S, m, 0, false, kSvcEnd, (uint32_t)st);
    const auto c1 = std::chrono::steady_clock::now();
    if (st2 == KBG_OK) st2 = comm_sync(S);
    const auto c2 = std::chrono::steady_clock::now();
    // FitError counts: each rank its own nodes, summed (allocate_serve does the same after the end message)
    if (st2 == KBG_OK && (st == KBG_OK || st == KBG_E_REF_PANIC))
      st2 = compute_fit_deltas(S, S.dec, S.dec_old_buf, g_svc_fit.dec_oldp, g_svc_fit.last);
    if (prof) {
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr, "[kbg svc] end message %.1f us, stream drain %.1f us, FitError counts %.1f us, cycle %.3f ms\n",
              us(c0, c1), us(c1, c2), us(c2, std::chrono::steady_clock::now()), S.stats.allocate_ms);
    }
  }
  g_svc_fit = SvcFit{};
  S.svc = nullptr;
  if (st2 != KBG_OK) return st2;
  g_err = err;
  return st;
}

// Rows and class-mask words from rank 0 into this rank's table.
kbg_status svc_apply_state(Session& S, const kbg::NodeDelta* nodes, size_t nn, const kbg::MaskDelta* masks, size_t nm) {
  for (size_t m = 0; m < nm;) {
    if (kbg_status st = stage_acquire(S); st != KBG_OK) return st;
    const int32_t cnt = (int32_t)std::min<size_t>(nm - m, (size_t)kbg::kMaskDeltaCap);
    std::memcpy(S.h_mdeltas, masks + m, (size_t)cnt * sizeof(kbg::MaskDelta));
    const kbg::MaskDelta* md = dev_ptr(S, S.h_mdeltas);
    if (!md) return fail(KBG_E_HIP, "hipHostGetDevicePointer of the mask-delta buffer failed");
    HIP_TRY(kbg::launch_mask_apply(S.d_class_mask, md, cnt, S.stream));
    if (kbg_status st = stage_release(S); st != KBG_OK) return st;
    m += cnt;
  }
  for (size_t i = 0; i < nn;) {
    if (kbg_status st = stage_acquire(S); st != KBG_OK) return st;
    int32_t cnt = 0;
    for (; i < nn && cnt < S.K; ++i) {
      const kbg::NodeDelta& d = nodes[i];
      if (d.node < S.tab_lo || d.node >= S.tab_lo + S.tab_n) continue;
      S.h_deltas[cnt] = d;
      S.h_deltas[cnt++].node = d.node - S.tab_lo;
    }
    if (cnt == 0) break;
    HIP_TRY(kbg::launch_apply(S.d_nodes, S.h_deltas_dev, cnt, S.stream));
    if (kbg_status st = stage_release(S); st != KBG_OK) return st;
  }
  return KBG_OK;
}

// Ranks != 0: serve rank 0's scans over this rank's words and follow its
// commits until the end message; the cycle ends with the same decision log,
// node state and plugin state as rank 0's.
kbg_status allocate_serve(Session& S, SvcLink& link, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.allocated || S.backfilled || S.preempted)
    return fail(KBG_E_INVALID, "allocate runs once per cycle, before backfill and preempt; call kbg_session_reset");
  const bool first = !S.cycle_started;
  if (first) begin_cycle(S);
  S.action = KBG_ACTION_ALLOCATE;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  std::vector<kbg_decision>& dec = S.dec;
  std::vector<Res>& dec_old = S.dec_old_buf;
  dec_old.assign(dec.size(), Res{});
  std::vector<uint64_t> dec_oldp(dec.size() * (size_t)S.PW);
  std::vector<LastEval> last(S.n_jobs);
  Engine E = first ? S.init : live_engine(S);
  Replayer rp(S, E);
  // rank 0's commits into this rank's mirror and decision log on a thread of
  // its own (in commit order), so the main thread is back at the next
  // message while they are applied; the engine replays them on another
  Logger lg(
      [&](const LogItem& it) {
        last[S.task_job[it.t]] = LastEval{it.t, (int32_t)dec.size(), it.node, it.ok ? it.kind : 0};
        if (!it.ok) return;
        dec_old.push_back(it.kind == KBG_KIND_ALLOCATE ? S.idle[it.node] : S.rel[it.node]);
        if (S.has_ports)
          dec_oldp.insert(dec_oldp.end(), S.node_ports.begin() + (size_t)it.node * S.PW,
                          S.node_ports.begin() + (size_t)(it.node + 1) * S.PW);
        const bool dup = mirror_add(S, it.t, it.node, it.kind);
        record_decision(S, it.t, it.node, it.kind, dup);
      },
      sched_getcpu());
  auto stop = [&]() {
    lg.join();
    rp.join();
  };
  std::vector<uint32_t> msg;
  kbg_status result = KBG_OK;
  int64_t evals = 0;
  for (;;) {
    if (kbg_status st = link.recv(S, msg); st != KBG_OK) {
      stop();
      return st;
    }
    const uint32_t kind = msg[0];
    size_t at = kSvcHead;
    const size_t args_w = msg[5], shapes_w = msg[6], rows_w = msg[7];
    const size_t nn = msg[2], nm = msg[3], no = msg[4];
    const size_t need = kSvcHead + args_w + shapes_w + rows_w + nn * kSvcNodeWords + nm * kSvcMaskWords + 2 * no;
    if (kind > kSvcState || need != msg.size() || (kind == kSvcLaunch && args_w * 4 < sizeof(kbg::FirstFitArgs))) {
      stop();
      comm_abort(S.comm);
      return fail(KBG_E_INVALID, "internal: malformed scan service message");
    }
    if (kind == kSvcAbort) {
      stop();
      return fail((kbg_status)msg[8], "the allocate failed on rank 0");
    }
    const uint32_t* args_p = msg.data() + at;
    at += args_w;
    const uint32_t* shapes_p = msg.data() + at;
    at += shapes_w;
    const uint32_t* rows_p = msg.data() + at;
    at += rows_w;
    const kbg::NodeDelta* nodes = reinterpret_cast<const kbg::NodeDelta*>(msg.data() + at);
    at += nn * kSvcNodeWords;
    const kbg::MaskDelta* masks = reinterpret_cast<const kbg::MaskDelta*>(msg.data() + at);
    at += nm * kSvcMaskWords;
    const uint32_t* outs = msg.data() + at;
    kbg_status st = svc_apply_state(S, nodes, nn, masks, nm);
    if (st == KBG_OK && kind == kSvcLaunch) {
      // this rank's part of the scan: rank 0's arguments, this rank's table, words and buffers
      thread_local kbg::FirstFitArgs a;
      std::memcpy(&a, args_p, sizeof(kbg::FirstFitArgs));
      const int32_t G = (int32_t)msg[9], ns = (int32_t)msg[10];
      char* up = S.stages[0].h_up;  // mapped staging (idle on this rank during the service)
      const size_t shapes_b = shapes_w ? ((size_t)ns * sizeof(kbg::TaskRec) + 15) & ~(size_t)15 : 0;
      if (G <= 0 || G > S.K || ns <= 0 || ns > G || shapes_b + rows_w * 4 > S.up_cap ||
          (shapes_w && shapes_w * 4 < (size_t)ns * sizeof(kbg::TaskRec)) || (rows_w && rows_w != (size_t)G) ||
          a.G != G || a.n_shapes != ns) {
        stop();
        comm_abort(S.comm);
        return fail(KBG_E_INVALID, "internal: malformed scan service launch");
      }
      if (shapes_w) std::memcpy(up, shapes_p, (size_t)ns * sizeof(kbg::TaskRec));
      if (rows_w) std::memcpy(up + shapes_b, rows_p, (size_t)G * 4);
      a.nodes = S.d_nodes.idle_cpu;
      a.stride = soa_stride(S);
      a.class_mask = S.d_class_mask;
      a.shapes = shapes_w ? dev_ptr(S, reinterpret_cast<const kbg::TaskRec*>(up)) : nullptr;
      a.row_shape = rows_w ? dev_ptr(S, reinterpret_cast<const uint32_t*>(up + shapes_b)) : nullptr;
      a.n_nodes = S.n_nodes;
      a.W = S.W;
      a.w_lo = std::min(S.W, S.shard * S.Wl);
      a.w_hi = std::min(S.W, (S.shard + 1) * S.Wl);
      a.tab_lo = S.tab_lo;
      a.tab_n = S.tab_n;
      a.splits = 1;
      a.split_words = a.w_hi - a.w_lo;
      a.info_stride = S.R;
      a.part0 = S.shard;
      a.mask_w0 = 0;
      a.mw = S.W;
      a.complete = a.w_hi - a.w_lo <= kbg::kFfRoundWords ? 1 : 0;
      a.avail = nullptr;
      a.info = S.d_svc;
      a.masks = reinterpret_cast<kbg::MaskPair*>(S.d_svc + fused_mask_off(S.K));
      const size_t info_w = (size_t)ns * S.R, mask_w = (size_t)ns * S.W * 4;
      if ((shapes_w && !a.shapes) || (rows_w && !a.row_shape)) {
        st = fail(KBG_E_HIP, "hipHostGetDevicePointer of a stage buffer failed");
      } else if (hipMemsetAsync(S.d_svc, 0, info_w * 4, S.stream) != hipSuccess ||
                 hipMemsetAsync(a.masks, 0, mask_w * 4, S.stream) != hipSuccess ||
                 kbg::launch_firstfit(a, S.int_mode ? 1 : 0, S.stream) != hipSuccess) {
        st = fail(KBG_E_HIP, "scan service launch failed");
      } else {
        st = link.sum(S, nullptr, info_w, mask_w);
        S.stats.scan_launches++;
      }
    }
    if (st != KBG_OK) {
      stop();
      comm_abort(S.comm);
      return st;
    }
    // rank 0's commits, in order: this rank's mirror and decision log (lg), engine (rp)
    std::vector<std::pair<int32_t, char>> v;
    std::vector<LogItem> items;
    v.reserve(no);
    items.reserve(no);
    for (size_t k = 0; k < no; ++k) {
      const int32_t t = (int32_t)outs[2 * k];
      const uint32_t w = outs[2 * k + 1];
      const bool ok = w != ~0u;
      const int32_t node = ok ? (int32_t)(w >> 1) : -1;
      const int32_t kd = ok && (w & 1u) ? KBG_KIND_PIPELINE : KBG_KIND_ALLOCATE;
      if (t < 0 || t >= S.n_tasks || node >= S.n_nodes) {
        stop();
        comm_abort(S.comm);
        return fail(KBG_E_INVALID, "internal: malformed scan service outcome");
      }
      items.push_back(LogItem{t, node, kd, ok, false, false, Res{}});
      v.emplace_back(t, (char)ok);
    }
    evals += (int64_t)no;
    if (!v.empty()) {
      lg.push(std::move(items));
      rp.push(std::move(v));
    }
    if (kind == kSvcEnd) {
      result = (kbg_status)msg[8];
      break;
    }
  }
  stop();
  if (!rp.error.empty()) return fail(KBG_E_INVALID, rp.error);
  if (kbg_status st = comm_sync(S); st != KBG_OK) return st;
  // the class-mask words this rank's mirror changed came from rank 0 already
  for (const uint32_t idx : S.mask_dirty) S.mask_dirty_flag[idx] = 0;
  S.mask_dirty.clear();
  if (result == KBG_OK || result == KBG_E_REF_PANIC) {  // as rank 0 (allocate_svc_root): the counts are summed
    SvcLink* const keep = S.svc;
    S.svc = &link;
    const kbg_status st = compute_fit_deltas(S, dec, dec_old, dec_oldp, last);
    S.svc = keep;
    if (st != KBG_OK) return st;
  }
  S.stats.task_evaluations += evals;
  S.fin = E;
  finalize_shares(S, S.fin);
  S.allocated = true;
  S.stats.allocate_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  if (result != KBG_OK) (void)fail(result, "the allocate on rank 0 ended with this status");
  return copy_log(S, out, cap, n_out, result);
}

// backfillAction.Execute (backfill.go:40-71). The order of the BestEffort
// tasks is fixed (ssn.Jobs, then each job's status index) and does not depend
// on outcomes, and a node only loses feasibility (its pod count grows), so
// the whole list is scanned in batches of K against the batch-start table and
// resolved in order exactly like allocate's rows, with no prediction.
kbg_status backfill_cycle(Session& S, kbg_decision* out, int32_t cap, int32_t* n_out) {
  using clk = std::chrono::steady_clock;
  if (S.backfilled || S.preempted)
    return fail(KBG_E_INVALID, "backfill runs once per cycle, before preempt; call kbg_session_reset");
  const auto t0 = clk::now();
  if (!S.cycle_started) begin_cycle(S);
  S.backfilled = true;
  S.action = KBG_ACTION_BACKFILL;
  std::vector<int32_t> be;
  for (int32_t j = 0; j < S.n_jobs; ++j)
    for (int32_t k = S.jt_off[j]; k < S.jt_off[j + 1]; ++k)
      if (S.be_task[S.jt[k]] && S.tstat[S.jt[k]] == KBG_PENDING) be.push_back(S.jt[k]);
  std::vector<int32_t> mark(S.n_nodes, -1), touched;
  Grouper grouper(S);
  Resolver rs{S, mark};
  kbg::Stage& sg = S.stages[0];
  int32_t pushed = S.res_stamp, rstamp = 0;
  kbg_status result = KBG_OK, st = KBG_OK;
  Engine& E = S.fin;
  // one synchronous scan of bt[0..n) against the table with every commit so far
  auto rescan = [&](const int32_t* b, int32_t n) -> kbg_status {
    kbg_status s2 = push_deltas(S, touched);
    if (s2 != KBG_OK) return s2;
    pushed = rstamp ? rstamp : pushed;
    touched.clear();
    const int32_t G = grouper.build(sg, b, n);
    if ((s2 = device_scan(S, sg, G, pushed)) != KBG_OK) return s2;
    rs.reset(sg);
    rstamp = ++S.res_stamp;
    S.mstamp = rstamp;
    return KBG_OK;
  };
  for (size_t done = 0; done < be.size() && result == KBG_OK;) {
    const int32_t cnt = (int32_t)std::min<size_t>(be.size() - done, (size_t)S.K);
    const int32_t* bt = be.data() + done;
    if ((st = rescan(bt, cnt)) != KBG_OK) return st;
    int32_t seg = 0;
    for (int32_t i = 0; i < cnt; ++i) {
      const int32_t t = bt[i];
      int32_t node = -1, kind = 0;
      int r = rs.resolve(sg.row_of[i - seg], t, &node, &kind);
      if (r == RES_TRUNC) {  // list exhausted: write back, rescan the rest of the batch
        S.stats.truncations++;
        if ((st = rescan(bt + i, cnt - i)) != KBG_OK) return st;
        seg = i;
        r = rs.resolve(sg.row_of[0], t, &node, &kind);
      }
      if (r == RES_PANIC) {
        result = fail(KBG_E_REF_PANIC, "backfill reached a node whose NodeInfo.Node is nil with the predicates plugin on "
                                       "(predicates.go:122-123)");
        break;
      }
      if (node < 0) continue;  // no node passes the predicates: the task stays Pending
      // ssn.Allocate -> NodeInfo.AddTask -> Idle.Sub panics when even the
      // tolerance does not cover the request (resource_info.go:100-110),
      // unless AddTask already failed on the pod key (node_info.go:101-106)
      if (!S.nil_node[node] && !node_has_key(S, t, node) && !kbg::res_le(S.treq[t], S.idle[node])) {
        result = fail(KBG_E_REF_PANIC, "backfill: Resource.Sub underflow on the node's Idle (resource_info.go:100-110)");
        break;
      }
      const bool dup = mirror_add(S, t, node, KBG_KIND_ALLOCATE);
      if (mark[node] != rstamp) {
        mark[node] = rstamp;
        touched.push_back(node);
      }
      // drf / proportion AllocateFunc (drf.go:130-139, proportion.go:196-206)
      const int32_t j = S.task_job[t];
      const Res& q = S.treq[t];
      if (S.has_drf) {
        kbg::res_add(E.jalloc[j], q);
        E.jshare[j] = share_of(E.jalloc[j], S.drf_total);
      }
      if (S.has_prop) {
        const int32_t jq = S.job_queue[j];
        kbg::res_add(E.qalloc[jq], q);
        E.qshare[jq] = share_of(E.qalloc[jq], S.q_deserved[jq]);
      }
      E.jready[j]++;
      record_decision(S, t, node, KBG_KIND_ALLOCATE, dup);
      if (!S.aff_gain_classes.empty() && i + 1 < cnt) {
        // pod affinity gave a class new nodes: rescan the rest of the batch
        for (int32_t c : S.aff_gain_classes) S.aff_gain_flag[c] = 0;
        S.aff_gain_classes.clear();
        if ((st = rescan(bt + i + 1, cnt - i - 1)) != KBG_OK) return st;
        seg = i + 1;
      }
    }
    if ((st = push_deltas(S, touched)) != KBG_OK) return st;
    touched.clear();
    pushed = rstamp;
    done += cnt;
  }
  HIP_TRY(hipStreamSynchronize(S.stream));
  S.stats.backfill_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  return copy_log(S, out, cap, n_out, result);
}

// ====================================================== preempt / reclaim
// preempt.go:43-253, reclaim.go:41-188, statement.go:35-217, session.go:318-352.
// The node loop of every reclaimer / preemptor runs on the device (one
// victim-scan launch over all nodes); the host replays the reference's
// control flow and, on the node the device names, its exact victim
// selection, eviction loop and pipeline.

void vt_delta(Session& S, int32_t kind, int32_t index, double a, double b, double c) {
  S.sdeltas.push_back(kbg::StateDelta{kind, index, {a, b, c}});
  if (!S.vt_sh_valid) return;
  switch (kind) {  // the device holds it from the next push on
    case 0: S.vt_sh_run[index] = a != 0.0; break;
    case 1: S.vt_sh_ready[index] = (int32_t)a; break;
    case 2:
    case 3: {
      double* v = (kind == 2 ? S.vt_sh_jalloc : S.vt_sh_qalloc).data() + 3 * (size_t)index;
      v[0] = a;
      v[1] = b;
      v[2] = c;
      break;
    }
  }
}

// Applies the queued state changes. Each carries the entry's new value, so
// only the last one of an entry is kept (the apply kernel writes in parallel).
// Node rows and victim-table entries changed by the host since the last
// scan, in one launch that reads them in place from host-mapped staging. The
// staging buffers are rewritten only once the previous launch has retired
// (the victim scan's synchronize, or an explicit one here).
kbg_status victim_push(Session& S, const std::vector<int32_t>& touched) {
  if (!S.mask_dirty.empty()) {  // class-mask words (ports / affinity) changed since the last scan
    if (S.vstage_busy) HIP_TRY(hipStreamSynchronize(S.stream));
    kbg_status st = push_mask_deltas(S);
    if (st != KBG_OK) return st;
  }
  if (!S.sdeltas.empty()) {  // last write of each entry wins: one stamp per (kind, index), no hashing
    const size_t sizes[4] = {std::max<size_t>(1, S.nt_task.size()), (size_t)std::max(1, S.n_jobs),
                             (size_t)std::max(1, S.n_jobs), (size_t)std::max(1, S.n_queues)};
    for (int k = 0; k < 4; ++k)
      if (S.sd_seen[k].size() < sizes[k]) S.sd_seen[k].assign(sizes[k], 0);
    if (++S.sd_gen == 0) {  // wrapped: clear the stamps
      for (auto& v : S.sd_seen) std::fill(v.begin(), v.end(), 0u);
      S.sd_gen = 1;
    }
    thread_local std::vector<kbg::StateDelta> uniq;
    uniq.clear();
    for (size_t i = S.sdeltas.size(); i-- > 0;) {
      const kbg::StateDelta& d = S.sdeltas[i];
      uint32_t& seen = S.sd_seen[d.kind][d.index];
      if (seen == S.sd_gen) continue;
      seen = S.sd_gen;
      uniq.push_back(d);
    }
    S.sdeltas.swap(uniq);
  }
  {  // few changes: in the kernel arguments
    int32_t nn = 0;
    for (int32_t n : touched) nn += n >= S.tab_lo && n < S.tab_lo + S.tab_n;
    if (nn <= kbg::kArgNodeDeltas && S.sdeltas.size() <= (size_t)kbg::kArgStateDeltas) {
      kbg::VictimPrepArgs a;
      a.nn = 0;
      for (int32_t n : touched) {
        if (n < S.tab_lo || n >= S.tab_lo + S.tab_n) continue;
        kbg::NodeDelta& d = a.nd[a.nn++];
        d.node = n - S.tab_lo;
        device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
      }
      a.ns = (int32_t)S.sdeltas.size();
      if (a.ns) std::memcpy(a.sd, S.sdeltas.data(), (size_t)a.ns * sizeof(kbg::StateDelta));
      S.sdeltas.clear();
      HIP_TRY(kbg::launch_victim_prep_inline(S.d_nodes, S.vt, a, S.stream));
      return KBG_OK;
    }
  }
  size_t ti = 0, si = 0;
  while (ti < touched.size() || si < S.sdeltas.size()) {
    if (S.vstage_busy) HIP_TRY(hipStreamSynchronize(S.stream));
    S.vstage_busy = false;
    if (kbg_status st = stage_acquire(S); st != KBG_OK) return st;
    int32_t nn = 0;
    for (; ti < touched.size() && nn < S.K; ++ti) {
      const int32_t n = touched[ti];
      if (n < S.tab_lo || n >= S.tab_lo + S.tab_n) continue;  // another rank's row
      kbg::NodeDelta& d = S.h_deltas[nn++];
      d.node = n - S.tab_lo;
      device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
    }
    const int32_t ns = (int32_t)std::min<size_t>(S.sdeltas.size() - si, (size_t)kbg::kMaskDeltaCap);
    if (ns > 0) std::memcpy(S.h_sdeltas, S.sdeltas.data() + si, (size_t)ns * sizeof(kbg::StateDelta));
    si += ns;
    if (nn + ns == 0) break;
    HIP_TRY(kbg::launch_victim_prep(S.d_nodes, S.vt, S.h_deltas_dev, nn, S.h_sdeltas_dev, ns, S.stream));
    S.vstage_busy = true;
    if (kbg_status st = stage_release(S); st != KBG_OK) return st;
  }
  S.sdeltas.clear();
  return KBG_OK;
}

// Device copies of the victim tables; the live parts (running flags, gang
// readiness, drf / proportion allocations) follow the host at every action.
kbg_status vt_setup(Session& S) {
  const size_t J = (size_t)std::max(1, S.n_jobs),
               Q = (size_t)std::max(1, S.n_queues);
  kbg_status st;
  if (S.vt_ready && S.vt_stale) {  // a session update changed the tasks behind them
    for (void* p : S.vt_allocs) {
      (void)hipFree(p);
      S.d_allocs.erase(std::find(S.d_allocs.begin(), S.d_allocs.end(), p));
    }
    S.vt_allocs.clear();
    S.vt_ready = false;
  }
  S.vt_stale = false;
  if (!S.vt_ready) {
    const size_t a0 = S.d_allocs.size();
    S.vt_sh_valid = false;  // new device tables: the live state goes up whole
    S.W32 = kbg::kbg_victim_words(S.n_nodes);
    kbg::VictimTables& v = S.vt;
    v.ntasks = S.d_nodes.ntasks;
    v.maxtasks = S.d_nodes.maxtasks;
    v.class_mask = S.d_class_mask;
    std::vector<uint8_t> pn(S.panic_node.begin(), S.panic_node.end());
    std::vector<int32_t> jq(S.job_queue), jm(S.n_jobs);
    for (int32_t j = 0; j < S.n_jobs; ++j) jm[j] = S.jobs_in[j].min_available;
    // candidate records in node-list order (position p = nt_off[n] + k)
    const size_t P = std::max<size_t>(1, S.nt_task.size());
    std::vector<double> cr(3 * P, 0.0), qd(3 * Q, 0.0);
    std::vector<int32_t> cjq(2 * P, 0);
    S.t_pos.assign(S.n_tasks, -1);
    for (size_t k = 0; k < S.nt_task.size(); ++k) {
      const int32_t t = S.nt_task[k];
      S.t_pos[t] = (int32_t)k;
      cjq[2 * k] = S.task_job[t];
      cjq[2 * k + 1] = S.job_queue[S.task_job[t]];
      cr[3 * k] = S.treq[t].c;
      cr[3 * k + 1] = S.treq[t].m;
      cr[3 * k + 2] = S.treq[t].g;
    }
    for (int32_t q = 0; q < S.n_queues; ++q) {
      qd[3 * q] = S.q_deserved[q].c;
      qd[3 * q + 1] = S.q_deserved[q].m;
      qd[3 * q + 2] = S.q_deserved[q].g;
    }
    uint8_t *dpn, *drun;
    int32_t *doff, *dcjq, *djq, *djm, *djr;
    double *dcr, *dja, *dqa, *dqd;
    // the live state (running flags, gang readiness, drf / proportion
    // allocations) goes up whole with the tables, as vt_sh_* records it
    const size_t Pn = S.nt_task.size();
    S.vt_sh_valid = true;
    S.vt_sh_run.resize(Pn);
    S.vt_sh_ready = S.committed_ready;
    S.vt_sh_jalloc.assign(3 * J, 0.0);
    S.vt_sh_qalloc.assign(3 * Q, 0.0);
    for (size_t k = 0; k < Pn; ++k) S.vt_sh_run[k] = S.trun[S.nt_task[k]];
    for (int32_t j = 0; j < S.n_jobs; ++j) std::memcpy(&S.vt_sh_jalloc[3 * (size_t)j], &S.fin.jalloc[j].c, 24);
    for (int32_t q = 0; q < S.n_queues; ++q) std::memcpy(&S.vt_sh_qalloc[3 * (size_t)q], &S.fin.qalloc[q].c, 24);
    S.sdeltas.clear();
    std::vector<int32_t> ready0(J, 0);
    std::copy(S.committed_ready.begin(), S.committed_ready.end(), ready0.begin());
    BulkUpload bu;  // every table (and the live state) in one block, one copy
    bu.add(&dpn, pn);
    bu.add(&doff, S.nt_off);
    bu.add(&dcjq, cjq);
    bu.add(&dcr, cr);
    bu.add(&drun, S.vt_sh_run);
    bu.add(&djq, jq);
    bu.add(&djm, jm);
    bu.add(&djr, ready0);
    bu.add(&dja, S.vt_sh_jalloc);
    bu.add(&dqa, S.vt_sh_qalloc);
    bu.add(&dqd, qd);
    bu.zeros(&S.d_vbits, 2 * (size_t)S.W32);  // other ranks' words stay 0
    bu.zeros(&S.d_vbits_red, 2 * (size_t)S.W32);
    // nodes of this process's range holding more than 128 candidates
    // (kbg_victim_big_kernel, up to kMaxNodeCandidates); every node holding
    // more is left out of the device scans and re-evaluated on the host when
    // a stop search reaches it (try_task marks it unknown after each scan)
    S.big_rows.clear();
    S.huge_nodes.clear();
    for (int32_t n = 0; n < S.n_nodes; ++n) {
      const int32_t L = S.nt_off[n + 1] - S.nt_off[n];
      if (L > kbg::kMaxNodeCandidates) S.huge_nodes.push_back(n);
      else if (L > 128 && n >= S.tab_lo && n < S.tab_lo + S.tab_n) S.big_rows.push_back(n - S.tab_lo);
    }
    bu.add(&S.d_big_rows, S.big_rows);
    if ((st = bu.commit(S))) return st;
    S.vt_allocs.assign(S.d_allocs.begin() + a0, S.d_allocs.end());
    if (!S.h_vbits) {
      const size_t vb = std::max<size_t>(2 * (size_t)S.W32 * sizeof(uint32_t), 64);  // W32 = 0: no nodes
      HIP_TRY(hipHostMalloc((void**)&S.h_vbits, vb, hipHostMallocCoherent | hipHostMallocMapped));
      HIP_TRY(hipHostGetDevicePointer((void**)&S.h_vbits_dev, S.h_vbits, 0));
      std::memset(S.h_vbits, 0, vb);  // the scan writes the bytes of its node blocks; the rest stays 0
    }
    if (S.h_vbig_cap < std::max<size_t>(1, S.big_rows.size())) {
      if (S.h_vbig) (void)hipHostFree(S.h_vbig);
      S.h_vbig = nullptr;
      S.h_vbig_cap = std::max<size_t>(64, S.big_rows.size());
      HIP_TRY(hipHostMalloc((void**)&S.h_vbig, S.h_vbig_cap, hipHostMallocCoherent | hipHostMallocMapped));
      HIP_TRY(hipHostGetDevicePointer((void**)&S.h_vbig_dev, S.h_vbig, 0));
    }
    // per job, the nodes holding its tasks Running at open (the only tasks a
    // victim fn can see; their job's readiness / allocation feed the fns)
    std::vector<std::vector<int32_t>> jn(S.n_jobs);
    for (int32_t n = 0; n < S.n_nodes; ++n)
      for (int32_t k = S.nt_off[n]; k < S.nt_off[n + 1]; ++k) {
        std::vector<int32_t>& l = jn[S.task_job[S.nt_task[k]]];
        if (l.empty() || l.back() != n) l.push_back(n);
      }
    S.jn_off.assign(S.n_jobs + 1, 0);
    S.jn_node.clear();
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      S.jn_node.insert(S.jn_node.end(), jn[j].begin(), jn[j].end());
      S.jn_off[j + 1] = (int32_t)S.jn_node.size();
    }
    S.vc.stop.assign(S.W32, 0u);
    S.vc.panic.assign(S.W32, 0u);
    S.vc.unk.assign(S.W32, 0u);

    if (!S.h_sdeltas) {
      HIP_TRY(hipHostMalloc((void**)&S.h_sdeltas, (size_t)kbg::kMaskDeltaCap * sizeof(kbg::StateDelta),
                            hipHostMallocMapped));
      HIP_TRY(hipHostGetDevicePointer((void**)&S.h_sdeltas_dev, S.h_sdeltas, 0));
    }
    v.panic_node = dpn;
    v.nt_off = doff;
    v.c_jq = reinterpret_cast<const int2*>(dcjq);
    v.c_req = dcr;
    v.c_run = drun;
    v.j_queue = djq;
    v.j_min = djm;
    v.j_ready = djr;
    v.j_alloc = dja;
    v.q_alloc = dqa;
    v.q_deserved = dqd;
    v.drf_total[0] = S.drf_total.c;
    v.drf_total[1] = S.drf_total.m;
    v.drf_total[2] = S.drf_total.g;
    S.vt_ready = true;
    HIP_TRY(hipStreamSynchronize(S.stream));  // host vectors end here
  }
  // live state: the first setup of the tables uploads it whole; later ones
  // queue the entries that differ from what the device holds (vt_sh_*), which
  // the first scan's prep launch applies (no copy, no synchronize here)
  const size_t P = S.nt_task.size();
  auto same3 = [](const double* a, const Res& r) {
    return std::memcmp(a, &r.c, 8) == 0 && std::memcmp(a + 1, &r.m, 8) == 0 && std::memcmp(a + 2, &r.g, 8) == 0;
  };
  if (!S.vt_sh_valid || S.vt_sh_run.size() != P || S.vt_sh_ready.size() != (size_t)S.n_jobs ||
      S.vt_sh_qalloc.size() != 3 * (size_t)S.n_queues) {
    S.vt_sh_valid = true;
    S.vt_sh_run.resize(P);
    S.vt_sh_ready = S.committed_ready;
    S.vt_sh_jalloc.assign(3 * J, 0.0);
    S.vt_sh_qalloc.assign(3 * Q, 0.0);
    for (size_t k = 0; k < P; ++k) S.vt_sh_run[k] = S.trun[S.nt_task[k]];
    for (int32_t j = 0; j < S.n_jobs; ++j) std::memcpy(&S.vt_sh_jalloc[3 * (size_t)j], &S.fin.jalloc[j].c, 24);
    for (int32_t q = 0; q < S.n_queues; ++q) std::memcpy(&S.vt_sh_qalloc[3 * (size_t)q], &S.fin.qalloc[q].c, 24);
    if (P > 0) HIP_TRY(hipMemcpyAsync(S.vt.c_run, S.vt_sh_run.data(), P, hipMemcpyHostToDevice, S.stream));
    if (S.n_jobs > 0)
      HIP_TRY(hipMemcpyAsync(S.vt.j_ready, S.vt_sh_ready.data(), (size_t)S.n_jobs * 4, hipMemcpyHostToDevice,
                             S.stream));
    HIP_TRY(hipMemcpyAsync(S.vt.j_alloc, S.vt_sh_jalloc.data(), S.vt_sh_jalloc.size() * 8, hipMemcpyHostToDevice,
                           S.stream));
    HIP_TRY(hipMemcpyAsync(S.vt.q_alloc, S.vt_sh_qalloc.data(), S.vt_sh_qalloc.size() * 8, hipMemcpyHostToDevice,
                           S.stream));
    HIP_TRY(hipStreamSynchronize(S.stream));
    S.sdeltas.clear();
  } else {
    for (size_t k = 0; k < P; ++k)
      if (S.vt_sh_run[k] != S.trun[S.nt_task[k]]) vt_delta(S, 0, (int32_t)k, S.trun[S.nt_task[k]] ? 1.0 : 0.0, 0, 0);
    for (int32_t j = 0; j < S.n_jobs; ++j) {
      if (S.vt_sh_ready[j] != S.committed_ready[j]) vt_delta(S, 1, j, (double)S.committed_ready[j], 0, 0);
      const Res& a = S.fin.jalloc[j];
      if (!same3(&S.vt_sh_jalloc[3 * (size_t)j], a)) vt_delta(S, 2, j, a.c, a.m, a.g);
    }
    for (int32_t q = 0; q < S.n_queues; ++q) {
      const Res& a = S.fin.qalloc[q];
      if (!same3(&S.vt_sh_qalloc[3 * (size_t)q], a)) vt_delta(S, 3, q, a.c, a.m, a.g);
    }
  }
  S.fin.jready = S.committed_ready;  // the job order keys read the live readiness
  return KBG_OK;
}

// ---- victim-scan stop maps kept current on the host (Session::VictimCache).
// A node's stop status for a preemptor depends on the node (static predicate,
// pod count, its Running tasks) and, through the victim fns, on the gang
// readiness and drf allocation of the jobs of those tasks and on the
// proportion allocation of their queues. Every change marks what it can
// affect unknown; a queue allocation change under a proportion fn affects
// every node and drops the maps.
void vc_dirty_node(Session& S, int32_t n) {
  if (S.vc.valid && n >= 0) S.vc.dirty(n);
}
void vc_dirty_job(Session& S, int32_t j) {
  if (!S.vc.valid) return;
  for (int32_t k = S.jn_off[j]; k < S.jn_off[j + 1]; ++k) vc_dirty_node(S, S.jn_node[k]);
}

// The plugin and gang state an event changes (drf.go:130-148,
// proportion.go:196-216, gang readiness), mirrored to the victim tables.
struct Live {
  Session& S;
  std::vector<int32_t>& touched;
  std::vector<int32_t>& mark;
  int32_t stamp;
  void touch(int32_t n) {
    vc_dirty_node(S, n);
    if (n >= 0 && mark[n] != stamp) {
      mark[n] = stamp;
      touched.push_back(n);
    }
  }
  void ready(int32_t j, int32_t d) {
    // the victim scan reads a job's readiness only through the gang fn's
    // `MinAvailable <= ready - 1` (gang.go:104-124): its nodes change only
    // when that test flips
    const int32_t ma = S.jobs_in[j].min_available, r0 = S.committed_ready[j];
    if ((S.vc.fns & kbg::VP_GANG) && ((ma <= r0 - 1) != (ma <= r0 + d - 1))) vc_dirty_job(S, j);
    S.committed_ready[j] += d;
    S.fin.jready[j] = S.committed_ready[j];
    vt_delta(S, 1, j, (double)S.committed_ready[j], 0, 0);
  }
  // AllocateFunc (+) / DeallocateFunc (-); false when Sub would panic
  bool plugins(int32_t t, bool add) {
    const int32_t j = S.task_job[t];
    const Res& r = S.treq[t];
    if (S.has_drf) {
      Res& a = S.fin.jalloc[j];
      if (add) kbg::res_add(a, r);
      else if (!kbg::res_sub(a, r)) return false;
      S.fin.jshare[j] = share_of(a, S.drf_total);
      vt_delta(S, 2, j, a.c, a.m, a.g);
      if (S.vc.fns & kbg::VP_DRF) vc_dirty_job(S, j);
    }
    if (S.has_prop) {
      if (S.vc.fns & kbg::VP_PROP) S.vc.valid = false;
      const int32_t q = S.job_queue[j];
      Res& a = S.fin.qalloc[q];
      if (add) kbg::res_add(a, r);
      else if (!kbg::res_sub(a, r)) return false;
      S.fin.qshare[q] = share_of(a, S.q_deserved[q]);
      vt_delta(S, 3, q, a.c, a.m, a.g);
    }
    return true;
  }
  // An AllocatedStatus pod enters (+1) or leaves (-1) the predicates'
  // podLister (api/helpers.go:63-70): the pod affinity counts and the class
  // masks follow (kbg_affinity.cpp); allocate's batch-cut bookkeeping is not
  // used by the victim actions.
  void lister(int32_t v, int32_t sign) {
    if (!S.has_aff) return;
    kbg::aff_place(S, v, S.task_node[v], sign, S.affm->st, true);
    for (int32_t c : S.aff_gain_classes) S.aff_gain_flag[c] = 0;
    S.aff_gain_classes.clear();
  }
  // job Releasing, NodeInfo.UpdateTask (Running copy out, Releasing copy
  // in), DeallocateFunc (session.go:323-349, statement.go:36-59)
  bool evict(int32_t v) {
    const int32_t j = S.task_job[v];
    if (ready_status(S.tstat[v])) ready(j, -1);
    if (allocated_status(S.tstat[v])) lister(v, -1);
    S.tstat[v] = KBG_RELEASING;
    const int32_t n = S.task_node[v];
    if (n >= 0) {
      if (!S.nil_node[n]) {
        const Res& r = S.treq[v];
        kbg::res_add(S.idle[n], r);                    // RemoveTask (node_info.go:148)
        kbg::res_add(S.rel[n], r);                     // AddTask as Releasing (:115-116)
        if (!kbg::res_sub(S.idle[n], r)) return false;
      }
      touch(n);
    }
    S.trun[v] = 0;
    if (S.t_pos[v] >= 0) vt_delta(S, 0, S.t_pos[v], 0, 0, 0);
    return plugins(v, false);
  }
  // job Pipelined, NodeInfo.AddTask as Pipelined, AllocateFunc (session.go:205-241, statement.go:110-151)
  // *dup: the node already held the pod key (node_info.go:101-106): unchanged
  bool pipeline(int32_t t, int32_t n, bool* dup) {
    const int32_t j = S.task_job[t];
    if (!ready_status(S.tstat[t])) ready(j, +1);
    S.tstat[t] = KBG_PIPELINED;
    *dup = node_has_key(S, t, n);
    if (!*dup) {
      if (!S.nil_node[n] && !kbg::res_sub(S.rel[n], S.treq[t])) return false;  // node_info.go:117-118
      S.ntasks[n]++;
      if (S.has_dupkeys && S.key_hot[S.task_key[t]]) {
        S.node_keys.insert(node_key_of(S, t, n));
        S.key_holder[node_key_of(S, t, n)] = t << 1 | 1;
      }
      if (S.has_ports) add_ports(S, S.task_class[t], n);  // the pod joins node.Pods()
      touch(n);
    }
    return plugins(t, true);
  }
  // statement.go:81-108: job Running again; node.AddTask fails (the task is
  // still there, as Releasing), so the node is unchanged; AllocateFunc. A
  // task whose copy a discard's RemoveTask took off the node (unpipeline_dup)
  // is added back as Running, unless another pod holds its key there now.
  // false: AddTask's Idle.Sub would panic.
  bool unevict(int32_t v) {
    const int32_t j = S.task_job[v];
    S.tstat[v] = KBG_RUNNING;
    lister(v, +1);
    ready(j, +1);
    const int32_t n = S.task_node[v];
    if (!S.t_detached.empty() && S.t_detached[v] && n >= 0 && !node_has_key(S, v, n)) {
      if (!S.nil_node[n] && !kbg::res_sub(S.idle[n], S.treq[v])) return false;  // node_info.go:123-124
      S.ntasks[n]++;
      S.node_keys.insert(node_key_of(S, v, n));
      S.key_holder[node_key_of(S, v, n)] = v << 1;
      S.trun[v] = 1;
      if (S.t_pos[v] >= 0) vt_delta(S, 0, S.t_pos[v], 1.0, 0, 0);
      S.t_detached[v] = 0;
      if (S.has_aff) {  // back among n's pods: n's predicate counts it again
        const auto fi = std::find(S.aff_filtered.begin(), S.aff_filtered.end(), std::make_pair(n, v));
        if (fi != S.aff_filtered.end()) {
          S.aff_filtered.erase(fi);
          kbg::aff_refresh_node(S, n);
        }
      }
      // back in node.Pods(): its host ports are used again (release_open_ports' reverse)
      const int32_t vs = S.tasks_in[v].spec;
      if (vs >= 0 && S.specs_in[vs].port_len > 0)
        restore_open_ports(S, n, &S.ports_in[S.specs_in[vs].port_off], S.specs_in[vs].port_len);
      touch(n);
    }
    plugins(v, true);
    return true;
  }
  // unpipeline of a pipeline whose AddTask found its pod key already on the
  // node (statement.go:156-192): NodeInfo.RemoveTask removes by key, so the
  // pod that held the key leaves the node (node_info.go:131-157), by the
  // status of its node copy: Releasing (Releasing -= req, Idle += req),
  // Pipelined (Releasing += req), anything else (Idle += req), and its host
  // ports leave node.Pods(). The holder is a session task on the node at open
  // (Running then — Releasing if evicted since — or any other status it kept),
  // a task placed this cycle (two Pending pods sharing a key: its copy is
  // Allocated or Pipelined, S.key_holder) or a pod outside the session jobs
  // (its copy from kbg_node_pod).
  kbg_status unpipeline_dup(int32_t t, int32_t n) {
    const int32_t j = S.task_job[t];
    ready(j, -1);
    S.tstat[t] = KBG_PENDING;
    if (node_has_key(S, t, n)) {
      const int64_t hk = node_key_of(S, t, n);
      int32_t h = -1;
      bool placed = false, placed_pipe = false;  // the holder took the key this cycle (its copy: Allocated / Pipelined)
      if (auto kh = S.key_holder.find(hk); kh != S.key_holder.end()) {
        h = kh->second >> 1;
        placed = S.tstat_in[h] == KBG_PENDING;
        placed_pipe = placed && (kh->second & 1);
      }
      for (int32_t k = S.nt_off[n]; k < S.nt_off[n + 1] && h < 0; ++k) {
        const int32_t u = S.nt_task[k];
        if (u != t && S.task_key[u] == S.task_key[t] && !S.t_detached[u]) h = u;
      }
      if (h < 0)  // a session task on the node at open in another status (it keeps it all cycle)
        for (int32_t u : S.node_task_order[n])
          if (u != t && S.task_key[u] == S.task_key[t] && S.tstat_in[u] != KBG_RUNNING && !S.t_detached[u]) {
            h = u;
            break;
          }
      const Session::Outsider* o = nullptr;
      if (h < 0) {
        auto oit = S.outsiders.find(hk);
        if (oit != S.outsiders.end() && oit->second.status != 0 && !S.outsider_gone.count(hk)) o = &oit->second;
      }
      if (h < 0 && !o)
        return fail(KBG_E_UNSUPPORTED, "statement discard of a pipeline whose pod key is held on the node by a pod "
                                       "outside the session jobs with no node_pods entry (node_info.go:131-157 "
                                       "removes it, its resources are unknown): supply node_pods");
      Res r;
      int32_t status;
      if (h >= 0) {
        r = S.treq[h];
        if (placed) status = placed_pipe ? KBG_PIPELINED : KBG_ALLOCATED;
        else status = S.tstat_in[h] != KBG_RUNNING ? S.tstat_in[h] : S.trun[h] ? KBG_RUNNING : KBG_RELEASING;
      } else {
        r = to_res(o->req);
        status = o->status;
      }
      if (!S.nil_node[n]) {
        if (status == KBG_RELEASING) {
          if (!kbg::res_sub(S.rel[n], r))
            return fail(KBG_E_REF_PANIC, "statement discard: RemoveTask Releasing.Sub underflow (node_info.go:143)");
          kbg::res_add(S.idle[n], r);
        } else if (status == KBG_PIPELINED) {
          kbg::res_add(S.rel[n], r);
        } else {
          kbg::res_add(S.idle[n], r);
        }
      }
      S.ntasks[n]--;
      S.node_keys.erase(hk);
      S.key_holder.erase(hk);
      if (h >= 0) {
        const int32_t hs = S.tasks_in[h].spec;
        if (placed) {  // its ports joined with its placement (add_ports)
          if (S.has_ports) remove_ports(S, S.task_class[h], n);
        } else if (hs >= 0 && S.specs_in[hs].port_len > 0) {
          release_open_ports(S, n, &S.ports_in[S.specs_in[hs].port_off], S.specs_in[hs].port_len);
        }
        if (S.trun[h]) {
          S.trun[h] = 0;  // no longer in node.Tasks: not a victim candidate
          if (S.t_pos[h] >= 0) vt_delta(S, 0, S.t_pos[h], 0, 0, 0);
        }
        S.t_detached[h] = 1;
        // the podLister Filter now leaves it out of n's predicate — unless it
        // was placed this cycle (its informer Spec.NodeName is "", kept)
        if (S.has_aff && !placed && allocated_status(S.tstat[h])) {
          S.aff_filtered.emplace_back(n, h);
          kbg::aff_refresh_node(S, n);
        }
      } else {
        if (!o->ports.empty()) release_open_ports(S, n, o->ports.data(), (int32_t)o->ports.size());
        S.outsider_gone.insert(hk);
      }
      touch(n);
    }
    if (!plugins(t, false))
      return fail(KBG_E_REF_PANIC, "statement discard: DeallocateFunc Sub underflow (resource_info.go:100-110)");
    return KBG_OK;
  }
  // statement.go:156-192: job Pending; node.RemoveTask; DeallocateFunc. A
  // task whose copy an earlier RemoveTask by key took off the node (a later
  // pipeline of the same statement that shared its key was discarded first):
  // RemoveTask finds nothing, the node is unchanged.
  bool unpipeline(int32_t t, int32_t n) {
    const int32_t j = S.task_job[t];
    ready(j, -1);
    S.tstat[t] = KBG_PENDING;
    if (!S.t_detached.empty() && S.t_detached[t]) {
      S.t_detached[t] = 0;
      return plugins(t, false);
    }
    if (!S.nil_node[n]) kbg::res_add(S.rel[n], S.treq[t]);  // node_info.go:145-146
    S.ntasks[n]--;
    if (S.has_dupkeys && S.key_hot[S.task_key[t]]) {
      S.node_keys.erase(node_key_of(S, t, n));
      S.key_holder.erase(node_key_of(S, t, n));
    }
    if (S.has_ports) remove_ports(S, S.task_class[t], n);  // the pod leaves node.Pods()
    touch(n);
    return plugins(t, false);
  }
};

// Victims of `t` on node n, exactly as the reference builds them: the
// filtered Running tasks in NodeInfo.Tasks order, then the victim fns of the
// deciding tier (session_plugins.go:59-140). false = a fn would panic.
bool host_victims(Session& S, int32_t mode, int32_t t, int32_t n, std::vector<int32_t>* victims) {
  const int32_t pj = S.task_job[t], pq = S.job_queue[pj];
  thread_local std::vector<int32_t> pre;
  thread_local std::vector<char> keep;
  pre.clear();
  for (int32_t k = S.nt_off[n]; k < S.nt_off[n + 1]; ++k) {
    const int32_t v = S.nt_task[k];
    if (!S.trun[v]) continue;
    const int32_t jv = S.task_job[v];
    bool f;
    if (mode == kbg::VM_PREEMPT_JOBS) f = S.job_queue[jv] == pq && jv != pj;
    else if (mode == kbg::VM_PREEMPT_TASKS) f = jv == pj;
    else f = S.job_queue[jv] != pq;
    if (f) pre.push_back(v);
  }
  victims->clear();
  if (pre.empty()) return true;
  const std::vector<int32_t>& tiers = mode == kbg::VM_RECLAIM ? S.tier_reclaim : S.tier_preempt;
  for (int32_t fns : tiers) {
    keep.assign(pre.size(), 1);
    if (fns & kbg::VP_GANG)  // gang.go:104-124
      for (size_t i = 0; i < pre.size(); ++i) {
        const int32_t jv = S.task_job[pre[i]];
        if (!(S.jobs_in[jv].min_available <= S.committed_ready[jv] - 1)) keep[i] = 0;
      }
    // the per-job / per-queue running allocations of the fns' maps
    // (`allocations`, drf.go:86-100, proportion.go:163-183): a node holds a
    // few dozen preemptees of a few jobs, so a flat list searched linearly
    // replaces the hash map (no allocation per call)
    thread_local std::vector<std::pair<int32_t, Res>> alloc;
    auto entry = [&](int32_t id, const Res& init) -> Res& {
      for (auto& e : alloc)
        if (e.first == id) return e.second;
      alloc.emplace_back(id, init);
      return alloc.back().second;
    };
    if (fns & kbg::VP_DRF) {  // drf.go:80-105
      Res la = S.fin.jalloc[pj];
      kbg::res_add(la, S.treq[t]);
      const double ls = share_of(la, S.drf_total);
      alloc.clear();
      for (size_t i = 0; i < pre.size(); ++i) {
        const int32_t jv = S.task_job[pre[i]];
        Res& a = entry(jv, S.fin.jalloc[jv]);
        if (!kbg::res_sub(a, S.treq[pre[i]])) return false;
        const double rs = share_of(a, S.drf_total);
        if (!(ls < rs || std::fabs(ls - rs) <= 0.000001)) keep[i] = 0;
      }
    }
    if (fns & kbg::VP_PROP) {  // proportion.go:161-186
      alloc.clear();
      for (size_t i = 0; i < pre.size(); ++i) {
        const int32_t q = S.job_queue[S.task_job[pre[i]]];
        const Res& r = S.treq[pre[i]];
        Res& a = entry(q, S.fin.qalloc[q]);
        if (a.c < r.c && a.m < r.m && a.g < r.g) {  // Resource.Less: skipped
          keep[i] = 0;
          continue;
        }
        if (!kbg::res_sub(a, r)) return false;
        if (!kbg::res_le(S.q_deserved[q], a)) keep[i] = 0;
      }
    }
    for (size_t i = 0; i < pre.size(); ++i)
      if (keep[i]) victims->push_back(pre[i]);
    if (!victims->empty()) return true;
  }
  return true;
}

// host_victims plus the rest of the reference's per-node test, for node n
// against the current host state: 0 the scan moves on, 1 stop, 2 panic.
// `v` receives the victims (valid when the result is 1).
int host_stop(Session& S, int32_t mode, int32_t t, int32_t n, std::vector<int32_t>& v) {
  const int32_t cls = S.task_class[t];
  if (!((S.h_class_mask[(size_t)cls * S.W + (n >> 6)] >> (n & 63)) & 1ull)) return 0;  // static predicate
  if (S.panic_node[n]) return 2;                                                      // predicates.go:122-123
  if (S.pred_active && S.ntasks[n] >= S.maxtasks[n]) return 0;                        // :125-127
  if (!host_victims(S, mode, t, n, &v)) return 2;
  if (v.empty()) return 0;
  Res all{};
  for (int32_t x : v) kbg::res_add(all, S.treq[x]);  // validateVictims (preempt.go:242-253)
  const Res& req = S.treq[t];
  return (all.c < req.c && all.m < req.m && all.g < req.g) ? 0 : 1;
}

// One statement (statement.go); a null statement is the session itself
// (reclaim uses ssn.Evict / ssn.Pipeline directly).
struct Stmt {
  struct Op {
    bool evict;
    int32_t task, node, by;
    bool dup;  // a pipeline the node's pod key table refused (the node is unchanged)
  };
  std::vector<Op> ops;
};

enum { TRY_NONE = 0, TRY_ASSIGNED = 1 };

// Opt-in cycle counters of the victim actions' host side (KBG_PROFILE_VICTIM=1):
// device scans, the stop search (with host re-evaluations), victim selection
// at the chosen node, evictions + pipeline, the action's own loop
struct VictimProfile {
  bool on = getenv("KBG_PROFILE_VICTIM") != nullptr;
  uint64_t scan = 0, walk = 0, select = 0, apply = 0, tries = 0, setup = 0, flush = 0;
  void print(const char* action, double ms) {
    if (!on || !tries) return;
    fprintf(stderr,
            "[kbg victim] %s %.3f ms, %llu tries, cycles/try: scan %.0f walk %.0f select %.0f apply %.0f; "
            "setup %.0f kcyc, flush %.0f kcyc\n",
            action, ms, (unsigned long long)tries, (double)scan / tries, (double)walk / tries, (double)select / tries,
            (double)apply / tries, setup / 1e3, flush / 1e3);
    scan = walk = select = apply = tries = setup = flush = 0;
  }
};
VictimProfile& vprof() {
  static VictimProfile p;
  return p;
}

// preempt.go:174-240 / reclaim.go:106-176 for one task: the device finds the
// first node where the reference stops; the host evicts there and pipelines.
kbg_status try_task(Session& S, Live& L, int32_t mode, int32_t t, Stmt* stmt, int32_t* outcome) {
  *outcome = TRY_NONE;
  kbg::VictimScan p{};
  p.n_nodes = S.n_nodes;
  p.node_lo = S.tab_lo;  // a node-axis shard scans its own nodes; the lowest stop is min-reduced over ranks
  p.node_n = S.tab_n;
  p.W = S.W;
  p.cls = S.task_class[t];
  p.cap_check = S.pred_active ? 1 : 0;
  p.mode = mode;
  const std::vector<int32_t>& tiers = mode == kbg::VM_RECLAIM ? S.tier_reclaim : S.tier_preempt;
  p.n_tiers = (int32_t)tiers.size();
  for (int32_t i = 0; i < p.n_tiers; ++i) p.tier_fns[i] = tiers[i];
  const int32_t pj = S.task_job[t];
  p.job = pj;
  p.queue = S.job_queue[pj];
  p.req[0] = S.treq[t].c;
  p.req[1] = S.treq[t].m;
  p.req[2] = S.treq[t].g;
  Res la = S.fin.jalloc[pj];
  kbg::res_add(la, S.treq[t]);
  p.ls = share_of(la, S.drf_total);
  S.stats.victim_tries++;
  const int32_t dfns = p.n_tiers ? p.tier_fns[0] : 0;
  // ls matters only to a drf fn in the deciding tier
  // the preemptor's job enters the preemptee filter only through its tasks
  // Running at open (reclaim filters by queue alone)
  const int32_t kjob = mode != kbg::VM_RECLAIM && S.jn_off[pj + 1] > S.jn_off[pj] ? pj : -1;
  const kbg::VictimKey key{mode, kjob, p.cls, p.queue, {p.req[0], p.req[1], p.req[2]}, (dfns & kbg::VP_DRF) ? p.ls : 0.0};
  Session::VictimCache& vc = S.vc;
  VictimProfile& vp = vprof();
  uint64_t c0 = vp.on ? cycles() : 0;
  if (vp.on) vp.tries++;
  if (!(vc.valid && vc.key == key)) {
    // device scan of every node against the current state
    kbg_status st = victim_push(S, L.touched);
    if (st != KBG_OK) return st;
    L.touched.clear();
    ++L.stamp;
    // one process: the scan writes its stop bytes straight into the mapped
    // host words and the big-node kernel one byte per big node (no copy);
    // sharded: device words, OR-reduced over the ranks, then copied
    const bool mapped = !S.comm;
    uint32_t* bits = mapped ? S.h_vbits_dev : S.d_vbits;
    const bool timed = (S.stats.victim_scans & 15) == 0 && p.node_n > 0;  // HIP-event time of every 16th launch
    HIP_TRY(kbg::launch_victim_scan(p, S.vt, bits, bits + S.W32, S.stream, timed ? S.ev[0] : nullptr,
                                    timed ? S.ev[1] : nullptr));
    if (!S.big_rows.empty())  // nodes with more than 128 candidates
      HIP_TRY(kbg::launch_victim_big(p, S.vt, S.d_big_rows, (int32_t)S.big_rows.size(), bits, bits + S.W32,
                                     mapped ? S.h_vbig_dev : nullptr, S.stream));
    if (!mapped) {  // disjoint words of the ranks: element-wise max is their OR
      if (kbg_status st2 =
              coll_rc(S, S.comm->coll->allreduce(S.d_vbits, S.d_vbits_red, 2 * (size_t)S.W32, kbg::kCollMax, S.stream));
          st2 != KBG_OK)
        return st2;
      HIP_TRY(hipMemcpyAsync(S.h_vbits, S.d_vbits_red, 2 * (size_t)S.W32 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                             S.stream));
    }
    if (kbg_status st2 = comm_sync(S); st2 != KBG_OK) return st2;
    S.vstage_busy = false;
    if (timed) {
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, S.ev[0], S.ev[1]));
      S.vk_timed_ms += ms;
      S.vk_timed++;
    }
    S.stats.victim_scans++;
    if (S.vk_timed) S.stats.victim_kernel_ms = S.vk_timed_ms / S.vk_timed * (double)S.stats.victim_scans;
    const volatile uint32_t* hb = S.h_vbits;
    for (int32_t w = 0; w < S.W32; ++w) {
      vc.stop[w] = hb[w];
      vc.panic[w] = hb[S.W32 + w];
    }
    if (mapped)
      for (size_t i = 0; i < S.big_rows.size(); ++i) {
        const uint8_t v = S.h_vbig[i];
        if (!v) continue;
        const int32_t n = S.tab_lo + S.big_rows[i];
        vc.stop[n >> 5] |= 1u << (n & 31);
        if (v & 2) vc.panic[n >> 5] |= 1u << (n & 31);
      }
    std::fill(vc.unk.begin(), vc.unk.end(), 0u);
    vc.lb = 0;
    for (int32_t hn : S.huge_nodes) vc.unk[hn >> 5] |= 1u << (hn & 31);  // not scanned on the device
    vc.key = key;
    vc.fns = dfns;
    vc.valid = true;
  }
  if (vp.on) {
    const uint64_t c1 = cycles();
    vp.scan += c1 - c0;
    c0 = c1;
  }
  // the first stop in node order: a node changed since the scan is
  // re-evaluated on the host (host_stop) when the search reaches it
  int32_t n = -1;
  bool pan = false;
  thread_local std::vector<int32_t> victims;
  bool have_victims = false;  // the stop node was just re-evaluated: its victims are in `victims`
  for (int32_t w = vc.lb; w < S.W32 && n < 0; ++w) {
    if (w == vc.lb && !(vc.stop[w] | vc.unk[w])) {  // nothing left below the next word
      vc.lb = w + 1;
      continue;
    }
    for (uint32_t cand = vc.stop[w] | vc.unk[w]; cand; cand &= cand - 1) {
      const int b = __builtin_ctz(cand);
      const uint32_t bit = 1u << b;
      const int32_t node = w * 32 + b;
      if (vc.unk[w] & bit) {
        vc.unk[w] &= ~bit;
        const int r = host_stop(S, mode, t, node, victims);
        S.stats.victim_host_evals++;
        vc.stop[w] = r ? (vc.stop[w] | bit) : (vc.stop[w] & ~bit);
        vc.panic[w] = r == 2 ? (vc.panic[w] | bit) : (vc.panic[w] & ~bit);
        if (!r) continue;
        have_victims = r == 1;
      }
      n = node;
      pan = (vc.panic[w] & bit) != 0;
      break;
    }
  }
  if (vp.on) {
    const uint64_t c1 = cycles();
    vp.walk += c1 - c0;
    c0 = c1;
  }
  if (n < 0) return KBG_OK;  // no node: the task stays Pending
  if (pan)
    return fail(KBG_E_REF_PANIC, "victim selection panics on node " + S.strs[S.nodes_in[n].name] +
                                     " (nil Node or Resource.Sub underflow in a victim fn)");
  if (!have_victims && (!host_victims(S, mode, t, n, &victims) || victims.empty()))
    return fail(KBG_E_INVALID, "internal: device and host victim selection disagree");
  Res all{};
  for (int32_t v : victims) kbg::res_add(all, S.treq[v]);
  const Res& req = S.treq[t];
  if (all.c < req.c && all.m < req.m && all.g < req.g)
    return fail(KBG_E_INVALID, "internal: device and host victim validation disagree");
  if (vp.on) {
    const uint64_t c1 = cycles();
    vp.select += c1 - c0;
    c0 = c1;
  }
  Res resreq = req;
  for (int32_t v : victims) {
    if (stmt) stmt->ops.push_back({true, v, -1, t, false});
    else S.evictions.push_back(kbg_eviction{v, t, S.action, 0});
    if (!L.evict(v)) return fail(KBG_E_REF_PANIC, "eviction: Resource.Sub underflow (resource_info.go:100-110)");
    if (kbg::res_le(resreq, S.treq[v])) break;  // preempt.go:221-224
    if (!kbg::res_sub(resreq, S.treq[v])) return fail(KBG_E_REF_PANIC, "preempt: resreq.Sub underflow (preempt.go:225)");
  }
  bool dup = false;
  if (!L.pipeline(t, n, &dup)) return fail(KBG_E_REF_PANIC, "pipeline: Releasing.Sub underflow (node_info.go:117-118)");
  if (stmt) stmt->ops.push_back({false, t, n, -1, dup});
  else append_log(S, t, n, KBG_KIND_PIPELINE, dup);
  if (vp.on) vp.apply += cycles() - c0;
  *outcome = TRY_ASSIGNED;
  return KBG_OK;
}

void stmt_commit(Session& S, Stmt& stmt) {  // statement.go:207-217
  for (auto& op : stmt.ops) {
    if (op.evict) S.evictions.push_back(kbg_eviction{op.task, op.by, S.action, 0});
    else append_log(S, op.task, op.node, KBG_KIND_PIPELINE, op.dup);
  }
  stmt.ops.clear();
}

kbg_status stmt_discard(Session& S, Live& L, Stmt& stmt) {  // statement.go:194-205
  // the one refusal (a key held by a pod outside the session jobs whose copy
  // the snapshot did not carry) is found before any operation is undone
  for (const Stmt::Op& op : stmt.ops) {
    if (op.evict || !op.dup) continue;
    const int64_t hk = node_key_of(S, op.task, op.node);
    auto oit = S.outsiders.find(hk);
    if (oit != S.outsiders.end() && oit->second.status == 0 && !S.outsider_gone.count(hk))
      return fail(KBG_E_UNSUPPORTED, "statement discard of a pipeline whose pod key is held on the node by a pod "
                                     "outside the session jobs with no node_pods entry (node_info.go:131-157 "
                                     "removes it, its resources are unknown): supply node_pods");
  }
  bool ok = true;
  for (size_t k = stmt.ops.size(); k-- > 0;) {
    const Stmt::Op& op = stmt.ops[k];
    if (op.evict) {
      if (!L.unevict(op.task)) return fail(KBG_E_REF_PANIC, "statement discard: unevict's AddTask Idle.Sub underflow");
    } else if (op.dup) {  // unpipeline's RemoveTask drops the pod that held the key
      if (kbg_status st = L.unpipeline_dup(op.task, op.node); st != KBG_OK) return st;
    } else {
      ok = L.unpipeline(op.task, op.node) && ok;
    }
  }
  stmt.ops.clear();
  return ok ? KBG_OK : fail(KBG_E_REF_PANIC, "statement discard: DeallocateFunc Sub underflow (resource_info.go:100-110)");
}

// Per job, its Pending tasks in TaskOrderFn order (a strict order, so the
// util.PriorityQueue pop sequence is this sorted order).
std::vector<std::vector<int32_t>> pending_by_job(const Session& S) {
  std::vector<std::vector<int32_t>> out(S.n_jobs);
  for (int32_t j = 0; j < S.n_jobs; ++j) {
    for (int32_t k = S.jt_off[j]; k < S.jt_off[j + 1]; ++k)
      if (S.tstat[S.jt[k]] == KBG_PENDING) out[j].push_back(S.jt[k]);
    std::sort(out[j].begin(), out[j].end(), [&](int32_t a, int32_t c) {
      if (S.task_order_prio && S.tasks_in[a].priority != S.tasks_in[c].priority)
        return S.tasks_in[a].priority > S.tasks_in[c].priority;
      return S.task_rank[a] < S.task_rank[c];
    });
  }
  return out;
}

kbg_status victim_action_check(Session&) { return KBG_OK; }  // nodes past kMaxNodeCandidates: host_stop

struct VictimRun {
  Session& S;
  std::vector<int32_t> mark, touched;
  Live L;
  explicit VictimRun(Session& s) : S(s), mark(s.n_nodes, -1), L{s, touched, mark, 0} {}
  // Node rows and plugin state reach the device before the next scan
  // (try_task) or at the end of the action (flush); between scans the host
  // stop maps carry the changes.
  kbg_status sync() { return KBG_OK; }
  kbg_status flush() {
    kbg_status st = victim_push(S, touched);
    touched.clear();
    ++L.stamp;
    return st;
  }
};

kbg_status reclaim_cycle(Session& S, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.reclaimed || S.allocated || S.backfilled || S.preempted)
    return fail(KBG_E_INVALID, "reclaim runs once per cycle, first; call kbg_session_reset");
  kbg_status st = victim_action_check(S);
  if (st != KBG_OK) return st;
  const auto t0 = std::chrono::steady_clock::now();
  if (!S.cycle_started) begin_cycle(S);
  S.reclaimed = true;
  S.action = KBG_ACTION_RECLAIM;
  S.vc.valid = false;  // other actions changed the session since any earlier scan
  if ((st = vt_setup(S)) != KBG_OK) return st;
  VictimRun R(S);
  auto queue_less = [&](int32_t a, int32_t b) {  // QueueOrderFn (proportion share, then UID)
    if (S.queue_order_prop && S.fin.qshare[a] != S.fin.qshare[b]) return S.fin.qshare[a] < S.fin.qshare[b];
    return S.queue_rank[a] < S.queue_rank[b];
  };
  auto job_less = [&](int32_t a, int32_t b) { return make_job_key(S, S.fin, a) < make_job_key(S, S.fin, b); };
  std::vector<int32_t> qheap;
  std::vector<std::vector<int32_t>> jheap(S.n_queues);
  std::vector<char> has_jobs(S.n_queues, 0);
  auto pending = pending_by_job(S);
  std::vector<size_t> next(S.n_jobs, 0);
  auto push = [&](std::vector<int32_t>& h, int32_t x, auto less) {
    h.push_back(x);
    go_up(h.data(), (int)h.size() - 1, less);
  };
  auto pop = [&](std::vector<int32_t>& h, auto less) {
    const int n = (int)h.size() - 1;
    std::swap(h[0], h[n]);
    go_down(h.data(), 0, n, less, S.heap_go111);
    const int32_t x = h.back();
    h.pop_back();
    return x;
  };
  for (int32_t j = 0; j < S.n_jobs; ++j) {  // reclaim.go:53-76
    const int32_t q = S.job_queue[j];
    push(qheap, q, queue_less);
    if (!pending[j].empty()) {
      has_jobs[q] = 1;
      push(jheap[q], j, job_less);
    }
  }
  kbg_status result = KBG_OK;
  while (!qheap.empty()) {  // reclaim.go:78-183
    const int32_t q = pop(qheap, queue_less);
    if (S.has_prop && S.q_has_attr[q] && kbg::res_le(S.q_deserved[q], S.fin.qalloc[q])) continue;  // Overused
    if (!has_jobs[q] || jheap[q].empty()) continue;
    const int32_t j = pop(jheap[q], job_less);
    if (next[j] >= pending[j].size()) continue;
    const int32_t t = pending[j][next[j]++];
    int32_t outcome;
    if ((result = try_task(S, R.L, kbg::VM_RECLAIM, t, nullptr, &outcome)) != KBG_OK) break;
    if ((result = R.sync()) != KBG_OK) break;
    if (outcome == TRY_ASSIGNED) push(qheap, q, queue_less);
  }
  if (result == KBG_OK || result == KBG_E_REF_PANIC) {
    kbg_status s2 = R.flush();
    if (s2 != KBG_OK) return s2;
  }
  HIP_TRY(hipStreamSynchronize(S.stream));
  S.vstage_busy = false;
  S.stats.reclaim_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  vprof().print("reclaim", S.stats.reclaim_ms);
  return copy_log(S, out, cap, n_out, result);
}

kbg_status preempt_cycle(Session& S, kbg_decision* out, int32_t cap, int32_t* n_out) {
  if (S.preempted) return fail(KBG_E_INVALID, "preempt runs once per cycle, last; call kbg_session_reset");
  kbg_status st = victim_action_check(S);
  if (st != KBG_OK) return st;
  const auto t0 = std::chrono::steady_clock::now();
  if (!S.cycle_started) begin_cycle(S);
  S.preempted = true;
  S.action = KBG_ACTION_PREEMPT;
  S.vc.valid = false;  // other actions changed the session since any earlier scan
  const uint64_t pc0 = vprof().on ? cycles() : 0;
  if ((st = vt_setup(S)) != KBG_OK) return st;
  VictimRun R(S);
  auto job_less = [&](int32_t a, int32_t b) { return make_job_key(S, S.fin, a) < make_job_key(S, S.fin, b); };
  auto job_ready = [&](int32_t j) { return !S.ready_gang || S.committed_ready[j] >= S.jobs_in[j].min_available; };
  std::vector<std::vector<int32_t>> jheap(S.n_queues);
  std::vector<char> has_jobs(S.n_queues, 0);
  std::vector<int32_t> queues, under;
  auto pending = pending_by_job(S);
  std::vector<size_t> next(S.n_jobs, 0);
  auto push = [&](std::vector<int32_t>& h, int32_t x) {
    h.push_back(x);
    go_up(h.data(), (int)h.size() - 1, job_less);
  };
  auto pop = [&](std::vector<int32_t>& h) {
    const int n = (int)h.size() - 1;
    std::swap(h[0], h[n]);
    go_down(h.data(), 0, n, job_less, S.heap_go111);
    const int32_t x = h.back();
    h.pop_back();
    return x;
  };
  for (int32_t j = 0; j < S.n_jobs; ++j) {  // preempt.go:54-77
    const int32_t q = S.job_queue[j];
    queues.push_back(q);
    if (!pending[j].empty()) {
      has_jobs[q] = 1;
      push(jheap[q], j);
      under.push_back(j);
    }
  }
  if (vprof().on) vprof().setup += cycles() - pc0;
  kbg_status result = KBG_OK;
  Stmt stmt;  // one statement object, emptied by every commit / discard (its ops keep their capacity)
  auto run = [&]() -> kbg_status {
    kbg_status s2;
    int32_t outcome;
    for (int32_t q : queues) {
      for (;;) {  // preempt.go:81-130: between jobs of the queue
        if (!has_jobs[q] || jheap[q].empty()) break;
        const int32_t pj = pop(jheap[q]);
        stmt.ops.clear();
        bool assigned = false;
        for (;;) {
          if (next[pj] >= pending[pj].size()) break;
          const int32_t t = pending[pj][next[pj]++];
          if ((s2 = try_task(S, R.L, kbg::VM_PREEMPT_JOBS, t, &stmt, &outcome)) != KBG_OK) return s2;
          if ((s2 = R.sync()) != KBG_OK) return s2;
          if (outcome == TRY_ASSIGNED) assigned = true;
          if (job_ready(pj)) {
            stmt_commit(S, stmt);
            break;
          }
        }
        if (!job_ready(pj)) {
          if ((s2 = stmt_discard(S, R.L, stmt)) != KBG_OK) return s2;
          if ((s2 = R.sync()) != KBG_OK) return s2;
          continue;
        }
        if (assigned) push(jheap[q], pj);
      }
      for (int32_t j : under) {  // preempt.go:132-166: between tasks of a job
        for (;;) {
          if (next[j] >= pending[j].size()) break;
          const int32_t t = pending[j][next[j]++];
          stmt.ops.clear();
          if ((s2 = try_task(S, R.L, kbg::VM_PREEMPT_TASKS, t, &stmt, &outcome)) != KBG_OK) return s2;
          stmt_commit(S, stmt);
          if ((s2 = R.sync()) != KBG_OK) return s2;
          if (outcome != TRY_ASSIGNED) break;
        }
      }
    }
    return KBG_OK;
  };
  result = run();
  const uint64_t pc1 = vprof().on ? cycles() : 0;
  if (result == KBG_OK || result == KBG_E_REF_PANIC) {
    kbg_status s2 = R.flush();
    if (s2 != KBG_OK) return s2;
  }
  if (vprof().on) vprof().flush += cycles() - pc1;
  HIP_TRY(hipStreamSynchronize(S.stream));
  S.vstage_busy = false;
  S.stats.preempt_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  vprof().print("preempt", S.stats.preempt_ms);
  return copy_log(S, out, cap, n_out, result);
}


// ================================================== resident session updates
// kbgpu.h kbg_session_update. The events edit the session's inputs the way the
// cache edits its objects (event_handlers.go:40-188, node_info.go:84-157);
// Snapshot's clones (cache.go:549-597) then equal those inputs: a clone
// re-adds a node's tasks to NewNodeInfo, and since Idle only decreases along
// AddTask (Releasing pods add to Releasing, no cache pod is Pipelined) the
// clone panics iff the final Idle drops below the tolerance, which is checked
// on the node rows an event touches.

bool terminated(int32_t status) { return status == KBG_SUCCEEDED || status == KBG_FAILED; }

struct UpdateCtx {
  std::vector<int32_t> nodes;  // node rows to rewrite in HBM
  std::vector<uint8_t> seen;
  bool rebuild = false;        // the static masks must be recompiled
  void touch(int32_t n) {
    if (!seen[n]) {
      seen[n] = 1;
      nodes.push_back(n);
    }
  }
};

// Sub with the reference's panic condition (resource_info.go:100-110)
bool kres_sub(kbg_resource& a, const Res& r) {
  Res x = to_res(a);
  if (!kbg::res_sub(x, r)) return false;
  a = to_kres(x);
  return true;
}
void kres_add(kbg_resource& a, const Res& r) {
  Res x = to_res(a);
  kbg::res_add(x, r);
  a = to_kres(x);
}

// NodeInfo.AddTask of session task t (node_info.go:101-129) on the inputs.
// false: the cache would panic.
bool in_node_add(Session& S, UpdateCtx& U, int32_t n, int32_t t) {
  kbg_node& nd = S.nodes_in[n];
  const int32_t key = S.canon[S.tasks_in[t].pod_key];
  std::vector<int32_t>& keys = S.node_key_order[n];
  if (std::find(keys.begin(), keys.end(), key) != keys.end()) return true;  // "already on node": unchanged
  const Res r = S.treq[t];
  if (nd.has_node) {
    switch (S.tasks_in[t].status) {
      case KBG_RELEASING:
        kres_add(nd.releasing, r);
        if (!kres_sub(nd.idle, r)) return false;
        break;
      case KBG_PIPELINED:
        if (!kres_sub(nd.releasing, r)) return false;
        break;
      default:
        if (!kres_sub(nd.idle, r)) return false;
    }
  }
  nd.num_tasks++;
  keys.push_back(key);
  if ((size_t)key >= S.kc_node.size()) S.kc_node.resize((size_t)key + 1, 0);
  S.kc_node[key]++;
  S.upd_keys.push_back(key);
  S.node_task_order[n].push_back(t);
  // the pod's host ports join the node's (one entry per pod and port: a port stays used while any pod lists it)
  const int32_t sp = S.tasks_in[t].spec;
  if (sp >= 0 && S.specs_in[sp].port_len > 0) {
    const kbg_spec& spec = S.specs_in[sp];
    std::vector<kbg_host_port> mine(S.ports_in.begin() + nd.port_off, S.ports_in.begin() + nd.port_off + nd.port_len);
    for (int32_t i = 0; i < spec.port_len; ++i)
      if (S.ports_in[spec.port_off + i].host_port > 0) mine.push_back(S.ports_in[spec.port_off + i]);
    nd.port_off = (int32_t)S.ports_in.size();
    nd.port_len = (int32_t)mine.size();
    S.ports_in.insert(S.ports_in.end(), mine.begin(), mine.end());
  }
  U.touch(n);
  return true;
}

// NodeInfo.RemoveTask(t) (node_info.go:131-157): the pod holding t's key
// leaves the node. 0 removed, 1 not found (an error), else a kbg_status.
int in_node_remove(Session& S, UpdateCtx& U, int32_t n, int32_t t) {
  kbg_node& nd = S.nodes_in[n];
  const int32_t key = S.canon[S.tasks_in[t].pod_key];
  std::vector<int32_t>& keys = S.node_key_order[n];
  auto kit = std::find(keys.begin(), keys.end(), key);
  if (kit == keys.end()) return 1;
  std::vector<int32_t>& tl = S.node_task_order[n];
  // a node's session tasks hold distinct keys (AddTask refuses a key already
  // there), so the task holding t's key is t itself whenever t is on the node;
  // otherwise another session task, or a pod outside the session jobs
  auto hit = std::find(tl.begin(), tl.end(), t);
  if (hit == tl.end())
    hit = std::find_if(tl.begin(), tl.end(), [&](int32_t u) { return S.canon[S.tasks_in[u].pod_key] == key; });
  const int64_t hk = ((int64_t)n << 32) | (uint32_t)key;
  auto oit = hit == tl.end() ? S.outsiders.find(hk) : S.outsiders.end();
  if (hit == tl.end() && (oit == S.outsiders.end() || oit->second.status == 0))
    return fail(KBG_E_UNSUPPORTED, "the pod key is held on the node by a pod outside the session jobs "
                                   "and the snapshot carried no node_pods (its resources are unknown): re-open");
  // the holder's copy: its ports, Resreq and status
  std::vector<kbg_host_port> gone;
  Res r;
  int32_t status;
  if (hit != tl.end()) {
    const int32_t u = *hit;
    const int32_t sp = S.tasks_in[u].spec;
    if (sp >= 0)
      for (int32_t i = 0; i < S.specs_in[sp].port_len; ++i) gone.push_back(S.ports_in[S.specs_in[sp].port_off + i]);
    r = S.treq[u];
    status = S.tasks_in[u].status;
  } else {
    gone = oit->second.ports;
    r = to_res(oit->second.req);
    status = oit->second.status;
  }
  if (!gone.empty()) {
    // the pod's host ports leave the node's: node.Pods() no longer lists it,
    // so a port stays used exactly while another pod's entry remains (the
    // node's list holds one entry per pod and port, kbgpu.h kbg_node)
    auto canon_ip = [&](int32_t id) { return S.strs[id].empty() ? std::string("0.0.0.0") : S.strs[id]; };
    auto canon_proto = [&](int32_t id) { return S.strs[id].empty() ? std::string("TCP") : S.strs[id]; };
    std::vector<kbg_host_port> mine(S.ports_in.begin() + nd.port_off, S.ports_in.begin() + nd.port_off + nd.port_len);
    for (const kbg_host_port& hp : gone) {
      if (hp.host_port <= 0) continue;
      const std::string ip = canon_ip(hp.host_ip), pr = canon_proto(hp.protocol);
      auto it = std::find_if(mine.begin(), mine.end(), [&](const kbg_host_port& x) {
        return x.host_port == hp.host_port && canon_ip(x.host_ip) == ip && canon_proto(x.protocol) == pr;
      });
      if (it != mine.end()) mine.erase(it);
    }
    nd.port_off = (int32_t)S.ports_in.size();
    nd.port_len = (int32_t)mine.size();
    S.ports_in.insert(S.ports_in.end(), mine.begin(), mine.end());
  }
  if (nd.has_node) {
    switch (status) {
      case KBG_RELEASING:
        if (!kres_sub(nd.releasing, r)) return fail(KBG_E_REF_PANIC, "RemoveTask: Releasing.Sub underflow");
        kres_add(nd.idle, r);
        break;
      case KBG_PIPELINED:
        kres_add(nd.releasing, r);
        break;
      default:
        kres_add(nd.idle, r);
    }
  }
  nd.num_tasks--;
  keys.erase(kit);
  if ((size_t)key < S.kc_node.size()) S.kc_node[key]--;
  S.upd_keys.push_back(key);
  if (hit != tl.end()) tl.erase(hit);
  else S.outsiders.erase(oit);  // the cache's node no longer holds it, for good
  U.touch(n);
  return 0;
}

// event_handlers.go deleteTask: the job side always, then the node side.
// Returns 0, 1 (the node side failed: updateTask stops there) or a status.
// A job's task order (JobInfo.Tasks insertion order) under an update: a task
// an event takes off its job (-1) and puts back (a sequence number) is moved
// to the end in event order. The moves are recorded per event and applied to
// each changed job's list once, after the events (finish_job_lists): a find
// and erase per event scanned the job's whole list (kept for small updates,
// whose lists the event loop prefetches and whose jobs are few).
void job_list_mark(Session& S, int32_t t, int64_t v) {
  if (!S.jmove_defer) {  // a small update: in place (the event loop has requested the list's lines)
    std::vector<int32_t>& jl = S.job_task_order[S.tasks_in[t].job];
    if (v < 0) jl.erase(std::find(jl.begin(), jl.end(), t));
    else jl.push_back(t);
    return;
  }
  if ((size_t)t >= S.jmove.size()) S.jmove.resize((size_t)std::max<int32_t>(S.n_tasks, t + 1), 0);
  const int32_t j = S.tasks_in[t].job;
  if ((size_t)j >= S.jmove_dirty.size()) S.jmove_dirty.resize(S.n_jobs, 0);
  if (!S.jmove_dirty[j]) {
    S.jmove_dirty[j] = 1;
    S.jmove_jobs.push_back(j);
  }
  S.jmove[t] = v;
  if (v < 0) S.jmove_out.push_back(t);
  else S.jmove_add.emplace_back(t, v);
}
void finish_job_lists(Session& S) {
  if (S.jmove_jobs.empty()) return;
  // each changed job's re-added tasks, in event order: counted, placed by offset
  std::vector<int32_t>& cnt = S.jmove_cnt;
  std::vector<int32_t>& pos = S.jmove_pos;
  if (cnt.size() < (size_t)S.n_jobs) {
    cnt.resize(S.n_jobs, 0);
    pos.resize(S.n_jobs, 0);
  }
  for (const auto& [t, v] : S.jmove_add)
    if (S.jmove[t] == v) cnt[S.tasks_in[t].job]++;
  int32_t total = 0;
  for (const int32_t j : S.jmove_jobs) {
    pos[j] = total;
    total += cnt[j];
  }
  S.jmove_flat.resize(total);
  for (const auto& [t, v] : S.jmove_add)
    if (S.jmove[t] == v) S.jmove_flat[pos[S.tasks_in[t].job]++] = t;
  thread_local std::vector<int32_t> kept;
  for (const int32_t j : S.jmove_jobs) {
    std::vector<int32_t>& jl = S.job_task_order[j];
    kept.clear();
    for (const int32_t t : jl)
      if ((size_t)t >= S.jmove.size() || S.jmove[t] == 0) kept.push_back(t);
    kept.insert(kept.end(), S.jmove_flat.begin() + (pos[j] - cnt[j]), S.jmove_flat.begin() + pos[j]);
    jl.assign(kept.begin(), kept.end());
    cnt[j] = 0;
    S.jmove_dirty[j] = 0;
  }
  for (const auto& [t, v] : S.jmove_add) S.jmove[t] = 0;
  for (const int32_t t : S.jmove_out) S.jmove[t] = 0;
  S.jmove_add.clear();
  S.jmove_out.clear();
  S.jmove_jobs.clear();
}

int in_delete_task(Session& S, UpdateCtx& U, int32_t t) {
  job_list_mark(S, t, -1);  // JobInfo.DeleteTaskInfo
  // sc.Nodes[NodeName] (task_cnode: a session node by name, or the node the
  // cache knows only from pods carrying that NodeName; kept current by the
  // events); -1: no NodeName, or no such NodeInfo
  const int32_t n = S.task_cnode[t];
  if (n < 0) return 0;
  return in_node_remove(S, U, n, t);
}

kbg_status in_add_task(Session& S, UpdateCtx& U, int32_t t) {  // event_handlers.go addTask
  job_list_mark(S, t, ++S.jmove_seq);                          // JobInfo.AddTaskInfo
  const int32_t n = S.task_cnode[t];
  if (n >= 0 && !terminated(S.tasks_in[t].status) && !in_node_add(S, U, n, t))
    return fail(KBG_E_REF_PANIC, "NodeInfo.AddTask: Resource.Sub underflow (node_info.go:117-123)");
  return KBG_OK;
}

kbg_status apply_event(Session& S, UpdateCtx& U, const kbg_event& e, const uint64_t* key_hash);
// The NodeName a pod event's node index stands for: the node's name, or for a
// node the cache knows only from pods the NodeName they carry (update_precheck
// refuses a nil node whose name the session does not know); "" for -1.
int32_t event_node_name(Session& S, const kbg_event& e) {
  const int32_t node = e.node;
  if (node < 0) return empty_str(S);
  const kbg_node& nd = S.nodes_in[node];
  if (nd.has_node) return nd.name;
  if (e.node_name && e.node_name[0]) {  // the caller names it: the node's name from now on
    const int32_t nm = S.canon[intern(S, e.node_name)];
    if (S.nil_name[node] < 0) S.nil_name[node] = nm;
    S.pod_only_of.emplace(nm, node);
    return nm;
  }
  return S.nil_name[node] < 0 ? nd.name : S.nil_name[node];
}
// The pods of node n as NodeInfo.Tasks holds them: (Resreq, status) of each
// session task and each pod outside the session jobs. false: an outsider
// whose copy the snapshot did not carry (no node_pods).
bool node_pods_of(const Session& S, int32_t n, std::vector<std::pair<Res, int32_t>>* out) {
  out->clear();
  for (const int32_t t : S.node_task_order[n]) out->emplace_back(S.treq[t], S.tasks_in[t].status);
  for (const int32_t key : S.node_key_order[n]) {
    bool session = false;
    for (const int32_t t : S.node_task_order[n]) session |= S.canon[S.tasks_in[t].pod_key] == key;
    if (session) continue;
    auto it = S.outsiders.find(((int64_t)n << 32) | (uint32_t)key);
    if (it == S.outsiders.end() || it->second.status == 0) return false;
    out->emplace_back(to_res(it->second.req), it->second.status);
  }
  return true;
}

// KBG_EV_NODE_SET: NodeInfo.SetNode with the whole Node (node_info.go:84-99),
// then the snapshot's clone (NewNodeInfo(node) + AddTask of every pod,
// cache.go:549-597). A node the cache knew only from a pod (Node nil, Name "")
// takes the Node's name: its pods' NodeName lookups (ssn.NodeIndex) find it
// from now on, so pods that were "ghosts" (allocated on a node outside the
// session) are not any more. New labels, taints or schedulability recompile
// the static predicate (a rebuild); an unchanged spec is a NODE_UPDATE.
kbg_status apply_node_set(Session& S, UpdateCtx& U, const kbg_event& e) {
  if (e.node < 0 || e.node >= S.n_nodes || !e.node_spec || !e.node_spec->name || e.node_spec->n_labels < 0 ||
      e.node_spec->n_taints < 0 || (e.node_spec->n_labels && !e.node_spec->labels) ||
      (e.node_spec->n_taints && !e.node_spec->taints))
    return fail(KBG_E_INVALID, "NODE_SET event");
  const kbg_node_spec& sp = *e.node_spec;
  kbg_node& nd = S.nodes_in[e.node];
  const int32_t name = intern(S, sp.name);
  if (nd.has_node && S.canon[nd.name] != S.canon[name]) return fail(KBG_E_INVALID, "NODE_SET: the node's name differs");
  thread_local std::vector<int32_t> labels;
  thread_local std::vector<kbg_taint> taints;
  labels.clear();
  taints.clear();
  for (int32_t i = 0; i < 2 * sp.n_labels; ++i) {
    if (!sp.labels[i]) return fail(KBG_E_INVALID, "NODE_SET: null label string");
    labels.push_back(intern(S, sp.labels[i]));
  }
  for (int32_t i = 0; i < sp.n_taints; ++i) {
    if (!sp.taints[3 * i] || !sp.taints[3 * i + 1] || !sp.taints[3 * i + 2])
      return fail(KBG_E_INVALID, "NODE_SET: null taint string");
    taints.push_back(kbg_taint{intern(S, sp.taints[3 * i]), intern(S, sp.taints[3 * i + 1]), intern(S, sp.taints[3 * i + 2])});
  }
  // the same labels (as a map: every new pair among the old ones, same count) and taints (in order)?
  bool same = nd.has_node && nd.label_len == sp.n_labels && nd.taint_len == sp.n_taints;
  const int32_t* old_l = S.labels_in.data() + 2 * (size_t)nd.label_off;
  for (int32_t i = 0; same && i < sp.n_labels; ++i) {
    bool found = false;
    for (int32_t k = 0; k < nd.label_len && !found; ++k)
      found = S.canon[old_l[2 * k]] == S.canon[labels[2 * i]] && S.canon[old_l[2 * k + 1]] == S.canon[labels[2 * i + 1]];
    same = found;
  }
  for (int32_t i = 0; same && i < sp.n_taints; ++i) {
    const kbg_taint& a = S.taints_in[nd.taint_off + i];
    same = S.canon[a.key] == S.canon[taints[i].key] && S.canon[a.value] == S.canon[taints[i].value] &&
           S.canon[a.effect] == S.canon[taints[i].effect];
  }
  if (same) {  // SetNode's resources and schedulability only
    kbg_event u = e;
    u.kind = KBG_EV_NODE_UPDATE;
    return apply_event(S, U, u, nullptr);
  }
  if (!nd.has_node) {
    // the clone: Idle = Allocatable - every pod, Releasing pods on Releasing (AddTask, node_info.go:101-129)
    std::vector<std::pair<Res, int32_t>> pods;
    if (!node_pods_of(S, e.node, &pods))
      return fail(KBG_E_UNSUPPORTED, "NODE_SET of a node holding a pod outside the session jobs whose copy the "
                                     "snapshot did not carry (node_pods): re-open");
    Res idle = to_res(e.resource), rel{};
    for (const auto& [r, st] : pods) {
      if (st == KBG_RELEASING) kbg::res_add(rel, r);
      if (st == KBG_PIPELINED) {
        if (!kbg::res_sub(rel, r)) return fail(KBG_E_REF_PANIC, "NodeInfo.AddTask: Releasing.Sub underflow");
        continue;
      }
      if (!kbg::res_sub(idle, r)) return fail(KBG_E_REF_PANIC, "NodeInfo.AddTask: Idle.Sub underflow (node_info.go:117-123)");
    }
    nd.idle = to_kres(idle);
    nd.releasing = to_kres(rel);
    nd.has_node = 1;
    S.node_of[S.canon[name]] = e.node;
    nd.name = name;
    for (int32_t t = 0; t < S.n_tasks; ++t)  // NodeIndex[NodeName] finds the node now
      if (S.task_live[t] && S.canon[S.tasks_in[t].node_name] == S.canon[name]) S.task_node[t] = S.task_cnode[t] = e.node;
  } else {
    Res idle = to_res(nd.idle);
    const Res a0 = to_res(nd.allocatable), a1 = to_res(e.resource);
    idle = Res{idle.c + (a1.c - a0.c), idle.m + (a1.m - a0.m), idle.g + (a1.g - a0.g)};
    if (nd.num_tasks > 0 && !kbg::res_le(Res{}, idle))
      return fail(KBG_E_REF_PANIC, "NodeInfo.SetNode: Idle.Sub underflow (node_info.go:84-99)");
    nd.idle = to_kres(idle);
  }
  nd.allocatable = e.resource;
  nd.max_task_num = e.max_task_num;
  nd.unschedulable = e.unschedulable;
  nd.label_off = (int32_t)(S.labels_in.size() / 2);
  nd.label_len = sp.n_labels;
  S.labels_in.insert(S.labels_in.end(), labels.begin(), labels.end());
  nd.taint_off = (int32_t)S.taints_in.size();
  nd.taint_len = sp.n_taints;
  S.taints_in.insert(S.taints_in.end(), taints.begin(), taints.end());
  U.rebuild = true;  // labels / taints / a new Node: the static predicate is recompiled
  U.touch(e.node);
  return KBG_OK;
}

// Structural events (kbgpu.h KBG_EV_NODE_ADD ... QUEUE_DELETE) on the inputs:
// what joins is appended (its pod events in the same batch find it), what
// leaves is marked; restructure() then rebuilds the session from the updated
// snapshot. update_precheck has validated every field.
kbg_status apply_structural(Session& S, UpdateCtx& U, const kbg_event& e) {
  switch (e.kind) {
    case KBG_EV_NODE_ADD: {  // cache.AddNode of a new name -> NewNodeInfo (event_handlers.go:232-240)
      kbg_node nd{};
      const int32_t n = S.n_nodes++;
      if (const kbg_node_spec* sp = e.node_spec) {
        nd.name = intern(S, sp->name);
        nd.has_node = 1;
        nd.allocatable = nd.idle = e.resource;  // Idle = Allocatable, Releasing empty (node_info.go:44-71)
        nd.max_task_num = e.max_task_num;
        nd.unschedulable = e.unschedulable;
        nd.label_off = (int32_t)(S.labels_in.size() / 2);
        nd.label_len = sp->n_labels;
        for (int32_t i = 0; i < 2 * sp->n_labels; ++i) S.labels_in.push_back(intern(S, sp->labels[i]));
        nd.taint_off = (int32_t)S.taints_in.size();
        nd.taint_len = sp->n_taints;
        for (int32_t i = 0; i < sp->n_taints; ++i)
          S.taints_in.push_back(kbg_taint{intern(S, sp->taints[3 * i]), intern(S, sp->taints[3 * i + 1]),
                                          intern(S, sp->taints[3 * i + 2])});
        S.node_of[S.canon[nd.name]] = n;
        S.nil_name.push_back(-1);
      } else {  // NewNodeInfo(nil): Name "", known by the NodeName that made it
        nd.name = empty_str(S);
        const int32_t nm = S.canon[intern(S, e.node_name)];
        S.nil_name.push_back(nm);
        S.pod_only_of[nm] = n;
      }
      nd.port_off = (int32_t)S.ports_in.size();
      S.nodes_in.push_back(nd);
      S.node_task_order.emplace_back();
      S.node_key_order.emplace_back();
      S.node_dead.push_back(0);
      U.seen.push_back(0);
      return KBG_OK;
    }
    case KBG_EV_NODE_DELETE: {  // cache.DeleteNode (event_handlers.go:262-268)
      const int32_t n = e.node;
      S.node_dead[n] = 1;
      const kbg_node& nd = S.nodes_in[n];
      if (nd.has_node) {
        auto it = S.node_of.find(S.canon[nd.name]);
        if (it != S.node_of.end() && it->second == n) S.node_of.erase(it);
      } else if (S.nil_name[n] >= 0) {
        auto it = S.pod_only_of.find(S.nil_name[n]);
        if (it != S.pod_only_of.end() && it->second == n) S.pod_only_of.erase(it);
      }
      return KBG_OK;
    }
    case KBG_EV_JOB_ADD: {  // cache.AddPodGroup of a new JobID -> NewJobInfo + SetPodGroup (event_handlers.go:344-358)
      kbg_job j{};
      j.uid = intern(S, e.name);
      j.queue = e.queue;
      j.min_available = e.min_available;
      j.priority = e.priority;
      j.creation_ns = e.creation_ns;
      S.jobs_in.push_back(j);
      S.job_task_order.emplace_back();
      S.job_dead.push_back(0);
      S.job_to_others.push_back(0);
      S.n_jobs++;
      return KBG_OK;
    }
    case KBG_EV_JOB_DELETE:  // UnsetPodGroup: its Running tasks are Others from now on (cache.go:570-582)
      S.job_dead[e.job] = 1;
      S.job_to_others[e.job] = 1;
      return KBG_OK;
    case KBG_EV_QUEUE_ADD:  // cache.AddQueue (event_handlers.go:635-640)
      S.queues_in.push_back(kbg_queue{intern(S, e.name), e.weight});
      S.queue_dead.push_back(0);
      S.n_queues++;
      return KBG_OK;
    case KBG_EV_QUEUE_DELETE:  // its jobs are not in the snapshot any more (cache.go:584-588)
      S.queue_dead[e.queue] = 1;
      for (int32_t j = 0; j < S.n_jobs; ++j)
        if (S.jobs_in[j].queue == e.queue) S.job_dead[j] = 1;
      return KBG_OK;
  }
  return fail(KBG_E_INVALID, "event kind");
}

// key_hash: StrIndex::hash of a POD_ADD's pod key when the caller computed it
// ahead (session_update's prefetch), else null
kbg_status apply_event(Session& S, UpdateCtx& U, const kbg_event& e, const uint64_t* key_hash) {
  auto status_ok = [](int32_t st) { return st > 0 && st <= KBG_UNKNOWN && !(st & (st - 1)); };
  switch (e.kind) {
    case KBG_EV_POD_UPDATE:
    case KBG_EV_POD_DELETE: {
      const int32_t t = e.task;
      if (t < 0 || t >= S.n_tasks || !S.task_live[t]) return fail(KBG_E_INVALID, "event task index");
      if (e.kind == KBG_EV_POD_UPDATE && (!status_ok(e.status) || e.node < -1 || e.node >= S.n_nodes))
        return fail(KBG_E_INVALID, "event status / node");
      S.pend_dirty_jobs.push_back(S.tasks_in[t].job);
      S.upd_tasks.push_back(t);
      const int r = in_delete_task(S, U, t);
      if (r > 1) return (kbg_status)r;
      if (e.kind == KBG_EV_POD_DELETE || r == 1) {  // deleted, or updateTask returned deleteTask's error
        S.task_live[t] = 0;
        // it leaves its job's rank order (an updated task keeps its place there:
        // same task, same UID; a task added by this update is not in it yet)
        const int32_t j = S.tasks_in[t].job;
        if ((size_t)j < S.job_rank_order.size()) {
          std::vector<int32_t>& ro = S.job_rank_order[j];
          auto it = std::find(ro.begin(), ro.end(), t);
          if (it != ro.end()) {
            if ((size_t)j < S.job_rank_key.size() && S.job_rank_key[j].size() == ro.size())
              S.job_rank_key[j].erase(S.job_rank_key[j].begin() + (it - ro.begin()));
            ro.erase(it);
          }
        }
        return KBG_OK;
      }
      S.tasks_in[t].status = e.status;
      S.tasks_in[t].node_name = event_node_name(S, e);
      S.task_node[t] = e.node >= 0 && S.nodes_in[e.node].has_node ? e.node : -1;  // ssn.NodeIndex finds it
      S.task_cnode[t] = e.node;
      if (e.status == KBG_PENDING) S.pend_new.push_back(t);
      return in_add_task(S, U, t);
    }
    case KBG_EV_POD_ADD: {
      if (e.job < 0 || e.job >= S.n_jobs || e.spec < -1 || e.spec >= (int32_t)S.specs_in.size() ||
          !status_ok(e.status) || e.node < -1 || e.node >= S.n_nodes || !e.uid || !e.pod_key)
        return fail(KBG_E_INVALID, "POD_ADD event");
      kbg_task k{};
      k.uid = append_str(S, e.uid);
      k.job = e.job;
      k.status = e.status;
      k.priority = e.priority;
      k.resreq = e.resource;
      k.spec = e.spec;
      k.node_name = event_node_name(S, e);
      k.pod_key = key_hash ? intern_h(S, e.pod_key, *key_hash) : intern(S, e.pod_key);
      const int32_t t = S.n_tasks++;
      S.tasks_in.push_back(k);
      S.task_live.push_back(1);
      S.treq.push_back(to_res(k.resreq));
      S.task_node.push_back(e.node >= 0 && S.nodes_in[e.node].has_node ? e.node : -1);
      S.task_cnode.push_back(e.node);
      S.task_ranks_stale = true;
      S.rank_dirty_jobs.push_back(e.job);
      S.pend_dirty_jobs.push_back(e.job);
      S.pend_new.push_back(t);
      S.upd_tasks.push_back(t);
      return in_add_task(S, U, t);
    }
    case KBG_EV_NODE_SET:
      return apply_node_set(S, U, e);
    case KBG_EV_NODE_ADD:
    case KBG_EV_NODE_DELETE:
    case KBG_EV_JOB_ADD:
    case KBG_EV_JOB_DELETE:
    case KBG_EV_QUEUE_ADD:
    case KBG_EV_QUEUE_DELETE:
      return apply_structural(S, U, e);
    case KBG_EV_NODE_UPDATE: {
      if (e.node < 0 || e.node >= S.n_nodes) return fail(KBG_E_INVALID, "event node index");
      kbg_node& nd = S.nodes_in[e.node];
      if (!nd.has_node)
        return fail(KBG_E_UNSUPPORTED, "KBG_EV_NODE_UPDATE of a node the cache only knows from a pod: send "
                                       "KBG_EV_NODE_SET (its name, labels and taints)");
      // SetNode (node_info.go:84-99) + the snapshot clone: Idle = Allocatable - every task
      Res idle = to_res(nd.idle);
      const Res a0 = to_res(nd.allocatable), a1 = to_res(e.resource);
      idle = Res{idle.c + (a1.c - a0.c), idle.m + (a1.m - a0.m), idle.g + (a1.g - a0.g)};
      if (nd.num_tasks > 0 && !kbg::res_le(Res{}, idle))
        return fail(KBG_E_REF_PANIC, "NodeInfo.SetNode: Idle.Sub underflow (node_info.go:84-99)");
      nd.idle = to_kres(idle);
      nd.allocatable = e.resource;
      nd.max_task_num = e.max_task_num;
      if ((nd.unschedulable != 0) != (e.unschedulable != 0)) U.rebuild = true;  // the static masks change
      nd.unschedulable = e.unschedulable;
      U.touch(e.node);
      return KBG_OK;
    }
  }
  return fail(KBG_E_INVALID, "event kind");
}

// The refusals of an event batch (KBG_E_INVALID, KBG_E_UNSUPPORTED), found by
// walking the events over an overlay of what they change — task liveness,
// each changed task's node and status, the session task holding a pod key on
// a node — before the first one is applied, so a refused batch leaves the
// session unchanged. The walk follows apply_event: deleteTask's node side
// (in_node_remove) finds the key's holder, addTask's (in_node_add) takes the
// key when no pod holds it (node_info.go:101-157).
kbg_status update_precheck(const Session& S, const kbg_event* ev, int32_t n) {
  auto status_ok = [](int32_t st) { return st > 0 && st <= KBG_UNKNOWN && !(st & (st - 1)); };
  bool port_specs = false;
  for (const kbg_spec& sp : S.specs_in) port_specs |= sp.has_host_ports != 0;
  bool structural = false;
  int32_t adds = 0;
  for (int32_t i = 0; i < n; ++i) {
    adds += ev[i].kind == KBG_EV_POD_ADD;
    structural |= ev[i].kind >= KBG_EV_NODE_ADD;
  }
  if (structural && S.comm)
    return fail(KBG_E_UNSUPPORTED, "structural events on a session sharded over a communicator: re-open it on every rank");
  // else no removal can be refused (a structural batch walks every pod's node: pods on deleted nodes)
  const bool holders = port_specs || !S.outsiders.empty() || structural;
  const int32_t T0 = S.n_tasks;
  std::vector<uint8_t> dead(S.n_tasks + adds, 0);
  for (int32_t t = 0; t < T0; ++t) dead[t] = !S.task_live[t];
  struct Now { int32_t node, status, key, spec; };
  std::unordered_map<int32_t, Now> now;            // tasks an earlier event of the batch changed or added
  std::unordered_map<int64_t, int32_t> hold;       // (node << 32 | key) -> holding session task, -1 none
  std::unordered_map<std::string, int32_t> fresh;  // pod keys the session has not interned yet
  auto task_now = [&](int32_t t) -> Now {
    auto it = now.find(t);
    if (it != now.end()) return it->second;
    const kbg_task& k = S.tasks_in[t];
    return Now{S.task_cnode[t], k.status, S.canon[k.pod_key], k.spec};
  };
  auto holder = [&](int32_t nd, int32_t key) -> int32_t {  // -2 / -3: a pod outside the session jobs (-3: unknown)
    const int64_t hk = ((int64_t)nd << 32) | (uint32_t)key;
    auto it = hold.find(hk);
    if (it != hold.end()) return it->second;
    if (nd >= S.n_nodes) return -1;  // a node this batch added: no pod yet
    auto ot = S.outsiders.find(hk);
    if (ot != S.outsiders.end()) return ot->second.status ? -2 : -3;
    for (int32_t u : S.node_task_order[nd])
      if (S.canon[S.tasks_in[u].pod_key] == key) return u;
    return -1;
  };
  int32_t T = T0;
  // structural events: the counts as the batch grows them, what it removed,
  // the names it gave (-1: removed by the batch)
  int32_t N = S.n_nodes, J = S.n_jobs, Q = S.n_queues;
  std::vector<uint8_t> ndead, jdead, qdead;
  std::vector<int32_t> jq, add_job;  // queues of the jobs this batch added; jobs of the tasks it added
  std::unordered_map<std::string, int32_t> bnodes, bjobs, bqueues;
  std::unordered_map<int32_t, int32_t> job_of_uid, queue_of_uid;  // canonical JobID / QueueID -> index
  if (structural) {
    ndead.assign(N, 0);
    jdead.assign(J, 0);
    qdead.assign(Q, 0);
    for (int32_t j = 0; j < J; ++j) job_of_uid.emplace(S.canon[S.jobs_in[j].uid], j);
    for (int32_t q = 0; q < Q; ++q) queue_of_uid.emplace(S.canon[S.queues_in[q].uid], q);
  }
  auto task_job = [&](int32_t t) { return t < T0 ? S.tasks_in[t].job : add_job[t - T0]; };
  auto job_queue_of = [&](int32_t j) { return j < S.n_jobs ? S.jobs_in[j].queue : jq[j - S.n_jobs]; };
  // a live name among the session's (or the batch's) nodes, jobs or queues
  auto node_live = [&](const std::string& nm) {
    if (auto b = bnodes.find(nm); b != bnodes.end()) return b->second >= 0;
    const int32_t id = S.canon_of.find(S.strs, nm.c_str());
    if (id < 0) return false;
    auto a = S.node_of.find(S.canon[id]);
    if (a != S.node_of.end() && !ndead[a->second]) return true;
    auto b = S.pod_only_of.find(S.canon[id]);
    return b != S.pod_only_of.end() && !ndead[b->second];
  };
  auto uid_live = [&](const std::unordered_map<std::string, int32_t>& batch,
                      const std::unordered_map<int32_t, int32_t>& have, const std::vector<uint8_t>& gone,
                      const std::string& nm) {
    if (auto b = batch.find(nm); b != batch.end()) return b->second >= 0;
    const int32_t id = S.canon_of.find(S.strs, nm.c_str());
    if (id < 0) return false;
    auto a = have.find(S.canon[id]);
    return a != have.end() && !gone[a->second];
  };
  auto node_name_of = [&](int32_t nd) -> std::string {  // "" : a pod-only node without a known name
    if (nd >= S.n_nodes) {
      for (const auto& [nm, i] : bnodes)
        if (i == nd) return nm;
      return "";
    }
    if (S.nodes_in[nd].has_node) return S.strs[S.nodes_in[nd].name];
    return S.nil_name[nd] >= 0 ? S.strs[S.nil_name[nd]] : "";
  };
  auto spec_ok = [](const kbg_node_spec* sp) {
    if (!sp || !sp->name || sp->n_labels < 0 || sp->n_taints < 0 || (sp->n_labels && !sp->labels) ||
        (sp->n_taints && !sp->taints))
      return false;
    for (int32_t k = 0; k < 2 * sp->n_labels; ++k)
      if (!sp->labels[k]) return false;
    for (int32_t k = 0; k < 3 * sp->n_taints; ++k)
      if (!sp->taints[k]) return false;
    return true;
  };
  std::vector<uint8_t> node_set(S.n_nodes, 0);  // nodes an earlier NODE_SET of the batch gave a Node
  std::unordered_map<int32_t, std::string> set_names;  // ... and the name it gave
  // a pod event's node: a node with a Node (now or from an earlier NODE_SET of
  // the batch), or a pod-only node whose NodeName the session knows
  auto nil_named = [&](const kbg_event& e) {
    const int32_t nd = e.node;
    return nd < 0 || nd >= S.n_nodes || S.nodes_in[nd].has_node || node_set[nd] || S.nil_name[nd] >= 0 ||
           (e.node_name && e.node_name[0]);
  };
  for (int32_t i = 0; i < n; ++i) {
    const kbg_event& e = ev[i];
    switch (e.kind) {
      case KBG_EV_POD_UPDATE:
      case KBG_EV_POD_DELETE: {
        const int32_t t = e.task;
        if (t < 0 || t >= T || dead[t]) return fail(KBG_E_INVALID, "event task index");
        if (e.kind == KBG_EV_POD_UPDATE && (!status_ok(e.status) || e.node < -1 || e.node >= N))
          return fail(KBG_E_INVALID, "event status / node");
        if (structural) {
          const int32_t on = task_now(t).node;
          if (jdead[task_job(t)] || (on >= 0 && ndead[on]) || (e.kind == KBG_EV_POD_UPDATE && e.node >= 0 && ndead[e.node]))
            return fail(KBG_E_UNSUPPORTED, "a pod event after its job or its node left the session in the same "
                                           "batch: send it in the next update");
        }
        if (e.kind == KBG_EV_POD_UPDATE && !nil_named(e))
          return fail(KBG_E_UNSUPPORTED, "a pod event naming a node the cache knows only from pods outside the "
                                         "session jobs (the NodeName is unknown to the session): re-open");
        if (!holders) {
          if (e.kind == KBG_EV_POD_DELETE) dead[t] = 1;
          break;
        }
        Now c = task_now(t);
        bool found = false;
        if (c.node >= 0) {
          const int32_t h = holder(c.node, c.key);
          if (h == -3)
            return fail(KBG_E_UNSUPPORTED, "the pod key is held on the node by a pod outside the session jobs "
                                           "and the snapshot carried no node_pods (its resources are unknown): re-open");
          if (h >= 0 || h == -2) {  // the holder leaves the node (in_node_remove)
            hold[((int64_t)c.node << 32) | (uint32_t)c.key] = -1;
            found = true;
          }
        }
        if (e.kind == KBG_EV_POD_DELETE || (c.node >= 0 && !found)) {  // deleted, or updateTask stopped
          dead[t] = 1;
          break;
        }
        c.node = e.node;
        c.status = e.status;
        now[t] = c;
        if (c.node >= 0 && !terminated(c.status) && holder(c.node, c.key) == -1)
          hold[((int64_t)c.node << 32) | (uint32_t)c.key] = t;
        break;
      }
      case KBG_EV_POD_ADD: {
        if (e.job < 0 || e.job >= J || e.spec < -1 || e.spec >= (int32_t)S.specs_in.size() ||
            !status_ok(e.status) || e.node < -1 || e.node >= N || !e.uid || !e.pod_key)
          return fail(KBG_E_INVALID, "POD_ADD event");
        if (structural) {
          if (jdead[e.job]) return fail(KBG_E_INVALID, "POD_ADD into a job that left the session in the same batch");
          if (e.node >= 0 && ndead[e.node])
            return fail(KBG_E_UNSUPPORTED, "POD_ADD onto a node that left the session in the same batch");
          add_job.push_back(e.job);
        }
        if (!nil_named(e))
          return fail(KBG_E_UNSUPPORTED, "a pod event naming a node the cache knows only from pods outside the "
                                         "session jobs (the NodeName is unknown to the session): re-open");
        const int32_t t = T++;
        if (!holders) break;
        int32_t key;
        const int32_t known = S.canon_of.find(S.strs, e.pod_key);
        if (known >= 0) {
          key = known;
        } else {
          key = (int32_t)S.strs.size() + (int32_t)fresh.size();
          key = fresh.emplace(e.pod_key, key).first->second;
        }
        const Now c{e.node, e.status, key, e.spec};
        now[t] = c;
        if (c.node >= 0 && e.job >= S.n_jobs && holder(c.node, c.key) <= -2)
          return fail(KBG_E_UNSUPPORTED, "POD_ADD of a pod of a job new to the session whose key a pod outside the "
                                         "session jobs holds on the node (the pod predates its PodGroup): re-open");
        if (c.node >= 0 && !terminated(c.status) && holder(c.node, c.key) == -1)
          hold[((int64_t)c.node << 32) | (uint32_t)c.key] = t;
        break;
      }
      case KBG_EV_NODE_UPDATE:
        if (e.node < 0 || e.node >= S.n_nodes) return fail(KBG_E_INVALID, "event node index");
        if (structural && ndead[e.node]) return fail(KBG_E_INVALID, "NODE_UPDATE of a node deleted in the batch");
        if (!S.nodes_in[e.node].has_node && !node_set[e.node])
          return fail(KBG_E_UNSUPPORTED, "KBG_EV_NODE_UPDATE of a node the cache only knows from a pod: send "
                                         "KBG_EV_NODE_SET (its name, labels and taints)");
        break;
      case KBG_EV_NODE_SET: {
        // every input apply_node_set rejects, so the apply step can only fail as the reference panics
        const kbg_node_spec* sp = e.node_spec;
        if (e.node < 0 || e.node >= N || !sp || !sp->name || sp->n_labels < 0 || sp->n_taints < 0 ||
            (sp->n_labels && !sp->labels) || (sp->n_taints && !sp->taints) || (structural && ndead[e.node]))
          return fail(KBG_E_INVALID, "NODE_SET event");
        if (e.node >= S.n_nodes) {  // the Node of a node this batch added without one (a pod's NodeName made it)
          if (!spec_ok(sp)) return fail(KBG_E_INVALID, "NODE_SET event");
          auto named = set_names.find(e.node);
          if (named != set_names.end() && named->second != sp->name)
            return fail(KBG_E_INVALID, "NODE_SET: the node's name differs");
          set_names.emplace(e.node, sp->name);
          break;
        }
        for (int32_t k = 0; k < 2 * sp->n_labels; ++k)
          if (!sp->labels[k]) return fail(KBG_E_INVALID, "NODE_SET: null label string");
        for (int32_t k = 0; k < 3 * sp->n_taints; ++k)
          if (!sp->taints[k]) return fail(KBG_E_INVALID, "NODE_SET: null taint string");
        // the Node's name must stay the node's (its own, or the one an earlier NODE_SET of the batch gave it)
        const kbg_node& nd = S.nodes_in[e.node];
        auto named = set_names.find(e.node);
        if (named != set_names.end()) {
          if (named->second != sp->name) return fail(KBG_E_INVALID, "NODE_SET: the node's name differs");
        } else if (nd.has_node) {
          const int32_t id = S.canon_of.find(S.strs, sp->name);
          if (id < 0 || S.canon[id] != S.canon[nd.name]) return fail(KBG_E_INVALID, "NODE_SET: the node's name differs");
        }
        set_names.emplace(e.node, sp->name);
        thread_local std::vector<std::pair<Res, int32_t>> pods;
        if (!S.nodes_in[e.node].has_node && !node_set[e.node] && !node_pods_of(S, e.node, &pods))
          return fail(KBG_E_UNSUPPORTED, "NODE_SET of a node holding a pod outside the session jobs whose copy the "
                                         "snapshot did not carry (node_pods): re-open");
        node_set[e.node] = 1;
        break;
      }
      case KBG_EV_NODE_ADD: {
        // with a Node (NewNodeInfo(node)), or without one: the node a pod's NodeName makes (NewNodeInfo(nil))
        if ((e.node_spec && !spec_ok(e.node_spec)) || (!e.node_spec && !(e.node_name && e.node_name[0])))
          return fail(KBG_E_INVALID, "NODE_ADD event");
        const std::string nm = e.node_spec ? e.node_spec->name : e.node_name;
        if (nm.empty() || node_live(nm))
          return fail(KBG_E_INVALID, "NODE_ADD of a node name the session holds (its Node: KBG_EV_NODE_SET)");
        bnodes[nm] = N++;
        ndead.push_back(0);
        break;
      }
      case KBG_EV_NODE_DELETE: {
        if (e.node < 0 || e.node >= N || ndead[e.node]) return fail(KBG_E_INVALID, "NODE_DELETE event node");
        const std::string nm = node_name_of(e.node);
        if (!nm.empty()) bnodes[nm] = -1;
        ndead[e.node] = 1;
        break;
      }
      case KBG_EV_JOB_ADD: {
        if (!e.name || !e.name[0] || e.queue < 0 || e.queue >= Q || qdead[e.queue])
          return fail(KBG_E_INVALID, "JOB_ADD event (name, queue)");
        if (uid_live(bjobs, job_of_uid, jdead, e.name))
          return fail(KBG_E_INVALID, "JOB_ADD of a JobID the session holds");
        bjobs[e.name] = J++;
        jdead.push_back(0);
        jq.push_back(e.queue);
        break;
      }
      case KBG_EV_JOB_DELETE:
        if (e.job < 0 || e.job >= J || jdead[e.job]) return fail(KBG_E_INVALID, "JOB_DELETE event job");
        jdead[e.job] = 1;
        for (auto& [nm, j] : bjobs)
          if (j == e.job) j = -1;
        break;
      case KBG_EV_QUEUE_ADD: {
        if (!e.name || !e.name[0]) return fail(KBG_E_INVALID, "QUEUE_ADD event name");
        if (uid_live(bqueues, queue_of_uid, qdead, e.name))
          return fail(KBG_E_INVALID, "QUEUE_ADD of a queue the session holds");
        bqueues[e.name] = Q++;
        qdead.push_back(0);
        break;
      }
      case KBG_EV_QUEUE_DELETE: {
        if (e.queue < 0 || e.queue >= Q || qdead[e.queue]) return fail(KBG_E_INVALID, "QUEUE_DELETE event queue");
        qdead[e.queue] = 1;
        for (auto& [nm, q] : bqueues)
          if (q == e.queue) q = -1;
        for (int32_t j = 0; j < J; ++j)  // its jobs leave ssn.Jobs (cache.go:584-588)
          if (!jdead[j] && job_queue_of(j) == e.queue) {
            jdead[j] = 1;
            for (auto& [nm, k] : bjobs)
              if (k == j) k = -1;
          }
        break;
      }
      default:
        return fail(KBG_E_INVALID, "event kind");
    }
  }
  return KBG_OK;
}

// After a batch with structural events: the session's updated snapshot as
// cache.Snapshot() would marshal it (cache.go:549-597) — live nodes, queues
// and jobs in their order, the new ones last; each job's tasks in JobInfo.Tasks
// order; the pods of jobs that left stay on their nodes as pods outside the
// session jobs (with their node copies when every pod on a live node has one),
// the Running tasks of a job whose PodGroup was deleted join Others — opened
// as a new session that replaces this one; renum[] maps the old indices.
struct Rebuilt {  // a session's updated snapshot (pointing into the session's own arrays too) and its renumbering
  std::vector<int32_t> rq, rj, rn, rt;
  std::vector<kbg_queue> queues;
  std::vector<kbg_job> jobs;
  std::vector<kbg_task> tasks;
  std::vector<kbg_resource> others;
  std::vector<kbg_node> nodes;
  std::vector<int32_t> node_tasks, node_keys;
  std::vector<kbg_node_pod> node_pods;
  std::vector<kbg_host_port> ports;
  std::vector<const char*> strs;
  kbg_snapshot sn{};
};
kbg_status rebuild_snapshot(const Session& S, Rebuilt& B) {
  const int32_t N = S.n_nodes, J = S.n_jobs, Q = S.n_queues, T = S.n_tasks;
  auto gone = [](const std::vector<uint8_t>& v, int32_t i) { return (size_t)i < v.size() && v[i] != 0; };
  std::vector<int32_t>&rq = B.rq, &rj = B.rj, &rn = B.rn, &rt = B.rt;
  rq.assign(Q, -1);
  rj.assign(J, -1);
  rn.assign(N, -1);
  rt.assign(T, -1);
  std::vector<kbg_queue>& queues = B.queues;
  for (int32_t q = 0; q < Q; ++q)
    if (!gone(S.queue_dead, q)) {
      rq[q] = (int32_t)queues.size();
      queues.push_back(S.queues_in[q]);
    }
  std::vector<kbg_job>& jobs = B.jobs;
  std::vector<kbg_task>& tasks = B.tasks;
  std::vector<kbg_resource>& others = B.others;
  others = S.others_in;
  for (int32_t j = 0; j < J; ++j) {
    if (gone(S.job_dead, j)) {
      if (gone(S.job_to_others, j))  // PodGroup == nil: its Running tasks are Others
        for (const int32_t t : S.job_task_order[j])
          if (S.task_live[t] && S.tasks_in[t].status == KBG_RUNNING) others.push_back(S.tasks_in[t].resreq);
      continue;
    }
    kbg_job jb = S.jobs_in[j];
    jb.queue = rq[jb.queue];
    if (jb.queue < 0) return fail(KBG_E_INVALID, "internal: a live job of a deleted queue");
    rj[j] = (int32_t)jobs.size();
    jobs.push_back(jb);
    for (const int32_t t : S.job_task_order[j]) {
      if (!S.task_live[t]) continue;
      rt[t] = (int32_t)tasks.size();
      kbg_task k = S.tasks_in[t];
      k.job = rj[j];
      tasks.push_back(k);
    }
  }
  // the pod behind each key of a live node: a task (of a session job or of one
  // that left) or a pod outside the session jobs
  auto holder_task = [&](int32_t n, int32_t key) -> int32_t {
    for (const int32_t t : S.node_task_order[n])
      if (S.canon[S.tasks_in[t].pod_key] == key) return t;
    return -1;
  };
  bool copies = true;
  for (int32_t n = 0; n < N && copies; ++n) {
    if (gone(S.node_dead, n) || S.node_key_order[n].size() == S.node_task_order[n].size()) continue;
    for (const int32_t key : S.node_key_order[n]) {
      if (holder_task(n, key) >= 0) continue;
      auto it = S.outsiders.find(((int64_t)n << 32) | (uint32_t)key);
      if (it == S.outsiders.end() || it->second.status == 0) {
        copies = false;
        break;
      }
    }
  }
  std::vector<kbg_node>& nodes = B.nodes;
  std::vector<int32_t>&node_tasks = B.node_tasks, &node_keys = B.node_keys;
  std::vector<kbg_node_pod>& node_pods = B.node_pods;
  std::vector<kbg_host_port>& ports = B.ports;
  ports = S.ports_in;  // the specs' ports keep their offsets
  for (int32_t n = 0; n < N; ++n) {
    if (gone(S.node_dead, n)) continue;
    kbg_node nd = S.nodes_in[n];
    nd.task_off = (int32_t)node_tasks.size();
    for (const int32_t t : S.node_task_order[n])
      if (rt[t] >= 0) node_tasks.push_back(rt[t]);
    nd.task_len = (int32_t)node_tasks.size() - nd.task_off;
    nd.key_off = (int32_t)node_keys.size();
    node_keys.insert(node_keys.end(), S.node_key_order[n].begin(), S.node_key_order[n].end());
    nd.key_len = (int32_t)node_keys.size() - nd.key_off;
    if (nd.key_len != nd.num_tasks) return fail(KBG_E_INVALID, "internal: node pod keys != num_tasks");
    if (copies) {  // NodeInfo.Tasks order: each pod's ports after the one before (kbg_node_pod)
      nd.port_off = (int32_t)ports.size();
      for (const int32_t key : S.node_key_order[n]) {
        const int32_t u = holder_task(n, key);
        const size_t p0 = ports.size();
        if (u >= 0) {
          const int32_t sp = S.tasks_in[u].spec;
          if (sp >= 0)
            for (int32_t i = 0; i < S.specs_in[sp].port_len; ++i)
              if (S.ports_in[S.specs_in[sp].port_off + i].host_port > 0)
                ports.push_back(S.ports_in[S.specs_in[sp].port_off + i]);
          node_pods.push_back(kbg_node_pod{S.tasks_in[u].resreq, S.tasks_in[u].status, (int32_t)(ports.size() - p0)});
        } else {
          const Session::Outsider& o = S.outsiders.at(((int64_t)n << 32) | (uint32_t)key);
          ports.insert(ports.end(), o.ports.begin(), o.ports.end());
          node_pods.push_back(kbg_node_pod{o.req, o.status, (int32_t)o.ports.size()});
        }
      }
      nd.port_len = (int32_t)ports.size() - nd.port_off;
    }
    rn[n] = (int32_t)nodes.size();
    nodes.push_back(nd);
  }
  std::vector<const char*>& strs = B.strs;
  strs.resize(S.strs.size());
  for (size_t i = 0; i < strs.size(); ++i) strs[i] = S.strs[i].c_str();
  kbg_snapshot& sn = B.sn;
  sn.strings = strs.data();
  sn.n_strings = (int32_t)strs.size();
  sn.nodes = nodes.data(), sn.n_nodes = (int32_t)nodes.size();
  sn.jobs = jobs.data(), sn.n_jobs = (int32_t)jobs.size();
  sn.queues = queues.data(), sn.n_queues = (int32_t)queues.size();
  sn.tasks = tasks.data(), sn.n_tasks = (int32_t)tasks.size();
  sn.others = others.data(), sn.n_others = (int32_t)others.size();
  sn.specs = S.specs_in.data(), sn.n_specs = (int32_t)S.specs_in.size();
  sn.terms = S.terms_in.data(), sn.n_terms = (int32_t)S.terms_in.size();
  sn.reqs = S.reqs_in.data(), sn.n_reqs = (int32_t)S.reqs_in.size();
  sn.values = S.values_in.data(), sn.n_values = (int32_t)S.values_in.size();
  sn.tolerations = S.tols_in.data(), sn.n_tolerations = (int32_t)S.tols_in.size();
  sn.labels = S.labels_in.data(), sn.n_labels = (int32_t)(S.labels_in.size() / 2);
  sn.taints = S.taints_in.data(), sn.n_taints = (int32_t)S.taints_in.size();
  sn.selectors = S.selectors_in.data(), sn.n_selectors = (int32_t)(S.selectors_in.size() / 2);
  sn.plugins = S.plugins_in.data(), sn.n_plugins = (int32_t)S.plugins_in.size();
  sn.tier_sizes = S.tier_sizes_in.data(), sn.n_tiers = (int32_t)S.tier_sizes_in.size();
  sn.ports = ports.data(), sn.n_ports = (int32_t)ports.size();
  sn.node_tasks = node_tasks.data(), sn.n_node_tasks = (int32_t)node_tasks.size();
  sn.pod_terms = S.pod_terms_in.data(), sn.n_pod_terms = (int32_t)S.pod_terms_in.size();
  sn.pod_labels = S.pod_labels_in.data(), sn.n_pod_labels = (int32_t)(S.pod_labels_in.size() / 2);
  sn.node_pod_keys = node_keys.data(), sn.n_node_pod_keys = (int32_t)node_keys.size();
  sn.node_pods = copies ? node_pods.data() : nullptr;
  sn.n_node_pods = copies ? (int32_t)node_pods.size() : 0;
  return KBG_OK;
}

kbg_status restructure(Session& S) {
  Rebuilt B;
  if (kbg_status st = rebuild_snapshot(S, B); st != KBG_OK) return st;
  const int32_t N = S.n_nodes;
  const std::vector<int32_t>& rn = B.rn;
  kbg_options o = S.opts;
  o.device = S.device;
  std::unique_ptr<Session> R(new Session());
  // the string table moves over as it is (the vector's elements keep their
  // addresses, so the snapshot's string pointers stay valid)
  R->strs = std::move(S.strs);
  R->canon = std::move(S.canon);
  R->canon_of = std::move(S.canon_of);
  R->adopt_strings = true;
  kbg_status st = open_session(*R, &B.sn, &o, nullptr);
  if (st != KBG_OK) {
    free_device(*R);
    return st;
  }
  // a node the cache knows only from pods keeps the NodeName that made it even
  // when no session task carries it any more (the snapshot has no field for
  // it: its Name is ""): pod events naming it find it (sc.Nodes[NodeName])
  std::unordered_map<int32_t, int32_t> named;
  for (int32_t n = 0; n < N; ++n) {
    const int32_t m = rn[n];
    if (m < 0 || S.nodes_in[n].has_node || S.nil_name[n] < 0 || R->nil_name[m] >= 0) continue;
    const int32_t nm = R->canon[S.nil_name[n]];
    R->nil_name[m] = nm;
    R->pod_only_of.emplace(nm, m);
    named.emplace(nm, m);
  }
  if (!named.empty())
    for (int32_t t = 0; t < R->n_tasks; ++t)
      if (R->task_cnode[t] < 0)
        if (auto it = named.find(R->canon[R->tasks_in[t].node_name]); it != named.end()) R->task_cnode[t] = it->second;
  R->updates = S.updates;
  R->rebuilds = S.rebuilds + 1;
  free_device(S);
  S = std::move(*R);
  S.renum[KBG_RENUM_TASKS] = std::move(B.rt);
  S.renum[KBG_RENUM_NODES] = std::move(B.rn);
  S.renum[KBG_RENUM_JOBS] = std::move(B.rj);
  S.renum[KBG_RENUM_QUEUES] = std::move(B.rq);
  return KBG_OK;
}

kbg_status session_update(Session& S, const kbg_event* ev, int32_t n) {
  const auto t0 = std::chrono::steady_clock::now();
  for (auto& r : S.renum) r.clear();
  bool structural = false;
  for (int32_t i = 0; i < n; ++i) structural |= ev[i].kind >= KBG_EV_NODE_ADD;
  if (structural) {
    S.node_dead.assign(S.n_nodes, 0);
    S.job_dead.assign(S.n_jobs, 0);
    S.job_to_others.assign(S.n_jobs, 0);
    S.queue_dead.assign(S.n_queues, 0);
  }
  if (n < 0 || (n > 0 && !ev)) return fail(KBG_E_INVALID, "events");
  // the cycle state goes back to "just opened"
  S.allocated = S.backfilled = S.reclaimed = S.preempted = S.cycle_started = false;
  static const bool prof = getenv("KBG_PROFILE_OPEN") != nullptr;
  auto tl = t0;
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[kbg update] %-20s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - tl).count());
    tl = now;
  };
  UpdateCtx U;
  U.seen.assign(S.n_nodes, 0);
  uint64_t kc[5] = {0, 0, 0, 0, 0}, kn[5] = {0, 0, 0, 0, 0};
  // An event touches a handful of rows of task-, node- and job-indexed state
  // spread over the whole session (cache misses, not work): the rows of the
  // events ahead are requested before they are applied, in three hops (the
  // task's row; what it names — its job's and nodes' list headers, its key;
  // then the lists themselves and the key's count), each hop's addresses
  // read from rows the hop before requested. Prefetches only; the order of
  // application is unchanged.
  constexpr int32_t kFar = 24, kMid = 12, kNear = 4;
  auto task_of = [&](const kbg_event& e) -> int32_t {
    const bool pod = e.kind == KBG_EV_POD_UPDATE || e.kind == KBG_EV_POD_DELETE;
    return pod && e.task >= 0 && e.task < S.n_tasks ? e.task : -1;
  };
  auto job_of_add = [&](const kbg_event& e) -> int32_t {
    return e.kind == KBG_EV_POD_ADD && e.job >= 0 && e.job < S.n_jobs ? e.job : -1;
  };
  auto node_ok = [&](int32_t nd) { return nd >= 0 && nd < S.n_nodes; };
  auto ahead_far = [&](const kbg_event& e) {
    if (const int32_t t = task_of(e); t >= 0) {
      __builtin_prefetch(&S.tasks_in[t]);
      __builtin_prefetch(&S.task_node[t]);
      __builtin_prefetch(&S.task_live[t]);
      __builtin_prefetch(&S.treq[t]);
    } else if (const int32_t j = job_of_add(e); j >= 0) {
      __builtin_prefetch(&S.job_task_order[j]);
    }
    if (node_ok(e.node)) {
      __builtin_prefetch(&S.nodes_in[e.node]);
      __builtin_prefetch(&S.node_key_order[e.node]);
      __builtin_prefetch(&S.node_task_order[e.node]);
    }
  };
  // a new pod's key: hashed here, its index slot requested, the hash kept
  // for the apply (events at least kMid ahead of the first)
  constexpr int32_t kRing = 32;
  static_assert(kRing > kMid, "the ring holds the hashes between the mid hop and the apply");
  uint64_t key_hash[kRing];
  auto ahead_mid = [&](const kbg_event& e, int32_t at) {
    if (e.kind == KBG_EV_POD_ADD && e.pod_key) {
      const uint64_t h = kbg::StrIndex::hash(std::string_view(e.pod_key));
      key_hash[at % kRing] = h;
      S.canon_of.prefetch(h);
    }
    if (const int32_t t = task_of(e); t >= 0) {
      const kbg_task& k = S.tasks_in[t];
      __builtin_prefetch(&S.job_task_order[k.job]);
      __builtin_prefetch(&S.canon[k.pod_key]);
      const int32_t on = S.task_node[t];  // the node the task leaves
      if (node_ok(on)) {
        __builtin_prefetch(&S.nodes_in[on]);
        __builtin_prefetch(&S.node_key_order[on]);
        __builtin_prefetch(&S.node_task_order[on]);
      }
    } else if (const int32_t j = job_of_add(e); j >= 0) {
      __builtin_prefetch(S.job_task_order[j].data() + S.job_task_order[j].size());
    }
    if (node_ok(e.node)) {
      __builtin_prefetch(S.node_key_order[e.node].data());
      __builtin_prefetch(S.node_task_order[e.node].data() + S.node_task_order[e.node].size());
    }
  };
  auto ahead_near = [&](const kbg_event& e) {
    if (const int32_t t = task_of(e); t >= 0) {
      const kbg_task& k = S.tasks_in[t];
      __builtin_prefetch(S.job_task_order[k.job].data());
      const int32_t key = S.canon[k.pod_key];
      if ((size_t)key < S.kc_node.size()) __builtin_prefetch(&S.kc_node[key]);
      const int32_t on = S.task_node[t];
      if (node_ok(on)) {
        __builtin_prefetch(S.node_key_order[on].data());
        __builtin_prefetch(S.node_task_order[on].data());
      }
    }
  };
  S.jmove_defer = (int64_t)n * 8 > (int64_t)S.n_tasks;
  for (int32_t i = 0; i < n; ++i) {
    if (i + kFar < n) ahead_far(ev[i + kFar]);
    if (i + kMid < n) ahead_mid(ev[i + kMid], i + kMid);
    if (i + kNear < n) ahead_near(ev[i + kNear]);
    const uint64_t c0 = prof ? __builtin_readcyclecounter() : 0;
    const bool hashed = i >= kMid && ev[i].kind == KBG_EV_POD_ADD && ev[i].pod_key;
    kbg_status st = apply_event(S, U, ev[i], hashed ? &key_hash[i % kRing] : nullptr);
    if (st != KBG_OK) return st;
    if (prof) {
      const int k = std::min(4, std::max(0, (int)ev[i].kind));
      kc[k] += __builtin_readcyclecounter() - c0;
      kn[k]++;
    }
  }
  finish_job_lists(S);
  if (prof)
    for (int k = 0; k < 5; ++k)
      if (kn[k]) fprintf(stderr, "[kbg update] event kind %d: %llu, %.0f cycles each\n", k, (unsigned long long)kn[k],
                         (double)kc[k] / kn[k]);
  phase("events");
  if (structural) {  // the sets of nodes, jobs or queues changed: the session is rebuilt from its snapshot
    if (kbg_status st = restructure(S); st != KBG_OK) return st;
    phase("restructure");
    S.updates++;
    S.update_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    S.stats.update_ms = S.update_ms;
    S.stats.update_rebuilds = S.rebuilds;
    return KBG_OK;
  }
  S.vt_stale = true;
  S.vc.valid = false;
  const bool had_masks = S.has_ports || S.has_aff;
  kbg_status st = KBG_OK;
  int outcome = DERIVE_OK;
  S.upd_nodes = U.nodes;
  S.upd_nodes_valid = true;
  if (!U.rebuild) st = derive_host(S, nullptr, &outcome);
  S.upd_nodes_valid = false;
  if (st != KBG_OK) return st;
  phase("derive");
  if (U.rebuild || outcome == DERIVE_REBUILD) {
    // new static classes or node flags: recompile and rebuild the device tables
    free_device(S);
    const int64_t rebuilds = S.rebuilds + 1;
    S.stats = kbg_stats{};
    if ((st = build(S, S.comm, [](const char*) {})) != KBG_OK) return st;
    S.rebuilds = rebuilds;
  } else {
    HIP_TRY(hipSetDevice(S.device));
    // the changed node rows, into the live table and the reset copy
    for (size_t i = 0; i < U.nodes.size();) {
      if ((st = stage_acquire(S)) != KBG_OK) return st;
      int32_t cnt = 0;
      for (; i < U.nodes.size() && cnt < S.K; ++i) {
        const int32_t nd = U.nodes[i];
        if (nd < S.tab_lo || nd >= S.tab_lo + S.tab_n) continue;
        kbg::NodeDelta& d = S.h_deltas[cnt++];
        d.node = nd - S.tab_lo;
        device_row(S, nd, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
      }
      if (cnt == 0) break;
      HIP_TRY(kbg::launch_apply(S.d_nodes0, S.h_deltas_dev, cnt, S.stream));  // read in place
      if ((st = stage_release(S)) != KBG_OK) return st;
    }
    // the live table restarts from the updated snapshot: the rows an action
    // committed since the last reset are stale whether or not an event touched them
    if ((st = copy_soa(S, S.d_nodes, S.d_nodes0)) != KBG_OK) return st;
    S.idle = S.idle0;
    S.rel = S.rel0;
    S.ntasks = S.ntasks0;
    S.node_keys = S.node_keys0;
    S.port_hold.clear();
    S.port_gone.clear();
    S.outsider_gone.clear();
    S.key_holder.clear();
    // host ports / pod affinity live in the class masks: refold them
    if (had_masks || S.has_ports || S.has_aff) {
      S.h_class_mask = S.h_class_mask_static;
      setup_host_ports(S);
      setup_affinity(S);
      S.mask_dirty.clear();
      std::fill(S.mask_dirty_flag.begin(), S.mask_dirty_flag.end(), 0);
      HIP_TRY(hipMemcpy(S.d_class_mask, S.h_class_mask.data(), S.h_class_mask.size() * 8, hipMemcpyHostToDevice));
    }
    S.h_class_mask0 = S.h_class_mask;
    S.stats.int_scan = S.int_mode ? 1 : 0;
  }
  phase("device rows");
  S.updates++;
  S.update_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  S.stats.update_ms = S.update_ms;
  S.stats.update_rebuilds = S.rebuilds;
  return KBG_OK;
}

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

// ============================================================ wire format
// kbgpu.h "Snapshot wire format". Host-only: no device is touched.
struct kbg_snapshot_blob {
  std::vector<std::string> strs;
  std::vector<const char*> ptrs;
  std::vector<std::vector<uint8_t>> arrays;
  kbg_snapshot snap{};
};

namespace {

constexpr char kSnapMagic[4] = {'K', 'B', 'G', 'S'};
constexpr int kSnapCounts = 22;

// Layout word of the wire format: a hash of the element size of every array
// (FNV-1a over the sizes). Blobs stay readable across ABI bumps that leave the
// snapshot structs unchanged; a struct change makes old blobs fail loudly.
uint32_t snapshot_layout() {
  const size_t sizes[] = {sizeof(kbg_node), sizeof(kbg_job), sizeof(kbg_queue), sizeof(kbg_task),
                          sizeof(kbg_resource), sizeof(kbg_spec), sizeof(kbg_term), sizeof(kbg_requirement),
                          sizeof(kbg_toleration), sizeof(kbg_taint), sizeof(kbg_plugin_option),
                          sizeof(kbg_host_port), sizeof(kbg_pod_term), sizeof(kbg_node_pod)};
  uint32_t h = 2166136261u;
  for (size_t v : sizes) {
    h ^= (uint32_t)v;
    h *= 16777619u;
  }
  return h;
}

// The arrays of a kbg_snapshot in declaration order: (pointer slot, count
// slot, element size, elements per count).
template <class F>
void for_each_array(kbg_snapshot& s, F f) {
  f((const void**)&s.nodes, &s.n_nodes, sizeof(kbg_node), 1);
  f((const void**)&s.jobs, &s.n_jobs, sizeof(kbg_job), 1);
  f((const void**)&s.queues, &s.n_queues, sizeof(kbg_queue), 1);
  f((const void**)&s.tasks, &s.n_tasks, sizeof(kbg_task), 1);
  f((const void**)&s.others, &s.n_others, sizeof(kbg_resource), 1);
  f((const void**)&s.specs, &s.n_specs, sizeof(kbg_spec), 1);
  f((const void**)&s.terms, &s.n_terms, sizeof(kbg_term), 1);
  f((const void**)&s.reqs, &s.n_reqs, sizeof(kbg_requirement), 1);
  f((const void**)&s.values, &s.n_values, sizeof(int32_t), 1);
  f((const void**)&s.tolerations, &s.n_tolerations, sizeof(kbg_toleration), 1);
  f((const void**)&s.labels, &s.n_labels, sizeof(int32_t), 2);
  f((const void**)&s.taints, &s.n_taints, sizeof(kbg_taint), 1);
  f((const void**)&s.selectors, &s.n_selectors, sizeof(int32_t), 2);
  f((const void**)&s.plugins, &s.n_plugins, sizeof(kbg_plugin_option), 1);
  f((const void**)&s.tier_sizes, &s.n_tiers, sizeof(int32_t), 1);
  f((const void**)&s.ports, &s.n_ports, sizeof(kbg_host_port), 1);
  f((const void**)&s.node_tasks, &s.n_node_tasks, sizeof(int32_t), 1);
  f((const void**)&s.pod_terms, &s.n_pod_terms, sizeof(kbg_pod_term), 1);
  f((const void**)&s.pod_labels, &s.n_pod_labels, sizeof(int32_t), 2);
  f((const void**)&s.node_pod_keys, &s.n_node_pod_keys, sizeof(int32_t), 1);
  f((const void**)&s.node_pods, &s.n_node_pods, sizeof(kbg_node_pod), 1);
}

struct Writer {
  uint8_t* out;
  int64_t cap, n = 0;
  void put(const void* p, size_t len) {
    if (out && n + (int64_t)len <= cap) std::memcpy(out + n, p, len);
    n += (int64_t)len;
  }
  void u32(uint32_t v) { put(&v, 4); }
};

kbg_status encode(const kbg_snapshot* snap, Writer& w) {
  kbg_status st = validate(snap);
  if (st != KBG_OK) return st;
  kbg_snapshot s = *snap;
  w.put(kSnapMagic, 4);
  w.u32(KBG_SNAPSHOT_FORMAT);
  w.u32(snapshot_layout());
  w.u32((uint32_t)s.n_strings);
  for_each_array(s, [&](const void**, int32_t* cnt, size_t, int) { w.u32((uint32_t)*cnt); });
  for (int32_t i = 0; i < s.n_strings; ++i) {
    const size_t len = std::strlen(s.strings[i]);
    w.u32((uint32_t)len);
    w.put(s.strings[i], len);
  }
  for_each_array(s, [&](const void** ptr, int32_t* cnt, size_t size, int per) {
    if (*cnt > 0) w.put(*ptr, (size_t)*cnt * per * size);
  });
  return KBG_OK;
}

}  // namespace

extern "C" {

kbg_status kbg_snapshot_encode(const kbg_snapshot* snap, uint8_t* out, int64_t cap, int64_t* n_out) {
  Writer w{out, out ? cap : 0};
  kbg_status st = encode(snap, w);
  if (st != KBG_OK) return st;
  if (n_out) *n_out = w.n;
  if (out && w.n > cap) return fail(KBG_E_CAPACITY, "snapshot buffer too small: need " + std::to_string(w.n));
  return KBG_OK;
}

static kbg_status snapshot_decode(const uint8_t* data, int64_t n, kbg_snapshot_blob** out) {
  int64_t pos = 0;
  auto take = [&](void* dst, int64_t len) {
    if (len < 0 || len > n - pos) return false;
    if (len > 0) std::memcpy(dst, data + pos, (size_t)len);
    pos += len;
    return true;
  };
  char magic[4];
  uint32_t fmt = 0, layout = 0, nstr = 0;
  if (!take(magic, 4) || std::memcmp(magic, kSnapMagic, 4) != 0) return fail(KBG_E_INVALID, "not a kbg snapshot");
  if (!take(&fmt, 4) || !take(&layout, 4) || fmt != KBG_SNAPSHOT_FORMAT || layout != snapshot_layout())
    return fail(KBG_E_INVALID, "snapshot format " + std::to_string(fmt) + " / layout " + std::to_string(layout) +
                                   " (this library: " + std::to_string(KBG_SNAPSHOT_FORMAT) + " / " +
                                   std::to_string(snapshot_layout()) + ")");
  if (!take(&nstr, 4) || nstr > (uint32_t)INT32_MAX) return fail(KBG_E_INVALID, "truncated snapshot header");
  auto blob = std::make_unique<kbg_snapshot_blob>();
  kbg_snapshot& s = blob->snap;
  s.n_strings = (int32_t)nstr;
  bool ok = true;
  int64_t array_bytes = 0;  // what the counts promise, checked against the input before any allocation
  for_each_array(s, [&](const void**, int32_t* cnt, size_t size, int per) {
    uint32_t v = 0;
    ok = ok && take(&v, 4) && v <= (uint32_t)INT32_MAX;
    *cnt = (int32_t)v;
    array_bytes += (int64_t)v * per * (int64_t)size;
  });
  if (!ok) return fail(KBG_E_INVALID, "truncated snapshot header");
  // every string takes at least its 4-byte length; every array its raw bytes
  if ((int64_t)nstr * 4 > n - pos || array_bytes > n - pos - (int64_t)nstr * 4)
    return fail(KBG_E_INVALID, "snapshot counts exceed the input");
  blob->strs.resize(nstr);
  for (uint32_t i = 0; i < nstr; ++i) {
    uint32_t len = 0;
    if (!take(&len, 4) || (int64_t)len > n - pos) return fail(KBG_E_INVALID, "truncated snapshot strings");
    blob->strs[i].assign((const char*)data + pos, len);
    pos += len;
  }
  blob->ptrs.resize(nstr);
  for (uint32_t i = 0; i < nstr; ++i) blob->ptrs[i] = blob->strs[i].c_str();
  s.strings = blob->ptrs.data();
  if (array_bytes != n - pos) return fail(KBG_E_INVALID, "snapshot arrays do not match the input length");
  blob->arrays.reserve(kSnapCounts);
  for_each_array(s, [&](const void** ptr, int32_t* cnt, size_t size, int per) {
    const int64_t len = (int64_t)*cnt * per * (int64_t)size;
    blob->arrays.emplace_back((size_t)len);
    std::vector<uint8_t>& a = blob->arrays.back();
    ok = ok && take(a.data(), len);
    *ptr = *cnt > 0 ? a.data() : nullptr;
  });
  if (!ok) return fail(KBG_E_INVALID, "truncated snapshot arrays");
  if (pos != n) return fail(KBG_E_INVALID, "trailing bytes after the snapshot");
  kbg_status st = validate(&s);
  if (st != KBG_OK) return st;
  *out = blob.release();
  return KBG_OK;
}

kbg_status kbg_snapshot_decode(const uint8_t* data, int64_t n, kbg_snapshot_blob** out) {
  if (!data || !out || n < 0) return fail(KBG_E_INVALID, "null argument");
  *out = nullptr;
  try {
    return snapshot_decode(data, n, out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::length_error&) {
    return fail(KBG_E_INVALID, "snapshot counts exceed the input");
  }
}

kbg_status kbg_snapshot_save(const kbg_snapshot* snap, const char* path) {
  if (!path) return fail(KBG_E_INVALID, "null path");
  int64_t n = 0;
  kbg_status st = kbg_snapshot_encode(snap, nullptr, 0, &n);
  if (st != KBG_OK) return st;
  std::vector<uint8_t> buf((size_t)n);
  if ((st = kbg_snapshot_encode(snap, buf.data(), n, &n)) != KBG_OK) return st;
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(KBG_E_INVALID, std::string("cannot open ") + path);
  const bool wrote = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
  if (std::fclose(f) != 0 || !wrote) return fail(KBG_E_INVALID, std::string("cannot write ") + path);
  return KBG_OK;
}

kbg_status kbg_snapshot_load(const char* path, kbg_snapshot_blob** out) {
  if (!path || !out) return fail(KBG_E_INVALID, "null argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(KBG_E_INVALID, std::string("cannot open ") + path);
  std::vector<uint8_t> buf;
  uint8_t chunk[1 << 16];
  size_t got;
  while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
  std::fclose(f);
  return kbg_snapshot_decode(buf.data(), (int64_t)buf.size(), out);
}

const kbg_snapshot* kbg_snapshot_blob_get(const kbg_snapshot_blob* b) { return b ? &b->snap : nullptr; }

void kbg_snapshot_blob_free(kbg_snapshot_blob* b) { delete b; }

}  // extern "C"
