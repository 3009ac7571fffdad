// Developer tool (not part of libkbgpu.so): times the host ordering engine of
// the allocate path alone, on a CPU-only machine. It includes the session
// source to reach the engine, runs open_session (which builds all host state
// and then stops at the missing device) and drives the predictor with every
// outcome = placed, i.e. the engine work of a cycle where everything fits.
#include <barrier>
#include <cmath>
#include <random>

#include "../csrc/kbg_session.cpp"

extern "C" double kbg_tool_engine_ns_per_step(const kbg_snapshot* snap, const kbg_options* o, int32_t reps,
                                              int64_t* steps_out, double* checksum, int32_t profile) {
  kbg::Session S;
  open_session(S, snap, o, nullptr);  // returns KBG_E_HIP on a machine without a device; host state is complete
  if (S.init.qlen == 0) return -1.0;
  double best = 1e30;
  int64_t steps = 0;
  uint64_t sum = 0;
  EngineProfile prof;
  for (int32_t r = 0; r < reps; ++r) {
    Engine E = S.init;
    prof = EngineProfile{};
    Ops ops{S, E, profile ? &prof : nullptr};
    steps = 0;
    sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const int32_t t = ops.next_task();
      if (t < 0) break;
      ops.apply(t, true);
      sum = (sum * 1000003u) ^ (uint64_t)t;  // order-sensitive
      ++steps;
    }
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, ns / std::max<int64_t>(1, steps));
  }
  if (steps_out) *steps_out = steps;
  if (checksum) *checksum = (double)(sum >> 11);
  if (profile && prof.steps)
    fprintf(stderr, "cycles/step: qpop %.1f apply %.1f jfix %.1f qpush %.1f\n", (double)prof.qpop / prof.steps,
            (double)prof.apply / prof.steps, (double)prof.jtop / prof.steps, (double)prof.qpush / prof.steps);
  return best;
}

// Host side of kbg_session_update without a device: opens the snapshot's host
// state, applies the events to the inputs and re-derives; returns the node
// rows (Idle, Releasing, task count) and the pending candidates in job order,
// for comparison with a fresh snapshot of the updated cache (CPU test).
extern "C" int32_t kbg_tool_update_nodes(const kbg_snapshot* snap, const kbg_options* o, const kbg_event* ev,
                                         int32_t n, double* idle, double* rel, int32_t* ntasks, int32_t* pend,
                                         int32_t* n_pend) {
  kbg::Session S;
  const auto i0 = std::chrono::steady_clock::now();
  if (ingest(S, snap, o) != KBG_OK) return -1;
  const auto i1 = std::chrono::steady_clock::now();
  kbg::StaticHost sh;
  int outcome;
  if (derive_host(S, &sh, &outcome) != KBG_OK) return -2;
  if (getenv("KBG_TOOL_TIME"))
    fprintf(stderr, "[tool] open: ingest %.3f ms, derive %.3f ms\n",
            std::chrono::duration<double, std::milli>(i1 - i0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - i1).count());
  S.n_classes = sh.n_classes;
  UpdateCtx U;
  U.seen.assign(S.n_nodes, 0);
  const auto t0 = std::chrono::steady_clock::now();
  S.jmove_defer = (int64_t)n * 8 > (int64_t)S.n_tasks;
  reserve_for_events(S, ev, n);  // as session_update
  for (int32_t i = 0; i < n; ++i)
    if (apply_event(S, U, ev[i], nullptr) != KBG_OK) return -3;
  finish_job_lists(S);
  const auto t1 = std::chrono::steady_clock::now();
  S.upd_nodes = U.nodes;  // as kbg_session_update hands them to the derive
  S.upd_nodes_valid = true;
  if (derive_host(S, nullptr, &outcome) != KBG_OK) return -4;
  if (getenv("KBG_TOOL_TIME"))
    fprintf(stderr, "[tool] %d events: apply %.3f ms, derive %.3f ms\n", n,
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  for (int32_t k = 0; k < S.n_nodes; ++k) {
    idle[3 * k] = S.idle[k].c;
    idle[3 * k + 1] = S.idle[k].m;
    idle[3 * k + 2] = S.idle[k].g;
    rel[3 * k] = S.rel[k].c;
    rel[3 * k + 1] = S.rel[k].m;
    rel[3 * k + 2] = S.rel[k].g;
    ntasks[k] = S.ntasks[k];
  }
  *n_pend = (int32_t)S.pend_all.size();
  std::copy(S.pend_all.begin(), S.pend_all.end(), pend);
  return outcome;
}

// Structural events (kbg_session_update KBG_EV_NODE_ADD ... QUEUE_DELETE)
// without a device: the session's host state opened from the snapshot, the
// batch prechecked and applied as the library does, then the updated snapshot
// the library would open from (rebuild_snapshot), encoded in the wire format
// into out (KBG_E_CAPACITY with *n_out = the size needed), and the four
// renumbering maps (tasks, nodes, jobs, queues; each renum[k] sized by the
// caller to the old count plus the batch's additions). Returns the precheck /
// apply status, or 100 + the status of opening the snapshot's host state (a
// session on it would not open: e.g. proportion's panic at OnSessionOpen).
// Test infrastructure only (tests/test_update_structural_host.py).
extern "C" int32_t kbg_tool_structural(const kbg_snapshot* snap, const kbg_options* o, const kbg_event* ev, int32_t n,
                                       uint8_t* out, int64_t cap, int64_t* n_out, int32_t* renum[4], int32_t lens[4]) {
  kbg::Session S;
  if (kbg_status st = ingest(S, snap, o); st != KBG_OK) return 100 + st;
  kbg::StaticHost sh;
  int outcome;
  if (kbg_status st = derive_host(S, &sh, &outcome); st != KBG_OK) return 100 + st;
  S.n_classes = sh.n_classes;
  if (kbg_status st = update_precheck(S, ev, n); st != KBG_OK) return st;
  S.node_dead.assign(S.n_nodes, 0);
  S.job_dead.assign(S.n_jobs, 0);
  S.job_to_others.assign(S.n_jobs, 0);
  S.queue_dead.assign(S.n_queues, 0);
  UpdateCtx U;
  U.seen.assign(S.n_nodes, 0);
  S.jmove_defer = (int64_t)n * 8 > (int64_t)S.n_tasks;
  for (int32_t i = 0; i < n; ++i)
    if (kbg_status st = apply_event(S, U, ev[i], nullptr); st != KBG_OK) return st;
  finish_job_lists(S);
  Rebuilt B;
  if (kbg_status st = rebuild_snapshot(S, B); st != KBG_OK) return st;
  const std::vector<int32_t>* maps[4] = {&B.rt, &B.rn, &B.rj, &B.rq};
  for (int k = 0; k < 4; ++k) {
    if ((int32_t)maps[k]->size() > lens[k]) return KBG_E_CAPACITY;
    lens[k] = (int32_t)maps[k]->size();
    std::copy(maps[k]->begin(), maps[k]->end(), renum[k]);
  }
  return kbg_snapshot_encode(&B.sn, out, cap, n_out);
}

// ---------------------------------------------------------------------------
// The owner-resolve protocol of a sharded allocate (allocate_sharded) without a
// device: each rank's host state is opened from the snapshot, the class masks
// come from a host evaluation of the static predicate programs (the same
// programs kbg_mask_kernel runs), the scan of the rank's own rows is a host
// walk of its mirror, and the collectives are either an in-process transport
// (R threads, kbg_tool_sharded_allocate_local) or a caller's callback
// (kbg_tool_sharded_allocate_rank: one rank per process, e.g. torch.distributed
// gloo in tests/test_shard_protocol.py). Test infrastructure only.
namespace {

bool host_req(const kbg::StaticHost& sh, const kbg::ReqProg& r, int32_t N, int32_t node) {
  switch (r.kind) {
    case kbg::REQ_FALSE: return false;
    case kbg::REQ_TRUE: return true;
    case kbg::REQ_ALL:
    case kbg::REQ_ANY:
    case kbg::REQ_NONE: {
      bool any = false, all = true;
      for (int32_t w = 0; w < sh.label_words; ++w) {
        const uint64_t m = sh.mask_pool[r.mask_off + w];
        const uint64_t b = sh.label_bits[(size_t)w * N + node] & m;
        any |= b != 0;
        all &= b == m;
      }
      return r.kind == kbg::REQ_ALL ? all : (r.kind == kbg::REQ_ANY ? any : !any);
    }
    case kbg::REQ_GT:
    case kbg::REQ_LT: {
      const size_t k = (size_t)r.col * N + node;
      if (!sh.num_ok[k]) return false;
      return r.kind == kbg::REQ_GT ? sh.num_vals[k] > r.value : sh.num_vals[k] < r.value;
    }
    case kbg::REQ_NAME_EQ: return (int64_t)sh.name_id[node] == r.value;
    case kbg::REQ_NAME_NE: return (int64_t)sh.name_id[node] != r.value;
  }
  return false;
}

void host_class_mask(Session& S, const kbg::StaticHost& sh) {
  const int32_t N = S.n_nodes;
  S.h_class_mask.assign((size_t)S.n_classes * S.W, 0);
  for (int32_t c = 0; c < S.n_classes; ++c) {
    const kbg::ClassProg& cp = sh.classes[c];
    for (int32_t n = 0; n < N; ++n) {
      const uint8_t fl = sh.node_flags[n];
      bool ok;
      if (cp.always || (fl & kbg::NF_NIL)) ok = true;
      else if (fl & (kbg::NF_UNSCHED | kbg::NF_DEAD)) ok = false;
      else {
        ok = cp.sel_req < 0 || host_req(sh, sh.reqs[cp.sel_req], N, n);
        if (ok && cp.has_affinity) {
          bool any_term = false;
          for (int32_t i = 0; i < cp.term_len && !any_term; ++i) {
            const kbg::TermProg& tp = sh.terms[cp.term_off + i];
            bool all = true;
            for (int32_t j = 0; j < tp.req_len && all; ++j) all = host_req(sh, sh.reqs[tp.req_off + j], N, n);
            any_term = all;
          }
          ok = any_term;
        }
        for (int32_t w = 0; ok && w < sh.taint_words; ++w)
          if (sh.taint_bits[(size_t)w * N + n] & ~sh.tol_pool[cp.tol_off + w]) ok = false;
      }
      if (ok) S.h_class_mask[(size_t)c * S.W + (n >> 6)] |= 1ull << (n & 63);
    }
  }
}

// Host state of rank `rank` of R (R = 1: the whole table), as build() leaves it
// minus the device.
kbg_status host_open(Session& S, const kbg_snapshot* snap, const kbg_options* o, int32_t R, int32_t rank) {
  kbg_status st = ingest(S, snap, o);
  if (st != KBG_OK) return st;
  kbg::StaticHost sh;
  int outcome;
  if ((st = derive_host(S, &sh, &outcome)) != KBG_OK) return st;
  const int32_t N = S.n_nodes;
  S.R = R;
  S.shard = rank;
  S.Wl = std::max(1, (S.W + R - 1) / R);
  S.tab_lo = std::min(N, rank * S.Wl * 64);
  S.tab_n = std::min(N, (rank + 1) * S.Wl * 64) - S.tab_lo;
  S.n_shapes_cap = std::max(S.n_shapes, 64);
  S.cand_cap = S.opts.full_scan ? (int64_t)S.K * S.M + (int64_t)std::min(S.K, S.n_shapes_cap) * (kFullScanGrow + S.M)
                                : (int64_t)S.K * (kGroupSlack + 1);
  const size_t up_cap = up_bytes_for(S.K);
  const size_t down_cap = (size_t)S.K + (size_t)S.cand_cap;  // the host scan's count + candidate lists
  for (kbg::Stage& g : S.stages) {
    g.h_up = (char*)std::malloc(up_cap);
    g.h_down = (uint32_t*)std::malloc(down_cap * 4);
  }
  host_class_mask(S, sh);
  S.h_class_mask_static = S.h_class_mask;
  setup_host_ports(S);
  setup_affinity(S);
  S.h_class_mask0 = S.h_class_mask;
  return KBG_OK;
}

void host_close(Session& S) {
  for (kbg::Stage& g : S.stages) {
    std::free(g.h_up);
    std::free(g.h_down);
    g.h_up = nullptr;
    g.h_down = nullptr;
  }
}

// first-fit candidates of each row over this rank's rows, from the mirror:
// what kbg_scan_kernel + kbg_select_kernel produce on the device
struct HostIO : ShardIO {
  kbg_status scan(Session& S, kbg::Stage& sg, int32_t G, int32_t base) override {
    sg.G = G;
    sg.base = base;
    sg.fused = false;  // candidate lists, as kbg_scan_kernel + kbg_select_kernel produce them
    sg.h_count = sg.h_down;
    sg.h_cand = sg.h_down + G;
    for (int32_t g = 0; g < G; ++g) {
      const kbg::TaskRec& r = sg.h_tasks[g];
      const uint32_t capn = sg.h_capoff[g + 1] - sg.h_capoff[g];
      uint32_t* c = sg.h_cand + sg.h_capoff[g];
      uint32_t found = 0;
      auto fits = [&](const Res& a) {
        if (S.int_mode) return a.c > r.req[0] && a.m > r.req[1] && a.g > r.req[2];
        return (r.req[0] < a.c || std::fabs(a.c - r.req[0]) < kbg::kMinMilliCPU) &&
               (r.req[1] < a.m || std::fabs(a.m - r.req[1]) < kbg::kMinMemory) &&
               (r.req[2] < a.g || std::fabs(a.g - r.req[2]) < kbg::kMinMilliGPU);
      };
      for (int32_t n = S.tab_lo; n < S.tab_lo + S.tab_n; ++n) {
        if (!((S.h_class_mask[(size_t)r.cls * S.W + (n >> 6)] >> (n & 63)) & 1ull)) continue;
        if (S.pred_active && S.ntasks[n] >= S.maxtasks[n]) continue;
        const bool mi = fits(S.idle[n]);
        if (!mi && !fits(S.rel[n])) continue;
        if (found < capn) c[found] = (uint32_t)n | (mi ? 0u : kbg::kCandPipelineBit);
        ++found;
      }
      sg.h_count[g] = std::min(found, capn) | (found > capn ? kbg::kCountIncompleteBit : 0u);
    }
    S.stats.scan_launches++;
    S.stats.evaluations += G;
    return KBG_OK;
  }
  kbg_status push(Session& S, const std::vector<int32_t>&) override {
    S.mask_dirty.clear();  // the host scan reads the mirror itself
    return KBG_OK;
  }
  kbg_status sync(Session&) override { return KBG_OK; }
};

// R ranks in one process: a barrier and one slot per rank
struct LocalHub {
  int32_t R;
  std::barrier<> bar;
  std::vector<std::vector<uint32_t>> slot;
  explicit LocalHub(int32_t r) : R(r), bar(r), slot(r) {}
};
struct LocalIO final : HostIO {
  LocalHub& hub;
  int32_t me;
  LocalIO(LocalHub& h, int32_t r) : hub(h), me(r) {}
  kbg_status bcast(uint32_t* buf, size_t n) override {
    if (me == 0) hub.slot[0].assign(buf, buf + n);
    hub.bar.arrive_and_wait();
    if (me != 0) std::copy(hub.slot[0].begin(), hub.slot[0].begin() + n, buf);
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status allreduce(uint32_t* buf, size_t n, bool sum) override {
    hub.slot[me].assign(buf, buf + n);
    hub.bar.arrive_and_wait();
    for (size_t i = 0; i < n; ++i) {
      uint32_t v = sum ? 0u : 0xffffffffu;
      for (int32_t r = 0; r < hub.R; ++r) v = sum ? v + hub.slot[r][i] : std::min(v, hub.slot[r][i]);
      buf[i] = v;
    }
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
};

typedef int32_t (*kbg_tool_coll)(void* user, int32_t op, uint32_t* buf, int64_t n);  // op 0 bcast, 1 min, 2 sum
struct CallbackIO final : HostIO {
  kbg_tool_coll fn;
  void* user;
  CallbackIO(kbg_tool_coll f, void* u) : fn(f), user(u) {}
  kbg_status bcast(uint32_t* buf, size_t n) override {
    return fn(user, 0, buf, (int64_t)n) == 0 ? KBG_OK : fail(KBG_E_RCCL, "bcast callback failed");
  }
  kbg_status allreduce(uint32_t* buf, size_t n, bool sum) override {
    return fn(user, sum ? 2 : 1, buf, (int64_t)n) == 0 ? KBG_OK : fail(KBG_E_RCCL, "allreduce callback failed");
  }
};

// stats of one rank's cycle for the caller: rounds, batches, mispredictions,
// truncations, task evaluations; with `times` also (ns) allocate, engine,
// resolve, device round trips, collectives, and the scan launches
void tool_stats(const Session& S, int64_t* st, int64_t* times = nullptr) {
  if (st) {
    st[0] = S.stats.owner_rounds;
    st[1] = S.stats.batches;
    st[2] = S.stats.mispredictions;
    st[3] = S.stats.truncations;
    st[4] = S.stats.task_evaluations;
  }
  if (times) {
    times[0] = (int64_t)(S.stats.allocate_ms * 1e6);
    times[1] = (int64_t)(S.stats.engine_ms * 1e6);
    times[2] = (int64_t)(S.stats.resolve_ms * 1e6);
    times[3] = (int64_t)(S.stats.device_ms * 1e6);
    times[4] = (int64_t)(S.stats.exchange_ms * 1e6);
    times[5] = S.stats.scan_launches;
  }
}

}  // namespace

// R ranks as threads; rank r's decision log at out + r * cap. Returns 0, or
// the first failing rank's status (negated) with its message in kbg_last_error.
extern "C" int32_t kbg_tool_sharded_allocate_local(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                   kbg_decision* out, int32_t cap, int32_t* n_out, int64_t* stats) {
  LocalHub hub(R);
  std::vector<kbg_status> res(R, KBG_OK);
  std::vector<std::string> err(R);
  std::vector<std::thread> th;
  for (int32_t r = 0; r < R; ++r)
    th.emplace_back([&, r]() {
      Session S;
      kbg_status st = host_open(S, snap, o, R, r);
      if (st == KBG_OK && S.has_aff) st = fail(KBG_E_UNSUPPORTED, "pod affinity: the library resolves on every rank");
      if (st == KBG_OK) {  // (an open failure is the same on every rank: no collective is left waiting)
        LocalIO io(hub, r);
        st = allocate_sharded(S, io, out + (size_t)r * cap, cap, n_out + r);
      }
      tool_stats(S, stats ? stats + 5 * r : nullptr);
      res[r] = st;
      err[r] = g_err;
      host_close(S);
    });
  for (auto& t : th) t.join();
  for (int32_t r = 0; r < R; ++r)
    if (res[r] != KBG_OK) {
      g_err = err[r];
      return -(int32_t)res[r];
    }
  return 0;
}

extern "C" int32_t kbg_tool_sharded_allocate_rank(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                  int32_t rank, kbg_tool_coll fn, void* user, kbg_decision* out,
                                                  int32_t cap, int32_t* n_out, int64_t* stats) {
  Session S;
  kbg_status st = host_open(S, snap, o, R, rank);
  if (st == KBG_OK && S.has_aff) st = fail(KBG_E_UNSUPPORTED, "pod affinity: the library resolves on every rank");
  if (st == KBG_OK) {
    CallbackIO io(fn, user);
    st = allocate_sharded(S, io, out, cap, n_out);
  }
  tool_stats(S, stats);
  host_close(S);
  return -(int32_t)st;
}

// ---------------------------------------------------------------------------
// The owner-resolve protocol with R real device sessions on ONE GPU: rank r is
// a session opened on `device` holding shard r of R (a communicator without
// RCCL: the scan, select and availability kernels run on the device over the
// rank's own words, the collectives are the in-process hub). Every rank but
// rank 0 has its first 64-node word at w_lo > 0, so this runs exactly the
// device code of a multi-GPU rank that a one-GPU box cannot host over RCCL
// (kbg_firstfit_kernel over [w_lo, w_hi), availability bit 1 << r per shape).
namespace {
struct DeviceLocalIO final : ShardIO {
  LocalHub& hub;
  int32_t me;
  DeviceLocalIO(LocalHub& h, int32_t r) : hub(h), me(r) {}
  kbg_status bcast(uint32_t* buf, size_t n) override {
    if (me == 0) hub.slot[0].assign(buf, buf + n);
    hub.bar.arrive_and_wait();
    if (me != 0) std::copy(hub.slot[0].begin(), hub.slot[0].begin() + n, buf);
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status allreduce(uint32_t* buf, size_t n, bool sum) override {
    hub.slot[me].assign(buf, buf + n);
    hub.bar.arrive_and_wait();
    for (size_t i = 0; i < n; ++i) {
      uint32_t v = sum ? 0u : 0xffffffffu;
      for (int32_t r = 0; r < hub.R; ++r) v = sum ? v + hub.slot[r][i] : std::min(v, hub.slot[r][i]);
      buf[i] = v;
    }
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status scan(Session& S, kbg::Stage& sg, int32_t G, int32_t base) override { return device_scan(S, sg, G, base); }
  kbg_status scan_avail(Session& S, kbg::Stage& sg, int32_t G, int32_t base, uint32_t* avail) override {
    kbg_status st = device_scan(S, sg, G, base);
    if (st != KBG_OK) return st;
    for (int32_t g = 0; g < G; ++g) avail[g] = sg.h_avail[sg.row_slot[g]];  // this rank's bit per shape slot
    return allreduce(avail, G, true);
  }
};
}  // namespace

extern "C" int32_t kbg_tool_sharded_allocate_device_t(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                      int32_t device, kbg_decision* out, int32_t cap, int32_t* n_out,
                                                      int64_t* stats, int64_t* times, int32_t cycles);
extern "C" int32_t kbg_tool_sharded_allocate_device(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                    int32_t device, kbg_decision* out, int32_t cap, int32_t* n_out,
                                                    int64_t* stats) {
  return kbg_tool_sharded_allocate_device_t(snap, o, R, device, out, cap, n_out, stats, nullptr, 1);
}
// The same, `cycles` allocate cycles in a row (each on the sessions reset to
// the snapshot), the last one's log and stats returned; `times` (6 per rank,
// tool_stats) of the last cycle.
extern "C" int32_t kbg_tool_sharded_allocate_device_t(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                      int32_t device, kbg_decision* out, int32_t cap, int32_t* n_out,
                                                      int64_t* stats, int64_t* times, int32_t cycles) {
  LocalHub hub(R);
  std::vector<kbg_status> res(R, KBG_OK);
  std::vector<std::string> err(R);
  std::vector<kbg_comm> comms(R);
  // every rank opens before any starts the protocol: an open failure returns
  // from all of them (no collective is left waiting)
  std::vector<std::unique_ptr<Session>> sess(R);
  std::vector<std::thread> th;
  for (int32_t r = 0; r < R; ++r) {
    comms[r].n_ranks = R;
    comms[r].rank = r;
    comms[r].device = device;
    sess[r].reset(new Session());
  }
  for (int32_t r = 0; r < R; ++r)
    th.emplace_back([&, r]() {
      kbg_status st = open_session(*sess[r], snap, o, &comms[r]);
      if (st == KBG_OK && sess[r]->has_aff) st = fail(KBG_E_UNSUPPORTED, "pod affinity: the library resolves on every rank");
      res[r] = st;
      err[r] = g_err;
    });
  for (auto& t : th) t.join();
  th.clear();
  bool opened = true;
  for (int32_t r = 0; r < R; ++r) opened &= res[r] == KBG_OK;
  if (opened)
    for (int32_t r = 0; r < R; ++r)
      th.emplace_back([&, r]() {
        Session& S = *sess[r];
        (void)hipSetDevice(S.device);
        DeviceLocalIO io(hub, r);
        kbg_status st = KBG_OK;
        for (int32_t c = 0; c < std::max(1, cycles) && st == KBG_OK; ++c) {
          if (c > 0) {
            st = session_reset(S);
            hub.bar.arrive_and_wait();  // every rank reset before any starts the next cycle
            if (st != KBG_OK) break;
          }
          S.stats = kbg_stats{};
          st = allocate_sharded(S, io, out + (size_t)r * cap, cap, n_out + r);
        }
        tool_stats(S, stats ? stats + 5 * r : nullptr, times ? times + 6 * r : nullptr);
        res[r] = st;
        err[r] = g_err;
      });
  for (auto& t : th) t.join();
  for (int32_t r = 0; r < R; ++r) free_device(*sess[r]);
  for (int32_t r = 0; r < R; ++r)
    if (res[r] != KBG_OK) {
      g_err = err[r];
      return -(int32_t)res[r];
    }
  return 0;
}

// ---------------------------------------------------------------------------
// The scan service (kbg_session.cpp allocate_svc_root / allocate_serve) with R
// device sessions on ONE GPU: rank r holds shard r of R (a communicator
// without RCCL); the messages and the sums of the ranks' launch results go
// through the in-process hub instead of RCCL, so this runs the device code
// and the message handling of a multi-GPU service on a one-GPU box.
namespace {
struct LocalSvc final : SvcLink {
  LocalHub& hub;
  int32_t me;
  LocalSvc(LocalHub& h, int32_t r) : hub(h), me(r) {}
  kbg_status send(Session&, const uint32_t* msg) override {
    hub.slot[0].assign(msg, msg + msg[1]);
    hub.bar.arrive_and_wait();  // the other ranks copy it
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status recv(Session&, std::vector<uint32_t>& msg) override {
    hub.bar.arrive_and_wait();
    msg = hub.slot[0];
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status sum(Session& S, kbg::Stage* sg, size_t info, size_t masks) override {
    std::vector<uint32_t>& b = hub.slot[me];
    b.assign(info + masks, 0u);
    if (hipStreamSynchronize(S.stream) != hipSuccess ||
        hipMemcpy(b.data(), S.d_svc, info * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(b.data() + info, S.d_svc + fused_mask_off(S.K), masks * 4, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(KBG_E_HIP, "scan service (local): device copy failed");
    hub.bar.arrive_and_wait();
    if (sg) {
      uint32_t* hi = sg->h_down;
      uint32_t* hm = sg->h_down + fused_mask_off(S.K);
      for (size_t i = 0; i < info + masks; ++i) {
        uint32_t v = 0;
        for (int32_t r = 0; r < hub.R; ++r) v += hub.slot[r][i];
        (i < info ? hi[i] : hm[i - info]) = v;
      }
    }
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
  kbg_status sum_host(Session&, uint32_t* buf, size_t n) override {
    hub.slot[me].assign(buf, buf + n);
    hub.bar.arrive_and_wait();
    for (size_t i = 0; i < n; ++i) {
      uint32_t v = 0;
      for (int32_t r = 0; r < hub.R; ++r) v += hub.slot[r][i];
      buf[i] = v;
    }
    hub.bar.arrive_and_wait();
    return KBG_OK;
  }
};
}  // namespace

// `cycles` allocate cycles through the scan service (each on the sessions
// reset to the snapshot), the last one's log per rank and tool_stats.
extern "C" int32_t kbg_tool_svc_allocate_device(const kbg_snapshot* snap, const kbg_options* o, int32_t R,
                                                int32_t device, kbg_decision* out, int32_t cap, int32_t* n_out,
                                                int64_t* stats, int64_t* times, int32_t cycles) {
  LocalHub hub(R);
  std::vector<kbg_status> res(R, KBG_OK);
  std::vector<std::string> err(R);
  std::vector<kbg_comm> comms(R);
  std::vector<std::unique_ptr<Session>> sess(R);
  std::vector<std::thread> th;
  for (int32_t r = 0; r < R; ++r) {
    comms[r].n_ranks = R;
    comms[r].rank = r;
    comms[r].device = device;
    sess[r].reset(new Session());
  }
  for (int32_t r = 0; r < R; ++r)
    th.emplace_back([&, r]() {
      res[r] = open_session(*sess[r], snap, o, &comms[r]);
      err[r] = g_err;
    });
  for (auto& t : th) t.join();
  th.clear();
  bool opened = true;
  for (int32_t r = 0; r < R; ++r) opened &= res[r] == KBG_OK;
  if (opened)
    for (int32_t r = 0; r < R; ++r)
      th.emplace_back([&, r]() {
        Session& S = *sess[r];
        (void)hipSetDevice(S.device);
        LocalSvc link(hub, r);
        kbg_status st = KBG_OK;
        for (int32_t c = 0; c < std::max(1, cycles) && st == KBG_OK; ++c) {
          if (c > 0) {
            st = session_reset(S);
            hub.bar.arrive_and_wait();
            if (st != KBG_OK) break;
          }
          S.stats = kbg_stats{};
          st = r == 0 ? allocate_svc_root(S, link, out + (size_t)r * cap, cap, n_out + r)
                      : allocate_serve(S, link, out + (size_t)r * cap, cap, n_out + r);
        }
        tool_stats(S, stats ? stats + 5 * r : nullptr, times ? times + 6 * r : nullptr);
        res[r] = st;
        err[r] = g_err;
      });
  for (auto& t : th) t.join();
  for (int32_t r = 0; r < R; ++r) free_device(*sess[r]);
  for (int32_t r = 0; r < R; ++r)
    if (res[r] != KBG_OK) {
      g_err = err[r];
      return -(int32_t)res[r];
    }
  return 0;
}

// ---------------------------------------------------------------------------
// The fused first-fit kernel alone on a device session: the first G pending
// tasks (session order) as one batch of rows (Grouper: full-scan or grouped
// per the options), launched `reps` times against the session's table;
// returns the median kernel time (HIP events) in microseconds, or < 0.
extern "C" double kbg_tool_firstfit_bench(const kbg_snapshot* snap, const kbg_options* o, int32_t G, int32_t reps) {
  Session S;
  if (open_session(S, snap, o, nullptr) != KBG_OK) return -1.0;
  std::vector<int32_t> bt;
  for (int32_t t : S.pend_all) {
    if ((int32_t)bt.size() == std::min(G, S.K)) break;
    bt.push_back(t);
  }
  Grouper grouper(S);
  kbg::Stage& sg = S.stages[0];
  const int32_t rows = grouper.build(sg, bt.data(), (int32_t)bt.size());
  std::vector<double> us;
  for (int32_t r = 0; r < reps; ++r) {
    S.ff_launch_seq = 0;  // every launch of the probe carries its events
    if (device_scan(S, sg, rows, S.res_stamp) != KBG_OK) {
      free_device(S);
      return -2.0;
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, sg.ev[0], sg.ev[1]);
    us.push_back(ms * 1e3);
  }
  free_device(S);
  std::sort(us.begin(), us.end());
  return us[us.size() / 2];
}

#ifdef KBG_FF_STAMPS
namespace kbg {
hipError_t read_ff_stamps(unsigned long long* out, int n_wg);
}
// One fused-kernel launch of G rows with phase stamps: out[wg][8] global
// 100 MHz clock values (slots 0 entry, 1 rows in LDS, 2 wave 0's scan done,
// 3 round barrier, 4 placement barrier, 5 wave 0's appends done, 6 end).
// Returns the number of workgroups, < 0 on failure.
extern "C" int32_t kbg_tool_firstfit_stamps(const kbg_snapshot* snap, const kbg_options* o, int32_t G,
                                            unsigned long long* out, int32_t max_wg) {
  Session S;
  if (open_session(S, snap, o, nullptr) != KBG_OK) return -1;
  std::vector<int32_t> bt;
  for (int32_t t : S.pend_all) {
    if ((int32_t)bt.size() == std::min(G, S.K)) break;
    bt.push_back(t);
  }
  Grouper grouper(S);
  kbg::Stage& sg = S.stages[0];
  const int32_t rows = grouper.build(sg, bt.data(), (int32_t)bt.size());
  for (int r = 0; r < 3; ++r)  // warm, then the stamped launch is the last one
    if (device_scan(S, sg, rows, S.res_stamp) != KBG_OK) {
      free_device(S);
      return -2;
    }
  const int32_t per = kbg::firstfit_geometry(rows, S.opts.full_scan != 0).rows;
  const int32_t n_wg = std::min((rows + per - 1) / per * sg.splits, max_wg);
  const bool ok = kbg::read_ff_stamps(out, n_wg) == hipSuccess;
  free_device(S);
  return ok ? n_wg : -3;
}
#endif


// Host cost of one fused launch (device_launch: arguments, the launch call,
// the completion event) and of the whole round trip (launch + wait), medians
// over `reps` launches of the first G pending tasks' rows; untimed != 0
// launches without the kernel's start / stop events.
extern "C" int32_t kbg_tool_launch_cost(const kbg_snapshot* snap, const kbg_options* o, int32_t G, int32_t reps,
                                        int32_t untimed, double* launch_us, double* roundtrip_us) {
  Session S;
  if (open_session(S, snap, o, nullptr) != KBG_OK) return -1;
  S.untimed_launches = untimed != 0;
  std::vector<int32_t> bt;
  for (int32_t t : S.pend_all) {
    if ((int32_t)bt.size() == std::min(G, S.K)) break;
    bt.push_back(t);
  }
  Grouper grouper(S);
  kbg::Stage& sg = S.stages[0];
  const int32_t rows = grouper.build(sg, bt.data(), (int32_t)bt.size());
  std::vector<double> l, rt;
  for (int32_t r = 0; r < reps; ++r) {
    S.ff_launch_seq = 0;  // timed variant: events on every launch
    const auto t0 = std::chrono::steady_clock::now();
    if (device_launch(S, sg, rows, S.res_stamp) != KBG_OK) return free_device(S), -2;
    const auto t1 = std::chrono::steady_clock::now();
    if (device_wait(S, sg) != KBG_OK) return free_device(S), -3;
    const auto t2 = std::chrono::steady_clock::now();
    l.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    rt.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
  }
  free_device(S);
  std::sort(l.begin(), l.end());
  std::sort(rt.begin(), rt.end());
  *launch_us = l[l.size() / 2];
  *roundtrip_us = rt[rt.size() / 2];
  return rows;
}

// ---------------------------------------------------------------------------
// CPU self-test of the host transport (kbg_comm.cpp HostColl) over host
// buffers: `iters` rounds of broadcast, sum / min / max all-reduce and
// all-gather of n words per rank (n past 1M words crosses the 4 MB chunks),
// every result checked against its closed form on this rank. One call per
// process; the ranks are processes naming the same segment. Returns 0, or
// -status with the message in kbg_last_error; *ops = collectives completed.
extern "C" int32_t kbg_tool_hostcomm_selftest(const char* name, int32_t R, int32_t rank, int64_t n, int32_t iters,
                                              int64_t* ops) {
  kbg_status st = KBG_OK;
  std::string err;
  std::unique_ptr<kbg::Coll> c = kbg::make_host_coll(name, R, rank, &st, &err, true);
  if (!c) {
    g_err = err;
    return -(int32_t)st;
  }
  auto val = [](int32_t r, int64_t i, int32_t it) { return (uint32_t)(r * 2654435761u + i * 40503u + it * 977u); };
  std::vector<uint32_t> a((size_t)n), b((size_t)n), g((size_t)n * R);
  int64_t done = 0;
  auto bad = [&](const char* what, int32_t it, int64_t i) {
    char m[160];
    snprintf(m, sizeof m, "self-test: %s wrong at iteration %d word %lld", what, it, (long long)i);
    g_err = m;
    if (ops) *ops = done;
    return -(int32_t)KBG_E_INVALID;
  };
  for (int32_t it = 0; it < iters; ++it) {
    for (int64_t i = 0; i < n; ++i) a[i] = rank == 0 ? val(0, i, it) : 0u;
    if ((st = c->bcast(a.data(), (size_t)n, nullptr)) != KBG_OK) break;
    ++done;
    for (int64_t i = 0; i < n; ++i)
      if (a[i] != val(0, i, it)) return bad("broadcast", it, i);
    for (int32_t op = 0; op < 3 && st == KBG_OK; ++op) {
      for (int64_t i = 0; i < n; ++i) a[i] = val(rank, i, it);
      if ((st = c->allreduce(a.data(), b.data(), (size_t)n, (kbg::CollOp)op, nullptr)) != KBG_OK) break;
      ++done;
      for (int64_t i = 0; i < n; ++i) {
        uint32_t want = val(0, i, it);
        for (int32_t r = 1; r < R; ++r) {
          const uint32_t v = val(r, i, it);
          want = op == 0 ? want + v : op == 1 ? std::min(want, v) : std::max(want, v);
        }
        if (b[i] != want) return bad(op == 0 ? "sum" : op == 1 ? "min" : "max", it, i);
      }
    }
    if (st != KBG_OK) break;
    for (int64_t i = 0; i < n; ++i) g[(size_t)rank * n + i] = val(rank, i, it) ^ 0x5a5a5a5au;
    if ((st = c->allgather(g.data() + (size_t)rank * n, g.data(), (size_t)n * 4, nullptr)) != KBG_OK) break;
    ++done;
    for (int32_t r = 0; r < R; ++r)
      for (int64_t i = 0; i < n; ++i)
        if (g[(size_t)r * n + i] != (val(r, i, it) ^ 0x5a5a5a5au)) return bad("all-gather", it, i);
  }
  if (ops) *ops = done;
  if (st != KBG_OK) {
    g_err = c->err;
    return -(int32_t)st;
  }
  return 0;
}
