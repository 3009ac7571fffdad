// kbg_allocate.ipp: the allocate cycle: predictor, committer, truth engine.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

// The host side of one allocate cycle runs on two threads:
//   predictor (pool thread) — the ordering engine: predicts batches of K task
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

// A helper thread of a cycle (predictor, builder, truth engine, logger) from
// a process-wide pool: every cycle starts four and joins them, and creating
// and joining an OS thread cost tens of microseconds each on the box (a
// resident churn cycle is about a millisecond). Same use as std::thread:
// construct with the function, join() waits until it has returned. A pool
// thread gets its CPU mask back after each function (pin_near narrows it).
// A forked child starts a pool of its own (the parent's threads are not in it).
class PoolThread {
  struct Slot {
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> fn;
    bool has = false, done = false;
  };
  struct Pool {
    std::mutex mu;
    std::vector<Slot*> idle;
    pid_t pid = 0;
  };
  static Pool& pool() {
    static Pool* p = new Pool();  // (never destroyed: its threads outlive static destruction)
    return *p;
  }
  static void loop(Slot* s) {
    cpu_set_t mask;
    const bool have_mask = pthread_getaffinity_np(pthread_self(), sizeof(mask), &mask) == 0;
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(s->mu);
        s->cv.wait(lk, [&] { return s->has; });
        fn = std::move(s->fn);
        s->has = false;
      }
      fn();
      fn = nullptr;  // (captured state released before the joiner returns)
      {
        std::lock_guard<std::mutex> lk(s->mu);
        s->done = true;
        s->cv.notify_all();
      }
      if (have_mask) (void)pthread_setaffinity_np(pthread_self(), sizeof(mask), &mask);
    }
  }
  Slot* slot_ = nullptr;

 public:
  PoolThread() = default;
  explicit PoolThread(std::function<void()> fn) {
    Pool& P = pool();
    Slot* s = nullptr;
    {
      std::lock_guard<std::mutex> lk(P.mu);
      if (P.pid != getpid()) {  // first use, or a forked child: the listed threads are not this process's
        P.idle.clear();
        P.pid = getpid();
      }
      if (!P.idle.empty()) {
        s = P.idle.back();
        P.idle.pop_back();
      }
    }
    if (!s) {
      s = new Slot();
      std::thread(loop, s).detach();
    }
    {
      std::lock_guard<std::mutex> lk(s->mu);
      s->fn = std::move(fn);
      s->done = false;
      s->has = true;
    }
    s->cv.notify_all();
    slot_ = s;
  }
  PoolThread(const PoolThread&) = delete;
  PoolThread& operator=(const PoolThread&) = delete;
  PoolThread& operator=(PoolThread&& o) noexcept {
    if (this != &o) {
      join();
      slot_ = o.slot_;
      o.slot_ = nullptr;
    }
    return *this;
  }
  ~PoolThread() { join(); }
  bool joinable() const { return slot_ != nullptr; }
  void join() {
    if (!slot_) return;
    Slot* s = slot_;
    slot_ = nullptr;
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv.wait(lk, [&] { return s->done; });
    }
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    P.idle.push_back(s);
  }
};

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
    pool_put(S.fit_h);
    if (S.fit_d) (void)hipFree(S.fit_d);
    S.fit_h = nullptr;
    S.fit_d = nullptr;
    S.fit_cap = 0;
    if (host_alloc((void**)&S.fit_h, bytes) != KBG_OK) return fail(KBG_E_HIP, "FitError staging");
    HIP_TRY(hipMalloc((void**)&S.fit_d, bytes));
    S.fit_cap = bytes;
  }
  if (out_bytes > S.fit_out_cap) {
    pool_put(S.fit_out);
    S.fit_out = nullptr;
    S.fit_out_cap = 0;
    if (host_alloc((void**)&S.fit_out, out_bytes) != KBG_OK) return fail(KBG_E_HIP, "FitError results");
    S.fit_out_cap = out_bytes;
  }
  int32_t* hoff = (int32_t*)S.fit_h;
  int32_t* hk = (int32_t*)(S.fit_h + o_hk);
  double* hold = (double*)(S.fit_h + o_hold);
  kbg::FitQuery* fq = (kbg::FitQuery*)(S.fit_h + o_q);
  trace_add("fit.count", E);
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
    if (i + 8 < Q) {  // the queried tasks are scattered over the task arrays
      const int32_t t8 = last[qj[i + 8]].task;
      __builtin_prefetch(&S.treq[t8]);
      __builtin_prefetch(&S.task_class[t8]);
    }
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
  trace_add("fit.staged", Q);
  HIP_TRY(kbg::launch_fitdelta(a, S.stream));
  HIP_TRY(hipStreamSynchronize(S.stream));
  trace_add("fit.kernel", 0);
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
    if (S.committed_ready[j] < S.job_min[j]) jobs.push_back(j);  // (job_min: jobs_in[j].min_available, compact)
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
  PoolThread th;
  std::mutex mu;
  SpinCV cv;
  std::deque<std::vector<Outcome>> q;
  bool done = false, busy = false;
  std::string error;
  // committer_cpu >= 0: on its own core of the committer's last-level cache
  // (after the predictor, logger and builder), never time-sharing the predictor's
  Replayer(Session& s, Engine& e, int committer_cpu = -1) : S(s), E(e) {
    th = PoolThread([this, committer_cpu]() {
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
  PoolThread th, bth;
  bool builder = false;       // a builder thread turns predicted batches into device rows (allocate_cycle)
  bool truth_mode = false;    // rollbacks copy a truth engine (rollback_truth): no batch checkpoints
  bool runs = false;          // consume a job's tasks of shapes known to fit nowhere as one entry (Batch::brun)
  std::vector<Batch*> all;    // every batch of this predictor (freed by finish)
  Predictor(Session& s, Engine& e, std::atomic<uint8_t>* f) : S(s), E(e), failed(f) {
    prof.on = getenv("KBG_PROFILE_ENGINE") != nullptr;
  }
  void start(int committer_cpu, bool with_builder = false) {
    builder = with_builder;
    th = PoolThread([this, committer_cpu]() { run(committer_cpu); });
    if (builder) bth = PoolThread([this, committer_cpu]() { build_run(committer_cpu); });
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
  PoolThread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::vector<LogItem>> q;
  bool done = false;
  explicit Logger(std::function<void(const LogItem&)> f, int committer_cpu) : fn(std::move(f)) {
    th = PoolThread([this, committer_cpu]() {
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
  ctr.add("flushed");
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
