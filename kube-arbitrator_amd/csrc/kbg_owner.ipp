// kbg_owner.ipp: sharded allocate over the owner-resolve protocol.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

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
