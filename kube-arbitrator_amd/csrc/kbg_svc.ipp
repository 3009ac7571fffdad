// kbg_svc.ipp: the scan service: rank 0 and the serving ranks.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

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
