// kbg_victims.ipp: preempt / reclaim and their victim scans.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

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
      pool_put(p);
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
