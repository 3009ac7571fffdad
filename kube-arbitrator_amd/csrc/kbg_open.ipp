// kbg_open.ipp: session open: ingest, the host derive and the device build.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

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
    // (a job's tasks usually share one (class, request): the last key found
    // answers most lookups without the hash map)
    kbg::ShapeKey last_key{-1, 0.0, 0.0, 0.0};
    int32_t last_id = -1;
    auto cand_shape = [&](int32_t t) {
      if (!S.pending_candidate[t]) return;
      int32_t& sh_t = S.shape_of_task[t];
      if (sh_t < 0) {
        const kbg::ShapeKey k{S.task_class[t], S.treq[t].c, S.treq[t].m, S.treq[t].g};
        if (last_id >= 0 && k == last_key) {
          sh_t = last_id;
        } else {
          auto it = S.shape_ids.emplace(k, S.n_shapes);
          if (it.second) S.n_shapes++;
          sh_t = last_id = it.first->second;
          last_key = k;
        }
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
  // (a rebuilt session arrives with its predecessor's stream and events, restructure)
  if (!S.stream) HIP_TRY(hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
  for (auto& e : S.ev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  if (!S.stage_ev) HIP_TRY(hipEventCreateWithFlags(&S.stage_ev, hipEventDisableTiming));
  if (!S.comm_ev) HIP_TRY(hipEventCreateWithFlags(&S.comm_ev, hipEventDisableTiming));
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
    for (int e = 0; e < 6; ++e)
      if (!g.ev[e]) HIP_TRY(hipEventCreate(&g.ev[e]));
    if (!g.ev[6]) HIP_TRY(hipEventCreateWithFlags(&g.ev[6], hipEventDisableTiming));
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
