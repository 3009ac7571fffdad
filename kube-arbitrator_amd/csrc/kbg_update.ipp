// kbg_update.ipp: resident session updates (kbg_session_update).
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

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
  // that left) or a pod outside the session jobs. Per node, its tasks' keys
  // sorted by (key, position): the first task in node order holding a key is
  // a binary search away (a node holds tens of pods; a linear scan per key
  // was quadratic, 40 ms at C4 with every task bound).
  std::vector<std::pair<int32_t, int32_t>> held;  // (canonical key, position in node_task_order[n])
  int32_t held_node = -1;
  auto holder_task = [&](int32_t n, int32_t key) -> int32_t {
    const std::vector<int32_t>& order = S.node_task_order[n];
    if (held_node != n) {
      held.clear();
      for (int32_t i = 0; i < (int32_t)order.size(); ++i) held.emplace_back(S.canon[S.tasks_in[order[i]].pod_key], i);
      std::sort(held.begin(), held.end());
      held_node = n;
    }
    auto it = std::lower_bound(held.begin(), held.end(), std::make_pair(key, INT32_MIN));
    return it != held.end() && it->first == key ? order[it->second] : -1;
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
  static const bool prof = getenv("KBG_PROFILE_OPEN") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!prof) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[kbg rebuild] %-20s %8.3f ms\n", name, std::chrono::duration<double, std::milli>(now - tl).count());
    tl = now;
  };
  Rebuilt B;
  if (kbg_status st = rebuild_snapshot(S, B); st != KBG_OK) return st;
  phase("snapshot");
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
  // the stream and its events move to the rebuilt session (creating and
  // destroying them cost milliseconds) once everything enqueued has run; the
  // old device tables and pinned buffers go back to the process's pool first,
  // so the new open takes them from there (an open that fails leaves the
  // session unusable either way: its events are applied)
  if (S.stream) HIP_TRY(hipStreamSynchronize(S.stream));
  for (kbg::Stage& g : S.stages) {
    if (g.inflight) HIP_TRY(hipEventSynchronize(g.ev[6]));
    g.inflight = false;
  }
  std::swap(R->stream, S.stream);
  for (size_t k = 0; k < std::size(S.ev); ++k) std::swap(R->ev[k], S.ev[k]);
  std::swap(R->stage_ev, S.stage_ev);
  std::swap(R->comm_ev, S.comm_ev);
  for (size_t g = 0; g < std::size(S.stages); ++g)
    for (size_t k = 0; k < std::size(S.stages[g].ev); ++k) std::swap(R->stages[g].ev[k], S.stages[g].ev[k]);
  free_device(S);
  phase("free device");
  kbg_status st = open_session(*R, &B.sn, &o, nullptr);
  phase("open");
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
  phase("pod-only names");
  S = std::move(*R);
  phase("session move");
  S.renum[KBG_RENUM_TASKS] = std::move(B.rt);
  S.renum[KBG_RENUM_NODES] = std::move(B.rn);
  S.renum[KBG_RENUM_JOBS] = std::move(B.rj);
  S.renum[KBG_RENUM_QUEUES] = std::move(B.rq);
  return KBG_OK;
}

// Room for a large batch's growth, reserved before its events apply: each
// target node's pod lists (a cycle's binds grow a node's lists by tens of
// entries, one reallocation per doubling otherwise) and the update's own
// per-event lists.
void reserve_for_events(Session& S, const kbg_event* ev, int32_t n) {
  if (n < 4096) return;
  thread_local std::vector<int32_t> adds;
  adds.assign(S.n_nodes, 0);
  for (int32_t i = 0; i < n; ++i) {
    const kbg_event& e = ev[i];
    if ((e.kind == KBG_EV_POD_UPDATE || e.kind == KBG_EV_POD_ADD) && e.node >= 0 && e.node < S.n_nodes &&
        !terminated(e.status))
      adds[e.node]++;
  }
  for (int32_t nd = 0; nd < S.n_nodes; ++nd)
    if (adds[nd]) {
      S.node_key_order[nd].reserve(S.node_key_order[nd].size() + adds[nd]);
      S.node_task_order[nd].reserve(S.node_task_order[nd].size() + adds[nd]);
    }
  S.upd_tasks.reserve(S.upd_tasks.size() + n);
  S.pend_dirty_jobs.reserve(S.pend_dirty_jobs.size() + n);
  S.upd_keys.reserve(S.upd_keys.size() + 2 * (size_t)n);
  S.jmove_out.reserve(S.jmove_out.size() + n);
  S.jmove_add.reserve(S.jmove_add.size() + n);
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
  reserve_for_events(S, ev, n);
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
