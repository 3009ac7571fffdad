// Inter-pod (anti)affinity on the device path: the vendor
// predicate InterPodAffinityMatches with meta == nil (vendor
// predicates.go:1155-1466), the slow path kube-batch's predicates plugin
// takes (pkg/scheduler/plugins/predicates/predicates.go:185-198), restated as
// counts over the session's AllocatedStatus pods (api/helpers.go:63-70) that
// the host keeps current as placements land, and folded into the class masks
// the scan kernel reads:
//
//  (A) existing pods' anti-affinity (:1244-1332): an allocated pod E with an
//      anti term T that selects the incoming pod forbids the (T.topologyKey,
//      E's node value) pair; a node fails if one of its label pairs is
//      forbidden. cntA[class][pair].
//  (B) the pod's affinity terms (:1402-1456): some allocated pod must match
//      every term's namespaces + selector and share every term's topology
//      value with the node; with no pod matching the selectors at all, the
//      pod passes iff it matches its own terms. nB[class] (pods matching the
//      selectors), cntB[class][node signature].
//  (C) the pod's anti terms: no allocated pod may match every term and share
//      the topology of every term up to the first empty topologyKey (an empty
//      key is an error, i.e. a failure, once reached). cntC[class][signature].
//
// (A) and (C) only remove nodes as pods are allocated (monotone, like the pod
// cap); (B) adds nodes. A placement that adds nodes to a class ends the
// allocate batch there (kbg_session.cpp), since the later rows of the batch
// were scanned against the old mask.
//
// The podLister Filter (vendor cache/node_info.go:692-702: a pod whose
// informer Spec.NodeName is the evaluated node but that the node's pods lack
// is left out of that node's predicate) arises within a session only for a
// holder a discarded statement's RemoveTask took off its node: aff_ok_node
// evaluates that node with the holder's counts taken out (S.aff_filtered).
// Tasks placed this session keep their informer Spec.NodeName "" (session.go
// sets task.NodeName only), so the Filter always keeps them.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>

#include "kbg_session.hpp"

namespace kbg {

namespace {

int64_t pair_key(int32_t k, int32_t v) { return ((int64_t)k << 32) | (uint32_t)v; }

bool allocated_status(int32_t s) {  // api/helpers.go:63-70 (the podLister's pods)
  return s == KBG_BOUND || s == KBG_BINDING || s == KBG_RUNNING || s == KBG_ALLOCATED;
}

// A class's forbidden pairs: a handful (one per distinct topology value of
// the pods that forbid them), so a flat list beats a hash map.
template <class K>
int32_t count_of(const std::vector<std::pair<K, int32_t>>& v, K k) {
  for (const auto& e : v)
    if (e.first == k) return e.second;
  return 0;
}
// adds d to k's count; returns {before, after}; drops entries that reach 0
template <class K>
std::pair<int32_t, int32_t> count_add(std::vector<std::pair<K, int32_t>>& v, K k, int32_t d) {
  size_t i = 0;
  while (i < v.size() && v[i].first != k) ++i;
  if (i == v.size()) v.emplace_back(k, 0);
  const int32_t b = v[i].second;
  const int32_t a = v[i].second += d;
  if (a == 0) {
    v[i] = v.back();
    v.pop_back();
  }
  return {b, a};
}

const int32_t* find_label(const std::vector<std::pair<int32_t, int32_t>>& ls, int32_t key) {
  auto it = std::lower_bound(ls.begin(), ls.end(), std::make_pair(key, INT32_MIN));
  return it != ls.end() && it->first == key ? &it->second : nullptr;
}

// metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:31-67)
// with NewRequirement validation (labels/selector.go:134-170).
AffSel compile_label_selector(const Session& S, const kbg_pod_term& pt) {
  AffSel s;
  if (!pt.has_selector) {
    s.nothing = true;
    return s;
  }
  if (pt.match_len == 0 && pt.expr_len == 0) {
    s.everything = true;
    return s;
  }
  for (int32_t i = 0; i < pt.match_len; ++i) {
    const int32_t k = S.selectors_in[2 * (pt.match_off + i)], v = S.selectors_in[2 * (pt.match_off + i) + 1];
    if (!label_key_valid(S.strs[k]) || !label_value_valid(S.strs[v])) {
      s.err = true;
      return s;
    }
    s.reqs.push_back(AffSelReq{S.canon[k], 0, {S.canon[v]}});
  }
  for (int32_t i = 0; i < pt.expr_len; ++i) {
    const kbg_requirement& r = S.reqs_in[pt.expr_off + i];
    const std::string& op = S.strs[r.op];
    int32_t o;
    if (op == "In") o = 0;
    else if (op == "NotIn") o = 1;
    else if (op == "Exists") o = 2;
    else if (op == "DoesNotExist") o = 3;
    else {
      s.err = true;
      return s;
    }
    if (!label_key_valid(S.strs[r.key]) || ((o == 0 || o == 1) && r.value_len == 0) ||
        ((o == 2 || o == 3) && r.value_len != 0)) {
      s.err = true;
      return s;
    }
    AffSelReq q{S.canon[r.key], o, {}};
    for (int32_t v = 0; v < r.value_len; ++v) {
      const int32_t id = S.values_in[r.value_off + v];
      if (!label_value_valid(S.strs[id])) {
        s.err = true;
        return s;
      }
      q.vals.push_back(S.canon[id]);
    }
    s.reqs.push_back(std::move(q));
  }
  return s;
}

bool selector_matches(const AffSel& s, const std::vector<std::pair<int32_t, int32_t>>& labels) {
  if (s.nothing) return false;
  if (s.everything) return true;
  for (const AffSelReq& r : s.reqs) {
    const int32_t* v = find_label(labels, r.key);
    const bool in = v && std::find(r.vals.begin(), r.vals.end(), *v) != r.vals.end();
    const bool ok = r.op == 0 ? in : r.op == 1 ? !in : r.op == 2 ? v != nullptr : v == nullptr;
    if (!ok) return false;
  }
  return true;
}

// PodMatchesTermsNamespaceAndSelector with GetNamespacesFromPodAffinityTerm
// (priorities/util/topologies.go:28-48): namespaces default to the owner's.
bool term_matches(const AffTerm& t, int32_t owner_ns, const AffSpec& target) {
  const bool in =
      t.ns.empty() ? target.ns == owner_ns : std::find(t.ns.begin(), t.ns.end(), target.ns) != t.ns.end();
  return in && selector_matches(t.sel, target.labels);
}

bool all_terms_match(const std::vector<AffTerm>& terms, int32_t owner_ns, const AffSpec& target) {
  for (const AffTerm& t : terms)
    if (!term_matches(t, owner_ns, target)) return false;
  return true;
}

bool ports_ok(const Session& S, int32_t c, int32_t n) {
  if (!S.has_ports) return true;
  for (int32_t w = 0; w < S.PW; ++w)
    if (S.node_ports[(size_t)n * S.PW + w] & S.cls_conf[(size_t)c * S.PW + w]) return false;
  return true;
}

// The class-mask bit of (c, n) from the static predicate, the port fit and
// the affinity counts; a change is queued for the device and reported.
void recompute_bit(Session& S, int32_t c, int32_t n) {
  S.affm->prof_recomputes++;
  const size_t idx = (size_t)c * S.W + (n >> 6);
  const uint64_t bit = 1ull << (n & 63);
  bool v = (S.h_class_mask_static[idx] & bit) != 0;
  if (v && !S.panic_node[n]) v = ports_ok(S, c, n) && aff_ok_node(S, c, n);
  const bool old = (S.h_class_mask[idx] & bit) != 0;
  if (v == old) return;
  vc_mask_changed(S, c, n);
  if (v) {
    S.h_class_mask[idx] |= bit;
    if (!S.aff_gain_flag[c]) {
      S.aff_gain_flag[c] = 1;
      S.aff_gain_classes.push_back(c);
    }
  } else {
    S.h_class_mask[idx] &= ~bit;
    S.mwmark[idx] = S.mstamp;  // a candidate list of this batch may hold the node: the resolver re-checks it
  }
  if (!S.mask_dirty_flag[idx]) {
    S.mask_dirty_flag[idx] = 1;
    S.mask_dirty.push_back((uint32_t)idx);
  }
}

void recompute_class(Session& S, int32_t c) {
  for (int32_t n = 0; n < S.n_nodes; ++n) recompute_bit(S, c, n);
}

}  // namespace

bool aff_ok(const Session& S, const AffState& st, int32_t c, int32_t n) {
  const AffinityModel& M = *S.affm;
  if (st.poison) return false;
  const auto& ca = st.cntA[c];
  if (!ca.empty())
    for (const auto& kv : M.node_labels[n])
      if (count_of(ca, pair_key(kv.first, kv.second)) > 0) return false;
  const AffClass& a = M.cls[c];
  if (a.hasB) {
    if (a.b_err) return false;
    if (st.nB[c] == 0) {
      if (!a.b_self) return false;
    } else {
      if (a.b_empty_key) return false;
      const int32_t sg = M.sigtabs[a.b_tab].sig[n];
      if (sg < 0 || count_of(st.cntB[c], sg) == 0) return false;
    }
  }
  if (a.hasC) {
    if (a.c_err) {
      if (st.allocated > 0) return false;
    } else {
      const int32_t sg = M.sigtabs[a.c_tab].sig[n];
      if (sg >= 0 && count_of(st.cntC[c], sg) > 0) return false;
    }
  }
  return true;
}

// The podLister's FilteredList(nodeInfo.Filter) (predicates.go:67-89) for
// node n: a pod whose informer Spec.NodeName is n but that n's pods lack
// (vendor cache/node_info.go:692-702) is not in the list n's predicate sees.
// Within a session that is a holder a discarded statement's RemoveTask took
// off its node (S.aff_filtered); its counts are taken out for n's own
// evaluation and put back.
bool aff_ok_node(Session& S, int32_t c, int32_t n) {
  AffState& st = S.affm->st;
  bool any = false;
  for (const auto& [fn, t] : S.aff_filtered)
    if (fn == n) {
      aff_place(S, t, n, -1, st, false);
      any = true;
    }
  const bool ok = aff_ok(S, st, c, n);
  if (any)
    for (const auto& [fn, t] : S.aff_filtered)
      if (fn == n) aff_place(S, t, n, +1, st, false);
  return ok;
}

void aff_refresh_node(Session& S, int32_t n) {
  if (!S.has_aff || n < 0) return;
  for (int32_t c = 0; c < S.n_classes; ++c) recompute_bit(S, c, n);
}

// One AllocatedStatus pod (task t) appears on (sign +1) or leaves (-1) node n
// (-1: a node outside the session).
void aff_place(Session& S, int32_t t, int32_t n, int32_t sign, AffState& st, bool update_bits) {
  const AffinityModel& M = *S.affm;
  const int32_t s = S.tasks_in[t].spec;
  if (s >= 0 && !M.spec_effect[s] && M.c_err_classes.empty()) {  // selects and is selected by nothing
    st.allocated += sign;
    return;
  }
  std::vector<int32_t> full;  // classes to recompute on every node
  auto crossed = [](int32_t before, int32_t after) { return (before == 0) != (after == 0); };
  {
    const int32_t b = st.allocated;
    st.allocated += sign;
    if (update_bits && crossed(b, st.allocated))
      for (int32_t c : M.c_err_classes) full.push_back(c);
  }
  if (s >= 0 && M.spec_poison[s]) {
    const int32_t b = st.poison;
    st.poison += sign;
    if (update_bits && crossed(b, st.poison)) {
      full.clear();
      for (int32_t c = 0; c < S.n_classes; ++c) full.push_back(c);
    }
  }
  if (s >= 0 && n >= 0) {
    const AffSpec& sp = M.specs[s];
    // (A) its anti terms forbid (key, value of node n) to the classes they select
    for (size_t k = 0; k < sp.anti.size(); ++k) {
      const AffTerm& term = sp.anti[k];
      const int32_t* v = find_label(M.node_labels[n], term.key);
      if (!v) continue;
      const int64_t pk = pair_key(term.key, *v);
      for (int32_t c : M.anti_match[s][k]) {
        const auto ba = count_add(st.cntA[c], pk, sign);
        if (update_bits && crossed(ba.first, ba.second)) {
          auto it = M.pair_nodes.find(pk);
          if (it != M.pair_nodes.end())
            for (int32_t m : it->second) recompute_bit(S, c, m);
        }
      }
    }
    // (B) it is a target of the affinity terms of these classes
    for (int32_t c : M.matchB[s]) {
      const AffClass& a = M.cls[c];
      const int32_t b = st.nB[c];
      st.nB[c] += sign;
      const bool first = update_bits && crossed(b, st.nB[c]);
      const AffSigTable* tb = a.b_tab >= 0 ? &M.sigtabs[a.b_tab] : nullptr;
      const int32_t sg = tb ? tb->sig[n] : -1;
      if (sg >= 0) {
        const auto ba = count_add(st.cntB[c], sg, sign);
        if (update_bits && !first && crossed(ba.first, ba.second))
          for (int32_t m : tb->nodes[sg]) recompute_bit(S, c, m);
      }
      if (!first) continue;
      if (sign > 0 && a.b_self) {
        // the first matching pod ends the "first pod of a series" pass: only
        // its topology domain stays (nothing with an empty key or without the
        // keys); every other constraint is unchanged, so the class mask is
        // ANDed with the domain (nil-Node nodes stay reachable)
        std::vector<uint64_t> keep(M.panic_words);
        if (!a.b_empty_key && sg >= 0)
          for (int32_t m : tb->nodes[sg]) keep[m >> 6] |= 1ull << (m & 63);
        for (int32_t w = 0; w < S.W; ++w) {
          const size_t idx = (size_t)c * S.W + w;
          const uint64_t old = S.h_class_mask[idx], nw = old & keep[w];
          if (nw == old) continue;
          for (uint64_t d = old & ~nw; d; d &= d - 1) vc_mask_changed(S, c, w * 64 + __builtin_ctzll(d));
          S.h_class_mask[idx] = nw;
          S.mwmark[idx] = S.mstamp;
          if (!S.mask_dirty_flag[idx]) {
            S.mask_dirty_flag[idx] = 1;
            S.mask_dirty.push_back((uint32_t)idx);
          }
        }
      } else if (sign > 0 && !a.b_empty_key && sg >= 0) {
        for (int32_t m : tb->nodes[sg]) recompute_bit(S, c, m);  // nothing passed before: its domain opens
      } else {
        full.push_back(c);
      }
    }
    // (C) ... and of the anti terms of these
    for (int32_t c : M.matchC[s]) {
      const AffClass& a = M.cls[c];
      const AffSigTable& tc = M.sigtabs[a.c_tab];
      const int32_t sg = tc.sig[n];
      if (sg < 0) continue;
      const auto ba = count_add(st.cntC[c], sg, sign);
      if (update_bits && crossed(ba.first, ba.second))
        for (int32_t m : tc.nodes[sg]) recompute_bit(S, c, m);
    }
  }
  if (!update_bits) return;
  std::sort(full.begin(), full.end());
  full.erase(std::unique(full.begin(), full.end()), full.end());
  for (int32_t c : full) recompute_class(S, c);
  // a node with filtered pods: its bits follow the counts without them (the
  // domain-wide updates above keep or recompute it with them)
  for (const auto& [fn, ft] : S.aff_filtered)
    for (int32_t c = 0; c < S.n_classes; ++c) recompute_bit(S, c, fn);
}

// Builds the model and the counts of the pods allocated at open, and folds
// the predicate into the class masks (after the static predicate and ports).
void setup_affinity(Session& S) {
  if (!S.has_aff) return;
  auto M = std::make_shared<AffinityModel>();
  S.affm = M;
  const int32_t N = S.n_nodes, C = S.n_classes, NS = (int32_t)S.specs_in.size();
  // node labels (labels.Set: the last value of a key wins), sorted by key
  M->node_labels.resize(N);
  for (int32_t n = 0; n < N; ++n) {
    const kbg_node& nd = S.nodes_in[n];
    std::map<int32_t, int32_t> lab;
    for (int32_t i = 0; i < nd.label_len; ++i)
      lab[S.canon[S.labels_in[2 * (nd.label_off + i)]]] = S.canon[S.labels_in[2 * (nd.label_off + i) + 1]];
    M->node_labels[n].assign(lab.begin(), lab.end());
  }
  // specs: namespace, labels, compiled terms
  M->specs.resize(NS);
  M->spec_poison.assign(NS, 0);
  for (int32_t s = 0; s < NS; ++s) {
    const kbg_spec& k = S.specs_in[s];
    AffSpec& a = M->specs[s];
    a.ns = S.canon[k.ns];
    std::map<int32_t, int32_t> lab;
    for (int32_t i = 0; i < k.pod_label_len; ++i)
      lab[S.canon[S.pod_labels_in[2 * (k.pod_label_off + i)]]] =
          S.canon[S.pod_labels_in[2 * (k.pod_label_off + i) + 1]];
    a.labels.assign(lab.begin(), lab.end());
    auto load = [&](int32_t off, int32_t len, std::vector<AffTerm>* out, bool* err) {
      for (int32_t i = 0; i < len; ++i) {
        const kbg_pod_term& pt = S.pod_terms_in[off + i];
        AffTerm t;
        t.sel = compile_label_selector(S, pt);
        if (t.sel.err) *err = true;
        for (int32_t v = 0; v < pt.ns_len; ++v) t.ns.push_back(S.canon[S.values_in[pt.ns_off + v]]);
        t.key = S.canon[pt.topology_key];
        t.key_empty = S.strs[pt.topology_key].empty();
        out->push_back(std::move(t));
      }
    };
    load(k.aff_off, k.aff_len, &a.aff, &a.aff_err);
    load(k.anti_off, k.anti_len, &a.anti, &a.anti_err);
    M->spec_poison[s] = a.anti_err ? 1 : 0;
  }
  // per class: (B) and (C) keys and node signatures
  M->cls.resize(C);
  std::map<std::vector<int32_t>, int32_t> tab_of;
  auto sig_table = [&](const std::vector<int32_t>& keys) -> int32_t {
    auto found = tab_of.find(keys);
    if (found != tab_of.end()) return found->second;
    const int32_t id = (int32_t)M->sigtabs.size();
    tab_of.emplace(keys, id);
    M->sigtabs.emplace_back();
    AffSigTable& tab = M->sigtabs.back();
    tab.keys = keys;
    tab.sig.assign(N, -1);
    std::map<std::vector<int32_t>, int32_t> ids;
    for (int32_t n = 0; n < N; ++n) {
      std::vector<int32_t> vals;
      bool all = true;
      for (int32_t key : keys) {
        const int32_t* v = find_label(M->node_labels[n], key);
        if (!v) {
          all = false;
          break;
        }
        vals.push_back(*v);
      }
      if (!all) continue;
      auto it = ids.find(vals);
      int32_t sg;
      if (it != ids.end()) {
        sg = it->second;
      } else {
        sg = (int32_t)ids.size();
        ids.emplace(vals, sg);
        tab.nodes.emplace_back();
      }
      tab.sig[n] = sg;
      tab.nodes[sg].push_back(n);
    }
    return id;
  };
  for (int32_t c = 0; c < C; ++c) {
    AffClass& a = M->cls[c];
    const int32_t s = S.class_spec[c];
    if (s < 0) continue;
    const AffSpec& sp = M->specs[s];
    if (!sp.aff.empty()) {
      a.hasB = true;
      a.b_err = sp.aff_err;
      std::vector<int32_t> keys;
      for (const AffTerm& t : sp.aff) {
        if (t.key_empty) a.b_empty_key = true;
        keys.push_back(t.key);
      }
      a.b_self = !a.b_err && all_terms_match(sp.aff, sp.ns, sp);  // targetPodMatchesAffinityOfPod(pod, pod)
      if (!a.b_err && !a.b_empty_key) a.b_tab = sig_table(keys);
    }
    if (!sp.anti.empty()) {
      a.hasC = true;
      a.c_err = sp.anti_err;
      if (a.c_err) M->c_err_classes.push_back(c);
      std::vector<int32_t> keys;
      for (const AffTerm& t : sp.anti) {
        if (t.key_empty) break;  // the error is reached once every earlier key matched
        keys.push_back(t.key);
      }
      if (!a.c_err) a.c_tab = sig_table(keys);
    }
  }
  // which classes each spec's pods select: as the owner of anti terms (A), as a target (B, C)
  M->anti_match.resize(NS);
  M->matchB.resize(NS);
  M->matchC.resize(NS);
  std::map<int32_t, char> anti_keys;
  for (int32_t s = 0; s < NS; ++s) {
    const AffSpec& sp = M->specs[s];
    M->anti_match[s].resize(sp.anti.size());
    for (size_t k = 0; k < sp.anti.size(); ++k) {
      const AffTerm& t = sp.anti[k];
      if (t.sel.err) continue;
      anti_keys[t.key] = 1;
      for (int32_t c = 0; c < C; ++c)
        if (S.class_spec[c] >= 0 && term_matches(t, sp.ns, M->specs[S.class_spec[c]]))
          M->anti_match[s][k].push_back(c);
    }
    for (int32_t c = 0; c < C; ++c) {
      const int32_t cs = S.class_spec[c];
      if (cs < 0) continue;
      const AffSpec& csp = M->specs[cs];
      if (M->cls[c].hasB && !M->cls[c].b_err && all_terms_match(csp.aff, csp.ns, sp)) M->matchB[s].push_back(c);
      if (M->cls[c].hasC && !M->cls[c].c_err && all_terms_match(csp.anti, csp.ns, sp)) M->matchC[s].push_back(c);
    }
  }
  for (int32_t n = 0; n < N; ++n)
    for (const auto& kv : M->node_labels[n])
      if (anti_keys.count(kv.first)) M->pair_nodes[pair_key(kv.first, kv.second)].push_back(n);
  M->spec_effect.assign(NS, 0);
  for (int32_t s = 0; s < NS; ++s) {
    bool e = M->spec_poison[s] || !M->matchB[s].empty() || !M->matchC[s].empty();
    for (const auto& l : M->anti_match[s]) e = e || !l.empty();
    M->spec_effect[s] = e ? 1 : 0;
  }
  // counts of the pods allocated at open
  AffState& st = M->st0;
  st.nB.assign(C, 0);
  st.cntA.assign(C, {});
  st.cntB.assign(C, {});
  st.cntC.assign(C, {});
  for (int32_t t = 0; t < S.n_tasks; ++t)
    if (S.task_live[t] && allocated_status(S.tasks_in[t].status)) aff_place(S, t, S.task_node[t], +1, st, false);
  M->st = st;
  // the predictor's failed-shape flags to clear when a class gains nodes
  M->class_shapes.assign(C, {});
  for (int32_t t = 0; t < S.n_tasks; ++t) {
    if (S.task_shape[t] < 0) continue;
    auto& v = M->class_shapes[S.task_class[t]];
    if (std::find(v.begin(), v.end(), S.task_shape[t]) == v.end()) v.push_back(S.task_shape[t]);
  }
  if (getenv("KBG_DEBUG_AFF")) {
    for (int32_t c = 0; c < C; ++c) {
      const AffClass& a = M->cls[c];
      int bits = 0;
      for (int32_t n = 0; n < N; ++n) bits += (S.h_class_mask[(size_t)c * S.W + (n >> 6)] >> (n & 63)) & 1;
      int ok = 0;
      for (int32_t n = 0; n < N; ++n) ok += aff_ok(S, M->st, c, n);
      const int32_t sp = S.class_spec[c];
      fprintf(stderr, "[aff] class %d spec %d hasB %d err %d self %d empty %d nB %d hasC %d cerr %d bits %d ok %d labels %zu ns %d\n",
              c, sp, a.hasB, a.b_err, a.b_self, a.b_empty_key, M->st.nB[c], a.hasC, a.c_err, bits, ok,
              sp >= 0 ? M->specs[sp].labels.size() : 0, sp >= 0 ? M->specs[sp].ns : -1);
    }
  }
  // fold into the class masks
  if (S.mask_dirty_flag.size() != S.h_class_mask.size()) S.mask_dirty_flag.assign(S.h_class_mask.size(), 0);
  S.mwmark.assign((size_t)C * S.W, -1);
  M->panic_words.assign(S.W, 0);
  for (int32_t n = 0; n < N; ++n)
    if (S.panic_node[n]) M->panic_words[n >> 6] |= 1ull << (n & 63);
  S.aff_gain_flag.assign(C, 0);
  S.aff_gain_classes.clear();
  for (int32_t c = 0; c < C; ++c)
    for (int32_t n = 0; n < N; ++n) {
      if (S.panic_node[n]) continue;
      if (!aff_ok(S, M->st, c, n)) S.h_class_mask[(size_t)c * S.W + (n >> 6)] &= ~(1ull << (n & 63));
    }
  S.mask_dirty.clear();
}

}  // namespace kbg
