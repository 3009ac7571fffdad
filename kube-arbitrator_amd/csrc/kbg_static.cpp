// Static part of the predicates plugin, compiled once per session into device
// programs (kbg_device.hpp ClassProg/TermProg/ReqProg) over node label/taint
// bitsets.
//
// Reference semantics restated here:
//   nodeSelector  -> labels.SelectorFromSet: every pair must be a valid
//                    requirement, otherwise the selector is EMPTY and matches
//                    every node (apimachinery labels/selector.go:849-866)
//   node affinity -> MatchNodeSelectorTerms: OR over terms; an empty term or a
//                    term whose requirements fail to build is skipped
//                    (k8s v1/helper/helpers.go:222-331, vendor
//                    predicates.go:807-850)
//   requirements  -> NewRequirement validation + Matches
//                    (labels/selector.go:134-236)
//   taints        -> NoSchedule/NoExecute taints must each be tolerated
//                    (predicates.go:1489-1517, helpers.go:412-441,
//                    core/v1/toleration.go:37-56)
#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "kbg_session.hpp"

namespace kbg {

namespace {

bool is_alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }

// ^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$  (validation.go:30-36)
bool qualified_token(const std::string& s) {
  if (s.empty() || !is_alnum(s[0]) || !is_alnum(s[s.size() - 1])) return false;
  return std::all_of(s.begin(), s.end(), [](char c) { return is_alnum(c) || c == '-' || c == '_' || c == '.'; });
}

// DNS-1123 subdomain (validation.go:125-140)
bool dns_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    size_t end = dot == std::string::npos ? s.size() : dot;
    if (end == start) return false;
    auto low = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!low(s[start]) || !low(s[end - 1])) return false;
    for (size_t i = start; i < end; ++i)
      if (!(low(s[i]) || s[i] == '-')) return false;
    if (dot == std::string::npos) return true;
    start = dot + 1;
  }
}

// IsQualifiedName (validation.go:42-70)
bool valid_label_key(const std::string& k) {
  const size_t slash = k.find('/');
  std::string name = k;
  if (slash != std::string::npos) {
    if (k.find('/', slash + 1) != std::string::npos) return false;
    if (slash == 0 || !dns_subdomain(k.substr(0, slash))) return false;
    name = k.substr(slash + 1);
  }
  return !name.empty() && name.size() <= 63 && qualified_token(name);
}

// IsValidLabelValue (validation.go:97-106)
bool valid_label_value(const std::string& v) { return v.size() <= 63 && (v.empty() || qualified_token(v)); }

}  // namespace

bool label_key_valid(const std::string& k) { return valid_label_key(k); }
bool label_value_valid(const std::string& v) { return valid_label_value(v); }

// strconv.ParseInt(s, 10, 64)
bool parse_go_int64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  uint64_t acc = 0;
  const uint64_t limit = neg ? (uint64_t)INT64_MAX + 1 : (uint64_t)INT64_MAX;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    const uint64_t d = (uint64_t)(s[i] - '0');
    if (acc > (limit - d) / 10) return false;
    acc = acc * 10 + d;
  }
  *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
  return true;
}

namespace {

struct Compiler {
  Session& S;
  // label dictionary: referenced (key,value) pairs and keys -> bit position
  std::map<std::pair<int32_t, int32_t>, int32_t> pair_bit;
  std::map<int32_t, int32_t> key_bit;
  std::map<int32_t, int32_t> num_col;  // Gt/Lt key -> numeric column
  int32_t nbits = 0;
  // programs (masks are stored as bit lists until the word width is known)
  std::vector<ReqProg> reqs;
  std::vector<std::vector<int32_t>> req_bits;  // per req: bits of its mask
  std::vector<TermProg> terms;
  std::vector<ClassProg> classes;

  explicit Compiler(Session& s) : S(s) {}

  int32_t bit_pair(int32_t k, int32_t v) {
    auto it = pair_bit.find({k, v});
    if (it != pair_bit.end()) return it->second;
    pair_bit[{k, v}] = nbits;
    return nbits++;
  }
  int32_t bit_key(int32_t k) {
    auto it = key_bit.find(k);
    if (it != key_bit.end()) return it->second;
    key_bit[k] = nbits;
    return nbits++;
  }
  int32_t add_req(int32_t kind, std::vector<int32_t> bits = {}, int32_t col = 0, int64_t value = 0) {
    ReqProg r{};
    r.kind = kind;
    r.col = col;
    r.value = value;
    reqs.push_back(r);
    req_bits.push_back(std::move(bits));
    return (int32_t)reqs.size() - 1;
  }
  const std::string& str(int32_t id) const { return S.strs[id]; }

  // NodeSelectorRequirementsAsSelector for one term; false => the term is skipped.
  bool compile_exprs(int32_t off, int32_t len, std::vector<int32_t>* out) {
    struct Tmp { int32_t kind; std::vector<int32_t> bits; int32_t col; int64_t val; };
    std::vector<Tmp> tmp;
    for (int32_t i = 0; i < len; ++i) {
      const kbg_requirement& r = S.reqs_in[off + i];
      const std::string& op = str(r.op);
      if (op != "In" && op != "NotIn" && op != "Exists" && op != "DoesNotExist" && op != "Gt" && op != "Lt") return false;
      if (!valid_label_key(str(r.key))) return false;
      const int32_t nv = r.value_len;
      if ((op == "In" || op == "NotIn") && nv == 0) return false;
      if ((op == "Exists" || op == "DoesNotExist") && nv != 0) return false;
      int64_t num = 0;
      if (op == "Gt" || op == "Lt") {
        if (nv != 1 || !parse_go_int64(str(S.values_in[r.value_off]), &num)) return false;
      }
      for (int32_t v = 0; v < nv; ++v)
        if (!valid_label_value(str(S.values_in[r.value_off + v]))) return false;
      const int32_t key = S.canon[r.key];
      Tmp t{REQ_FALSE, {}, 0, 0};
      if (op == "In" || op == "NotIn") {
        for (int32_t v = 0; v < nv; ++v) t.bits.push_back(bit_pair(key, S.canon[S.values_in[r.value_off + v]]));
        t.kind = op == "In" ? REQ_ANY : REQ_NONE;
      } else if (op == "Exists" || op == "DoesNotExist") {
        t.bits.push_back(bit_key(key));
        t.kind = op == "Exists" ? REQ_ANY : REQ_NONE;
      } else {
        auto it = num_col.find(key);
        int32_t col = it != num_col.end() ? it->second : (int32_t)num_col.size();
        if (it == num_col.end()) num_col[key] = col;
        t.kind = op == "Gt" ? REQ_GT : REQ_LT;
        t.col = col;
        t.val = num;
      }
      tmp.push_back(std::move(t));
    }
    for (auto& t : tmp) out->push_back(add_req(t.kind, std::move(t.bits), t.col, t.val));
    return true;
  }

  // NodeSelectorRequirementsAsFieldSelector; false => the term is skipped.
  bool compile_fields(int32_t off, int32_t len, std::vector<int32_t>* out) {
    for (int32_t i = 0; i < len; ++i) {
      const kbg_requirement& r = S.reqs_in[off + i];
      const std::string& op = str(r.op);
      if ((op != "In" && op != "NotIn") || r.value_len != 1) return false;
    }
    for (int32_t i = 0; i < len; ++i) {
      const kbg_requirement& r = S.reqs_in[off + i];
      const bool in = str(r.op) == "In";
      const int32_t val = S.values_in[r.value_off];
      if (str(r.key) == "metadata.name") {  // algorithm/types.go:30-32
        out->push_back(add_req(in ? REQ_NAME_EQ : REQ_NAME_NE, {}, 0, S.canon[val]));
      } else {  // fields.Set.Get of an absent key is ""
        const bool eq = str(val).empty();
        out->push_back(add_req((in ? eq : !eq) ? REQ_TRUE : REQ_FALSE));
      }
    }
    return true;
  }

  ClassProg compile_spec(const kbg_spec* sp) {
    ClassProg c{};
    c.sel_req = -1;
    c.tol_off = 0;
    if (!sp) return c;
    if (sp->selector_len > 0) {
      bool valid = true;
      std::vector<int32_t> bits;
      for (int32_t i = 0; i < sp->selector_len && valid; ++i) {
        const int32_t k = S.selectors_in[2 * (sp->selector_off + i)], v = S.selectors_in[2 * (sp->selector_off + i) + 1];
        if (!valid_label_key(str(k)) || !valid_label_value(str(v))) valid = false;
        else bits.push_back(bit_pair(S.canon[k], S.canon[v]));
      }
      if (valid) c.sel_req = add_req(REQ_ALL, bits);
    }
    if (sp->has_required_affinity) {
      c.has_affinity = 1;
      c.term_off = (int32_t)terms.size();
      for (int32_t ti = 0; ti < sp->term_len; ++ti) {
        const kbg_term& t = S.terms_in[sp->term_off + ti];
        if (t.expr_len == 0 && t.field_len == 0) continue;
        std::vector<int32_t> ids;
        if (t.expr_len > 0 && !compile_exprs(t.expr_off, t.expr_len, &ids)) continue;
        if (t.field_len > 0 && !compile_fields(t.field_off, t.field_len, &ids)) continue;
        // requirement ids of one term are contiguous by construction
        TermProg tp{ids.empty() ? 0 : ids.front(), (int32_t)ids.size()};
        terms.push_back(tp);
      }
      c.term_len = (int32_t)terms.size() - c.term_off;
    }
    return c;
  }
};

std::string spec_key(const Session& S, const kbg_spec* sp) {
  if (!sp) return "-";
  std::string k;
  auto add = [&](int32_t id) {
    const std::string& s = S.strs[id];
    k += std::to_string(s.size());
    k += ':';
    k += s;
  };
  std::vector<std::pair<std::string, std::string>> sel;
  for (int32_t i = 0; i < sp->selector_len; ++i)
    sel.emplace_back(S.strs[S.selectors_in[2 * (sp->selector_off + i)]], S.strs[S.selectors_in[2 * (sp->selector_off + i) + 1]]);
  std::sort(sel.begin(), sel.end());
  k += "S";
  for (auto& p : sel) k += std::to_string(p.first.size()) + ":" + p.first + std::to_string(p.second.size()) + ":" + p.second;
  k += "A" + std::to_string(sp->has_required_affinity);
  if (sp->has_required_affinity)
    for (int32_t ti = 0; ti < sp->term_len; ++ti) {
      const kbg_term& t = S.terms_in[sp->term_off + ti];
      k += "T";
      for (int pass = 0; pass < 2; ++pass) {
        const int32_t off = pass ? t.field_off : t.expr_off, len = pass ? t.field_len : t.expr_len;
        k += pass ? "F" : "E";
        for (int32_t i = 0; i < len; ++i) {
          const kbg_requirement& r = S.reqs_in[off + i];
          k += "R";
          add(r.key);
          add(r.op);
          for (int32_t v = 0; v < r.value_len; ++v) add(S.values_in[r.value_off + v]);
        }
      }
    }
  k += "O";
  for (int32_t i = 0; i < sp->toleration_len; ++i) {
    const kbg_toleration& t = S.tols_in[sp->toleration_off + i];
    k += "t";
    add(t.key);
    add(t.op);
    add(t.value);
    add(t.effect);
  }
  k += "P";  // host ports (vendor predicates.go:1031-1051): part of the class, checked dynamically
  for (int32_t i = 0; i < sp->port_len; ++i) {
    const kbg_host_port& hp = S.ports_in[sp->port_off + i];
    k += "p";
    add(hp.host_ip);
    add(hp.protocol);
    k += std::to_string(hp.host_port);
  }
  if (S.has_aff) {  // inter-pod (anti)affinity: what other pods' terms select, and the pod's own terms
    k += "N";
    add(sp->ns);
    std::vector<std::pair<std::string, std::string>> lab;
    for (int32_t i = 0; i < sp->pod_label_len; ++i)
      lab.emplace_back(S.strs[S.pod_labels_in[2 * (sp->pod_label_off + i)]],
                       S.strs[S.pod_labels_in[2 * (sp->pod_label_off + i) + 1]]);
    std::stable_sort(lab.begin(), lab.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t i = 0; i < lab.size(); ++i) {
      if (i + 1 < lab.size() && lab[i + 1].first == lab[i].first) continue;  // the last value of a key wins
      k += "l" + std::to_string(lab[i].first.size()) + ":" + lab[i].first + std::to_string(lab[i].second.size()) +
           ":" + lab[i].second;
    }
    for (int pass = 0; pass < 2; ++pass) {
      const int32_t off = pass ? sp->anti_off : sp->aff_off, len = pass ? sp->anti_len : sp->aff_len;
      k += pass ? "X" : "Y";
      for (int32_t i = 0; i < len; ++i) {
        const kbg_pod_term& t = S.pod_terms_in[off + i];
        k += "q" + std::to_string(t.has_selector);
        for (int32_t m = 0; m < t.match_len; ++m) {
          add(S.selectors_in[2 * (t.match_off + m)]);
          add(S.selectors_in[2 * (t.match_off + m) + 1]);
        }
        k += "e";
        for (int32_t m = 0; m < t.expr_len; ++m) {
          const kbg_requirement& r = S.reqs_in[t.expr_off + m];
          k += "R";
          add(r.key);
          add(r.op);
          for (int32_t v = 0; v < r.value_len; ++v) add(S.values_in[r.value_off + v]);
        }
        k += "n";
        for (int32_t m = 0; m < t.ns_len; ++m) add(S.values_in[t.ns_off + m]);
        k += "k";
        add(t.topology_key);
      }
    }
  }
  return k;
}

}  // namespace

// Builds classes for every pending task (allocate and backfill candidates), the node bitsets and the device
// programs; fills S.task_class and S.static_host (uploaded by the caller).
void compile_static_predicates(Session& S, StaticHost* out) {
  Compiler C(S);
  out->n_classes = 0;
  S.task_class.assign(S.n_tasks, 0);
  S.class_spec.assign(1, -1);
  if (!S.pred_active) {
    ClassProg c{};
    c.sel_req = -1;
    c.always = 1;
    C.classes.push_back(c);
    S.spec_class.assign(S.specs_in.size(), 0);
    S.nospec_class = 0;
  } else {
    std::unordered_map<std::string, int32_t> class_of_key;
    std::vector<int32_t> class_spec;
    // a spec's class is its key's: each spec's key is built once (the tasks
    // share a few specs), classes numbered in order of their first task
    std::vector<int32_t> memo(S.specs_in.size() + 1, -1);  // [spec + 1] -> class; [0]: no spec
    for (int32_t t = 0; t < S.n_tasks; ++t) {
      if (!S.pending_candidate[t] && !S.be_task[t]) continue;  // allocate and backfill candidates
      const int32_t sp = S.tasks_in[t].spec;
      int32_t& m = memo[(size_t)(sp + 1)];
      if (m < 0) {
        const kbg_spec* spec = sp >= 0 ? &S.specs_in[sp] : nullptr;
        std::string key = spec_key(S, spec);
        auto it = class_of_key.find(key);
        if (it == class_of_key.end()) {
          const int32_t id = (int32_t)class_spec.size();
          class_of_key.emplace(std::move(key), id);
          class_spec.push_back(sp);
          m = id;
        } else {
          m = it->second;
        }
      }
      S.task_class[t] = m;
    }
    if (class_spec.empty()) class_spec.push_back(-1);
    S.class_spec = class_spec;
    // the class of every spec (for tasks that become candidates in a session
    // update): a spec whose key no candidate had at compile time has none
    S.spec_class.assign(S.specs_in.size(), -1);
    for (size_t sp = 0; sp < S.specs_in.size(); ++sp) {
      auto it = class_of_key.find(spec_key(S, &S.specs_in[sp]));
      if (it != class_of_key.end()) S.spec_class[sp] = it->second;
    }
    auto it0 = class_of_key.find(spec_key(S, nullptr));
    S.nospec_class = it0 != class_of_key.end() ? it0->second : -1;
    for (int32_t sp : class_spec) C.classes.push_back(C.compile_spec(sp >= 0 ? &S.specs_in[sp] : nullptr));

    // taint dictionary over NoSchedule/NoExecute taints of the session nodes
    std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> taint_bit;
    for (int32_t n = 0; n < S.n_nodes; ++n) {
      const kbg_node& nd = S.nodes_in[n];
      for (int32_t i = 0; i < nd.taint_len; ++i) {
        const kbg_taint& t = S.taints_in[nd.taint_off + i];
        const std::string& eff = S.strs[t.effect];
        if (eff != "NoSchedule" && eff != "NoExecute") continue;
        auto key = std::make_tuple(S.canon[t.key], S.canon[t.value], S.canon[t.effect]);
        if (!taint_bit.count(key)) {
          const int32_t b = (int32_t)taint_bit.size();
          taint_bit[key] = b;
        }
      }
    }
    out->taint_words = std::max<int32_t>(1, ((int32_t)taint_bit.size() + 63) / 64);
    out->taint_bits.assign((size_t)out->taint_words * S.n_nodes, 0);
    for (int32_t n = 0; n < S.n_nodes; ++n) {
      const kbg_node& nd = S.nodes_in[n];
      for (int32_t i = 0; i < nd.taint_len; ++i) {
        const kbg_taint& t = S.taints_in[nd.taint_off + i];
        auto it = taint_bit.find(std::make_tuple(S.canon[t.key], S.canon[t.value], S.canon[t.effect]));
        if (it == taint_bit.end()) continue;
        out->taint_bits[(size_t)(it->second / 64) * S.n_nodes + n] |= 1ull << (it->second % 64);
      }
    }
    // tolerated mask per class (ToleratesTaint over the dictionary)
    out->tol_pool.assign((size_t)out->taint_words * C.classes.size(), 0);
    for (size_t c = 0; c < C.classes.size(); ++c) {
      C.classes[c].tol_off = (int32_t)(c * out->taint_words);
      const int32_t sp = class_spec[c];
      if (sp < 0) continue;
      const kbg_spec& spec = S.specs_in[sp];
      for (auto& kv : taint_bit) {
        const std::string& tkey = S.strs[std::get<0>(kv.first)];
        const std::string& tval = S.strs[std::get<1>(kv.first)];
        const std::string& teff = S.strs[std::get<2>(kv.first)];
        bool tolerated = false;
        for (int32_t i = 0; i < spec.toleration_len && !tolerated; ++i) {
          const kbg_toleration& tol = S.tols_in[spec.toleration_off + i];
          const std::string& e = S.strs[tol.effect];
          const std::string& k = S.strs[tol.key];
          const std::string& op = S.strs[tol.op];
          if (!e.empty() && e != teff) continue;
          if (!k.empty() && k != tkey) continue;
          if (op.empty() || op == "Equal") tolerated = S.strs[tol.value] == tval;
          else if (op == "Exists") tolerated = true;
        }
        if (tolerated) out->tol_pool[c * out->taint_words + kv.second / 64] |= 1ull << (kv.second % 64);
      }
    }
  }

  // node label bitsets, numeric columns, names, flags
  const int32_t N = S.n_nodes;
  out->label_words = std::max<int32_t>(1, (C.nbits + 63) / 64);
  out->label_bits.assign((size_t)out->label_words * N, 0);
  out->n_numcols = (int32_t)C.num_col.size();
  out->num_vals.assign((size_t)std::max<int32_t>(1, out->n_numcols) * N, 0);
  out->num_ok.assign((size_t)std::max<int32_t>(1, out->n_numcols) * N, 0);
  out->name_id.assign(N, -1);
  out->node_flags.assign(N, 0);
  if (out->taint_bits.empty()) {
    out->taint_words = 1;
    out->taint_bits.assign(N, 0);
    out->tol_pool.assign(C.classes.size(), 0);
  }
  for (int32_t n = 0; n < N; ++n) {
    const kbg_node& nd = S.nodes_in[n];
    out->name_id[n] = S.canon[nd.name];
    if (!nd.has_node) out->node_flags[n] |= NF_NIL;
    if (nd.unschedulable) out->node_flags[n] |= NF_UNSCHED;
    if (S.ghost) out->node_flags[n] |= NF_DEAD;
    // labels.Set semantics: last value of a key wins
    std::map<int32_t, int32_t> lab;
    for (int32_t i = 0; i < nd.label_len; ++i)
      lab[S.canon[S.labels_in[2 * (nd.label_off + i)]]] = S.canon[S.labels_in[2 * (nd.label_off + i) + 1]];
    for (auto& kv : lab) {
      auto kb = C.key_bit.find(kv.first);
      if (kb != C.key_bit.end()) out->label_bits[(size_t)(kb->second / 64) * N + n] |= 1ull << (kb->second % 64);
      auto pb = C.pair_bit.find({kv.first, kv.second});
      if (pb != C.pair_bit.end()) out->label_bits[(size_t)(pb->second / 64) * N + n] |= 1ull << (pb->second % 64);
      auto nc = C.num_col.find(kv.first);
      if (nc != C.num_col.end()) {
        int64_t v;
        if (parse_go_int64(S.strs[kv.second], &v)) {
          out->num_vals[(size_t)nc->second * N + n] = v;
          out->num_ok[(size_t)nc->second * N + n] = 1;
        }
      }
    }
  }
  // masks for ALL/ANY/NONE requirements
  out->mask_pool.clear();
  for (size_t r = 0; r < C.reqs.size(); ++r) {
    C.reqs[r].mask_off = (int32_t)out->mask_pool.size();
    for (int32_t w = 0; w < out->label_words; ++w) out->mask_pool.push_back(0);
    for (int32_t b : C.req_bits[r]) out->mask_pool[C.reqs[r].mask_off + b / 64] |= 1ull << (b % 64);
  }
  if (out->mask_pool.empty()) out->mask_pool.push_back(0);
  out->reqs = C.reqs;
  if (out->reqs.empty()) out->reqs.push_back(ReqProg{});
  out->terms = C.terms;
  if (out->terms.empty()) out->terms.push_back(TermProg{0, 0});
  out->classes = C.classes;
  out->n_classes = (int32_t)C.classes.size();
}

}  // namespace kbg
