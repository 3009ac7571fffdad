// kbref — CPU restatement of kube-batch v0.4's allocate hot path.
//
// TEST INFRASTRUCTURE ONLY. This program is the parity oracle for the
// MI355X path in kube-arbitrator_amd/. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may run it, and only as the checker or as
// the timed CPU baseline — never as the product path.
//
// It restates, object for object, what the reference does between
// cache.Snapshot() and the end of allocate.Execute():
//   pkg/scheduler/cache/event_handlers.go:40-61,232-240,344-358,458-470,635-640,726-736 (cache builders)
//   pkg/scheduler/cache/cache.go:549-597 (Snapshot)
//   pkg/scheduler/framework/{framework.go:26-54, session.go:63-316, session_plugins.go:23-295}
//   pkg/scheduler/util/priority_queue.go:25-88 + Go 1.11 container/heap (up/down/Push/Pop)
//   pkg/scheduler/api/{resource_info.go, node_info.go, job_info.go, helpers.go, helpers/helpers.go}
//   pkg/scheduler/plugins/{drf,proportion,gang,priority,predicates}
//   pkg/scheduler/actions/allocate/allocate.go:41-176
//   pkg/scheduler/actions/backfill/backfill.go:40-71 (fixture "actions": [..., "backfill"])
//   pkg/scheduler/actions/{reclaim/reclaim.go:41-188, preempt/preempt.go:43-253}, framework/statement.go
//   vendor/k8s.io/kubernetes/pkg/scheduler/algorithm/predicates/predicates.go:797-862,1031-1051,1489-1517
//   vendor/k8s.io/kubernetes/pkg/scheduler/cache/host_ports.go:29-135, node_info.go:593-605 (host ports)
//   vendor/k8s.io/kubernetes/pkg/apis/core/v1/helper/helpers.go:222-331,412-441
//   vendor/k8s.io/api/core/v1/toleration.go:37-56
//   vendor/k8s.io/apimachinery/pkg/labels/selector.go:134-236,849-866
//   vendor/k8s.io/apimachinery/pkg/util/validation/validation.go:30-160
//   vendor/k8s.io/apimachinery/pkg/api/resource quantity MilliValue/Value (ceil)
//
// Parity pinning: the reference's own tests are restated as fixtures under
// tests/golden/ref_* (allocate_test.go:140-300 cases 1-2, node_info_test.go,
// job_info_test.go, cache_test.go). Those pin the data model and the
// drf/proportion/queue path. The predicate truth tables, gang and priority
// paths are pinned by hand-derived KATs (tests/golden/kat_*) and by the
// reference's e2e specs (test/e2e/{job,predicates,queue}.go) restated as
// multi-cycle fake-cluster runs whose conditions the oracle must reach
// (tests/e2e_sim.py, tests/test_e2e_scenarios.py): "restated, not executed",
// because no Go toolchain exists here.
//
// Go map iteration order (random in the reference) is replaced by insertion
// order everywhere; SURVEY F4 makes that order an input of both sides.
//
// Inter-pod (anti)affinity (vendor predicates.go:1155-1466, the meta == nil
// slow path) and host ports run in every action, with the podLister and
// node.Pods() read live. Nothing is rejected as "unsupported" by the oracle;
// the device path refuses only nodes with more than 1024 Running candidates
// in a victim scan.

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "json.hpp"

using kbjson::Value;

namespace ref {

struct RefPanic : std::runtime_error {
  explicit RefPanic(const std::string& m) : std::runtime_error(m) {}
};
struct Unsupported : std::runtime_error {
  explicit Unsupported(const std::string& m) : std::runtime_error(m) {}
};
struct BadInput : std::runtime_error {
  explicit BadInput(const std::string& m) : std::runtime_error(m) {}
};

// ---------------------------------------------------------------- Resource
// pkg/scheduler/api/resource_info.go:26-168
static const double kMinMilliCPU = 10;
static const double kMinMilliGPU = 10;
static const double kMinMemory = 10.0 * 1024 * 1024;

struct Resource {
  double MilliCPU = 0, Memory = 0, MilliGPU = 0;
  int MaxTaskNum = 0;

  bool IsEmpty() const {  // :75-77
    return MilliCPU < kMinMilliCPU && Memory < kMinMemory && MilliGPU < kMinMilliGPU;
  }
  Resource& Add(const Resource& rr) {  // :92-97
    MilliCPU += rr.MilliCPU;
    Memory += rr.Memory;
    MilliGPU += rr.MilliGPU;
    return *this;
  }
  bool Less(const Resource& rr) const {  // :138-140 (every dimension strictly less)
    return MilliCPU < rr.MilliCPU && Memory < rr.Memory && MilliGPU < rr.MilliGPU;
  }
  bool LessEqual(const Resource& rr) const {  // :142-146
    return (MilliCPU < rr.MilliCPU || std::fabs(rr.MilliCPU - MilliCPU) < kMinMilliCPU) &&
           (Memory < rr.Memory || std::fabs(rr.Memory - Memory) < kMinMemory) &&
           (MilliGPU < rr.MilliGPU || std::fabs(rr.MilliGPU - MilliGPU) < kMinMilliGPU);
  }
  Resource& Sub(const Resource& rr) {  // :100-110 — panics when rr does not fit
    if (rr.LessEqual(*this)) {
      MilliCPU -= rr.MilliCPU;
      Memory -= rr.Memory;
      MilliGPU -= rr.MilliGPU;
      return *this;
    }
    throw RefPanic("Resource is not sufficient to do operation");
  }
  Resource& FitDelta(const Resource& rr) {  // :116-129
    if (rr.MilliCPU > 0) MilliCPU -= rr.MilliCPU + kMinMilliCPU;
    if (rr.Memory > 0) Memory -= rr.Memory + kMinMemory;
    if (rr.MilliGPU > 0) MilliGPU -= rr.MilliGPU + kMinMilliGPU;
    return *this;
  }
  Resource& Multi(double ratio) {  // :131-136
    MilliCPU = MilliCPU * ratio;
    Memory = Memory * ratio;
    MilliGPU = MilliGPU * ratio;
    return *this;
  }
  double Get(int d) const { return d == 0 ? MilliCPU : d == 1 ? Memory : MilliGPU; }  // :153-164
};

// Go math.Min (handles signed zeros / NaN) — api/helpers/helpers.go:25-33
static double go_min(double x, double y) {
  if (std::isinf(x) && x < 0) return x;
  if (std::isinf(y) && y < 0) return y;
  if (std::isnan(x) || std::isnan(y)) return NAN;
  if (x == 0 && x == y) return std::signbit(x) ? x : y;
  return x < y ? x : y;
}
static Resource helpers_min(const Resource& l, const Resource& r) {
  Resource res;
  res.MilliCPU = go_min(l.MilliCPU, r.MilliCPU);
  res.MilliGPU = go_min(l.MilliGPU, r.MilliGPU);
  res.Memory = go_min(l.Memory, r.Memory);
  return res;
}
static double helpers_share(double l, double r) {  // helpers/helpers.go:35-48
  if (r == 0) return l == 0 ? 0 : 1;
  return l / r;
}

// ---------------------------------------------------------------- Quantity
// k8s.io/apimachinery/pkg/api/resource: MilliValue() = ScaledValue(-3),
// Value() = ScaledValue(0); both round toward +inf (quantity.go:684-703).
static int64_t quantity_scaled(const std::string& q, int scale) {
  size_t p = 0;
  bool neg = false;
  if (p < q.size() && (q[p] == '+' || q[p] == '-')) { neg = q[p] == '-'; p++; }
  __int128 num = 0;
  int frac = 0, ndig = 0;
  bool seen_dot = false;
  while (p < q.size() && ((q[p] >= '0' && q[p] <= '9') || q[p] == '.')) {
    if (q[p] == '.') { if (seen_dot) throw BadInput("bad quantity " + q); seen_dot = true; p++; continue; }
    if (ndig < 36) { num = num * 10 + (q[p] - '0'); if (seen_dot) frac++; ndig++; }
    else if (!seen_dot) throw BadInput("quantity too large " + q);
    p++;
  }
  if (ndig == 0) throw BadInput("bad quantity " + q);
  std::string suf = q.substr(p);
  int dec_exp = 0, bin_exp = 0;
  if (suf.empty()) {}
  else if (suf == "n") dec_exp = -9;
  else if (suf == "u") dec_exp = -6;
  else if (suf == "m") dec_exp = -3;
  else if (suf == "k") dec_exp = 3;
  else if (suf == "M") dec_exp = 6;
  else if (suf == "G") dec_exp = 9;
  else if (suf == "T") dec_exp = 12;
  else if (suf == "P") dec_exp = 15;
  else if (suf == "E") dec_exp = 18;
  else if (suf == "Ki") bin_exp = 10;
  else if (suf == "Mi") bin_exp = 20;
  else if (suf == "Gi") bin_exp = 30;
  else if (suf == "Ti") bin_exp = 40;
  else if (suf == "Pi") bin_exp = 50;
  else if (suf == "Ei") bin_exp = 60;
  else if (suf[0] == 'e' || suf[0] == 'E') dec_exp = (int)strtol(suf.c_str() + 1, nullptr, 10);
  else throw BadInput("bad quantity suffix " + q);
  __int128 den = 1;
  for (int i = 0; i < frac; i++) den *= 10;
  int e10 = dec_exp + scale;
  const __int128 lim = (__int128)1 << 100;
  for (int i = 0; i < bin_exp; i++) { num *= 2; if (num > lim) throw BadInput("quantity overflow " + q); }
  for (; e10 > 0; e10--) { num *= 10; if (num > lim) throw BadInput("quantity overflow " + q); }
  for (; e10 < 0; e10++) den *= 10;
  __int128 v;
  if (!neg) v = (num + den - 1) / den;
  else v = -(num / den);
  if (v > (__int128)INT64_MAX || v < -(__int128)INT64_MAX) throw BadInput("quantity overflow " + q);
  return (int64_t)v;
}

// pkg/scheduler/api/resource_info.go:58-73 (NewResource over a ResourceList)
static Resource new_resource(const Value* rl) {
  Resource r;
  if (!rl || !rl->is_obj()) return r;
  for (auto& kv : rl->obj) {
    std::string q = kv.second.is_str() ? kv.second.s : (kv.second.kind == Value::Int ? std::to_string(kv.second.i) : "");
    if (kv.second.kind == Value::Double) throw BadInput("use string quantities");
    if (kv.first == "cpu") r.MilliCPU += (double)quantity_scaled(q, 3);
    else if (kv.first == "memory") r.Memory += (double)quantity_scaled(q, 0);
    else if (kv.first == "pods") r.MaxTaskNum += (int)quantity_scaled(q, 0);
    else if (kv.first == "nvidia.com/gpu") r.MilliGPU += (double)quantity_scaled(q, 3);
  }
  return r;
}

// ------------------------------------------------------- label validation
// apimachinery/pkg/util/validation/validation.go:30-160
static bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
static bool qualified_name_re(const std::string& s) {  // ^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$
  if (s.empty()) return false;
  if (!alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
static bool dns1123_label(const std::string& s) {  // [a-z0-9]([-a-z0-9]*[a-z0-9])?
  if (s.empty()) return false;
  auto lc = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
  if (!lc(s.front()) || !lc(s.back())) return false;
  for (char c : s)
    if (!(lc(c) || c == '-')) return false;
  return true;
}
static bool is_dns1123_subdomain(const std::string& s) {
  if (s.size() > 253) return false;
  size_t st = 0;
  for (;;) {
    size_t d = s.find('.', st);
    std::string part = s.substr(st, d == std::string::npos ? std::string::npos : d - st);
    if (!dns1123_label(part)) return false;
    if (d == std::string::npos) return true;
    st = d + 1;
  }
}
static bool is_qualified_name(const std::string& v) {
  size_t slash = v.find('/');
  std::string name;
  if (slash == std::string::npos) name = v;
  else {
    if (v.find('/', slash + 1) != std::string::npos) return false;
    std::string prefix = v.substr(0, slash);
    name = v.substr(slash + 1);
    if (prefix.empty() || !is_dns1123_subdomain(prefix)) return false;
  }
  if (name.empty() || name.size() > 63) return false;
  return qualified_name_re(name);
}
static bool is_valid_label_value(const std::string& v) {
  if (v.size() > 63) return false;
  return v.empty() || qualified_name_re(v);
}
// strconv.ParseInt(s, 10, 64)
static bool go_parse_int64(const std::string& s, int64_t* out) {
  size_t p = 0;
  bool neg = false;
  if (s.empty()) return false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; p = 1; }
  if (p >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; p < s.size(); p++) {
    if (s[p] < '0' || s[p] > '9') return false;
    v = v * 10 + (unsigned)(s[p] - '0');
    if (v > (unsigned __int128)INT64_MAX + 1) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

// ------------------------------------------------------------ k8s objects
typedef std::vector<std::pair<std::string, std::string>> StrMap;  // ordered map
static const std::string* map_get(const StrMap& m, const std::string& k) {
  for (auto& kv : m)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
static StrMap parse_strmap(const Value* v) {
  StrMap m;
  if (!v || !v->is_obj()) return m;
  for (auto& kv : v->obj) {
    if (!kv.second.is_str()) throw BadInput("label map values must be strings");
    bool dup = false;
    for (auto& e : m) if (e.first == kv.first) { e.second = kv.second.s; dup = true; }
    if (!dup) m.emplace_back(kv.first, kv.second.s);
  }
  return m;
}

struct Taint { std::string key, value, effect; };
struct Toleration { std::string key, op, value, effect; };
struct NodeSelectorRequirement { std::string key, op; std::vector<std::string> values; };
struct NodeSelectorTerm { std::vector<NodeSelectorRequirement> exprs, fields; };

struct Pod {
  std::string uid, ns, name, phase, nodeName, controller;
  bool has_priority = false;
  int32_t priority = 0;
  bool deleting = false;
  StrMap annotations, labels, nodeSelector;
  bool has_affinity = false, has_node_affinity = false, has_required = false;
  std::vector<NodeSelectorTerm> terms;
  bool has_pod_affinity = false, has_pod_anti_affinity = false;
  struct LabelSelector {  // metav1.LabelSelector; absent = nil (selects nothing)
    bool present = false;
    StrMap matchLabels;
    std::vector<NodeSelectorRequirement> exprs;
  };
  struct AffinityTerm {  // v1.PodAffinityTerm
    LabelSelector selector;
    std::vector<std::string> namespaces;
    std::string topologyKey;
  };
  std::vector<AffinityTerm> aff_terms, anti_terms;  // RequiredDuringSchedulingIgnoredDuringExecution
  std::vector<Toleration> tolerations;
  std::vector<Value> containers_requests;
  bool has_host_port = false;
  struct Port { std::string ip, protocol; int64_t port; };
  std::vector<Port> ports;  // GetContainerPorts(pod) (vendor scheduler/util/utils.go:30-41)
  Resource resreq;
};

struct Node {
  std::string name;
  Resource allocatable, capacity;
  StrMap labels;
  std::vector<Taint> taints;
  bool unschedulable = false;
};

struct PodGroup { std::string ns, name, queue; int32_t minMember = 0; int64_t creation = 0; };
struct PDB { std::string ns, name, controller; int32_t minAvailable = 0; int64_t creation = 0; };

static std::vector<NodeSelectorRequirement> parse_reqs(const Value* v) {
  std::vector<NodeSelectorRequirement> out;
  if (!v || !v->is_arr()) return out;
  for (auto& e : v->arr) {
    NodeSelectorRequirement r;
    r.key = e.str("key");
    r.op = e.str("operator");
    if (const Value* vals = e.get("values"))
      for (auto& s : vals->arr) r.values.push_back(s.s);
    out.push_back(r);
  }
  return out;
}

static Pod parse_pod(const Value& v) {
  Pod p;
  p.uid = v.str("uid");
  p.ns = v.str("namespace");
  p.name = v.str("name");
  p.phase = v.str("phase", "Pending");
  p.nodeName = v.str("nodeName");
  p.controller = v.str("controller");
  if (const Value* pr = v.get("priority"); pr && !pr->is_null()) { p.has_priority = true; p.priority = (int32_t)pr->i; }
  p.deleting = v.boolean("deleting") || (v.get("deletionTimestamp") && !v.get("deletionTimestamp")->is_null());
  p.annotations = parse_strmap(v.get("annotations"));
  p.labels = parse_strmap(v.get("labels"));
  p.nodeSelector = parse_strmap(v.get("nodeSelector"));
  if (const Value* aff = v.get("affinity"); aff && aff->is_obj()) {
    p.has_affinity = true;
    if (const Value* na = aff->get("nodeAffinity"); na && na->is_obj()) {
      p.has_node_affinity = true;
      if (const Value* rq = na->get("requiredDuringSchedulingIgnoredDuringExecution"); rq && rq->is_obj()) {
        p.has_required = true;
        if (const Value* ts = rq->get("nodeSelectorTerms"); ts && ts->is_arr())
          for (auto& t : ts->arr) {
            NodeSelectorTerm term;
            term.exprs = parse_reqs(t.get("matchExpressions"));
            term.fields = parse_reqs(t.get("matchFields"));
            p.terms.push_back(term);
          }
      }
    }
    auto parse_terms = [](const Value* pa, std::vector<Pod::AffinityTerm>* out) {
      const Value* rq = pa->get("requiredDuringSchedulingIgnoredDuringExecution");
      if (!rq || !rq->is_arr()) return;
      for (auto& t : rq->arr) {
        Pod::AffinityTerm term;
        if (const Value* ls = t.get("labelSelector"); ls && ls->is_obj()) {
          term.selector.present = true;
          term.selector.matchLabels = parse_strmap(ls->get("matchLabels"));
          term.selector.exprs = parse_reqs(ls->get("matchExpressions"));
        }
        if (const Value* ns = t.get("namespaces"); ns && ns->is_arr())
          for (auto& x : ns->arr) term.namespaces.push_back(x.s);
        term.topologyKey = t.str("topologyKey");
        out->push_back(term);
      }
    };
    if (const Value* pa = aff->get("podAffinity"); pa && pa->is_obj()) {
      p.has_pod_affinity = true;
      parse_terms(pa, &p.aff_terms);
    }
    if (const Value* pa = aff->get("podAntiAffinity"); pa && pa->is_obj()) {
      p.has_pod_anti_affinity = true;
      parse_terms(pa, &p.anti_terms);
    }
  }
  if (const Value* ts = v.get("tolerations"); ts && ts->is_arr())
    for (auto& t : ts->arr) p.tolerations.push_back({t.str("key"), t.str("operator"), t.str("value"), t.str("effect")});
  // TaskInfo.Resreq = Σ containers' requests (job_info.go:64-70)
  if (const Value* cs = v.get("containers"); cs && cs->is_arr()) {
    for (auto& c : cs->arr) {
      p.resreq.Add(new_resource(c.get("requests")));
      if (const Value* ports = c.get("ports"); ports && ports->is_arr())
        for (auto& pt : ports->arr) {
          p.ports.push_back({pt.str("hostIP"), pt.str("protocol"), pt.integer("hostPort")});
          if (pt.integer("hostPort") > 0) p.has_host_port = true;
        }
    }
  }
  return p;
}

// ---------------------------------------------------------------- api types
// pkg/scheduler/api/types.go:20-60
enum TaskStatus {
  Pending = 1 << 0, Allocated = 1 << 1, Pipelined = 1 << 2, Binding = 1 << 3, Bound = 1 << 4,
  Running = 1 << 5, Releasing = 1 << 6, Succeeded = 1 << 7, Failed = 1 << 8, Unknown = 1 << 9
};
static bool AllocatedStatus(int s) { return s == Bound || s == Binding || s == Running || s == Allocated; }  // helpers.go:63-70

static int get_task_status(const Pod& p) {  // api/helpers.go:35-61
  if (p.phase == "Running") return p.deleting ? Releasing : Running;
  if (p.phase == "Pending") {
    if (p.deleting) return Releasing;
    return p.nodeName.empty() ? Pending : Bound;
  }
  if (p.phase == "Unknown") return Unknown;
  if (p.phase == "Succeeded") return Succeeded;
  if (p.phase == "Failed") return Failed;
  return Unknown;
}

struct TaskInfo {
  std::string uid, job, name, ns, nodeName;
  Resource resreq;
  int status = Pending;
  int32_t priority = 1;
  const Pod* pod = nullptr;
  int spec_class = -1;  // identity of the static predicate inputs (oracle-internal cache key)
};

static std::string pod_key(const Pod* p) { return p->ns.empty() ? p->name : p->ns + "/" + p->name; }

// Insertion-ordered map (replaces Go maps whose iteration order is random).
template <class V>
struct OMap {
  std::list<std::pair<std::string, V>> items;
  std::unordered_map<std::string, typename std::list<std::pair<std::string, V>>::iterator> idx;
  V* find(const std::string& k) {
    auto it = idx.find(k);
    return it == idx.end() ? nullptr : &it->second->second;
  }
  void set(const std::string& k, V v) {
    auto it = idx.find(k);
    if (it != idx.end()) { it->second->second = v; return; }
    items.emplace_back(k, v);
    idx[k] = std::prev(items.end());
  }
  bool erase(const std::string& k) {
    auto it = idx.find(k);
    if (it == idx.end()) return false;
    items.erase(it->second);
    idx.erase(it);
    return true;
  }
  size_t size() const { return items.size(); }
};

struct NodeInfo {  // api/node_info.go:26-42
  std::string name;
  const Node* node = nullptr;
  Resource releasing, idle, used, allocatable, capability;
  OMap<TaskInfo*> tasks;  // keyed by PodKey; the node owns clones

  static NodeInfo* make(const Node* n) {  // :44-71
    NodeInfo* ni = new NodeInfo();
    if (n) {
      ni->name = n->name;
      ni->node = n;
      ni->idle = n->allocatable;
      ni->allocatable = n->allocatable;
      ni->capability = n->capacity;
    }
    return ni;
  }
  void SetNode(const Node* n) {  // :84-99 (Releasing and Used are not reset, as in the reference)
    name = n->name;
    node = n;
    allocatable = n->allocatable;
    capability = n->capacity;
    idle = n->allocatable;
    for (auto& kv : tasks.items) {
      if (kv.second->status == Releasing) releasing.Add(kv.second->resreq);
      idle.Sub(kv.second->resreq);
      used.Add(kv.second->resreq);
    }
  }
  bool AddTask(const TaskInfo* task) {  // :101-129
    std::string key = pod_key(task->pod);
    if (tasks.find(key)) return false;  // "already on node" error
    TaskInfo* ti = new TaskInfo(*task);
    if (node) {
      switch (ti->status) {
        case Releasing: releasing.Add(ti->resreq); idle.Sub(ti->resreq); break;
        case Pipelined: releasing.Sub(ti->resreq); break;
        default: idle.Sub(ti->resreq);
      }
      used.Add(ti->resreq);
    }
    tasks.set(key, ti);
    return true;
  }
  bool RemoveTask(const TaskInfo* ti) {  // :131-157
    std::string key = pod_key(ti->pod);
    TaskInfo** t = tasks.find(key);
    if (!t) return false;
    TaskInfo* task = *t;
    if (node) {
      switch (task->status) {
        case Releasing: releasing.Sub(task->resreq); idle.Add(task->resreq); break;
        case Pipelined: releasing.Add(task->resreq); break;
        default: idle.Add(task->resreq);
      }
      used.Sub(task->resreq);
    }
    tasks.erase(key);
    return true;
  }
  NodeInfo* Clone() const {  // :73-81
    NodeInfo* res = make(node);
    for (auto& kv : tasks.items) res->AddTask(kv.second);
    return res;
  }
};

struct JobInfo {  // api/job_info.go:118-145
  std::string uid, name, ns, queue;
  int priority = 0;
  int32_t minAvailable = 0;
  std::map<std::string, Resource> nodesFitDelta;
  // B-omp only: the last evaluated task's FitDelta entries in node order,
  // turned into nodesFitDelta when allocate ends (same map, built once)
  std::vector<std::pair<const NodeInfo*, Resource>> fit_log;
  bool fit_log_pending = false;
  std::map<int, OMap<TaskInfo*>> statusIndex;
  OMap<TaskInfo*> tasks;
  Resource allocated, totalRequest;
  int64_t creation = 0;
  const PodGroup* podGroup = nullptr;
  const PDB* pdb = nullptr;

  void addTaskIndex(TaskInfo* ti) { statusIndex[ti->status].set(ti->uid, ti); }
  void AddTaskInfo(TaskInfo* ti) {  // :228-237
    tasks.set(ti->uid, ti);
    addTaskIndex(ti);
    totalRequest.Add(ti->resreq);
    if (AllocatedStatus(ti->status)) allocated.Add(ti->resreq);
  }
  void deleteTaskIndex(TaskInfo* ti) {  // :254-262
    auto it = statusIndex.find(ti->status);
    if (it != statusIndex.end()) {
      it->second.erase(ti->uid);
      if (it->second.size() == 0) statusIndex.erase(it);
    }
  }
  bool DeleteTaskInfo(TaskInfo* ti) {  // :264-280
    TaskInfo** t = tasks.find(ti->uid);
    if (!t) return false;
    TaskInfo* task = *t;
    totalRequest.Sub(task->resreq);
    if (AllocatedStatus(task->status)) allocated.Sub(task->resreq);
    tasks.erase(task->uid);
    deleteTaskIndex(task);
    return true;
  }
  void UpdateTaskStatus(TaskInfo* task, int status) {  // :239-252
    DeleteTaskInfo(task);
    task->status = status;
    AddTaskInfo(task);
  }
  void SetPodGroup(const PodGroup* pg, const std::string& defaultQueue) {  // :166-186
    name = pg->name;
    ns = pg->ns;
    minAvailable = pg->minMember;
    if (!pg->queue.empty()) queue = pg->queue;
    else if (!defaultQueue.empty()) queue = defaultQueue;
    else queue = pg->ns;
    creation = pg->creation;
    podGroup = pg;
  }
  void SetPDB(const PDB* p, const std::string& defaultQueue) {  // :188-200
    name = p->name;
    minAvailable = p->minAvailable;
    ns = p->ns;
    queue = defaultQueue.empty() ? p->ns : defaultQueue;
    creation = p->creation;
    pdb = p;
  }
  JobInfo* Clone() const {  // :282-313
    JobInfo* info = new JobInfo();
    info->uid = uid; info->name = name; info->ns = ns; info->queue = queue;
    info->minAvailable = minAvailable;
    info->pdb = pdb; info->podGroup = podGroup;
    info->creation = creation;
    for (auto& kv : tasks.items) info->AddTaskInfo(new TaskInfo(*kv.second));
    return info;
  }
  std::string FitError() const {  // :329-358
    if (nodesFitDelta.empty()) return "0 nodes are available";
    std::map<std::string, int> reasons;
    for (auto& kv : nodesFitDelta) {
      if (kv.second.Get(0) < 0) reasons["cpu"]++;
      if (kv.second.Get(1) < 0) reasons["memory"]++;
      if (kv.second.Get(2) < 0) reasons["GPU"]++;
    }
    std::vector<std::string> rs;
    for (auto& kv : reasons) rs.push_back(std::to_string(kv.second) + " insufficient " + kv.first);
    std::sort(rs.begin(), rs.end());
    std::string j;
    for (size_t i = 0; i < rs.size(); i++) j += (i ? ", " : "") + rs[i];
    return "0/" + std::to_string(nodesFitDelta.size()) + " nodes are available, " + j + ".";
  }
};

struct QueueInfo { std::string uid, name; int32_t weight = 0; };  // api/queue_info.go:27-54

// -------------------------------------------------------------- the cache
struct ClusterInfo {
  std::vector<NodeInfo*> nodes;
  std::vector<JobInfo*> jobs;
  std::vector<QueueInfo*> queues;
  std::vector<TaskInfo*> others;
};

struct SchedulerCache {
  std::string defaultQueue;
  OMap<NodeInfo*> nodes;
  OMap<JobInfo*> jobs;
  OMap<QueueInfo*> queues;

  // event_handlers.go:40-61
  void addTask(TaskInfo* pi) {
    if (!pi->job.empty()) {
      if (!jobs.find(pi->job)) { JobInfo* j = new JobInfo(); j->uid = pi->job; jobs.set(pi->job, j); }
      (*jobs.find(pi->job))->AddTaskInfo(pi);
    }
    if (!pi->nodeName.empty()) {
      if (!nodes.find(pi->nodeName)) nodes.set(pi->nodeName, NodeInfo::make(nullptr));
      NodeInfo* node = *nodes.find(pi->nodeName);
      if (!(pi->status == Succeeded || pi->status == Failed)) node->AddTask(pi);
    }
  }
  // job_info.go:53-62 getJobID
  static std::string job_id_of(const Pod& p) {
    if (const std::string* gn = map_get(p.annotations, "scheduling.k8s.io/group-name"); gn && !gn->empty())
      return p.ns + "/" + *gn;
    return p.controller;
  }
  // job_info.go:64-89 NewTaskInfo
  void addPod(const Pod* p, int spec_class) {
    TaskInfo* ti = new TaskInfo();
    ti->uid = p->uid;
    ti->job = job_id_of(*p);
    ti->name = p->name;
    ti->ns = p->ns;
    ti->nodeName = p->nodeName;
    ti->status = get_task_status(*p);
    ti->priority = p->has_priority ? p->priority : 1;
    ti->pod = p;
    ti->resreq = p->resreq;
    ti->spec_class = spec_class;
    addTask(ti);
  }
  void addNode(const Node* n) {  // :232-240
    if (NodeInfo** ni = nodes.find(n->name)) (*ni)->SetNode(n);  // a pod named it first: NodeInfo(nil)
    else nodes.set(n->name, NodeInfo::make(n));
  }
  void setPodGroup(const PodGroup* pg) {  // :344-358
    std::string id = pg->ns + "/" + pg->name;
    if (!jobs.find(id)) { JobInfo* j = new JobInfo(); j->uid = id; jobs.set(id, j); }
    (*jobs.find(id))->SetPodGroup(pg, defaultQueue);
  }
  void setPDB(const PDB* p) {  // :458-470
    std::string id = p->controller;
    if (!jobs.find(id)) { JobInfo* j = new JobInfo(); j->uid = id; jobs.set(id, j); }
    (*jobs.find(id))->SetPDB(p, defaultQueue);
  }
  void addQueue(const std::string& name, int32_t weight) {  // :635-640, :726-736
    QueueInfo* q = new QueueInfo();
    q->uid = name; q->name = name; q->weight = weight;
    queues.set(name, q);
  }
  ClusterInfo Snapshot() {  // cache.go:549-597
    ClusterInfo s;
    for (auto& kv : nodes.items) s.nodes.push_back(kv.second->Clone());
    std::set<std::string> qs;
    for (auto& kv : queues.items) { s.queues.push_back(new QueueInfo(*kv.second)); qs.insert(kv.second->uid); }
    for (auto& kv : jobs.items) {
      JobInfo* v = kv.second;
      if (!v->podGroup && !v->pdb) {
        if (auto* rt = (v->statusIndex.count(Running) ? &v->statusIndex[Running] : nullptr))
          for (auto& t : rt->items) s.others.push_back(new TaskInfo(*t.second));
        continue;
      }
      if (!qs.count(v->queue)) continue;
      s.jobs.push_back(v->Clone());
    }
    return s;
  }
};

// ------------------------------------------------------ Go container/heap
// pkg/scheduler/util/priority_queue.go:25-88 over Go 1.11 container/heap.
// down()'s right-child test is "!Less(j1, j2)" in Go <= 1.11 and
// "Less(j2, j1)" in later releases; the rule is a run parameter.
static bool g_heap_go111 = true;

template <class T>
struct PriorityQueue {
  std::vector<T*> items;
  std::function<bool(T*, T*)> less;
  explicit PriorityQueue(std::function<bool(T*, T*)> l) : less(std::move(l)) {}
  bool Less(int i, int j) { return less(items[i], items[j]); }
  void Swap(int i, int j) { std::swap(items[i], items[j]); }
  void up(int j) {
    for (;;) {
      int i = (j - 1) / 2;  // Go truncated division: j=0 -> 0
      if (i == j || !Less(j, i)) break;
      Swap(i, j);
      j = i;
    }
  }
  void down(int i0, int n) {
    int i = i0;
    for (;;) {
      int j1 = 2 * i + 1;
      if (j1 >= n || j1 < 0) break;
      int j = j1;
      int j2 = j1 + 1;
      if (j2 < n && (g_heap_go111 ? !Less(j1, j2) : Less(j2, j1))) j = j2;
      if (!Less(j, i)) break;
      Swap(i, j);
      i = j;
    }
  }
  void Push(T* x) { items.push_back(x); up((int)items.size() - 1); }
  T* Pop() {
    if (items.empty()) return nullptr;
    int n = (int)items.size() - 1;
    Swap(0, n);
    down(0, n);
    T* it = items.back();
    items.pop_back();
    return it;
  }
  bool Empty() const { return items.empty(); }
  int Len() const { return (int)items.size(); }
};

// -------------------------------------------------------------- framework
struct PluginOption {
  std::string name;
  bool jobOrderDisabled = false, jobReadyDisabled = false, taskOrderDisabled = false;
  bool preemptableDisabled = false, reclaimableDisabled = false, queueOrderDisabled = false, predicateDisabled = false;
};
typedef std::vector<std::vector<PluginOption>> Tiers;

struct Decision { TaskInfo* task; std::string node; int kind; int dispatched_at = -1; const char* action = ""; };
// One committed eviction (cache.Evict), in commit order.
struct Eviction { std::string task, by, action; };
enum { KIND_ALLOCATE = 0, KIND_PIPELINE = 1 };

struct Session;
typedef std::function<int(void*, void*)> CompareFn;
typedef std::function<bool(void*)> ValidateFn;
typedef std::function<bool(TaskInfo*, NodeInfo*)> PredFn;  // true = nil error
struct EventHandler { std::function<void(TaskInfo*)> allocate, deallocate; };

struct Session {  // framework/session.go:35-61
  std::vector<JobInfo*> jobs;
  std::unordered_map<std::string, JobInfo*> jobIndex;
  std::vector<NodeInfo*> nodes;
  std::unordered_map<std::string, NodeInfo*> nodeIndex;
  std::vector<QueueInfo*> queues;
  std::unordered_map<std::string, QueueInfo*> queueIndex;
  std::vector<TaskInfo*> others;
  Tiers tiers;

  std::vector<EventHandler> eventHandlers;
  std::map<std::string, CompareFn> jobOrderFns, queueOrderFns, taskOrderFns;
  std::map<std::string, PredFn> predicateFns;
  std::map<std::string, ValidateFn> overusedFns, jobReadyFns;
  typedef std::function<std::vector<TaskInfo*>(TaskInfo*, const std::vector<TaskInfo*>&)> VictimFn;
  std::map<std::string, VictimFn> preemptableFns, reclaimableFns;
  std::vector<Eviction> evictions;
  const char* action = "";  // the action whose decisions are being logged
  // A pending pod declares hostPort under an active predicates plugin: the
  // device path refuses reclaim/preempt for such sessions (kbgpu.h), so the
  // oracle draws the same boundary there.
  bool pending_host_ports = false;
  bool pod_affinity_terms = false;  // some task of the session carries a required pod (anti)affinity term

  // run-time bookkeeping for the decision log
  std::vector<Decision> decisions;
  std::unordered_map<TaskInfo*, int> decisionOf;
  std::vector<std::pair<std::string, std::string>> binds;  // (ns/name, node) in dispatch order
  int64_t predicate_calls = 0;
  int64_t dup_discards = 0;  // statement discards whose unpipeline removed another pod holding the key (stats only)
  int64_t dup_discards_placed = 0;  // ... a holder placed this session (informer Spec.NodeName "", stats only)
  int threads = 1;  // > 1: allocate's node loop evaluated by a team of threads (B-omp CPU baseline only)
  size_t min_parallel_nodes = 512;  // B-omp: smaller clusters walk the nodes on one thread
  std::vector<TaskInfo*> evaluated;  // every task whose node loop ran, in order

  // session_plugins.go:142-156
  bool Overused(QueueInfo* q) {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        auto it = overusedFns.find(p.name);
        if (it == overusedFns.end()) continue;
        if (it->second(q)) return true;
      }
    return false;
  }
  // :158-176
  bool JobReady(JobInfo* j) {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (p.jobReadyDisabled) continue;
        auto it = jobReadyFns.find(p.name);
        if (it == jobReadyFns.end()) continue;
        if (!it->second(j)) return false;
      }
    return true;
  }
  // :196-221
  bool JobOrderFn(JobInfo* l, JobInfo* r) {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (p.jobOrderDisabled) continue;
        auto it = jobOrderFns.find(p.name);
        if (it == jobOrderFns.end()) continue;
        int j = it->second(l, r);
        if (j != 0) return j < 0;
      }
    if (l->creation == r->creation) return l->uid < r->uid;
    return l->creation < r->creation;
  }
  // :223-245
  bool QueueOrderFn(QueueInfo* l, QueueInfo* r) {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (p.queueOrderDisabled) continue;
        auto it = queueOrderFns.find(p.name);
        if (it == queueOrderFns.end()) continue;
        int j = it->second(l, r);
        if (j != 0) return j < 0;
      }
    return l->uid < r->uid;
  }
  // :247-276
  bool TaskOrderFn(TaskInfo* l, TaskInfo* r) {
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (p.taskOrderDisabled) continue;
        auto it = taskOrderFns.find(p.name);
        if (it == taskOrderFns.end()) continue;
        int j = it->second(l, r);
        if (j != 0) return j < 0;
      }
    return l->uid < r->uid;
  }
  // :278-295
  bool PredicateFn(TaskInfo* t, NodeInfo* n, bool count = true) {
    if (count) predicate_calls++;
    for (auto& tier : tiers)
      for (auto& p : tier) {
        if (p.predicateDisabled) continue;
        auto it = predicateFns.find(p.name);
        if (it == predicateFns.end()) continue;
        if (!it->second(t, n)) return false;
      }
    return true;
  }

  // session_plugins.go:59-140: the first tier with a registered, enabled fn
  // decides; its fns' candidate lists are intersected in plugin order (Go nil
  // slices: an empty result falls through to the next tier, where it stays empty).
  std::vector<TaskInfo*> victims_of(bool preempt, TaskInfo* t, const std::vector<TaskInfo*>& tasks) {
    std::vector<TaskInfo*> victims;
    bool init = false;
    for (auto& tier : tiers) {
      for (auto& p : tier) {
        if (preempt ? p.preemptableDisabled : p.reclaimableDisabled) continue;
        auto& fns = preempt ? preemptableFns : reclaimableFns;
        auto it = fns.find(p.name);
        if (it == fns.end()) continue;
        std::vector<TaskInfo*> cand = it->second(t, tasks);
        if (!init) {
          victims = cand;
          init = true;
        } else {
          std::vector<TaskInfo*> inter;
          for (TaskInfo* v : victims)
            for (TaskInfo* c : cand)
              if (v->uid == c->uid) inter.push_back(v);
          victims = inter;
        }
      }
      if (!victims.empty()) return victims;
    }
    return victims;
  }
  // job/node side of an eviction (session.go:323-349, statement.go:36-59):
  // Releasing in the job, NodeInfo.UpdateTask on the node, DeallocateFunc
  void evict_state(TaskInfo* reclaimee) {
    auto jit = jobIndex.find(reclaimee->job);
    if (jit != jobIndex.end()) jit->second->UpdateTaskStatus(reclaimee, Releasing);
    auto nit = nodeIndex.find(reclaimee->nodeName);
    if (nit != nodeIndex.end()) {
      nit->second->RemoveTask(reclaimee);  // node_info.go:159-165
      nit->second->AddTask(reclaimee);
    }
    for (auto& eh : eventHandlers)
      if (eh.deallocate) eh.deallocate(reclaimee);
  }
  // session.go:318-352 (the fake cache's Evict succeeds and is recorded)
  void Evict(TaskInfo* reclaimee, const std::string& by) {
    evictions.push_back({reclaimee->uid, by, action});
    evict_state(reclaimee);
  }

  // session.go:295-316
  void dispatch(TaskInfo* task) {
    binds.emplace_back(pod_key(task->pod), task->nodeName);
    auto d = decisionOf.find(task);
    if (d != decisionOf.end()) decisions[d->second].dispatched_at = (int)decisions.size() - 1;
    auto j = jobIndex.find(task->job);
    if (j != jobIndex.end()) j->second->UpdateTaskStatus(task, Binding);
  }
  // session.go:205-241
  void Pipeline(TaskInfo* task, NodeInfo* nodeHint) {
    auto jit = jobIndex.find(task->job);
    if (jit != jobIndex.end()) jit->second->UpdateTaskStatus(task, Pipelined);
    task->nodeName = nodeHint->name;
    auto nit = nodeIndex.find(nodeHint->name);
    if (nit != nodeIndex.end()) nit->second->AddTask(task);
    decisionOf[task] = (int)decisions.size();
    decisions.push_back({task, nodeHint->name, KIND_PIPELINE, -1, action});
    for (auto& eh : eventHandlers)
      if (eh.allocate) eh.allocate(task);
  }
  // session.go:243-293
  void Allocate(TaskInfo* task, NodeInfo* nodeHint) {
    JobInfo* job = nullptr;
    auto jit = jobIndex.find(task->job);
    if (jit != jobIndex.end()) { job = jit->second; job->UpdateTaskStatus(task, Allocated); }
    task->nodeName = nodeHint->name;
    auto nit = nodeIndex.find(nodeHint->name);
    if (nit != nodeIndex.end()) nit->second->AddTask(task);
    decisionOf[task] = (int)decisions.size();
    decisions.push_back({task, nodeHint->name, KIND_ALLOCATE, -1, action});
    for (auto& eh : eventHandlers)
      if (eh.allocate) eh.allocate(task);
    if (!job) throw RefPanic("JobReady on nil job");
    if (JobReady(job)) {
      auto it = job->statusIndex.find(Allocated);
      if (it != job->statusIndex.end()) {
        std::vector<TaskInfo*> batch;
        for (auto& kv : it->second.items) batch.push_back(kv.second);
        for (TaskInfo* t : batch) dispatch(t);
      }
    }
  }
};

// ---------------------------------------------------------------- plugins
// drf: pkg/scheduler/plugins/drf/drf.go:55-166
struct DRF {
  Resource total;
  std::unordered_map<std::string, std::pair<Resource, double>> opts;  // job -> (allocated, share)
  double calc(const Resource& a) const {
    double res = 0;
    for (int d = 0; d < 3; d++) {
      double s = helpers_share(a.Get(d), total.Get(d));
      if (s > res) res = s;
    }
    return res;
  }
  void open(Session* ssn) {
    for (NodeInfo* n : ssn->nodes) total.Add(n->allocatable);
    for (JobInfo* job : ssn->jobs) {
      Resource a;
      for (auto& kv : job->statusIndex)
        if (AllocatedStatus(kv.first))
          for (auto& t : kv.second.items) a.Add(t.second->resreq);
      opts[job->uid] = {a, calc(a)};
    }
    ssn->jobOrderFns["drf"] = [this](void* l, void* r) {
      double ls = opts[((JobInfo*)l)->uid].second, rs = opts[((JobInfo*)r)->uid].second;
      if (ls == rs) return 0;
      if (ls < rs) return -1;
      return 1;
    };
    // drf.go:80-105: a preemptee is a victim when the preemptor job's share
    // with the preemptor placed does not exceed the preemptee job's share with
    // this and the earlier preemptees of that job removed (within 1e-6).
    ssn->preemptableFns["drf"] = [this](TaskInfo* preemptor, const std::vector<TaskInfo*>& preemptees) {
      std::vector<TaskInfo*> victims;
      auto lit = opts.find(preemptor->job);
      if (lit == opts.end()) throw RefPanic("drf: preemptor job has no attributes (nil dereference)");
      Resource lalloc = lit->second.first;
      lalloc.Add(preemptor->resreq);
      const double ls = calc(lalloc);
      std::map<std::string, Resource> allocations;
      for (TaskInfo* p : preemptees) {
        auto al = allocations.find(p->job);
        if (al == allocations.end()) {
          auto rit = opts.find(p->job);
          if (rit == opts.end()) throw RefPanic("drf: preemptee job has no attributes (nil dereference)");
          al = allocations.emplace(p->job, rit->second.first).first;
        }
        const double rs = calc(al->second.Sub(p->resreq));
        if (ls < rs || std::fabs(ls - rs) <= 0.000001) victims.push_back(p);  // shareDelta drf.go:29
      }
      return victims;
    };
    ssn->eventHandlers.push_back({[this](TaskInfo* t) {
      auto& a = opts[t->job];
      a.first.Add(t->resreq);
      a.second = calc(a.first);
    }, [this](TaskInfo* t) {  // drf.go:140-148
      auto& a = opts[t->job];
      a.first.Sub(t->resreq);
      a.second = calc(a.first);
    }});
  }
};

// proportion: pkg/scheduler/plugins/proportion/proportion.go:54-237
struct QueueAttr { std::string id, name; int32_t weight = 0; double share = 0; Resource deserved, allocated, request; };
struct Proportion {
  Resource total;
  OMap<QueueAttr*> opts;  // insertion order = first job of the queue in ssn.Jobs order
  static void update_share(QueueAttr* a) {
    double res = 0;
    for (int d = 0; d < 3; d++) {
      double s = helpers_share(a->allocated.Get(d), a->deserved.Get(d));
      if (s > res) res = s;
    }
    a->share = res;
  }
  void open(Session* ssn) {
    for (NodeInfo* n : ssn->nodes) total.Add(n->allocatable);
    for (TaskInfo* t : ssn->others) total.Sub(t->resreq);
    for (JobInfo* job : ssn->jobs) {
      if (!opts.find(job->queue)) {
        QueueInfo* q = ssn->queueIndex[job->queue];
        QueueAttr* a = new QueueAttr();
        a->id = q->uid; a->name = q->name; a->weight = q->weight;
        opts.set(job->queue, a);
      }
      QueueAttr* a = *opts.find(job->queue);
      for (auto& kv : job->statusIndex) {
        if (AllocatedStatus(kv.first)) {
          for (auto& t : kv.second.items) { a->allocated.Add(t.second->resreq); a->request.Add(t.second->resreq); }
        } else if (kv.first == Pending) {
          for (auto& t : kv.second.items) a->request.Add(t.second->resreq);
        }
      }
    }
    Resource remaining = total;
    std::set<std::string> meet;
    for (;;) {
      int32_t totalWeight = 0;
      for (auto& kv : opts.items) if (!meet.count(kv.second->id)) totalWeight += kv.second->weight;
      if (totalWeight == 0) break;
      Resource deserved;
      for (auto& kv : opts.items) {
        QueueAttr* a = kv.second;
        if (meet.count(a->id)) continue;
        Resource part = remaining;
        a->deserved.Add(part.Multi((double)a->weight / (double)totalWeight));
        if (!a->deserved.LessEqual(a->request)) {
          a->deserved = helpers_min(a->deserved, a->request);
          meet.insert(a->id);
        }
        update_share(a);
        deserved.Add(a->deserved);
      }
      remaining.Sub(deserved);
      if (remaining.IsEmpty()) break;
    }
    ssn->queueOrderFns["proportion"] = [this](void* l, void* r) {
      double ls = (*opts.find(((QueueInfo*)l)->uid))->share, rs = (*opts.find(((QueueInfo*)r)->uid))->share;
      if (ls == rs) return 0;
      if (ls < rs) return -1;
      return 1;
    };
    ssn->overusedFns["proportion"] = [this](void* q) {
      QueueAttr* a = *opts.find(((QueueInfo*)q)->uid);
      return a->deserved.LessEqual(a->allocated);
    };
    // proportion.go:161-186: reclaimees of a queue are victims while the
    // queue's allocation with them removed (cumulatively, in list order)
    // still covers its deserved share; one the allocation cannot cover
    // (Less: every dimension short) is skipped.
    ssn->reclaimableFns["proportion"] = [this, ssn](TaskInfo*, const std::vector<TaskInfo*>& reclaimees) {
      std::vector<TaskInfo*> victims;
      std::map<std::string, Resource> allocations;
      for (TaskInfo* r : reclaimees) {
        JobInfo* job = ssn->jobIndex[r->job];
        QueueAttr** ap = opts.find(job->queue);
        if (!ap) throw RefPanic("proportion: reclaimee queue has no attributes (nil dereference)");
        auto al = allocations.find(job->queue);
        if (al == allocations.end()) al = allocations.emplace(job->queue, (*ap)->allocated).first;
        if (al->second.Less(r->resreq)) continue;
        al->second.Sub(r->resreq);
        if ((*ap)->deserved.LessEqual(al->second)) victims.push_back(r);
      }
      return victims;
    };
    ssn->eventHandlers.push_back({[this, ssn](TaskInfo* t) {
      JobInfo* job = ssn->jobIndex[t->job];
      QueueAttr* a = *opts.find(job->queue);
      a->allocated.Add(t->resreq);
      update_share(a);
    }, [this, ssn](TaskInfo* t) {  // proportion.go:207-216
      JobInfo* job = ssn->jobIndex[t->job];
      QueueAttr* a = *opts.find(job->queue);
      a->allocated.Sub(t->resreq);
      update_share(a);
    }});
  }
};

// gang: pkg/scheduler/plugins/gang/gang.go:44-190
static int32_t readyTaskNum(JobInfo* job) {
  int occ = 0;
  for (auto& kv : job->statusIndex)
    if (AllocatedStatus(kv.first) || kv.first == Succeeded || kv.first == Pipelined) occ += (int)kv.second.size();
  return occ;
}
static bool jobReady(JobInfo* job) { return readyTaskNum(job) >= job->minAvailable; }
static void gang_open(Session* ssn) {
  ssn->jobOrderFns["gang"] = [](void* l, void* r) {
    JobInfo* lv = (JobInfo*)l;
    JobInfo* rv = (JobInfo*)r;
    bool lr = jobReady(lv), rr = jobReady(rv);
    if (lr && rr) return 0;
    if (lr) return 1;
    if (rr) return -1;
    if (lv->creation == rv->creation) {
      if (lv->uid < rv->uid) return -1;
    } else if (lv->creation < rv->creation) {
      return -1;
    }
    return 1;
  };
  ssn->jobReadyFns["gang"] = [](void* j) { return jobReady((JobInfo*)j); };
  // gang.go:104-127: a preemptee is a victim when its job stays at or above
  // MinAvailable without it (registered for both preempt and reclaim)
  Session::VictimFn fn = [ssn](TaskInfo*, const std::vector<TaskInfo*>& preemptees) {
    std::vector<TaskInfo*> victims;
    for (TaskInfo* p : preemptees) {
      auto it = ssn->jobIndex.find(p->job);
      if (it == ssn->jobIndex.end()) throw RefPanic("gang: preemptee job not in session (nil dereference)");
      if (it->second->minAvailable <= readyTaskNum(it->second) - 1) victims.push_back(p);
    }
    return victims;
  };
  ssn->reclaimableFns["gang"] = fn;
  ssn->preemptableFns["gang"] = fn;
}

// priority: pkg/scheduler/plugins/priority/priority.go:36-77
static void priority_open(Session* ssn) {
  ssn->taskOrderFns["priority"] = [](void* l, void* r) {
    TaskInfo* lv = (TaskInfo*)l;
    TaskInfo* rv = (TaskInfo*)r;
    if (lv->priority == rv->priority) return 0;
    if (lv->priority > rv->priority) return -1;
    return 1;
  };
  ssn->jobOrderFns["priority"] = [](void* l, void* r) {
    JobInfo* lv = (JobInfo*)l;
    JobInfo* rv = (JobInfo*)r;
    if (lv->priority > rv->priority) return -1;
    if (lv->priority < rv->priority) return 1;
    return 0;
  };
}

// ------------------------------------------------------------- predicates
// NewRequirement validation + Matches (labels/selector.go:134-236)
struct Req { bool ok = true; std::string key, op; std::vector<std::string> vals; int64_t num = 0; };
static Req make_requirement(const std::string& key, const std::string& op, const std::vector<std::string>& vals) {
  Req r;
  r.key = key; r.op = op; r.vals = vals;
  if (!is_qualified_name(key)) { r.ok = false; return r; }
  if (op == "In" || op == "NotIn") { if (vals.empty()) r.ok = false; }
  else if (op == "=" ) { if (vals.size() != 1) r.ok = false; }
  else if (op == "Exists" || op == "DoesNotExist") { if (!vals.empty()) r.ok = false; }
  else if (op == "Gt" || op == "Lt") {
    if (vals.size() != 1) r.ok = false;
    else if (!go_parse_int64(vals[0], &r.num)) r.ok = false;
  } else r.ok = false;
  if (!r.ok) return r;
  for (auto& v : vals)
    if (!is_valid_label_value(v)) { r.ok = false; return r; }
  return r;
}
static bool req_matches(const Req& r, const StrMap& ls) {
  const std::string* v = map_get(ls, r.key);
  auto has = [&](const std::string& x) { return std::find(r.vals.begin(), r.vals.end(), x) != r.vals.end(); };
  if (r.op == "In" || r.op == "=") return v && has(*v);
  if (r.op == "NotIn") return !v || !has(*v);
  if (r.op == "Exists") return v != nullptr;
  if (r.op == "DoesNotExist") return v == nullptr;
  if (r.op == "Gt" || r.op == "Lt") {
    if (!v) return false;
    int64_t lv;
    if (!go_parse_int64(*v, &lv)) return false;
    return (r.op == "Gt" && lv > r.num) || (r.op == "Lt" && lv < r.num);
  }
  return false;
}
// v1/helper/helpers.go:222-252 NodeSelectorRequirementsAsSelector (error => term skipped)
static bool term_labels_match(const std::vector<NodeSelectorRequirement>& nsm, const StrMap& labels) {
  for (auto& e : nsm) {
    std::string op;
    if (e.op == "In" || e.op == "NotIn" || e.op == "Exists" || e.op == "DoesNotExist" || e.op == "Gt" || e.op == "Lt") op = e.op;
    else return false;
    Req r = make_requirement(e.key, op, e.values);
    if (!r.ok) return false;
  }
  for (auto& e : nsm)
    if (!req_matches(make_requirement(e.key, e.op, e.values), labels)) return false;
  return true;
}
// v1/helper/helpers.go:256-284 NodeSelectorRequirementsAsFieldSelector
static bool term_fields_match(const std::vector<NodeSelectorRequirement>& nsm, const Node* node) {
  for (auto& e : nsm) {
    if (e.op != "In" && e.op != "NotIn") return false;
    if (e.values.size() != 1) return false;
  }
  for (auto& e : nsm) {
    std::string fv = e.key == "metadata.name" ? node->name : "";
    if (e.op == "In" && fv != e.values[0]) return false;
    if (e.op == "NotIn" && fv == e.values[0]) return false;
  }
  return true;
}
// vendor predicates.go:807-850 podMatchesNodeSelectorAndAffinityTerms
static bool pod_matches_node_selector(const Pod* pod, const Node* node) {
  if (!pod->nodeSelector.empty()) {
    // labels.SelectorFromSet: any invalid pair => empty selector (matches all)
    bool valid = true;
    for (auto& kv : pod->nodeSelector)
      if (!make_requirement(kv.first, "=", {kv.second}).ok) { valid = false; break; }
    if (valid)
      for (auto& kv : pod->nodeSelector) {
        const std::string* v = map_get(node->labels, kv.first);
        if (!v || *v != kv.second) return false;
      }
  }
  if (pod->has_affinity && pod->has_node_affinity) {
    if (!pod->has_required) return true;
    // MatchNodeSelectorTerms (helpers.go:302-331)
    for (auto& t : pod->terms) {
      if (t.exprs.empty() && t.fields.empty()) continue;
      if (!t.exprs.empty() && !term_labels_match(t.exprs, node->labels)) continue;
      if (!t.fields.empty() && !term_fields_match(t.fields, node)) continue;
      return true;
    }
    return false;
  }
  return true;
}
// toleration.go:37-56 + helpers.go:412-441 + predicates.go:1489-1517
static bool tolerates(const Toleration& t, const Taint& taint) {
  if (!t.effect.empty() && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
  if (t.op == "Exists") return true;
  return false;
}
static bool pod_tolerates_node_taints(const Pod* pod, const Node* node) {
  for (auto& taint : node->taints) {
    if (taint.effect != "NoSchedule" && taint.effect != "NoExecute") continue;
    bool ok = false;
    for (auto& t : pod->tolerations)
      if (tolerates(t, taint)) { ok = true; break; }
    if (!ok) return false;
  }
  return true;
}

// pkg/scheduler/plugins/predicates/predicates.go:112-202
struct Predicates {
  Session* ssn = nullptr;
  bool faithful_scan = false;  // replay the podLister's per-call O(allocated pods) walk (F7)
  bool ghost = false;          // some allocated-status pod names a node outside the session
  std::unique_ptr<std::atomic<int8_t>[]> static_cache;  // [class][node]: -1 unknown
  size_t static_nodes = 0;

  // ---- PodAffinityChecker.InterPodAffinityMatches with meta == nil (vendor
  // predicates.go:1155-1182), the slow path kube-batch takes
  // (pkg/scheduler/plugins/predicates/predicates.go:185-198).
  // podLister.FilteredList(nodeInfo.Filter, Everything()) (predicates.go:67-89,
  // vendor cache/node_info.go:692-702): every AllocatedStatus task of every job
  // as a pod whose Spec.NodeName is the task's NodeName, minus the pods whose
  // informer Spec.NodeName is this node but that are missing from its pods.
  std::vector<TaskInfo*> filtered_pods(NodeInfo* node) {
    std::vector<TaskInfo*> out;
    for (JobInfo* job : ssn->jobs)
      for (auto& kv : job->statusIndex) {
        if (!AllocatedStatus(kv.first)) continue;
        for (auto& t : kv.second.items) {
          TaskInfo* task = t.second;
          bool keep;
          // podFilter(task.Pod) (predicates.go:79): the informer pod's
          // Spec.NodeName, which Allocate / Pipeline never change
          // (session.go:218,260 set task.NodeName only)
          if (task->pod->nodeName != node->node->name) keep = true;
          else {
            keep = false;
            for (auto& nt : node->tasks.items)
              if (nt.second->pod->name == task->pod->name && nt.second->pod->ns == task->pod->ns) { keep = true; break; }
          }
          if (keep) out.push_back(task);
        }
      }
    return out;
  }
  // metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:31-67)
  struct Selector { bool err = false, nothing = false, everything = false; std::vector<Req> reqs; };
  static Selector as_selector(const Pod::LabelSelector& ls) {
    Selector s;
    if (!ls.present) { s.nothing = true; return s; }
    if (ls.matchLabels.empty() && ls.exprs.empty()) { s.everything = true; return s; }
    for (auto& kv : ls.matchLabels) {
      Req r = make_requirement(kv.first, "=", {kv.second});
      if (!r.ok) { s.err = true; return s; }
      s.reqs.push_back(r);
    }
    for (auto& e : ls.exprs) {
      if (e.op != "In" && e.op != "NotIn" && e.op != "Exists" && e.op != "DoesNotExist") { s.err = true; return s; }
      Req r = make_requirement(e.key, e.op, e.values);
      if (!r.ok) { s.err = true; return s; }
      s.reqs.push_back(r);
    }
    return s;
  }
  static bool selector_matches(const Selector& s, const StrMap& labels) {
    if (s.nothing) return false;
    if (s.everything) return true;
    for (auto& r : s.reqs)
      if (!req_matches(r, labels)) return false;
    return true;
  }
  // priorities/util/topologies.go:28-48 (namespaces default to the term owner's)
  static bool ns_and_selector_match(const Pod* owner, const Pod::AffinityTerm& term, const Selector& sel,
                                    const Pod* target) {
    bool in = false;
    if (term.namespaces.empty()) in = target->ns == owner->ns;
    else
      for (auto& n : term.namespaces)
        if (n == target->ns) { in = true; break; }
    return in && selector_matches(sel, target->labels);
  }
  // topologies.go:52-71
  static bool same_topology(const Node* a, const Node* b, const std::string& key) {
    if (key.empty()) return false;
    const std::string* va = map_get(a->labels, key);
    const std::string* vb = map_get(b->labels, key);
    return va && vb && *va == *vb;
  }
  // podMatchesPodAffinityTerms (vendor predicates.go:1189-1214): {match, selector match, error}.
  // getAffinityTermProperties builds every term's selector before any match,
  // so a selector error in any term is returned first.
  struct TermsMatch { bool match = false, sel = false, err = false; };
  TermsMatch pod_matches_terms(const Pod* pod, TaskInfo* target, NodeInfo* node,
                               const std::vector<Pod::AffinityTerm>& terms) {
    TermsMatch r;
    std::vector<Selector> sels;
    for (auto& t : terms) {
      sels.push_back(as_selector(t.selector));
      if (sels.back().err) { r.err = true; return r; }
    }
    for (size_t i = 0; i < terms.size(); ++i)  // podMatchesAllAffinityTermProperties
      if (!ns_and_selector_match(pod, terms[i], sels[i], target->pod)) return r;
    auto it = ssn->nodeIndex.find(target->nodeName);  // c.info.GetNodeInfo
    if (it == ssn->nodeIndex.end() || !it->second->node) { r.err = true; return r; }
    for (auto& t : terms) {
      if (t.topologyKey.empty()) { r.err = true; return r; }
      if (!same_topology(node->node, it->second->node, t.topologyKey)) { r.sel = true; return r; }
    }
    r.match = r.sel = true;
    return r;
  }
  // targetPodMatchesAffinityOfPod(pod, pod) (vendor predicates/metadata.go)
  static bool pod_matches_own_affinity(const Pod* pod) {
    if (pod->aff_terms.empty()) return false;
    std::vector<Selector> sels;
    for (auto& t : pod->aff_terms) {
      sels.push_back(as_selector(t.selector));
      if (sels.back().err) return false;
    }
    for (size_t i = 0; i < pod->aff_terms.size(); ++i)
      if (!ns_and_selector_match(pod, pod->aff_terms[i], sels[i], pod)) return false;
    return true;
  }
  bool inter_pod_affinity_ok(TaskInfo* task, NodeInfo* node) {
    const Pod* pod = task->pod;
    std::vector<TaskInfo*> pods = filtered_pods(node);
    // satisfiesExistingPodsAntiAffinity (:1293-1332) via
    // getMatchingAntiAffinityTopologyPairsOfPods (:1270-1289)
    std::set<std::pair<std::string, std::string>> pairs;
    for (TaskInfo* e : pods) {
      auto it = ssn->nodeIndex.find(e->nodeName);
      if (it == ssn->nodeIndex.end() || !it->second->node) return false;  // GetNodeInfo error (not IsNotFound)
      const Node* enode = it->second->node;
      for (auto& term : e->pod->anti_terms) {  // :1247-1268
        Selector sel = as_selector(term.selector);
        if (sel.err) return false;
        if (!ns_and_selector_match(e->pod, term, sel, pod)) continue;
        if (const std::string* v = map_get(enode->labels, term.topologyKey)) pairs.insert({term.topologyKey, *v});
      }
    }
    for (auto& kv : node->node->labels)
      if (pairs.count({kv.first, kv.second})) return false;
    if (pod->aff_terms.empty() && pod->anti_terms.empty()) return true;
    // satisfiesPodsAffinityAntiAffinity, slow path (:1402-1457)
    bool matchFound = false, termsSelectorMatchFound = false;
    for (TaskInfo* e : pods) {
      if (!matchFound && !pod->aff_terms.empty()) {
        TermsMatch m = pod_matches_terms(pod, e, node, pod->aff_terms);
        if (m.err) return false;
        if (m.sel) termsSelectorMatchFound = true;
        if (m.match) matchFound = true;
      }
      if (!pod->anti_terms.empty()) {
        TermsMatch m = pod_matches_terms(pod, e, node, pod->anti_terms);
        if (m.err || m.match) return false;
      }
    }
    if (!matchFound && !pod->aff_terms.empty()) {
      if (termsSelectorMatchFound) return false;
      if (!pod_matches_own_affinity(pod)) return false;
    }
    return true;
  }
  bool static_ok(TaskInfo* task, NodeInfo* node, size_t node_pos) {
    auto calc = [&]() -> bool {
      if (!pod_matches_node_selector(task->pod, node->node)) return false;
      if (node->node->unschedulable) return false;  // predicates.go:105-110
      if (!pod_tolerates_node_taints(task->pod, node->node)) return false;
      return true;
    };
    if (faithful_scan || task->spec_class < 0 || !static_cache) return calc();
    std::atomic<int8_t>& slot = static_cache[(size_t)task->spec_class * static_nodes + node_pos];
    const int8_t known = slot.load(std::memory_order_relaxed);
    if (known >= 0) return known != 0;
    bool r = calc();
    slot.store(r ? 1 : 0, std::memory_order_relaxed);
    return r;
  }
  std::unordered_map<NodeInfo*, size_t> pos;
  // PodFitsHostPorts(task.Pod, nil, NewNodeInfo(node.Pods()...)) — vendor
  // predicates.go:1031-1051: every wanted port checked against the HostPortInfo
  // of the pods on the node (host_ports.go CheckConflict; sanitize "" -> 0.0.0.0
  // and TCP; port <= 0 is never recorded and never conflicts).
  static bool fits_host_ports(TaskInfo* task, NodeInfo* node) {
    const auto& want = task->pod->ports;
    if (want.empty()) return true;
    auto ip_of = [](const std::string& ip) { return ip.empty() ? std::string("0.0.0.0") : ip; };
    auto proto_of = [](const std::string& p) { return p.empty() ? std::string("TCP") : p; };
    for (auto& w : want) {
      if (w.port <= 0) continue;
      const std::string wip = ip_of(w.ip), wproto = proto_of(w.protocol);
      for (auto& kv : node->tasks.items)
        for (auto& e : kv.second->pod->ports) {
          if (e.port <= 0 || e.port != w.port || proto_of(e.protocol) != wproto) continue;
          const std::string eip = ip_of(e.ip);
          if (wip == "0.0.0.0" || eip == "0.0.0.0" || eip == wip) return false;
        }
    }
    return true;
  }

  void open(Session* s, bool active, int n_classes) {
    ssn = s;
    for (size_t i = 0; i < s->nodes.size(); i++) pos[s->nodes[i]] = i;
    static_nodes = s->nodes.size();
    if (n_classes > 0) {
      const size_t n = (size_t)n_classes * static_nodes;
      static_cache.reset(new std::atomic<int8_t>[n]);
      for (size_t i = 0; i < n; ++i) static_cache[i].store(-1, std::memory_order_relaxed);
    }
    // Without any pod (anti)affinity term in the session the inter-pod
    // predicate reduces to the GetNodeInfo errors of allocated pods whose node
    // is outside the session (SURVEY A10 "ghost" pods); otherwise it runs in full.
    if (active)
    for (JobInfo* job : s->jobs)
      for (auto& kv : job->tasks.items) {
        TaskInfo* t = kv.second;
        if (!t->pod->aff_terms.empty() || !t->pod->anti_terms.empty()) s->pod_affinity_terms = true;
        if (AllocatedStatus(t->status) && !s->nodeIndex.count(t->nodeName)) ghost = true;
        if (t->status == Pending && t->pod->has_host_port) s->pending_host_ports = true;
      }
    s->predicateFns["predicates"] = [this](TaskInfo* task, NodeInfo* node) -> bool {
      // cache.NewNodeInfo(node.Pods()...).SetNode(node.Node): nil node => nil dereference
      if (!node->node) throw RefPanic("predicate on a NodeInfo without Node (nil dereference)");
      if (node->allocatable.MaxTaskNum <= (int)node->tasks.size()) return false;  // :125-127
      if (!static_ok(task, node, pos[node])) return false;                       // :130-141,158-183
      if (!fits_host_ports(task, node)) return false;                            // :144-155
      if (faithful_scan || ssn->pod_affinity_terms) return inter_pod_affinity_ok(task, node);  // :186-198
      return !ghost;
    };
  }
};

// ---------------------------------------------------------------- allocate
// B-omp (the multi-core CPU baseline only): allocate.go:119-162 for one task
// with PredicateFn and the two fits evaluated on a persistent team of
// ssn->threads threads (PredicateFn reads the session only). The node axis is
// cut into chunks of kChunk nodes handed out in node order from one counter;
// a thread stops taking chunks once a chunk at or below the one it would take
// holds a stop (Idle or Releasing fit, or a PredicateFn panic), so an early
// first fit costs one round of chunks and a task that fits nowhere is spread
// over every thread. The calling thread then walks the evaluated prefix in
// node order exactly like the sequential loop: the first node whose Idle or
// Releasing fits wins; NodesFitDelta gets the predicate-passing nodes before
// it; a panic is rethrown when the walk reaches its node. One parallel region
// for the whole run (the team spins between tasks): no fork/join per task.
struct NodeTeam {
  static constexpr size_t kChunk = 64;
  Session* ssn = nullptr;
  TaskInfo* task = nullptr;
  size_t N = 0, n_chunks = 0;
  std::vector<int8_t> st;  // per node: 0 predicates fail, 1 Idle fits, 2 Releasing fits, 3 neither, 4 panic, -1 not evaluated
  std::vector<std::string> panic;
  std::atomic<uint64_t> gen{0};
  std::atomic<size_t> next{0};
  std::atomic<size_t> best{SIZE_MAX};  // lowest chunk holding a stop
  std::atomic<int> done{0};
  std::atomic<bool> quit{false};
  std::vector<std::thread> team;

  explicit NodeTeam(int workers) {
    for (int w = 0; w < workers; ++w) team.emplace_back([this] { loop(); });
  }
  ~NodeTeam() {
    quit.store(true, std::memory_order_release);
    gen.fetch_add(1, std::memory_order_release);
    for (auto& t : team) t.join();
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g;
      while ((g = gen.load(std::memory_order_acquire)) == seen) __builtin_ia32_pause();
      seen = g;
      if (quit.load(std::memory_order_acquire)) return;
      work();
      done.fetch_add(1, std::memory_order_release);
    }
  }
  void work() {
    for (;;) {
      const size_t c = next.fetch_add(1, std::memory_order_relaxed);
      if (c >= n_chunks || c > best.load(std::memory_order_relaxed)) return;
      const size_t lo = c * kChunk, hi = std::min(N, lo + kChunk);
      for (size_t i = lo; i < hi; ++i) {
        NodeInfo* node = ssn->nodes[i];
        int8_t v;
        try {
          if (!ssn->PredicateFn(task, node, false)) v = 0;
          else if (task->resreq.LessEqual(node->idle)) v = 1;
          else if (task->resreq.LessEqual(node->releasing)) v = 2;
          else v = 3;
        } catch (const RefPanic& e) {
          v = 4;
          panic[i] = e.what();
        }
        st[i] = v;
        if (v == 1 || v == 2 || v == 4) {  // the walk stops here: the rest of the chunk is not needed
          size_t b = best.load(std::memory_order_relaxed);
          while (c < b && !best.compare_exchange_weak(b, c, std::memory_order_relaxed)) {
          }
          break;
        }
      }
    }
  }
  // Evaluates the task's node loop; returns the index one past the last node
  // the sequential walk needs (every node below it evaluated).
  size_t run(Session* s, TaskInfo* t) {
    ssn = s;
    task = t;
    N = s->nodes.size();
    n_chunks = (N + kChunk - 1) / kChunk;
    if (st.size() < N) {
      st.resize(N);
      panic.resize(N);
    }
    next.store(0, std::memory_order_relaxed);
    best.store(SIZE_MAX, std::memory_order_relaxed);
    done.store(0, std::memory_order_relaxed);
    gen.fetch_add(1, std::memory_order_release);  // publishes the task and the reset counters
    work();
    while (done.load(std::memory_order_acquire) != (int)team.size()) __builtin_ia32_pause();
    const size_t b = best.load(std::memory_order_relaxed);
    return b == SIZE_MAX ? N : std::min(N, (b + 1) * kChunk);
  }
};

static bool threaded_node_loop(Session* ssn, JobInfo* job, TaskInfo* task) {
  static std::unique_ptr<NodeTeam> team;
  if (!team || (int)team->team.size() != ssn->threads - 1) {
    team.reset();
    team.reset(new NodeTeam(ssn->threads - 1));
  }
  const size_t end = team->run(ssn, task);
  job->fit_log.clear();
  job->fit_log_pending = true;
  for (size_t i = 0; i < end; ++i) {
    ssn->predicate_calls++;
    const int8_t v = team->st[i];
    if (v == 4) throw RefPanic(team->panic[i]);
    if (v == 0) continue;
    NodeInfo* node = ssn->nodes[i];
    if (v == 1) {
      ssn->Allocate(task, node);
      return true;
    }
    Resource fd = node->idle;
    fd.FitDelta(task->resreq);
    job->fit_log.emplace_back(node, fd);
    if (v == 2) {
      ssn->Pipeline(task, node);
      return true;
    }
  }
  return false;
}

// kbref --budget SECONDS: stop the actions after this much wall time (CPU
// baselines that cannot finish, e.g. B-faithful at C2-C4) and report the
// placements reached; 0 = no budget
double g_budget_s = 0;
std::chrono::steady_clock::time_point g_budget_t0;
struct BudgetExceeded {};
inline void budget_check(size_t evaluated) {
  if (g_budget_s <= 0 || (evaluated & 63) != 0) return;
  if (std::chrono::duration<double>(std::chrono::steady_clock::now() - g_budget_t0).count() > g_budget_s)
    throw BudgetExceeded{};
}

// pkg/scheduler/actions/allocate/allocate.go:41-176
static void allocate_execute(Session* ssn) {
  PriorityQueue<QueueInfo> queues([ssn](QueueInfo* l, QueueInfo* r) { return ssn->QueueOrderFn(l, r); });
  OMap<PriorityQueue<JobInfo>*> jobsMap;
  for (JobInfo* job : ssn->jobs) {
    if (!jobsMap.find(job->queue))
      jobsMap.set(job->queue, new PriorityQueue<JobInfo>([ssn](JobInfo* l, JobInfo* r) { return ssn->JobOrderFn(l, r); }));
    auto q = ssn->queueIndex.find(job->queue);
    if (q != ssn->queueIndex.end()) queues.Push(q->second);
    (*jobsMap.find(job->queue))->Push(job);
  }
  std::unordered_map<std::string, PriorityQueue<TaskInfo>*> pendingTasks;
  for (;;) {
    if (queues.Empty()) break;
    QueueInfo* queue = queues.Pop();
    if (ssn->Overused(queue)) continue;
    PriorityQueue<JobInfo>** jobsp = jobsMap.find(queue->uid);
    if (!jobsp || (*jobsp)->Empty()) continue;
    PriorityQueue<JobInfo>* jobs = *jobsp;
    JobInfo* job = jobs->Pop();
    if (!pendingTasks.count(job->uid)) {
      auto* tasks = new PriorityQueue<TaskInfo>([ssn](TaskInfo* l, TaskInfo* r) { return ssn->TaskOrderFn(l, r); });
      auto it = job->statusIndex.find(Pending);
      if (it != job->statusIndex.end())
        for (auto& kv : it->second.items) {
          if (kv.second->resreq.IsEmpty()) continue;  // BestEffort left to backfill
          tasks->Push(kv.second);
        }
      pendingTasks[job->uid] = tasks;
    }
    PriorityQueue<TaskInfo>* tasks = pendingTasks[job->uid];
    while (!tasks->Empty()) {
      TaskInfo* task = tasks->Pop();
      ssn->evaluated.push_back(task);
      budget_check(ssn->evaluated.size());
      bool assigned = false;
      if (!job->nodesFitDelta.empty()) job->nodesFitDelta.clear();
      // B-omp: the same loop, predicates evaluated by the node team; below
      // min_parallel_nodes the hand-off per task costs more than the whole walk
      if (ssn->threads > 1 && ssn->nodes.size() >= ssn->min_parallel_nodes) {
        if (threaded_node_loop(ssn, job, task)) { jobs->Push(job); break; }
        continue;
      }
      for (NodeInfo* node : ssn->nodes) {
        if (!ssn->PredicateFn(task, node)) continue;
        if (task->resreq.LessEqual(node->idle)) {
          ssn->Allocate(task, node);
          assigned = true;
          break;
        } else {
          Resource fd = node->idle;
          fd.FitDelta(task->resreq);
          job->nodesFitDelta[node->name] = fd;
        }
        if (task->resreq.LessEqual(node->releasing)) {
          ssn->Pipeline(task, node);
          assigned = true;
          break;
        }
      }
      if (assigned) { jobs->Push(job); break; }
    }
    queues.Push(queue);
  }
  for (JobInfo* job : ssn->jobs)
    if (job->fit_log_pending) {
      job->nodesFitDelta.clear();
      for (auto& e : job->fit_log) job->nodesFitDelta[e.first->name] = e.second;
      job->fit_log.clear();
      job->fit_log_pending = false;
    }
}

// backfill.go:40-71: every Pending task of every job (ssn.Jobs order, status
// index order) that requests nothing goes to the first node whose PredicateFn
// passes, through ssn.Allocate. Go ranges over the live Pending map while
// Allocate removes the current task from it; removing the entry being visited
// does not change which entries the range yields, so a copy is equivalent.
static void backfill_execute(Session* ssn) {
  for (JobInfo* job : ssn->jobs) {
    auto it = job->statusIndex.find(Pending);
    if (it == job->statusIndex.end()) continue;
    std::vector<TaskInfo*> pending;
    for (auto& kv : it->second.items) pending.push_back(kv.second);
    for (TaskInfo* task : pending) {
      if (!task->resreq.IsEmpty()) continue;  // "backfill for other case" is a TODO in v0.4
      for (NodeInfo* node : ssn->nodes) {
        if (!ssn->PredicateFn(task, node)) continue;
        ssn->Allocate(task, node);
        break;
      }
    }
  }
}

// framework/statement.go:35-217. Evict/Pipeline change the session at once
// and are recorded; Commit sends the evictions to the cache (recorded here);
// Discard undoes in reverse order — unevict's node.AddTask finds the task
// still on the node (it was re-added as Releasing) and fails, so the node
// keeps it as Releasing while the job and the plugins see it Running again.
struct Statement {
  Session* ssn;
  struct Op { bool evict; TaskInfo* task; std::string by; };
  std::vector<Op> ops;
  explicit Statement(Session* s) : ssn(s) {}
  void Evict(TaskInfo* reclaimee, const std::string& by) {  // :35-67
    ssn->evict_state(reclaimee);
    ops.push_back({true, reclaimee, by});
  }
  void Pipeline(TaskInfo* task, NodeInfo* node) {  // :110-151
    auto jit = ssn->jobIndex.find(task->job);
    if (jit != ssn->jobIndex.end()) jit->second->UpdateTaskStatus(task, Pipelined);
    task->nodeName = node->name;
    auto nit = ssn->nodeIndex.find(node->name);
    if (nit != ssn->nodeIndex.end()) nit->second->AddTask(task);
    for (auto& eh : ssn->eventHandlers)
      if (eh.allocate) eh.allocate(task);
    ops.push_back({false, task, ""});
  }
  void Discard() {  // :194-205
    for (size_t k = ops.size(); k-- > 0;) {
      TaskInfo* t = ops[k].task;
      auto jit = ssn->jobIndex.find(t->job);
      auto nit = ssn->nodeIndex.find(t->nodeName);
      if (ops[k].evict) {  // unevict :81-108
        if (jit != ssn->jobIndex.end()) jit->second->UpdateTaskStatus(t, Running);
        if (nit != ssn->nodeIndex.end()) nit->second->AddTask(t);  // already on the node: error, no change
        for (auto& eh : ssn->eventHandlers)
          if (eh.allocate) eh.allocate(t);
      } else {  // unpipeline :156-192
        if (jit != ssn->jobIndex.end()) jit->second->UpdateTaskStatus(t, Pending);
        if (nit != ssn->nodeIndex.end()) {
          TaskInfo** held = nit->second->tasks.find(pod_key(t->pod));
          if (held && (*held)->uid != t->uid) {
            ssn->dup_discards++;
            if ((*held)->pod->nodeName.empty()) ssn->dup_discards_placed++;
          }
          nit->second->RemoveTask(t);
        }
        for (auto& eh : ssn->eventHandlers)
          if (eh.deallocate) eh.deallocate(t);
      }
    }
  }
  void Commit() {  // :207-217
    for (auto& op : ops) {
      if (op.evict) ssn->evictions.push_back({op.task->uid, op.by, ssn->action});
      else ssn->decisions.push_back({op.task, op.task->nodeName, KIND_PIPELINE, -1, ssn->action});
    }
  }
};

// preempt.go:182-240: the first node (ssn.Nodes order) whose PredicateFn
// passes and whose filtered tasks yield validated victims; victims are evicted
// in order until the request is covered, then the preemptor is pipelined.
// Clones of the node's tasks are evicted (node.Tasks order = insertion order).
static bool preempt_one(Session* ssn, Statement& stmt, TaskInfo* preemptor,
                        const std::function<bool(TaskInfo*)>& filter) {
  Resource resreq = preemptor->resreq;
  for (NodeInfo* node : ssn->nodes) {
    if (!ssn->PredicateFn(preemptor, node)) continue;
    std::vector<TaskInfo*> preemptees;
    for (auto& kv : node->tasks.items)
      if (filter(kv.second)) preemptees.push_back(new TaskInfo(*kv.second));
    std::vector<TaskInfo*> victims = ssn->victims_of(true, preemptor, preemptees);
    if (victims.empty()) continue;  // validateVictims :242-253
    Resource all;
    for (TaskInfo* v : victims) all.Add(v->resreq);
    if (all.Less(resreq)) continue;
    for (TaskInfo* v : victims) {
      stmt.Evict(v, preemptor->uid);
      if (resreq.LessEqual(v->resreq)) break;
      resreq.Sub(v->resreq);
    }
    stmt.Pipeline(preemptor, node);
    return true;
  }
  return false;
}

static void preempt_execute(Session* ssn) {  // preempt.go:43-171
  OMap<PriorityQueue<JobInfo>*> preemptorsMap;
  std::unordered_map<std::string, PriorityQueue<TaskInfo>*> preemptorTasks;
  std::vector<JobInfo*> underRequest;
  std::vector<QueueInfo*> queues;
  auto job_less = [ssn](JobInfo* l, JobInfo* r) { return ssn->JobOrderFn(l, r); };
  auto task_less = [ssn](TaskInfo* l, TaskInfo* r) { return ssn->TaskOrderFn(l, r); };
  for (JobInfo* job : ssn->jobs) {
    auto q = ssn->queueIndex.find(job->queue);
    if (q == ssn->queueIndex.end()) continue;
    queues.push_back(q->second);
    auto pit = job->statusIndex.find(Pending);
    if (pit != job->statusIndex.end() && pit->second.size() != 0) {
      if (!preemptorsMap.find(job->queue)) preemptorsMap.set(job->queue, new PriorityQueue<JobInfo>(job_less));
      (*preemptorsMap.find(job->queue))->Push(job);
      underRequest.push_back(job);
      auto* tasks = new PriorityQueue<TaskInfo>(task_less);
      for (auto& kv : pit->second.items) tasks->Push(kv.second);
      preemptorTasks[job->uid] = tasks;
    }
  }
  for (QueueInfo* queue : queues) {
    for (;;) {  // preemption between jobs within the queue
      PriorityQueue<JobInfo>** pp = preemptorsMap.find(queue->uid);
      if (!pp || (*pp)->Empty()) break;
      JobInfo* preemptorJob = (*pp)->Pop();
      Statement stmt(ssn);
      bool assigned = false;
      for (;;) {
        PriorityQueue<TaskInfo>* tasks = preemptorTasks[preemptorJob->uid];
        if (tasks->Empty()) break;
        TaskInfo* preemptor = tasks->Pop();
        if (preempt_one(ssn, stmt, preemptor, [&](TaskInfo* t) {
              if (t->status != Running) return false;
              auto jit = ssn->jobIndex.find(t->job);
              if (jit == ssn->jobIndex.end()) return false;
              return jit->second->queue == preemptorJob->queue && preemptor->job != t->job;
            }))
          assigned = true;
        if (ssn->JobReady(preemptorJob)) {
          stmt.Commit();
          break;
        }
      }
      if (!ssn->JobReady(preemptorJob)) {
        stmt.Discard();
        continue;
      }
      if (assigned) (*pp)->Push(preemptorJob);
    }
    for (JobInfo* job : underRequest) {  // preemption between tasks within a job
      for (;;) {
        auto it = preemptorTasks.find(job->uid);
        if (it == preemptorTasks.end() || it->second->Empty()) break;
        TaskInfo* preemptor = it->second->Pop();
        Statement stmt(ssn);
        const bool assigned = preempt_one(ssn, stmt, preemptor, [&](TaskInfo* t) {
          return t->status == Running && preemptor->job == t->job;
        });
        stmt.Commit();
        if (!assigned) break;
      }
    }
  }
}

static void reclaim_execute(Session* ssn) {  // reclaim.go:41-188
  PriorityQueue<QueueInfo> queues([ssn](QueueInfo* l, QueueInfo* r) { return ssn->QueueOrderFn(l, r); });
  OMap<PriorityQueue<JobInfo>*> preemptorsMap;
  std::unordered_map<std::string, PriorityQueue<TaskInfo>*> preemptorTasks;
  auto job_less = [ssn](JobInfo* l, JobInfo* r) { return ssn->JobOrderFn(l, r); };
  auto task_less = [ssn](TaskInfo* l, TaskInfo* r) { return ssn->TaskOrderFn(l, r); };
  for (JobInfo* job : ssn->jobs) {
    auto q = ssn->queueIndex.find(job->queue);
    if (q == ssn->queueIndex.end()) continue;
    queues.Push(q->second);
    auto pit = job->statusIndex.find(Pending);
    if (pit != job->statusIndex.end() && pit->second.size() != 0) {
      if (!preemptorsMap.find(job->queue)) preemptorsMap.set(job->queue, new PriorityQueue<JobInfo>(job_less));
      (*preemptorsMap.find(job->queue))->Push(job);
      auto* tasks = new PriorityQueue<TaskInfo>(task_less);
      for (auto& kv : pit->second.items) tasks->Push(kv.second);
      preemptorTasks[job->uid] = tasks;
    }
  }
  for (;;) {
    if (queues.Empty()) break;
    QueueInfo* queue = queues.Pop();
    if (ssn->Overused(queue)) continue;
    PriorityQueue<JobInfo>** jp = preemptorsMap.find(queue->uid);
    if (!jp || (*jp)->Empty()) continue;
    JobInfo* job = (*jp)->Pop();
    auto tit = preemptorTasks.find(job->uid);
    if (tit == preemptorTasks.end() || tit->second->Empty()) continue;
    TaskInfo* task = tit->second->Pop();
    Resource resreq = task->resreq;
    bool assigned = false;
    for (NodeInfo* n : ssn->nodes) {
      if (!ssn->PredicateFn(task, n)) continue;
      std::vector<TaskInfo*> reclaimees;
      for (auto& kv : n->tasks.items) {
        TaskInfo* t = kv.second;
        if (t->status != Running) continue;
        auto jit = ssn->jobIndex.find(t->job);
        if (jit == ssn->jobIndex.end()) continue;
        if (jit->second->queue != job->queue) reclaimees.push_back(new TaskInfo(*t));
      }
      std::vector<TaskInfo*> victims = ssn->victims_of(false, task, reclaimees);
      if (victims.empty()) continue;
      Resource all;
      for (TaskInfo* v : victims) all.Add(v->resreq);
      if (all.Less(resreq)) continue;
      for (TaskInfo* v : victims) {
        ssn->Evict(v, task->uid);
        if (resreq.LessEqual(v->resreq)) break;
        resreq.Sub(v->resreq);
      }
      ssn->Pipeline(task, n);
      assigned = true;
      break;
    }
    if (assigned) queues.Push(queue);
  }
}

// ---------------------------------------------------------------- driver
struct World {
  std::vector<Node> nodes;
  std::vector<Pod> pods;
  std::vector<PodGroup> pgs;
  std::vector<PDB> pdbs;
  std::vector<int> pod_class;
};

static Tiers parse_tiers(const Value* v) {
  Tiers t;
  if (!v || v->is_null()) {  // pkg/scheduler/util.go:30-40 default conf
    t = {{{"priority"}, {"gang"}}, {{"drf"}, {"predicates"}, {"proportion"}}};
    return t;
  }
  for (auto& tier : v->arr) {
    std::vector<PluginOption> ps;
    const Value* plugins = tier.is_obj() ? tier.get("plugins") : &tier;
    for (auto& p : plugins->arr) {
      PluginOption o;
      o.name = p.str("name");
      o.jobOrderDisabled = p.boolean("disableJobOrder");
      o.jobReadyDisabled = p.boolean("disableJobReady");
      o.taskOrderDisabled = p.boolean("disableTaskOrder");
      o.preemptableDisabled = p.boolean("disablePreemptable");
      o.reclaimableDisabled = p.boolean("disableReclaimable");
      o.queueOrderDisabled = p.boolean("disableQueueOrder");
      o.predicateDisabled = p.boolean("disablePredicate");
      ps.push_back(o);
    }
    t.push_back(ps);
  }
  return t;
}

static std::string res_json(const Resource& r) {
  return "[" + kbjson::num(r.MilliCPU) + "," + kbjson::num(r.Memory) + "," + kbjson::num(r.MilliGPU) + "]";
}

template <class T>
static void reorder(std::vector<T*>& v, const Value* order, std::function<std::string(T*)> key) {
  if (!order || !order->is_arr()) return;
  std::unordered_map<std::string, T*> m;
  for (T* x : v) m[key(x)] = x;
  std::vector<T*> out;
  std::unordered_set<T*> used;
  for (auto& k : order->arr) {
    auto it = m.find(k.s);
    if (it != m.end() && !used.count(it->second)) { out.push_back(it->second); used.insert(it->second); }
  }
  for (T* x : v) if (!used.count(x)) out.push_back(x);
  v = out;
}

size_t g_min_parallel_nodes = 512;  // kbref --min-parallel-nodes
static std::string run_session(const Value& fx, bool faithful, bool no_cache, int threads) {
  World w;
  std::string defaultQueue;
  if (const Value* o = fx.get("options")) {
    defaultQueue = o->str("defaultQueue");
    std::string rule = o->str("heapDownRule", "go1.11");
    g_heap_go111 = rule != "go1.13";
  }
  if (const Value* ns = fx.get("nodes"))
    for (auto& n : ns->arr) {
      Node node;
      node.name = n.str("name");
      node.allocatable = new_resource(n.get("allocatable"));
      node.capacity = n.get("capacity") ? new_resource(n.get("capacity")) : node.allocatable;
      node.labels = parse_strmap(n.get("labels"));
      node.unschedulable = n.boolean("unschedulable");
      if (const Value* ts = n.get("taints"))
        for (auto& t : ts->arr) node.taints.push_back({t.str("key"), t.str("value"), t.str("effect")});
      w.nodes.push_back(node);
    }
  if (const Value* ps = fx.get("pods")) {
    w.pods.reserve(ps->arr.size());
    for (auto& p : ps->arr) w.pods.push_back(parse_pod(p));
  }
  if (const Value* gs = fx.get("podGroups"))
    for (auto& g : gs->arr)
      w.pgs.push_back({g.str("namespace"), g.str("name"), g.str("queue"), (int32_t)g.integer("minMember"), g.integer("creationTimestamp")});
  if (const Value* ds = fx.get("pdbs"))
    for (auto& d : ds->arr)
      w.pdbs.push_back({d.str("namespace"), d.str("name"), d.str("controller"), (int32_t)d.integer("minAvailable"), d.integer("creationTimestamp")});

  // static-predicate identity of each pod spec (oracle-side cache only)
  std::unordered_map<std::string, int> spec_ids;
  if (const Value* ps = fx.get("pods"))
    for (size_t i = 0; i < ps->arr.size(); i++) {
      const Value& p = ps->arr[i];
      std::string key;
      for (const char* f : {"nodeSelector", "affinity", "tolerations"}) {
        const Value* v = p.get(f);
        key += f;
        key += ':';
        // structural identity: re-serialise via parse result order
        std::function<void(const Value*)> ser = [&](const Value* x) {
          if (!x) { key += "~"; return; }
          switch (x->kind) {
            case Value::Null: key += "n"; break;
            case Value::Bool: key += x->b ? "T" : "F"; break;
            case Value::Int: key += "i" + std::to_string(x->i); break;
            case Value::Double: key += "d" + kbjson::num(x->d); break;
            case Value::String: key += kbjson::quote(x->s); break;
            case Value::Array: key += "["; for (auto& e : x->arr) { ser(&e); key += ","; } key += "]"; break;
            case Value::Object: key += "{"; for (auto& e : x->obj) { key += kbjson::quote(e.first) + ":"; ser(&e.second); key += ","; } key += "}"; break;
          }
        };
        ser(v);
      }
      auto it = spec_ids.find(key);
      int id = it == spec_ids.end() ? (int)spec_ids.size() : it->second;
      if (it == spec_ids.end()) spec_ids[key] = id;
      w.pod_class.push_back(no_cache ? -1 : id);
    }

  int n_pod_classes = 0;
  for (int c : w.pod_class) n_pod_classes = std::max(n_pod_classes, c + 1);
  SchedulerCache cache;
  cache.defaultQueue = defaultQueue;
  for (auto& n : w.nodes) cache.addNode(&n);
  {
    std::unordered_set<std::string> uids;
    for (size_t i = 0; i < w.pods.size(); i++) {
      if (!uids.insert(w.pods[i].uid).second) throw BadInput("duplicate pod uid " + w.pods[i].uid);
      cache.addPod(&w.pods[i], w.pod_class[i]);
    }
  }
  for (auto& g : w.pgs) cache.setPodGroup(&g);
  for (auto& d : w.pdbs) cache.setPDB(&d);
  if (const Value* qs = fx.get("queues"))
    for (auto& q : qs->arr) cache.addQueue(q.str("name"), (int32_t)q.integer("weight"));
  if (const Value* nss = fx.get("namespaces"))
    for (auto& n : nss->arr) cache.addQueue(n.is_str() ? n.s : n.str("name"), 1);

  ClusterInfo snap = cache.Snapshot();
  if (const Value* so = fx.get("sessionOrder")) {
    reorder<NodeInfo>(snap.nodes, so->get("nodes"), [](NodeInfo* n) { return n->name; });
    reorder<JobInfo>(snap.jobs, so->get("jobs"), [](JobInfo* j) { return j->uid; });
    reorder<QueueInfo>(snap.queues, so->get("queues"), [](QueueInfo* q) { return q->uid; });
  }

  // framework.OpenSession (framework.go:26-46, session.go:63-128)
  Session* ssn = new Session();
  ssn->jobs = snap.jobs;  // JobValid is a no-op at this point
  for (JobInfo* j : ssn->jobs) ssn->jobIndex[j->uid] = j;
  ssn->nodes = snap.nodes;
  for (NodeInfo* n : ssn->nodes) ssn->nodeIndex[n->name] = n;
  ssn->queues = snap.queues;
  for (QueueInfo* q : ssn->queues) ssn->queueIndex[q->uid] = q;
  ssn->others = snap.others;
  ssn->tiers = parse_tiers(fx.get("tiers"));

  std::set<std::string> names;
  for (auto& tier : ssn->tiers)
    for (auto& p : tier) names.insert(p.name);
  DRF drf;
  Proportion prop;
  Predicates preds;
  preds.faithful_scan = faithful;
  ssn->threads = std::max(1, threads);
  ssn->min_parallel_nodes = g_min_parallel_nodes;
  // OnSessionOpen in plugin registration (tier) order; the plugins touch disjoint state.
  std::set<std::string> opened;
  for (auto& tier : ssn->tiers)
    for (auto& p : tier) {
      if (opened.count(p.name)) continue;
      opened.insert(p.name);
      if (p.name == "drf") drf.open(ssn);
      else if (p.name == "proportion") prop.open(ssn);
      else if (p.name == "gang") gang_open(ssn);
      else if (p.name == "priority") priority_open(ssn);
      else if (p.name == "predicates") {
        bool active = false;
        for (auto& t2 : ssn->tiers)
          for (auto& p2 : t2)
            if (p2.name == "predicates" && !p2.predicateDisabled) active = true;
        preds.open(ssn, active, n_pod_classes);
      }
      // unknown plugin names are skipped (framework.go:30-35 logs an error)
    }

  // conf "actions" (util.go:30-61); fixtures without the field run allocate only
  std::vector<std::string> actions = {"allocate"};
  if (const Value* a = fx.get("actions")) {
    actions.clear();
    for (auto& x : a->arr) actions.push_back(x.s);
  }
  auto t0 = std::chrono::steady_clock::now();
  g_budget_t0 = t0;
  try {
  for (auto& a : actions) {
    if (a == "allocate") { ssn->action = ""; allocate_execute(ssn); }
    else if (a == "backfill") { ssn->action = "backfill"; backfill_execute(ssn); }
    else if (a == "reclaim") { ssn->action = "reclaim"; reclaim_execute(ssn); }
    else if (a == "preempt") { ssn->action = "preempt"; preempt_execute(ssn); }
    else throw BadInput("unsupported action " + a);
  }
  } catch (const BudgetExceeded&) {
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return "{\"status\":\"budget\",\"stats\":{\"seconds\":" + kbjson::num(secs) +
           ",\"predicate_calls\":" + std::to_string(ssn->predicate_calls) +
           ",\"decisions\":" + std::to_string(ssn->decisions.size()) +
           ",\"evaluated\":" + std::to_string(ssn->evaluated.size()) + "}}";
  }
  auto t1 = std::chrono::steady_clock::now();
  double secs = std::chrono::duration<double>(t1 - t0).count();

  // ---- output
  std::string o = "{\"status\":\"ok\",\"decisions\":[";
  for (size_t i = 0; i < ssn->decisions.size(); i++) {
    auto& d = ssn->decisions[i];
    if (i) o += ",";
    o += "{\"task\":" + kbjson::quote(d.task->uid) + ",\"job\":" + kbjson::quote(d.task->job) +
         ",\"node\":" + kbjson::quote(d.node) + ",\"kind\":\"" + (d.kind == KIND_ALLOCATE ? "allocate" : "pipeline") +
         "\",\"dispatched_at\":" + std::to_string(d.dispatched_at) + (*d.action ? ",\"action\":\"" + std::string(d.action) + "\"" : std::string()) + "}";
  }
  o += "],\"evaluated\":[";
  for (size_t i = 0; i < ssn->evaluated.size(); i++) o += (i ? "," : "") + kbjson::quote(ssn->evaluated[i]->uid);
  o += "],\"binds\":{";
  for (size_t i = 0; i < ssn->binds.size(); i++)
    o += (i ? "," : "") + kbjson::quote(ssn->binds[i].first) + ":" + kbjson::quote(ssn->binds[i].second);
  o += "},\"evictions\":[";
  for (size_t i = 0; i < ssn->evictions.size(); i++) {
    auto& e = ssn->evictions[i];
    o += (i ? "," : "") + std::string("{\"task\":") + kbjson::quote(e.task) + ",\"by\":" + kbjson::quote(e.by) +
         ",\"action\":" + kbjson::quote(e.action) + "}";
  }
  o += "],\"jobs\":[";
  for (size_t i = 0; i < ssn->jobs.size(); i++) {
    JobInfo* j = ssn->jobs[i];
    o += (i ? "," : "");
    o += "{\"uid\":" + kbjson::quote(j->uid) + ",\"queue\":" + kbjson::quote(j->queue) +
         ",\"ready_num\":" + std::to_string(readyTaskNum(j)) + ",\"min_available\":" + std::to_string(j->minAvailable) +
         ",\"ready\":" + (readyTaskNum(j) >= j->minAvailable ? "true" : "false") +
         ",\"allocated\":" + res_json(j->allocated);
    if (names.count("drf")) o += ",\"drf_share\":" + kbjson::num(drf.opts[j->uid].second);
    o += ",\"fit_error\":" + kbjson::quote(j->FitError()) + "}";
  }
  o += "],\"queues\":[";
  bool first = true;
  for (auto& kv : prop.opts.items) {
    QueueAttr* a = kv.second;
    o += (first ? "" : ",");
    first = false;
    o += "{\"uid\":" + kbjson::quote(a->id) + ",\"share\":" + kbjson::num(a->share) + ",\"deserved\":" + res_json(a->deserved) +
         ",\"allocated\":" + res_json(a->allocated) + ",\"request\":" + res_json(a->request) + "}";
  }
  o += "],\"nodes\":[";
  for (size_t i = 0; i < ssn->nodes.size(); i++) {
    NodeInfo* n = ssn->nodes[i];
    o += (i ? "," : "");
    o += "{\"name\":" + kbjson::quote(n->name) + ",\"idle\":" + res_json(n->idle) + ",\"releasing\":" + res_json(n->releasing) +
         ",\"used\":" + res_json(n->used) + ",\"ntasks\":" + std::to_string(n->tasks.size()) + "}";
  }
  o += "],\"stats\":{\"seconds\":" + kbjson::num(secs) + ",\"predicate_calls\":" + std::to_string(ssn->predicate_calls) +
       ",\"decisions\":" + std::to_string(ssn->decisions.size()) + ",\"dup_discards\":" +
       std::to_string(ssn->dup_discards) + ",\"dup_discards_placed\":" + std::to_string(ssn->dup_discards_placed) + "}}";
  return o;
}

// Data-model KATs (node_info_test.go, job_info_test.go): explicit op sequences.
static std::string run_ops(const Value& fx) {
  std::vector<Pod> pods;
  if (const Value* ps = fx.get("pods"))
    for (auto& p : ps->arr) pods.push_back(parse_pod(p));
  auto find_pod = [&](const std::string& name) -> const Pod* {
    for (auto& p : pods) if (p.ns + "/" + p.name == name || p.name == name) return &p;
    throw BadInput("unknown pod " + name);
  };
  auto make_task = [&](const Pod* p) {
    TaskInfo* ti = new TaskInfo();
    ti->uid = p->uid; ti->job = SchedulerCache::job_id_of(*p); ti->name = p->name; ti->ns = p->ns;
    ti->nodeName = p->nodeName; ti->status = get_task_status(*p); ti->priority = p->has_priority ? p->priority : 1;
    ti->pod = p; ti->resreq = p->resreq;
    return ti;
  };
  std::string kind = fx.str("kind");
  std::string o = "{\"status\":\"ok\",";
  if (kind == "nodeinfo_ops") {
    const Value& nv = *fx.get("node");
    Node* node = new Node();
    node->name = nv.str("name");
    node->allocatable = new_resource(nv.get("allocatable"));
    node->capacity = nv.get("capacity") ? new_resource(nv.get("capacity")) : node->allocatable;
    NodeInfo* ni = NodeInfo::make(node);
    for (auto& op : fx.get("ops")->arr) {
      const Pod* p = find_pod(op.str("pod"));
      if (op.str("op") == "add") ni->AddTask(make_task(p));
      else ni->RemoveTask(make_task(p));
    }
    o += "\"idle\":" + res_json(ni->idle) + ",\"used\":" + res_json(ni->used) + ",\"releasing\":" + res_json(ni->releasing) +
         ",\"allocatable\":" + res_json(ni->allocatable) + ",\"tasks\":[";
    bool f = true;
    for (auto& kv : ni->tasks.items) { o += (f ? "" : ",") + kbjson::quote(kv.first); f = false; }
    o += "]}";
  } else if (kind == "jobinfo_ops") {
    JobInfo* ji = new JobInfo();
    ji->uid = fx.str("uid");
    for (auto& op : fx.get("ops")->arr) {
      const Pod* p = find_pod(op.str("pod"));
      if (op.str("op") == "add") ji->AddTaskInfo(make_task(p));
      else { TaskInfo* t = make_task(p); ji->DeleteTaskInfo(t); }
    }
    o += "\"allocated\":" + res_json(ji->allocated) + ",\"total_request\":" + res_json(ji->totalRequest) + ",\"status_index\":{";
    bool f = true;
    for (auto& kv : ji->statusIndex) {
      o += (f ? "" : ",") + std::string("\"") + std::to_string(kv.first) + "\":[";
      f = false;
      std::vector<std::string> ids;
      for (auto& t : kv.second.items) ids.push_back(t.first);
      std::sort(ids.begin(), ids.end());
      for (size_t i = 0; i < ids.size(); i++) o += (i ? "," : "") + kbjson::quote(ids[i]);
      o += "]";
    }
    o += "}}";
  } else if (kind == "cache_ops") {  // cache_test.go: AddNode / AddPod in the listed order
    std::vector<Node*> nodes;
    if (const Value* ns = fx.get("nodes"))
      for (auto& nv : ns->arr) {
        Node* node = new Node();
        node->name = nv.str("name");
        node->allocatable = new_resource(nv.get("allocatable"));
        node->capacity = nv.get("capacity") ? new_resource(nv.get("capacity")) : node->allocatable;
        nodes.push_back(node);
      }
    SchedulerCache c;
    for (auto& op : fx.get("ops")->arr) {
      if (op.str("op") == "add_node") {
        const Node* n = nullptr;
        for (const Node* x : nodes)
          if (x->name == op.str("node")) n = x;
        if (!n) throw BadInput("unknown node " + op.str("node"));
        c.addNode(n);
      } else {
        c.addPod(find_pod(op.str("pod")), 0);
      }
    }
    o += "\"nodes\":{";
    bool f = true;
    for (auto& kv : c.nodes.items) {
      const NodeInfo* ni = kv.second;
      o += std::string(f ? "" : ",") + kbjson::quote(kv.first) + ":{\"idle\":" + res_json(ni->idle) +
           ",\"used\":" + res_json(ni->used) + ",\"releasing\":" + res_json(ni->releasing) +
           ",\"allocatable\":" + res_json(ni->allocatable) + ",\"tasks\":[";
      f = false;
      bool g = true;
      for (auto& t : ni->tasks.items) { o += (g ? "" : ",") + kbjson::quote(t.first); g = false; }
      o += "]}";
    }
    o += "},\"jobs\":{";
    f = true;
    for (auto& kv : c.jobs.items) {
      const JobInfo* ji = kv.second;
      o += std::string(f ? "" : ",") + kbjson::quote(kv.first) + ":{\"status_index\":{";
      f = false;
      bool g = true;
      for (auto& si : ji->statusIndex) {
        o += (g ? "" : ",") + std::string("\"") + std::to_string(si.first) + "\":[";
        g = false;
        std::vector<std::string> ids;
        for (auto& t : si.second.items) ids.push_back(t.first);
        std::sort(ids.begin(), ids.end());
        for (size_t i = 0; i < ids.size(); i++) o += (i ? "," : "") + kbjson::quote(ids[i]);
        o += "]";
      }
      o += "},\"allocated\":" + res_json(ji->allocated) + ",\"total_request\":" + res_json(ji->totalRequest) + "}";
    }
    o += "}}";
  } else if (kind == "quantity") {
    o += "\"values\":[";
    bool f = true;
    for (auto& q : fx.get("quantities")->arr) {
      o += (f ? "" : ",");
      f = false;
      o += "[" + std::to_string(quantity_scaled(q.s, 3)) + "," + std::to_string(quantity_scaled(q.s, 0)) + "]";
    }
    o += "]}";
  } else {
    throw BadInput("unknown kind " + kind);
  }
  return o;
}

}  // namespace ref

int main(int argc, char** argv) {
  std::string in, out;
  bool faithful = false, no_cache = false;
  int threads = 1;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "--faithful") faithful = true;
    else if (a == "--no-cache") no_cache = true;
    else if (a == "--threads" && i + 1 < argc) threads = std::atoi(argv[++i]);
    else if (a == "--min-parallel-nodes" && i + 1 < argc) ref::g_min_parallel_nodes = std::atol(argv[++i]);
    else if (a == "--budget" && i + 1 < argc) ref::g_budget_s = std::atof(argv[++i]);
    else if (a == "-o" && i + 1 < argc) out = argv[++i];
    else in = a;
  }
  if (in.empty()) {
    fprintf(stderr, "usage: kbref [--faithful] [--no-cache] [--threads N] [--min-parallel-nodes N] [--budget SECONDS] fixture.json [-o out.json]\n");
    return 2;
  }
  std::string result;
  int rc = 0;
  try {
    Value fx = kbjson::parse_file(in);
    std::string kind = fx.str("kind", "session");
    result = kind == "session" ? ref::run_session(fx, faithful, no_cache, threads) : ref::run_ops(fx);
  } catch (const ref::RefPanic& e) {
    result = std::string("{\"status\":\"ref_panic\",\"error\":") + kbjson::quote(e.what()) + "}";
  } catch (const ref::Unsupported& e) {
    result = std::string("{\"status\":\"unsupported\",\"error\":") + kbjson::quote(e.what()) + "}";
  } catch (const std::exception& e) {
    result = std::string("{\"status\":\"bad_input\",\"error\":") + kbjson::quote(e.what()) + "}";
    rc = 3;
  }
  if (out.empty()) {
    fwrite(result.data(), 1, result.size(), stdout);
    fputc('\n', stdout);
  } else {
    FILE* f = fopen(out.c_str(), "wb");
    if (!f) { perror("open output"); return 4; }
    fwrite(result.data(), 1, result.size(), f);
    fclose(f);
  }
  return rc;
}
