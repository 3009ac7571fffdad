// kbg_wire.ipp: the snapshot wire format (kbg_snapshot_encode / decode / save / load).
// Part of kbg_session.cpp (one translation unit: included at its end; not
// compiled on its own).

// ============================================================ wire format
// kbgpu.h "Snapshot wire format". Host-only: no device is touched.
struct kbg_snapshot_blob {
  std::vector<std::string> strs;
  std::vector<const char*> ptrs;
  std::vector<std::vector<uint8_t>> arrays;
  kbg_snapshot snap{};
};

namespace {

constexpr char kSnapMagic[4] = {'K', 'B', 'G', 'S'};
constexpr int kSnapCounts = 22;

// Layout word of the wire format: a hash of the element size of every array
// (FNV-1a over the sizes). Blobs stay readable across ABI bumps that leave the
// snapshot structs unchanged; a struct change makes old blobs fail loudly.
uint32_t snapshot_layout() {
  const size_t sizes[] = {sizeof(kbg_node), sizeof(kbg_job), sizeof(kbg_queue), sizeof(kbg_task),
                          sizeof(kbg_resource), sizeof(kbg_spec), sizeof(kbg_term), sizeof(kbg_requirement),
                          sizeof(kbg_toleration), sizeof(kbg_taint), sizeof(kbg_plugin_option),
                          sizeof(kbg_host_port), sizeof(kbg_pod_term), sizeof(kbg_node_pod)};
  uint32_t h = 2166136261u;
  for (size_t v : sizes) {
    h ^= (uint32_t)v;
    h *= 16777619u;
  }
  return h;
}

// The arrays of a kbg_snapshot in declaration order: (pointer slot, count
// slot, element size, elements per count).
template <class F>
void for_each_array(kbg_snapshot& s, F f) {
  f((const void**)&s.nodes, &s.n_nodes, sizeof(kbg_node), 1);
  f((const void**)&s.jobs, &s.n_jobs, sizeof(kbg_job), 1);
  f((const void**)&s.queues, &s.n_queues, sizeof(kbg_queue), 1);
  f((const void**)&s.tasks, &s.n_tasks, sizeof(kbg_task), 1);
  f((const void**)&s.others, &s.n_others, sizeof(kbg_resource), 1);
  f((const void**)&s.specs, &s.n_specs, sizeof(kbg_spec), 1);
  f((const void**)&s.terms, &s.n_terms, sizeof(kbg_term), 1);
  f((const void**)&s.reqs, &s.n_reqs, sizeof(kbg_requirement), 1);
  f((const void**)&s.values, &s.n_values, sizeof(int32_t), 1);
  f((const void**)&s.tolerations, &s.n_tolerations, sizeof(kbg_toleration), 1);
  f((const void**)&s.labels, &s.n_labels, sizeof(int32_t), 2);
  f((const void**)&s.taints, &s.n_taints, sizeof(kbg_taint), 1);
  f((const void**)&s.selectors, &s.n_selectors, sizeof(int32_t), 2);
  f((const void**)&s.plugins, &s.n_plugins, sizeof(kbg_plugin_option), 1);
  f((const void**)&s.tier_sizes, &s.n_tiers, sizeof(int32_t), 1);
  f((const void**)&s.ports, &s.n_ports, sizeof(kbg_host_port), 1);
  f((const void**)&s.node_tasks, &s.n_node_tasks, sizeof(int32_t), 1);
  f((const void**)&s.pod_terms, &s.n_pod_terms, sizeof(kbg_pod_term), 1);
  f((const void**)&s.pod_labels, &s.n_pod_labels, sizeof(int32_t), 2);
  f((const void**)&s.node_pod_keys, &s.n_node_pod_keys, sizeof(int32_t), 1);
  f((const void**)&s.node_pods, &s.n_node_pods, sizeof(kbg_node_pod), 1);
}

struct Writer {
  uint8_t* out;
  int64_t cap, n = 0;
  void put(const void* p, size_t len) {
    if (out && n + (int64_t)len <= cap) std::memcpy(out + n, p, len);
    n += (int64_t)len;
  }
  void u32(uint32_t v) { put(&v, 4); }
};

kbg_status encode(const kbg_snapshot* snap, Writer& w) {
  kbg_status st = validate(snap);
  if (st != KBG_OK) return st;
  kbg_snapshot s = *snap;
  w.put(kSnapMagic, 4);
  w.u32(KBG_SNAPSHOT_FORMAT);
  w.u32(snapshot_layout());
  w.u32((uint32_t)s.n_strings);
  for_each_array(s, [&](const void**, int32_t* cnt, size_t, int) { w.u32((uint32_t)*cnt); });
  for (int32_t i = 0; i < s.n_strings; ++i) {
    const size_t len = std::strlen(s.strings[i]);
    w.u32((uint32_t)len);
    w.put(s.strings[i], len);
  }
  for_each_array(s, [&](const void** ptr, int32_t* cnt, size_t size, int per) {
    if (*cnt > 0) w.put(*ptr, (size_t)*cnt * per * size);
  });
  return KBG_OK;
}

}  // namespace

extern "C" {

kbg_status kbg_snapshot_encode(const kbg_snapshot* snap, uint8_t* out, int64_t cap, int64_t* n_out) {
  Writer w{out, out ? cap : 0};
  kbg_status st = encode(snap, w);
  if (st != KBG_OK) return st;
  if (n_out) *n_out = w.n;
  if (out && w.n > cap) return fail(KBG_E_CAPACITY, "snapshot buffer too small: need " + std::to_string(w.n));
  return KBG_OK;
}

static kbg_status snapshot_decode(const uint8_t* data, int64_t n, kbg_snapshot_blob** out) {
  int64_t pos = 0;
  auto take = [&](void* dst, int64_t len) {
    if (len < 0 || len > n - pos) return false;
    if (len > 0) std::memcpy(dst, data + pos, (size_t)len);
    pos += len;
    return true;
  };
  char magic[4];
  uint32_t fmt = 0, layout = 0, nstr = 0;
  if (!take(magic, 4) || std::memcmp(magic, kSnapMagic, 4) != 0) return fail(KBG_E_INVALID, "not a kbg snapshot");
  if (!take(&fmt, 4) || !take(&layout, 4) || fmt != KBG_SNAPSHOT_FORMAT || layout != snapshot_layout())
    return fail(KBG_E_INVALID, "snapshot format " + std::to_string(fmt) + " / layout " + std::to_string(layout) +
                                   " (this library: " + std::to_string(KBG_SNAPSHOT_FORMAT) + " / " +
                                   std::to_string(snapshot_layout()) + ")");
  if (!take(&nstr, 4) || nstr > (uint32_t)INT32_MAX) return fail(KBG_E_INVALID, "truncated snapshot header");
  auto blob = std::make_unique<kbg_snapshot_blob>();
  kbg_snapshot& s = blob->snap;
  s.n_strings = (int32_t)nstr;
  bool ok = true;
  int64_t array_bytes = 0;  // what the counts promise, checked against the input before any allocation
  for_each_array(s, [&](const void**, int32_t* cnt, size_t size, int per) {
    uint32_t v = 0;
    ok = ok && take(&v, 4) && v <= (uint32_t)INT32_MAX;
    *cnt = (int32_t)v;
    array_bytes += (int64_t)v * per * (int64_t)size;
  });
  if (!ok) return fail(KBG_E_INVALID, "truncated snapshot header");
  // every string takes at least its 4-byte length; every array its raw bytes
  if ((int64_t)nstr * 4 > n - pos || array_bytes > n - pos - (int64_t)nstr * 4)
    return fail(KBG_E_INVALID, "snapshot counts exceed the input");
  blob->strs.resize(nstr);
  for (uint32_t i = 0; i < nstr; ++i) {
    uint32_t len = 0;
    if (!take(&len, 4) || (int64_t)len > n - pos) return fail(KBG_E_INVALID, "truncated snapshot strings");
    blob->strs[i].assign((const char*)data + pos, len);
    pos += len;
  }
  blob->ptrs.resize(nstr);
  for (uint32_t i = 0; i < nstr; ++i) blob->ptrs[i] = blob->strs[i].c_str();
  s.strings = blob->ptrs.data();
  if (array_bytes != n - pos) return fail(KBG_E_INVALID, "snapshot arrays do not match the input length");
  blob->arrays.reserve(kSnapCounts);
  for_each_array(s, [&](const void** ptr, int32_t* cnt, size_t size, int per) {
    const int64_t len = (int64_t)*cnt * per * (int64_t)size;
    blob->arrays.emplace_back((size_t)len);
    std::vector<uint8_t>& a = blob->arrays.back();
    ok = ok && take(a.data(), len);
    *ptr = *cnt > 0 ? a.data() : nullptr;
  });
  if (!ok) return fail(KBG_E_INVALID, "truncated snapshot arrays");
  if (pos != n) return fail(KBG_E_INVALID, "trailing bytes after the snapshot");
  kbg_status st = validate(&s);
  if (st != KBG_OK) return st;
  *out = blob.release();
  return KBG_OK;
}

kbg_status kbg_snapshot_decode(const uint8_t* data, int64_t n, kbg_snapshot_blob** out) {
  if (!data || !out || n < 0) return fail(KBG_E_INVALID, "null argument");
  *out = nullptr;
  try {
    return snapshot_decode(data, n, out);
  } catch (const std::bad_alloc&) {
    return fail(KBG_E_NOMEM, "host allocation failed");
  } catch (const std::length_error&) {
    return fail(KBG_E_INVALID, "snapshot counts exceed the input");
  }
}

kbg_status kbg_snapshot_save(const kbg_snapshot* snap, const char* path) {
  if (!path) return fail(KBG_E_INVALID, "null path");
  int64_t n = 0;
  kbg_status st = kbg_snapshot_encode(snap, nullptr, 0, &n);
  if (st != KBG_OK) return st;
  std::vector<uint8_t> buf((size_t)n);
  if ((st = kbg_snapshot_encode(snap, buf.data(), n, &n)) != KBG_OK) return st;
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(KBG_E_INVALID, std::string("cannot open ") + path);
  const bool wrote = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
  if (std::fclose(f) != 0 || !wrote) return fail(KBG_E_INVALID, std::string("cannot write ") + path);
  return KBG_OK;
}

kbg_status kbg_snapshot_load(const char* path, kbg_snapshot_blob** out) {
  if (!path || !out) return fail(KBG_E_INVALID, "null argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(KBG_E_INVALID, std::string("cannot open ") + path);
  std::vector<uint8_t> buf;
  uint8_t chunk[1 << 16];
  size_t got;
  while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.insert(buf.end(), chunk, chunk + got);
  std::fclose(f);
  return kbg_snapshot_decode(buf.data(), (int64_t)buf.size(), out);
}

const kbg_snapshot* kbg_snapshot_blob_get(const kbg_snapshot_blob* b) { return b ? &b->snap : nullptr; }

void kbg_snapshot_blob_free(kbg_snapshot_blob* b) { delete b; }

}  // extern "C"
