// kbg_svc_link.ipp: the scan service's transport (SvcLink), its messages and the device side of a served launch.
// Part of kbg_session.cpp (one translation unit: included there inside its
// anonymous namespace, after the parts before it; not compiled on its own).

// ============================================ the scan service: transport
// Sharded allocate as ONE committer: rank 0 runs the single-GPU
// pipeline (ordering engine, in-order commit, overlapped and reused scans)
// and every scan it launches is a message to the other ranks: the launch's
// arguments, the node rows and class-mask words its commits wrote since the
// last message (every rank writes the rows it holds), and the committed
// outcomes (each rank replays them into its mirror, decision log and engine,
// beside its scans). Every rank runs the fused kernel over its own words into
// a zeroed (slot, rank) info array and a [slot][W] mask array; one summing
// all-reduce over the ranks (disjoint words: the sum is the union) gives rank
// 0 the whole table's lists, joined in node order like a split launch's
// parts. Rank 0's collectives are enqueued on its stream (no host wait); the
// other ranks wait for each message.

enum : uint32_t { kSvcLaunch = 0, kSvcEnd = 1, kSvcAbort = 2, kSvcState = 3 };
constexpr size_t kSvcHead = 16;          // header words: kind, words, nodes, masks, outcomes, args, shapes, rowshape,
                                         // status, G, slots
constexpr size_t kSvcMaxWords = 1u << 19;  // one message (2 MB); a longer state goes out in kSvcState chunks
constexpr size_t kSvcNodeWords = sizeof(kbg::NodeDelta) / 4, kSvcMaskWords = sizeof(kbg::MaskDelta) / 4;
constexpr size_t kSvcStreamWords = 2 * 2048;  // rank 0 streams its commits once this many words wait
static_assert(sizeof(kbg::NodeDelta) % 4 == 0 && sizeof(kbg::MaskDelta) % 4 == 0, "message words");

inline void svc_put(std::vector<uint32_t>& m, const void* p, size_t bytes) {
  const size_t o = m.size();
  m.resize(o + (bytes + 3) / 4, 0u);
  if (bytes) std::memcpy(&m[o], p, bytes);
}

// Rank 0: the pending state (rows, mask words, outcomes) in messages of kind
// `kind` (kSvcState chunks first when it does not fit into one message with
// `reserve` more words); leaves the last part for the caller when `keep` is set.
kbg_status svc_flush_state(Session& S, std::vector<uint32_t>& m, size_t reserve, bool keep, uint32_t kind,
                           uint32_t status) {
  size_t ni = 0, mi = 0, oi = 0;
  for (;;) {
    const size_t room = kSvcMaxWords - kSvcHead - reserve;
    const size_t nn = std::min(S.svc_nodes.size() - ni, room / kSvcNodeWords);
    const size_t nm = std::min(S.svc_masks.size() - mi, (room - nn * kSvcNodeWords) / kSvcMaskWords);
    const size_t no = std::min((S.svc_out.size() - oi) / 2,
                               (room - nn * kSvcNodeWords - nm * kSvcMaskWords) / 2);
    const bool last = ni + nn == S.svc_nodes.size() && mi + nm == S.svc_masks.size() && oi + 2 * no == S.svc_out.size();
    m.assign(kSvcHead, 0u);
    m[0] = last ? kind : kSvcState;
    m[2] = (uint32_t)nn;
    m[3] = (uint32_t)nm;
    m[4] = (uint32_t)no;
    m[8] = status;
    svc_put(m, S.svc_nodes.data() + ni, nn * sizeof(kbg::NodeDelta));
    svc_put(m, S.svc_masks.data() + mi, nm * sizeof(kbg::MaskDelta));
    svc_put(m, S.svc_out.data() + oi, no * 8);
    ni += nn;
    mi += nm;
    oi += 2 * no;
    if (last && keep) break;  // the caller appends its part and sends
    m[1] = (uint32_t)m.size();
    if (kbg_status st = S.svc->send(S, m.data()); st != KBG_OK) return st;
    if (last) break;
  }
  S.svc_nodes.clear();
  S.svc_masks.clear();
  S.svc_out.clear();
  return KBG_OK;
}

// Rank 0's part of a scan: the launch message, its own words, the sum.
kbg_status svc_launch(Session& S, kbg::Stage& sg, kbg::FirstFitArgs& a, int32_t G, int32_t base) {
  const int32_t ns = sg.n_slots;
  // the arguments go out before this rank's words are set in them (each rank sets its own)
  const size_t args_w = (sizeof(kbg::FirstFitArgs) + 3) / 4;
  const size_t shapes_w = a.shapes ? ((size_t)ns * sizeof(kbg::TaskRec) + 3) / 4 : 0;
  const size_t rows_w = a.row_shape ? (size_t)G : 0;
  thread_local std::vector<uint32_t> m;
  if (kbg_status st = svc_flush_state(S, m, args_w + shapes_w + rows_w, true, kSvcLaunch, 0); st != KBG_OK) return st;
  m[5] = (uint32_t)args_w;
  m[6] = (uint32_t)shapes_w;
  m[7] = (uint32_t)rows_w;
  m[9] = (uint32_t)G;
  m[10] = (uint32_t)ns;
  // payload order: args, shapes, rows, then the state svc_flush_state put
  std::vector<uint32_t> state(m.begin() + kSvcHead, m.end());
  m.resize(kSvcHead);
  svc_put(m, &a, sizeof(kbg::FirstFitArgs));
  if (shapes_w) svc_put(m, sg.h_shapes, (size_t)ns * sizeof(kbg::TaskRec));
  if (rows_w) svc_put(m, sg.h_rowshape, (size_t)G * 4);
  m.insert(m.end(), state.begin(), state.end());
  m[1] = (uint32_t)m.size();
  if (kbg_status st = S.svc->send(S, m.data()); st != KBG_OK) return st;
  // this rank's words, every rank's info column and the whole mask width
  a.w_lo = std::min(S.W, S.shard * S.Wl);
  a.w_hi = std::min(S.W, (S.shard + 1) * S.Wl);
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
  HIP_TRY(hipMemsetAsync(S.d_svc, 0, info_w * 4, S.stream));
  HIP_TRY(hipMemsetAsync(a.masks, 0, mask_w * 4, S.stream));
  sg.timed = !S.untimed_launches && S.ff_launch_seq++ % ff_time_every(S) == 0;
  HIP_TRY(kbg::launch_firstfit(a, S.int_mode ? 1 : 0, S.stream, sg.timed ? sg.ev[0] : nullptr,
                               sg.timed ? sg.ev[1] : nullptr));
  trace_add("l.firstfit");
  if (kbg_status st = S.svc->sum(S, &sg, info_w, mask_w); st != KBG_OK) return st;
  HIP_TRY(hipEventRecord(sg.ev[6], S.stream));
  sg.splits = S.R;  // device_wait joins the ranks' parts in node order
  sg.fused = true;
  sg.G = G;
  sg.base = base;
  sg.inflight = true;
  return KBG_OK;
}

kbg_status svc_sum_counts(Session& S, int32_t* counts, size_t n) {
  return S.svc->sum_host(S, reinterpret_cast<uint32_t*>(counts), n);
}

// Writes the rows of the nodes touched by the last commits back to HBM (only
// the rows this process holds; every shard's host mirror saw every commit).
// The pinned staging buffers (h_deltas, h_mdeltas, h_sdeltas) are read by
// the stream when a copy or kernel executes, not when it is enqueued, and the
// stream may still be behind (a scan enqueued earlier runs first): a writer
// waits for the last reader (stage_acquire) and every enqueued reader marks
// the stream (stage_release).
kbg_status stage_acquire(Session& S) {
  if (S.stage_pending) {
    HIP_TRY(hipEventSynchronize(S.stage_ev));
    S.stage_pending = false;
  }
  return KBG_OK;
}
kbg_status stage_release(Session& S) {
  HIP_TRY(hipEventRecord(S.stage_ev, S.stream));
  S.stage_pending = true;
  return KBG_OK;
}

// Class-mask words changed on the host (host ports, pod affinity) into HBM;
// every shard holds the whole mask.
kbg_status push_mask_deltas(Session& S) {
  for (size_t m = 0; m < S.mask_dirty.size();) {
    kbg_status st = stage_acquire(S);
    if (st != KBG_OK) return st;
    const int32_t cnt = (int32_t)std::min<size_t>(S.mask_dirty.size() - m, (size_t)kbg::kMaskDeltaCap);
    for (int32_t k = 0; k < cnt; ++k) {
      const uint32_t idx = S.mask_dirty[m + k];
      S.h_mdeltas[k] = kbg::MaskDelta{idx, 0u, S.h_class_mask[idx]};
      S.mask_dirty_flag[idx] = 0;
    }
    if (S.svc) S.svc_masks.insert(S.svc_masks.end(), S.h_mdeltas, S.h_mdeltas + cnt);  // for every rank's table
    const kbg::MaskDelta* md = dev_ptr(S, S.h_mdeltas);
    if (!md) return fail(KBG_E_HIP, "hipHostGetDevicePointer of the mask-delta buffer failed");
    HIP_TRY(kbg::launch_mask_apply(S.d_class_mask, md, cnt, S.stream));  // read in place
    if ((st = stage_release(S)) != KBG_OK) return st;
    m += cnt;
  }
  S.mask_dirty.clear();
  return KBG_OK;
}

kbg_status push_deltas(Session& S, const std::vector<int32_t>& touched) {
  kbg_status st = push_mask_deltas(S);
  if (st != KBG_OK) return st;
  if (S.svc)  // the scan service: every rank's rows go out with the next message (each rank writes its own)
    for (const int32_t n : touched) {
      kbg::NodeDelta d{};
      d.node = n;
      device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
      S.svc_nodes.push_back(d);
    }
  size_t i = 0;
  while (i < touched.size()) {
    if ((st = stage_acquire(S)) != KBG_OK) return st;
    int32_t cnt = 0;
    for (; i < touched.size() && cnt < S.K; ++i) {
      const int32_t n = touched[i];
      if (n < S.tab_lo || n >= S.tab_lo + S.tab_n) continue;
      kbg::NodeDelta& d = S.h_deltas[cnt++];
      d.node = n - S.tab_lo;
      device_row(S, n, &d.idle[0], &d.idle[1], &d.idle[2], &d.rel[0], &d.rel[1], &d.rel[2], &d.ntasks, &d.maxtasks);
    }
    if (cnt == 0) break;
    HIP_TRY(kbg::launch_apply(S.d_nodes, S.h_deltas_dev, cnt, S.stream));  // read in place
    if ((st = stage_release(S)) != KBG_OK) return st;
  }
  return KBG_OK;
}

// Groups the tasks of a batch into device rows and sizes their candidate
// lists. Full-scan mode: one row per task (every evaluation scans the whole
// table — the SURVEY §8(d) roofline rule) with M + r slots, r = the number of
// earlier rows of the same (class, request) shape in this scan: each earlier
// commit can exhaust at most one node of the list, so a row rarely runs out
// before the table does. Grouped mode: one row per distinct shape with (tasks
// of the shape + slack) slots; tasks of a shape share the row and a cursor.
constexpr int32_t kGroupSlack = 512;     // extra candidate slots per shape row (grouped mode)
constexpr int32_t kContendedSlack = 4096;  // the same in a rescan of the contended part of a cycle
constexpr int32_t kFullScanGrow = 1024;  // cap on a full-scan row's extra slots
constexpr int32_t kFullScanK = 8192;     // default batch of the full-scan mode

// Bytes of one stage's row buffer for batches of K tasks: the rows
// (TaskRec, padded) and their candidate offsets, then (fused full-scan path)
// each row's shape slot and the shape table.
inline size_t up_bytes_for(int32_t K) {
  const size_t rows = (size_t)kbg::kbg_pad_rows(K) * sizeof(kbg::TaskRec) + ((size_t)K + 1) * 4;
  return ((rows + 15) & ~(size_t)15) + (((size_t)K * 4 + 15) & ~(size_t)15) + (size_t)K * sizeof(kbg::TaskRec);
}

// A row whose scan found no fitting node in a complete walk of the table.
inline bool row_fits_nowhere(const kbg::Stage& g, int32_t r) {
  if (g.fused) return (g.h_info[g.row_slot[r]] & (kbg::kInfoAnyBit | kbg::kCountIncompleteBit)) == 0;
  return g.h_count[r] == 0;
}
// A row with some fitting node in the words its scan covered (listed or not).
inline bool row_fits_somewhere(const kbg::Stage& g, int32_t r) {
  if (g.fused) return (g.h_info[g.row_slot[r]] & kbg::kInfoAnyBit) != 0;
  return g.h_count[r] != 0;
}

struct Grouper {
  Session& S;
  std::vector<int32_t> shape_row, shape_stamp, count, ext_slot;
  int32_t stamp = 0;
  explicit Grouper(Session& s) : S(s), shape_row(s.n_shapes, -1), shape_stamp(s.n_shapes, -1) {}
  // `slack`: grouped mode's extra candidate slots per shape row (the
  // contended part of a cycle asks for long lists: few nodes still fit a
  // shape there, and a list that holds all of them needs no rescan to
  // learn that the shape fits nowhere)
  int32_t build(kbg::Stage& sg, const int32_t* bt, int32_t n, int32_t slack = kGroupSlack) {
    sg.h_tasks = (kbg::TaskRec*)sg.h_up;
    ++stamp;
    sg.row_of.resize(n);
    sg.row_shape.clear();
    count.clear();
    int32_t G = 0;
    for (int32_t i = 0; i < n; ++i) {
      const int32_t t = bt[i];
      int32_t g;
      const int32_t sh = S.task_shape[t];
      const bool seen = shape_stamp[sh] == stamp;
      if (!S.opts.full_scan && seen) {
        g = shape_row[sh];
      } else {
        g = G++;
        // full-scan: count[g] = earlier rows of this shape in the scan (the list grows with them)
        count.push_back(S.opts.full_scan && seen ? count[shape_row[sh]] + 1 : 0);
        shape_stamp[sh] = stamp;
        shape_row[sh] = g;
        sg.row_shape.push_back(sh);
        kbg::TaskRec& r = sg.h_tasks[g];
        const Res& q = S.treq[t];
        if (S.be_task[t]) {  // backfill: PredicateFn only — every node fits (a > -inf in both modes)
          r.req[0] = r.req[1] = r.req[2] = -INFINITY;
        } else if (S.int_mode) {  // thresholds: LessEqual(q, a) == (a > q - min), exact (kbg_device.hpp)
          r.req[0] = q.c - kbg::kMinMilliCPU;
          r.req[1] = q.m - kbg::kMinMemory;
          r.req[2] = q.g - kbg::kMinMilliGPU;
        } else {
          r.req[0] = q.c;
          r.req[1] = q.m;
          r.req[2] = q.g;
        }
        r.cls = S.task_class[t];
        r.flags = (S.be_task[t] || kbg::res_le(q, Res{})) ? kbg::kRowRelZeroFits : 0;
      }
      sg.row_of[i] = g;
      if (!S.opts.full_scan) count[g]++;
    }
    const int32_t Gp = kbg::kbg_pad_rows(G);
    for (int32_t g = G; g < Gp; ++g) sg.h_tasks[g] = sg.h_tasks[0];  // padding rows: scanned, never stored
    sg.h_capoff = (uint32_t*)(sg.h_up + (size_t)Gp * sizeof(kbg::TaskRec));
    sg.h_capoff[0] = 0;
    // full-scan: rows of one shape in one scan evaluate identical inputs
    // against the same table, so their lists are one sequence. Every row is
    // evaluated against the whole table on the device; the list is written
    // once, for the shape's last row (a long list: every commit before it can
    // exhaust one node), and the shape's other rows read it (Resolver).
    if (S.opts.full_scan) {
      sg.row_ext.resize(G);
      for (int32_t g = 0; g < G; ++g) sg.row_ext[g] = shape_row[sg.row_shape[g]];
    }
    int32_t grow_cap = kFullScanGrow;
    if (S.opts.full_scan) {  // more shapes than the buffers were sized for: shorter long lists
      int64_t longs = 0;
      for (int32_t g = 0; g < G; ++g) longs += sg.row_ext[g] == g;
      const int64_t spare = S.cand_cap - (int64_t)G * S.M;
      if (longs * kFullScanGrow > spare) grow_cap = (int32_t)std::max<int64_t>(0, spare / std::max<int64_t>(1, longs));
    }
    if (!S.opts.full_scan && slack > kGroupSlack) {  // within the candidate buffer (sized for K x (kGroupSlack + 1))
      const int64_t room = (S.cand_cap - n) / std::max(1, G);
      slack = (int32_t)std::max<int64_t>(kGroupSlack, std::min<int64_t>(slack, room));
    }
    const int32_t cap_want = std::max(4096, slack);
    for (int32_t g = 0; g < G; ++g) {
      uint32_t want;
      if (!S.opts.full_scan) want = (uint32_t)std::min(count[g] + slack, cap_want);
      else if (sg.row_ext[g] != g) want = 0;  // its list is the shape's long one (Resolver: alias rows)
      else want = (uint32_t)(S.M + std::min(2 * count[g] + (g >> 3) + 64, grow_cap));
      sg.h_capoff[g + 1] = sg.h_capoff[g] + want;
      // the fused kernel reads the row's want from its flags (kbg_device.hpp FirstFitArgs)
      sg.h_tasks[g].flags = (sg.h_tasks[g].flags & kbg::kRowRelZeroFits) | (int32_t)(want << kbg::kRowWantShift);
    }
    // Fused path: grouped rows are their own shapes; full-scan rows name the
    // slot of their shape (the shape's last row, which writes the list; the
    // shape table holds that row's record, so no launch reads all G records)
    sg.row_slot.resize(G);
    if (S.opts.full_scan) {
      const size_t rows_b = ((size_t)Gp * sizeof(kbg::TaskRec) + ((size_t)G + 1) * 4 + 15) & ~(size_t)15;
      sg.h_rowshape = (uint32_t*)(sg.h_up + rows_b);
      sg.h_shapes = (kbg::TaskRec*)(sg.h_up + rows_b + (((size_t)G * 4 + 15) & ~(size_t)15));
      ext_slot.resize(G);
      int32_t ns = 0;
      for (int32_t g = 0; g < G; ++g)
        if (sg.row_ext[g] == g) {
          ext_slot[g] = ns;
          sg.h_shapes[ns++] = sg.h_tasks[g];
        }
      sg.slot_rows.assign(ns, 0);
      for (int32_t g = 0; g < G; ++g) {
        const int32_t sl = ext_slot[sg.row_ext[g]];
        sg.row_slot[g] = sl;
        sg.h_rowshape[g] = (uint32_t)sl | (sg.row_ext[g] == g ? kbg::kRowWriter : 0u);
        sg.slot_rows[sl]++;
      }
      sg.n_slots = ns;
    } else {
      for (int32_t g = 0; g < G; ++g) sg.row_slot[g] = g;
      sg.h_rowshape = nullptr;
      sg.h_shapes = sg.h_tasks;
      sg.n_slots = G;
      sg.slot_rows.clear();
    }
    return G;
  }
};

// In-order commit against the candidate lists of one scan. A node the list
// names is taken as it is unless a resolution newer than the scan touched it
// (mark > base: resources, pod count, or a class-mask bit it lost); those are
// re-checked on the host mirror. A row's cursor only moves forward: a
// candidate found infeasible for a (class, request) shape stays infeasible
// for every later task of that shape (monotonicity). In full-scan mode every
// task has its own row, and rows of one shape in one scan hold the same list
// (same inputs, same table): the prefix an earlier row of the shape rejected
// is skipped instead of re-checked (`shape_skip`).
enum { RES_OK = 0, RES_TRUNC = 1, RES_PANIC = 2 };
// The in-order commit's view of one node, in one cache line: what a
// re-check of a candidate touched since its scan reads (Idle, Releasing, pod
// count and cap, the stamp of the node's last commit, the nil-Node panic
// flag), instead of five separate arrays. The allocate committer keeps it
// current with every commit (mirror_row).
struct alignas(64) MirrorRow {
  double ic, im, ig, rc, rm, rg;
  int32_t nt, mt;
  int32_t mark;
  int32_t panic;
};
static_assert(sizeof(MirrorRow) == 64, "one cache line per node");
inline void mirror_row(const Session& S, MirrorRow& q, int32_t nd) {
  q.ic = S.idle[nd].c;
  q.im = S.idle[nd].m;
  q.ig = S.idle[nd].g;
  q.rc = S.rel[nd].c;
  q.rm = S.rel[nd].m;
  q.rg = S.rel[nd].g;
  q.nt = S.ntasks[nd];
}
struct Resolver {
  Session& S;
  std::vector<int32_t>& mark;
  const kbg::Stage* sg = nullptr;
  int32_t base = 0;
  std::vector<int32_t> cursor;
  std::vector<int32_t> shape_skip, skip_stamp;
  int32_t skip_gen = 0;
  // per shape, the first node not yet found infeasible this action (nullptr:
  // off). Nodes only lose room while an allocate runs (a pod-affinity gain
  // resets its class's shapes), so what a shape rejected under one scan
  // stays rejected under every later scan: a fresh stage's cursor starts
  // there instead of re-checking the nodes the earlier batches filled.
  int32_t* floor = nullptr;
  // the committer's packed mirror (nullptr: the separate arrays and `mark`)
  const MirrorRow* rows = nullptr;
  void reset(const kbg::Stage& stage) {
    sg = &stage;
    base = stage.base;
    cursor.assign(stage.G, 0);
    if (S.opts.full_scan) {
      if (shape_skip.size() < (size_t)S.n_shapes) {
        shape_skip.assign(S.n_shapes, 0);
        skip_stamp.assign(S.n_shapes, -1);
      }
      ++skip_gen;
    }
  }
  bool dirty(int32_t t, int32_t nd) const {
    return mark[nd] > base || (S.has_aff && S.mwmark[(size_t)S.task_class[t] * S.W + (nd >> 6)] > base);
  }
  // the host mirror's verdict on node nd for task t, for a candidate touched
  // since the scan: 1 Allocate, 2 Pipeline, 0 it no longer fits
  int recheck(int32_t t, int32_t nd, const Res& r) const {
    if (S.pred_active && S.ntasks[nd] >= S.maxtasks[nd]) return 0;
    if ((S.has_ports || S.has_aff) &&
        !((S.h_class_mask[(size_t)S.task_class[t] * S.W + (nd >> 6)] >> (nd & 63)) & 1ull))
      return 0;
    if (S.be_task[t]) return 1;  // backfill: PredicateFn only, always ssn.Allocate
    if (kbg::res_le(r, S.idle[nd])) return 1;
    if (kbg::res_le(r, S.rel[nd])) return 2;
    return 0;
  }
  // Fused stages: the row's shape list as word masks (kbg_device.hpp
  // FirstFitArgs); the cursor is the next node to look at, in node order.
  int resolve_mask(int32_t g, int32_t t, int32_t* node, int32_t* kind) {
    const int32_t sl = sg->row_slot[g];
    const uint32_t info = sg->h_info[sl];
    const int32_t wl = sg->w_lo;
    const kbg::MaskPair* m = sg->h_mask + (size_t)sl * sg->mw - wl;  // indexed by global word
    const int32_t end = (wl + (int32_t)(info & kbg::kInfoWordsMask)) * 64;
    const Res& r = S.treq[t];
    int32_t sh = -1;
    int32_t& k = cursor[g];
    if (k < wl * 64) k = wl * 64;
    if (S.opts.full_scan) {
      sh = sg->row_shape[g];
      if (skip_stamp[sh] == skip_gen) k = std::max(k, shape_skip[sh]);  // what earlier rows of the shape rejected
    }
    int32_t* const fl = floor ? floor + S.task_shape[t] : nullptr;
    if (fl && k < *fl) k = *fl;
    int res = -1;
    int64_t steps = 0, rechecks = 0;
    // A word's candidates are taken lowest first by clearing bits (a short
    // dependency chain: the checks of successive candidates overlap), the
    // mirror's rows through pointers held in registers. In contended
    // cycles most candidates are nodes touched since the scan that no
    // longer fit, so this loop is the in-order commit's hot spot.
    const char* panic = S.panic_node.data();
    const int32_t* mk = mark.data();
    const int32_t* nt = S.ntasks.data();
    const int32_t* mt = S.maxtasks.data();
    const Res* idle = S.idle.data();
    const Res* rel = S.rel.data();
    const bool cap = S.pred_active, masked = S.has_ports || S.has_aff, aff = S.has_aff, be = S.be_task[t];
    const uint64_t* cmask = S.h_class_mask.data() + (size_t)S.task_class[t] * S.W;
    const int32_t bs = base;
    if (rows) {  // the same walk over one cache line per candidate
      const int32_t* awm = aff ? S.mwmark.data() + (size_t)S.task_class[t] * S.W : nullptr;
      const double rc_ = r.c, rm_ = r.m, rg_ = r.g;
      auto fits = [&](double a0, double a1, double a2) {  // Resource.LessEqual (resource_info.go:142-146)
        return (rc_ < a0 || __builtin_fabs(a0 - rc_) < kbg::kMinMilliCPU) &&
               (rm_ < a1 || __builtin_fabs(a1 - rm_) < kbg::kMinMemory) &&
               (rg_ < a2 || __builtin_fabs(a2 - rg_) < kbg::kMinMilliGPU);
      };
      while (k < end && res < 0) {
        const int32_t w = k >> 6;
        uint64_t bits = m[w].f & (~0ull << (k & 63));
        const bool wdirty = aff && awm[w] > bs;
        while (bits) {
          const int32_t nd = (w << 6) | __builtin_ctzll(bits);
          bits &= bits - 1;
          if (bits) __builtin_prefetch(rows + ((w << 6) | __builtin_ctzll(bits)));
          const MirrorRow& q = rows[nd];
          ++steps;
          if (q.panic) {
            k = nd;
            res = RES_PANIC;
            break;
          }
          if (!(q.mark > bs || wdirty)) {
            k = nd;
            *node = nd;
            *kind = ((m[w].i >> (nd & 63)) & 1ull) ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
            res = RES_OK;
            break;
          }
          ++rechecks;  // touched since the scan: re-check on the host mirror
          if (cap && q.nt >= q.mt) continue;
          if (masked && !((cmask[w] >> (nd & 63)) & 1ull)) continue;
          const int v = be ? 1 : fits(q.ic, q.im, q.ig) ? 1 : fits(q.rc, q.rm, q.rg) ? 2 : 0;
          if (v) {
            k = nd;
            *node = nd;
            *kind = v == 1 ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
            res = RES_OK;
            break;
          }
        }
        if (res < 0) k = (w + 1) << 6;
      }
    }
    while (k < end && res < 0) {
      const int32_t w = k >> 6;
      uint64_t bits = m[w].f & (~0ull << (k & 63));
      while (bits) {
        const int32_t nd = (w << 6) | __builtin_ctzll(bits);
        bits &= bits - 1;
        ++steps;
        if (panic[nd]) {
          k = nd;
          res = RES_PANIC;
          break;
        }
        if (!(mk[nd] > bs || (aff && S.mwmark[(size_t)S.task_class[t] * S.W + w] > bs))) {
          k = nd;
          *node = nd;
          *kind = ((m[w].i >> (nd & 63)) & 1ull) ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
          res = RES_OK;
          break;
        }
        ++rechecks;  // touched since the scan: re-check on the host mirror (recheck())
        if (cap && nt[nd] >= mt[nd]) continue;
        if (masked && !((cmask[w] >> (nd & 63)) & 1ull)) continue;
        const int v = be ? 1 : kbg::res_le(r, idle[nd]) ? 1 : kbg::res_le(r, rel[nd]) ? 2 : 0;
        if (v) {
          k = nd;
          *node = nd;
          *kind = v == 1 ? KBG_KIND_ALLOCATE : KBG_KIND_PIPELINE;
          res = RES_OK;
          break;
        }
      }
      if (res < 0) k = (w + 1) << 6;
    }
    S.stats.resolve_steps += steps;
    S.stats.resolve_rechecks += rechecks;
    if (sh >= 0 && res != RES_PANIC) {  // nodes before k are infeasible for the shape from now on
      shape_skip[sh] = k;
      skip_stamp[sh] = skip_gen;
    }
    if (fl && res != RES_PANIC) *fl = k;
    if (res >= 0) return res;
    if (info & kbg::kCountIncompleteBit) return RES_TRUNC;
    *node = -1;
    return RES_OK;
  }
  int resolve(int32_t g, int32_t t, int32_t* node, int32_t* kind) {
    if (sg->fused) return resolve_mask(g, t, node, kind);
    if (S.opts.full_scan && sg->h_capoff[g + 1] == sg->h_capoff[g])
      g = sg->row_ext[g];  // an alias row: its shape's long list (Grouper::build), this row's cursor
    const uint32_t cnt = sg->h_count[g];
    const int32_t n = (int32_t)(cnt & kbg::kCountMask);
    const uint32_t* c = sg->h_cand + sg->h_capoff[g];
    const Res& r = S.treq[t];
    int32_t sh = -1;
    if (S.opts.full_scan) {
      sh = sg->row_shape[g];
      // the skip may pass this row's own M entries: the loop moves to the long list
      if (skip_stamp[sh] == skip_gen) cursor[g] = std::max(cursor[g], shape_skip[sh]);
    }
    int res = -1;
    int32_t& k = cursor[g];
    const int32_t k0 = k;
    int64_t rechecks = 0;
    int32_t n_end = n;
    uint32_t cnt_end = cnt;
    for (;; ++k) {
      if (k >= n_end) {  // full-scan: continue in the shape's longest list of this scan
        if (sh < 0 || !(cnt_end & kbg::kCountIncompleteBit)) break;
        const int32_t g2 = sg->row_ext[g];
        const uint32_t cnt2 = sg->h_count[g2];
        if (g2 == g || (int32_t)(cnt2 & kbg::kCountMask) <= n_end) break;
        c = sg->h_cand + sg->h_capoff[g2];
        n_end = (int32_t)(cnt2 & kbg::kCountMask);
        cnt_end = cnt2;
        if (k >= n_end) break;
      }
      const int32_t nd = (int32_t)(c[k] & ~kbg::kCandPipelineBit);
      if (S.panic_node[nd]) {
        res = RES_PANIC;
        break;
      }
      if (!dirty(t, nd)) {
        *node = nd;
        *kind = (c[k] & kbg::kCandPipelineBit) ? KBG_KIND_PIPELINE : KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      // touched since the scan: re-check on the host mirror
      ++rechecks;
      if (S.pred_active && S.ntasks[nd] >= S.maxtasks[nd]) continue;
      if ((S.has_ports || S.has_aff) &&
          !((S.h_class_mask[(size_t)S.task_class[t] * S.W + (nd >> 6)] >> (nd & 63)) & 1ull))
        continue;
      if (S.be_task[t]) {  // backfill: PredicateFn only, always ssn.Allocate
        *node = nd;
        *kind = KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      if (kbg::res_le(r, S.idle[nd])) {
        *node = nd;
        *kind = KBG_KIND_ALLOCATE;
        res = RES_OK;
        break;
      }
      if (kbg::res_le(r, S.rel[nd])) {
        *node = nd;
        *kind = KBG_KIND_PIPELINE;
        res = RES_OK;
        break;
      }
    }
    S.stats.resolve_steps += k - k0 + (k < n_end ? 1 : 0);
    S.stats.resolve_rechecks += rechecks;
    if (sh >= 0 && res != RES_PANIC) {  // entries before k are infeasible for the shape from now on
      shape_skip[sh] = k;
      skip_stamp[sh] = skip_gen;
    }
    if (res >= 0) return res;
    if (cnt_end & kbg::kCountIncompleteBit) return RES_TRUNC;
    *node = -1;
    return RES_OK;
  }
};

// NodeInfo.AddTask on the host mirror (node_info.go:101-129): Allocated ->
// Idle -= req; Pipelined -> Releasing -= req; both add a task.
void clear_mask_bit(Session& S, int32_t c, int32_t nd) {
  const uint32_t idx = (uint32_t)((size_t)c * S.W + (nd >> 6));
  const uint64_t bit = 1ull << (nd & 63);
  if (!(S.h_class_mask[idx] & bit)) return;
  S.h_class_mask[idx] &= ~bit;
  vc_mask_changed(S, c, nd);
  if (!S.mask_dirty_flag[idx]) {
    S.mask_dirty_flag[idx] = 1;
    S.mask_dirty.push_back(idx);
  }
}

// The bit of (c, n) from the static predicate, the port fit and the pod
// affinity counts (a nil-Node node stays reachable: SetNode panics first).
void refresh_mask_bit(Session& S, int32_t c, int32_t n) {
  const uint32_t idx = (uint32_t)((size_t)c * S.W + (n >> 6));
  const uint64_t bit = 1ull << (n & 63);
  bool v = (S.h_class_mask_static[idx] & bit) != 0;
  if (v && !S.panic_node[n]) {
    for (int32_t w = 0; w < S.PW && v; ++w)
      v = (S.node_ports[(size_t)n * S.PW + w] & S.cls_conf[(size_t)c * S.PW + w]) == 0;
    if (v && S.has_aff) v = kbg::aff_ok_node(S, c, n);
  }
  if (v == ((S.h_class_mask[idx] & bit) != 0)) return;
  S.h_class_mask[idx] ^= bit;
  vc_mask_changed(S, c, n);
  if (!S.mask_dirty_flag[idx]) {
    S.mask_dirty_flag[idx] = 1;
    S.mask_dirty.push_back(idx);
  }
}

// The pod joins node.Pods(), so its ports join the node's HostPortInfo
// (vendor cache/node_info.go:593-605): every class that conflicts with a newly
// used (ip, protocol, port) loses the node.
void add_ports(Session& S, int32_t c, int32_t nd) {
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  const uint64_t* add = &S.cls_add[(size_t)c * S.PW];
  for (int32_t w = 0; w < S.PW; ++w) {
    for (uint64_t b = add[w]; b; b &= b - 1)  // holders, for a statement discard (remove_ports)
      S.port_hold[((int64_t)nd << 32) | (uint32_t)(w * 64 + __builtin_ctzll(b))]++;
    uint64_t nb = add[w] & ~np[w];
    np[w] |= nb;
    while (nb) {
      const int32_t a = w * 64 + __builtin_ctzll(nb);
      nb &= nb - 1;
      for (int32_t c2 : S.atom_cls[a]) clear_mask_bit(S, c2, nd);
    }
  }
}

// The pod leaves node.Pods() (statement.go:156-192 unpipeline ->
// NodeInfo.RemoveTask): an atom no other pod holds — and that no pod held at
// open — is free again, and the classes it blocked get the node back where
// nothing else forbids it.
int32_t open_ports_left(const Session& S, int32_t nd, int32_t a) {  // entries of open pods still on the node
  const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
  auto o = S.port_open.find(k);
  if (o == S.port_open.end()) return 0;
  auto g = S.port_gone.find(k);
  return o->second - (g == S.port_gone.end() ? 0 : g->second);
}
void remove_ports(Session& S, int32_t c, int32_t nd) {
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  const uint64_t* add = &S.cls_add[(size_t)c * S.PW];
  for (int32_t w = 0; w < S.PW; ++w)
    for (uint64_t b = add[w]; b; b &= b - 1) {
      const int32_t a = w * 64 + __builtin_ctzll(b);
      auto it = S.port_hold.find(((int64_t)nd << 32) | (uint32_t)a);
      if (it == S.port_hold.end() || --it->second > 0) continue;
      S.port_hold.erase(it);
      const uint64_t bit = 1ull << (a & 63);
      if (open_ports_left(S, nd, a) > 0) continue;  // a pod on the node at open still holds it
      np[w] &= ~bit;
      for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
    }
}

// The port atom of one of a pod's host-port entries (-1: no atom; every port
// a pod on a node uses is one).
int32_t port_atom(const Session& S, const kbg_host_port& hp) {
  if (hp.host_port <= 0) return -1;
  const std::string ip = S.strs[hp.host_ip].empty() ? std::string("0.0.0.0") : S.strs[hp.host_ip];
  const std::string pr = S.strs[hp.protocol].empty() ? std::string("TCP") : S.strs[hp.protocol];
  auto ai = S.atom_of.find(ip + "|" + pr + "|" + std::to_string(hp.host_port));
  return ai == S.atom_of.end() ? -1 : ai->second;
}

// A pod that was on the node at open leaves node.Pods() (a statement
// discard's RemoveTask by key of the pod holding the key): each of its port
// entries goes; an atom no pod holds any more is free again.
void release_open_ports(Session& S, int32_t nd, const kbg_host_port* ports, int32_t n) {
  if (!S.has_ports) return;
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  for (int32_t i = 0; i < n; ++i) {
    const int32_t a = port_atom(S, ports[i]);
    if (a < 0) continue;
    const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
    S.port_gone[k]++;
    if (open_ports_left(S, nd, a) > 0 || S.port_hold.count(k)) continue;
    const uint64_t bit = 1ull << (a & 63);
    if (!(np[a / 64] & bit)) continue;
    np[a / 64] &= ~bit;
    for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
  }
}

// The reverse: a discarded statement's unevict adds that pod back to the node
// (statement.go:81-108 node.AddTask), so it is in node.Pods() again and its
// port entries are used again (vendor cache/node_info.go:593-605): every class
// one of them conflicts with loses the node.
void restore_open_ports(Session& S, int32_t nd, const kbg_host_port* ports, int32_t n) {
  if (!S.has_ports) return;
  uint64_t* np = &S.node_ports[(size_t)nd * S.PW];
  for (int32_t i = 0; i < n; ++i) {
    const int32_t a = port_atom(S, ports[i]);
    if (a < 0) continue;
    const int64_t k = ((int64_t)nd << 32) | (uint32_t)a;
    auto g = S.port_gone.find(k);
    if (g != S.port_gone.end() && --g->second <= 0) S.port_gone.erase(g);
    const uint64_t bit = 1ull << (a & 63);
    if (np[a / 64] & bit) continue;
    np[a / 64] |= bit;
    for (int32_t c2 : S.atom_cls[a]) refresh_mask_bit(S, c2, nd);
  }
}

// NodeInfo.Tasks already holds the task's PodKey (node_info.go:101-106)
inline int64_t node_key_of(const Session& S, int32_t t, int32_t nd) {
  return ((int64_t)nd << 32) | (uint32_t)S.task_key[t];
}
bool node_has_key(const Session& S, int32_t t, int32_t nd) {
  return S.has_dupkeys && S.key_hot[S.task_key[t]] && S.node_keys.count(node_key_of(S, t, nd)) != 0;
}

// Returns true when the node already held the task's pod key: the decision
// stands, the node is unchanged (AddTask's error), the pod is not among
// node.Pods() (ports), but it is an Allocated pod of its job (the podLister).
bool mirror_add(Session& S, int32_t t, int32_t nd, int32_t kind) {
  const bool dup = node_has_key(S, t, nd);
  if (!dup) {
    if (!S.nil_node[nd]) {
      if (kind == KBG_KIND_ALLOCATE) kbg::res_sub(S.idle[nd], S.treq[t]);
      else kbg::res_sub(S.rel[nd], S.treq[t]);
    }
    S.ntasks[nd]++;
    if (S.has_ports) add_ports(S, S.task_class[t], nd);
    if (S.has_dupkeys && S.key_hot[S.task_key[t]]) {
      S.node_keys.insert(node_key_of(S, t, nd));
      S.key_holder[node_key_of(S, t, nd)] = t << 1 | (kind != KBG_KIND_ALLOCATE);
    }
  }
  // an Allocated pod joins the podLister (api/helpers.go:63-70); Pipelined does not
  if (S.has_aff && kind == KBG_KIND_ALLOCATE) {
    static const bool prof = getenv("KBG_PROFILE_AFF") != nullptr;
    const uint64_t c0 = prof ? __builtin_readcyclecounter() : 0;
    kbg::aff_place(S, t, nd, +1, S.affm->st, true);
    if (prof) {
      S.affm->prof_cycles += __builtin_readcyclecounter() - c0;
      S.affm->prof_calls++;
    }
  }
  return dup;
}

// Which pod keys can collide: a candidate task's key that another candidate
// shares or that some node already holds (a StatefulSet pod recreated while
// its predecessor is still on a node). Usually none: then nothing is tracked.
// Kept as counts per canonical key — candidate (Pending) tasks holding it,
// node entries holding it — so an update adjusts the keys its events and
// touched tasks changed instead of rescanning every task and node.
void pod_key_refresh(Session& S, int32_t k) {
  const bool hot = S.kc_cand[k] >= 2 || (S.kc_cand[k] >= 1 && S.kc_node[k] >= 1);
  if (hot != (S.key_hot[k] != 0)) {
    S.n_hot += hot ? 1 : -1;
    S.key_hot[k] = hot ? 1 : 0;
  }
}
void setup_pod_keys(Session& S, bool incr = false, const std::vector<int32_t>* touched = nullptr,
                    const std::vector<uint8_t>* was = nullptr) {
  const size_t NS = S.strs.size();
  S.task_key.resize(S.n_tasks);
  if (!incr || S.kc_cand.empty()) {
    for (int32_t t = 0; t < S.n_tasks; ++t) S.task_key[t] = S.canon[S.tasks_in[t].pod_key];
    S.kc_cand.assign(NS, 0);
    S.kc_node.assign(NS, 0);
    S.key_hot.assign(NS, 0);
    S.n_hot = 0;
    for (int32_t t = 0; t < S.n_tasks; ++t)
      if (S.pending_candidate[t] || S.be_task[t]) S.kc_cand[S.task_key[t]]++;  // (false for removed tasks)
    for (int32_t n = 0; n < S.n_nodes; ++n)
      for (int32_t k : S.node_key_order[n]) S.kc_node[k]++;
    for (size_t k = 0; k < NS; ++k) pod_key_refresh(S, (int32_t)k);
  } else {
    S.kc_cand.resize(NS, 0);
    if (S.kc_node.size() < NS) S.kc_node.resize(NS, 0);
    S.key_hot.resize(NS, 0);
    for (size_t i = 0; i < touched->size(); ++i) {
      const int32_t t = (*touched)[i];
      const int32_t k = S.task_key[t] = S.canon[S.tasks_in[t].pod_key];
      const bool was_c = ((*was)[i] & 3) != 0, now_c = S.pending_candidate[t] || S.be_task[t];
      if (was_c == now_c) continue;
      S.kc_cand[k] += now_c ? 1 : -1;
      pod_key_refresh(S, k);
    }
    for (int32_t k : S.upd_keys) pod_key_refresh(S, k);  // node entries added / removed by the events
  }
  S.upd_keys.clear();
  S.has_dupkeys = S.n_hot > 0;
  S.node_keys.clear();
  if (S.has_dupkeys)
    for (int32_t n = 0; n < S.n_nodes; ++n)
      for (int32_t k : S.node_key_order[n])
        if (S.key_hot[k]) S.node_keys.insert(((int64_t)n << 32) | (uint32_t)k);
  S.node_keys0 = S.node_keys;
}

// Builds the port-atom dictionary (distinct sanitized (ip, protocol, port)
// with port > 0 over the nodes' used ports and the candidate classes' wanted
// ports), each class's conflict set (host_ports.go CheckConflict: same
// protocol and port, and either side 0.0.0.0 or the same ip) and folds the
// nodes' current conflicts into the class masks.
void setup_host_ports(Session& S) {
  S.has_ports = false;
  if (!S.pred_active) return;
  const int32_t C = (int32_t)S.class_spec.size();
  auto ip_of = [&](int32_t id) { return S.strs[id].empty() ? std::string("0.0.0.0") : S.strs[id]; };
  auto proto_of = [&](int32_t id) { return S.strs[id].empty() ? std::string("TCP") : S.strs[id]; };
  typedef std::tuple<std::string, std::string, int32_t> Atom;
  std::map<Atom, int32_t> atoms;
  std::vector<Atom> atom_list;
  auto atom = [&](const kbg_host_port& hp) {
    Atom a{ip_of(hp.host_ip), proto_of(hp.protocol), hp.host_port};
    auto it = atoms.find(a);
    if (it != atoms.end()) return it->second;
    const int32_t id = (int32_t)atom_list.size();
    atoms.emplace(a, id);
    atom_list.push_back(a);
    return id;
  };
  std::vector<std::vector<int32_t>> want(C);
  bool any = false;
  // only classes some candidate task uses (a resident session keeps classes
  // whose tasks have left; they must not switch the port machinery on)
  std::vector<uint8_t> in_use(C, 0);
  for (int32_t t = 0; t < S.n_tasks; ++t)
    if (S.pending_candidate[t] || S.be_task[t]) in_use[S.task_class[t]] = 1;
  for (int32_t c = 0; c < C; ++c) {
    const int32_t sp = S.class_spec[c];
    if (sp < 0 || !in_use[c]) continue;
    const kbg_spec& spec = S.specs_in[sp];
    for (int32_t i = 0; i < spec.port_len; ++i) {
      const kbg_host_port& hp = S.ports_in[spec.port_off + i];
      if (hp.host_port <= 0) continue;
      want[c].push_back(atom(hp));
      any = true;
    }
  }
  if (!any) return;
  std::vector<std::vector<int32_t>> used(S.n_nodes);
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    const kbg_node& nd = S.nodes_in[n];
    for (int32_t i = 0; i < nd.port_len; ++i) {
      const kbg_host_port& hp = S.ports_in[nd.port_off + i];
      if (hp.host_port > 0) used[n].push_back(atom(hp));
    }
  }
  S.has_ports = true;
  const int32_t A = (int32_t)atom_list.size();
  S.PW = (A + 63) / 64;
  S.cls_conf.assign((size_t)C * S.PW, 0);
  S.cls_add.assign((size_t)C * S.PW, 0);
  S.atom_cls.assign(A, {});
  for (int32_t c = 0; c < C; ++c)
    for (int32_t w : want[c]) {
      S.cls_add[(size_t)c * S.PW + w / 64] |= 1ull << (w % 64);
      const Atom& wa = atom_list[w];
      for (int32_t a = 0; a < A; ++a) {
        const Atom& ea = atom_list[a];
        if (std::get<1>(ea) != std::get<1>(wa) || std::get<2>(ea) != std::get<2>(wa)) continue;
        if (std::get<0>(wa) == "0.0.0.0" || std::get<0>(ea) == "0.0.0.0" || std::get<0>(ea) == std::get<0>(wa))
          S.cls_conf[(size_t)c * S.PW + a / 64] |= 1ull << (a % 64);
      }
    }
  for (int32_t c = 0; c < C; ++c)
    for (int32_t a = 0; a < A; ++a)
      if ((S.cls_conf[(size_t)c * S.PW + a / 64] >> (a % 64)) & 1ull) S.atom_cls[a].push_back(c);
  S.atom_of.clear();
  for (int32_t a = 0; a < A; ++a)
    S.atom_of[std::get<0>(atom_list[a]) + "|" + std::get<1>(atom_list[a]) + "|" + std::to_string(std::get<2>(atom_list[a]))] = a;
  S.port_open.clear();  // one entry per pod and port: how many pods at open use each atom
  for (int32_t n = 0; n < S.n_nodes; ++n)
    for (int32_t a : used[n]) S.port_open[((int64_t)n << 32) | (uint32_t)a]++;
  S.node_ports.assign((size_t)S.n_nodes * S.PW, 0);
  S.mask_dirty_flag.assign(S.h_class_mask.size(), 0);
  S.mask_dirty.clear();
  for (int32_t n = 0; n < S.n_nodes; ++n) {
    for (int32_t a : used[n]) S.node_ports[(size_t)n * S.PW + a / 64] |= 1ull << (a % 64);
    if (S.panic_node[n]) continue;  // SetNode(nil) panics before any check: keep the node reachable
    for (int32_t c = 0; c < C; ++c) {
      bool conflict = false;
      for (int32_t w = 0; w < S.PW && !conflict; ++w)
        conflict = (S.node_ports[(size_t)n * S.PW + w] & S.cls_conf[(size_t)c * S.PW + w]) != 0;
      if (conflict) S.h_class_mask[(size_t)c * S.W + (n >> 6)] &= ~(1ull << (n & 63));
    }
  }
  S.node_ports0 = S.node_ports;
}
kbg_status validate(const kbg_snapshot* s) {
  if (!s) return fail(KBG_E_INVALID, "null snapshot");
  auto in = [](int32_t v, int32_t n) { return v >= 0 && v < n; };
  auto range = [](int32_t off, int32_t len, int32_t n) { return off >= 0 && len >= 0 && (int64_t)off + len <= n; };
  if (s->n_strings < 0 || (s->n_strings > 0 && !s->strings)) return fail(KBG_E_INVALID, "strings");
  {  // every count non-negative, every non-empty array present (encode must never emit an unreadable blob)
    const std::pair<const void*, int32_t> arrays[] = {
        {s->nodes, s->n_nodes},         {s->jobs, s->n_jobs},           {s->queues, s->n_queues},
        {s->tasks, s->n_tasks},         {s->others, s->n_others},       {s->specs, s->n_specs},
        {s->terms, s->n_terms},         {s->reqs, s->n_reqs},           {s->values, s->n_values},
        {s->tolerations, s->n_tolerations}, {s->labels, s->n_labels},   {s->taints, s->n_taints},
        {s->selectors, s->n_selectors}, {s->plugins, s->n_plugins},     {s->tier_sizes, s->n_tiers},
        {s->ports, s->n_ports},         {s->node_tasks, s->n_node_tasks}, {s->pod_terms, s->n_pod_terms},
        {s->pod_labels, s->n_pod_labels}, {s->node_pod_keys, s->n_node_pod_keys}, {s->node_pods, s->n_node_pods}};
    for (const auto& a : arrays)
      if (a.second < 0 || (a.second > 0 && !a.first)) return fail(KBG_E_INVALID, "negative count or null array");
  }
  for (int32_t i = 0; i < s->n_strings; ++i)
    if (!s->strings[i]) return fail(KBG_E_INVALID, "null string " + std::to_string(i));
  const int32_t NS = s->n_strings;
  for (int32_t i = 0; i < s->n_nodes; ++i) {
    const kbg_node& n = s->nodes[i];
    if (!in(n.name, NS) || !range(n.label_off, n.label_len, s->n_labels) || !range(n.taint_off, n.taint_len, s->n_taints) ||
        !range(n.port_off, n.port_len, s->n_ports))
      return fail(KBG_E_INVALID, "node " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_labels * 2; ++i)
    if (!in(s->labels[i], NS)) return fail(KBG_E_INVALID, "label string");
  for (int32_t i = 0; i < s->n_selectors * 2; ++i)
    if (!in(s->selectors[i], NS)) return fail(KBG_E_INVALID, "selector string");
  for (int32_t i = 0; i < s->n_taints; ++i) {
    const kbg_taint& t = s->taints[i];
    if (!in(t.key, NS) || !in(t.value, NS) || !in(t.effect, NS)) return fail(KBG_E_INVALID, "taint");
  }
  for (int32_t i = 0; i < s->n_queues; ++i)
    if (!in(s->queues[i].uid, NS)) return fail(KBG_E_INVALID, "queue");
  for (int32_t i = 0; i < s->n_jobs; ++i)
    if (!in(s->jobs[i].uid, NS) || !in(s->jobs[i].queue, s->n_queues)) return fail(KBG_E_INVALID, "job " + std::to_string(i));
  for (int32_t i = 0; i < s->n_tasks; ++i) {
    const kbg_task& t = s->tasks[i];
    if (!in(t.uid, NS) || !in(t.job, s->n_jobs) || !(t.spec == -1 || in(t.spec, s->n_specs)) || !in(t.node_name, NS) ||
        !in(t.pod_key, NS))
      return fail(KBG_E_INVALID, "task " + std::to_string(i));
    if (t.status <= 0 || t.status > KBG_UNKNOWN || (t.status & (t.status - 1))) return fail(KBG_E_INVALID, "task status");
  }
  if (s->n_pod_terms < 0 || (s->n_pod_terms > 0 && !s->pod_terms)) return fail(KBG_E_INVALID, "pod_terms");
  if (s->n_pod_labels < 0 || (s->n_pod_labels > 0 && !s->pod_labels)) return fail(KBG_E_INVALID, "pod_labels");
  for (int32_t i = 0; i < s->n_specs; ++i) {
    const kbg_spec& p = s->specs[i];
    if (!range(p.selector_off, p.selector_len, s->n_selectors) || !range(p.term_off, p.term_len, s->n_terms) ||
        !range(p.toleration_off, p.toleration_len, s->n_tolerations) || !range(p.port_off, p.port_len, s->n_ports) ||
        !in(p.ns, NS) || !range(p.pod_label_off, p.pod_label_len, s->n_pod_labels) ||
        !range(p.aff_off, p.aff_len, s->n_pod_terms) || !range(p.anti_off, p.anti_len, s->n_pod_terms))
      return fail(KBG_E_INVALID, "spec " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_pod_labels * 2; ++i)
    if (!in(s->pod_labels[i], NS)) return fail(KBG_E_INVALID, "pod label string");
  for (int32_t i = 0; i < s->n_pod_terms; ++i) {
    const kbg_pod_term& t = s->pod_terms[i];
    if (!range(t.match_off, t.match_len, s->n_selectors) || !range(t.expr_off, t.expr_len, s->n_reqs) ||
        !range(t.ns_off, t.ns_len, s->n_values) || !in(t.topology_key, NS))
      return fail(KBG_E_INVALID, "pod term " + std::to_string(i));
  }
  for (int32_t i = 0; i < s->n_terms; ++i) {
    const kbg_term& t = s->terms[i];
    if (!range(t.expr_off, t.expr_len, s->n_reqs) || !range(t.field_off, t.field_len, s->n_reqs))
      return fail(KBG_E_INVALID, "term");
  }
  for (int32_t i = 0; i < s->n_reqs; ++i) {
    const kbg_requirement& r = s->reqs[i];
    if (!in(r.key, NS) || !in(r.op, NS) || !range(r.value_off, r.value_len, s->n_values)) return fail(KBG_E_INVALID, "req");
  }
  for (int32_t i = 0; i < s->n_values; ++i)
    if (!in(s->values[i], NS)) return fail(KBG_E_INVALID, "value");
  if (s->n_ports < 0 || (s->n_ports > 0 && !s->ports)) return fail(KBG_E_INVALID, "ports");
  if (s->n_node_tasks < 0 || (s->n_node_tasks > 0 && !s->node_tasks)) return fail(KBG_E_INVALID, "node_tasks");
  for (int32_t i = 0; i < s->n_nodes; ++i)
    if (!range(s->nodes[i].task_off, s->nodes[i].task_len, s->n_node_tasks))
      return fail(KBG_E_INVALID, "node task list " + std::to_string(i));
  for (int32_t i = 0; i < s->n_node_tasks; ++i)
    if (!in(s->node_tasks[i], s->n_tasks)) return fail(KBG_E_INVALID, "node task index");
  for (int32_t i = 0; i < s->n_nodes; ++i) {  // NodeInfo.Tasks keys: one per pod on the node
    const kbg_node& n = s->nodes[i];
    if (!range(n.key_off, n.key_len, s->n_node_pod_keys) || n.key_len != n.num_tasks)
      return fail(KBG_E_INVALID, "node pod keys " + std::to_string(i) + " (key_len must equal num_tasks)");
  }
  for (int32_t i = 0; i < s->n_node_pod_keys; ++i)
    if (!in(s->node_pod_keys[i], NS)) return fail(KBG_E_INVALID, "node pod key string");
  if (s->n_node_pods != 0 && s->n_node_pods != s->n_node_pod_keys)
    return fail(KBG_E_INVALID, "node_pods: none or one per node_pod_keys entry");
  for (int32_t i = 0; i < s->n_nodes && s->n_node_pods; ++i) {  // each pod's ports: the node's, in order
    const kbg_node& n = s->nodes[i];
    int64_t pl = 0;
    for (int32_t k = 0; k < n.key_len; ++k) {
      const kbg_node_pod& q = s->node_pods[n.key_off + k];
      if (q.port_len < 0 || q.status <= 0 || q.status > KBG_UNKNOWN || (q.status & (q.status - 1)))
        return fail(KBG_E_INVALID, "node pod " + std::to_string(n.key_off + k));
      pl += q.port_len;
    }
    if (pl != n.port_len) return fail(KBG_E_INVALID, "node " + std::to_string(i) + ": node_pods port_len sum != port_len");
  }
  for (int32_t i = 0; i < s->n_ports; ++i)
    if (!in(s->ports[i].host_ip, NS) || !in(s->ports[i].protocol, NS)) return fail(KBG_E_INVALID, "port");
  for (int32_t i = 0; i < s->n_tolerations; ++i) {
    const kbg_toleration& t = s->tolerations[i];
    if (!in(t.key, NS) || !in(t.op, NS) || !in(t.value, NS) || !in(t.effect, NS)) return fail(KBG_E_INVALID, "toleration");
  }
  int32_t np = 0;
  for (int32_t i = 0; i < s->n_tiers; ++i) {
    if (s->tier_sizes[i] < 0) return fail(KBG_E_INVALID, "tier size");
    np += s->tier_sizes[i];
  }
  if (np != s->n_plugins) return fail(KBG_E_INVALID, "tier sizes do not sum to n_plugins");
  for (int32_t i = 0; i < s->n_plugins; ++i)
    if (!in(s->plugins[i].name, NS)) return fail(KBG_E_INVALID, "plugin name");
  return KBG_OK;
}

template <class T>
std::vector<T> copy_arr(const T* p, int32_t n) {
  return (p && n > 0) ? std::vector<T>(p, p + n) : std::vector<T>();
}

constexpr int64_t kRankGap = int64_t(1) << 20;  // task_rank spacing at open (kbg_session.hpp)

std::vector<int32_t> ranks_of(const Session& S, const std::vector<int32_t>& ids) {
  std::vector<int32_t> idx(ids.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return S.strs[ids[a]] < S.strs[ids[b]]; });
  std::vector<int32_t> rank(ids.size());
  int32_t r = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    if (i > 0 && S.strs[ids[idx[i]]] != S.strs[ids[idx[i - 1]]]) ++r;
    rank[idx[i]] = r;
  }
  return rank;
}
