// Device-side data layout and kernel launchers of the MI355X allocate path.
//
// Node table (HBM, struct-of-arrays, one entry per ssn.Nodes position):
//   idle_{cpu,mem,gpu}, rel_{cpu,mem,gpu}  f64[N]   NodeInfo.Idle / .Releasing
//   ntasks, maxtasks                       i32[N]   len(NodeInfo.Tasks), Allocatable.MaxTaskNum
// 56 B of dynamic state per node; the static part of the predicate
// (selector/affinity, taints, unschedulable) is resolved once per session into
// class_mask[class][word] (1 bit per node) by kbg_build_class_mask.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kbg {

// resource_info.go:54-56 LessEqual tolerances
constexpr double kMinMilliCPU = 10.0;
constexpr double kMinMemory = 10.0 * 1024.0 * 1024.0;
constexpr double kMinMilliGPU = 10.0;

// select kernel result encoding
constexpr uint32_t kCandPipelineBit = 0x80000000u;  // candidate fits Releasing only
constexpr uint32_t kCountIncompleteBit = 0x40000000u;
constexpr uint32_t kCountMask = 0x3fffffffu;

struct NodeSoA {
  double* idle_cpu;
  double* idle_mem;
  double* idle_gpu;
  double* rel_cpu;
  double* rel_mem;
  double* rel_gpu;
  int32_t* ntasks;
  int32_t* maxtasks;
};

// One task evaluation request (32 B, SURVEY §8(d) task record).
// General mode: req = Resreq and the kernel evaluates LessEqual with the
// reference's expression `r < a || |a - r| < min` per dimension.
// Integer mode (the session proved every node value and request an exact
// integer of magnitude <= 2^51, with the pending requests' sum <= 2^51 so the
// values stay exact integers for the whole cycle): req = Resreq - min, and
// `r <= a` is exactly `a > req`: if r < a then a > r - min; if |a - r| < min
// then a - r > -min; conversely a > r - min gives r < a or r - min < a <= r,
// i.e. |a - r| < min — every operation exact on such integers.
struct TaskRec {
  double req[3];
  int32_t cls;
  int32_t flags;  // kRowRelZeroFits: LessEqual(Resreq, 0) (the Releasing fit on a zero-Releasing node)
};
constexpr int32_t kRowRelZeroFits = 1;

// Scan rows per workgroup (one per lane for the write-out). The host pads
// every batch's rows to a multiple of this with copies of a real row, so the
// kernel's row loop has no bound checks (kbg_pad_rows).
constexpr int kScanRowsPerBlock = 64;
inline int32_t kbg_pad_rows(int32_t g) { return (g + kScanRowsPerBlock - 1) / kScanRowsPerBlock * kScanRowsPerBlock; }

// Node row written back after the host commits placements (AddTask delta).
struct NodeDelta {
  int32_t node;
  int32_t ntasks;
  double idle[3];
  double rel[3];
  int32_t maxtasks;  // Allocatable pods (changes only through a session update)
  int32_t pad;
};

// One class-mask word rewritten by the host (host-port conflicts).
struct MaskDelta {
  uint32_t index;
  uint32_t pad;
  uint64_t value;
};
constexpr int32_t kMaskDeltaCap = 8192;

// ---- preempt / reclaim victim scan (preempt.go:182-240, reclaim.go:106-135)
enum VictimPlugin : int32_t { VP_GANG = 1, VP_DRF = 2, VP_PROP = 4 };
enum VictimMode : int32_t { VM_PREEMPT_JOBS = 0, VM_PREEMPT_TASKS = 1, VM_RECLAIM = 2 };
constexpr int kMaxVictimTiers = 8;
constexpr int kVictimChunks = 16;                      // 64-candidate chunks per node in one victim scan
constexpr int kMaxNodeCandidates = 64 * kVictimChunks;  // victim candidates per node

// One reclaimer / preemptor against every node.
struct VictimScan {
  int32_t n_nodes, W, cls, cap_check;  // n_nodes: global N
  int32_t node_lo, node_n;             // node range this launch covers (the shard's node table, tab_lo based)
  int32_t mode;                        // VictimMode
  int32_t n_tiers;                     // tiers holding an enabled victim fn, in order
  int32_t tier_fns[kMaxVictimTiers];   // VictimPlugin bits of each (every fn keeps the preemptee order,
                                       // so the intersection does not depend on the fns' order)
  int32_t job, queue;                  // the preemptor's
  double req[3];                       // its Resreq
  double ls;                           // drf: its job's share with it placed
};

struct VictimTables {
  const int32_t* ntasks;        // node table rows (node - VictimScan.node_lo)
  const int32_t* maxtasks;
  const uint8_t* panic_node;    // nil Node under an active predicates plugin
  const uint64_t* class_mask;
  const int32_t* nt_off;        // [N+1] candidate lists: session tasks Running on the node at open,
                                //       in NodeInfo.Tasks order; position p = nt_off[n] + k
  const int2* c_jq;             // [P] {job, queue} of the candidate at position p (coalesced per lane)
  const double* c_req;          // [P][3] its Resreq
  uint8_t* c_run;               // [P] node-side status still Running
  const int32_t* j_queue;       // per job
  const int32_t* j_min;
  int32_t* j_ready;             // gang readyTaskNum
  double* j_alloc;              // [J][3] drf attr.allocated
  double* q_alloc;              // [Q][3] proportion attr.allocated
  const double* q_deserved;     // [Q][3]
  double drf_total[3];
};

// A host-side change to the victim tables.
struct StateDelta {
  int32_t kind;   // 0 candidate running flag (index = candidate position), 1 job ready, 2 job drf alloc, 3 queue alloc
  int32_t index;
  double v[3];
};

// ---- static predicate programs (built on host, evaluated on device) ----
enum ReqKind : int32_t {
  REQ_FALSE = 0,
  REQ_TRUE = 1,
  REQ_ALL = 2,      // (label_bits & mask) == mask
  REQ_ANY = 3,      // (label_bits & mask) != 0
  REQ_NONE = 4,     // (label_bits & mask) == 0
  REQ_GT = 5,       // numeric label column > value
  REQ_LT = 6,       // numeric label column < value
  REQ_NAME_EQ = 7,  // node name id == value
  REQ_NAME_NE = 8,  // node name id != value
};

struct ReqProg {
  int32_t kind;
  int32_t mask_off;  // offset (in u64 words) into the mask pool, label_words wide
  int32_t col;       // numeric column for GT/LT
  int32_t pad;
  int64_t value;
};

struct TermProg {
  int32_t req_off, req_len;  // AND of reqs; a skipped term is not emitted
};

struct ClassProg {
  int32_t sel_req;           // index of the nodeSelector requirement, -1 = none
  int32_t has_affinity;      // required node affinity present: OR over terms
  int32_t term_off, term_len;
  int32_t tol_off;           // offset into the tolerated-mask pool (taint_words wide)
  int32_t always;            // 1 = predicate always true for this class (predicates inactive)
};

struct StaticTables {
  int32_t n_nodes;
  int32_t label_words;       // u64 words per node label bitset
  int32_t taint_words;       // u64 words per node taint bitset
  int32_t n_numcols;
  const uint64_t* label_bits;    // [label_words][N]  (word-major => coalesced)
  const uint64_t* taint_bits;    // [taint_words][N]
  const int64_t* num_vals;       // [n_numcols][N]
  const uint8_t* num_ok;         // [n_numcols][N]
  const int32_t* name_id;        // [N]
  const uint8_t* node_flags;     // [N] bit0 = unschedulable, bit1 = nil Node, bit2 = ghost-failed
  const uint64_t* mask_pool;
  const uint64_t* tol_pool;
  const ReqProg* reqs;
  const TermProg* terms;
  const ClassProg* classes;
};

enum NodeFlag : uint8_t { NF_UNSCHED = 1, NF_NIL = 2, NF_DEAD = 4 };

// ---- launchers (all asynchronous on `stream`) ----
hipError_t launch_build_class_mask(const StaticTables& t, int32_t n_classes, int32_t W, uint64_t* class_mask,
                                   hipStream_t stream);

// Words a row takes in one shard slot of the feasibility bitmaps: Wl rounded
// up to whole quads (a quad = the 4 words one scan workgroup produces).
__host__ __device__ inline int32_t kbg_slot_words(int32_t Wl) { return (Wl + 3) & ~3; }

// Feasibility bitmaps of a batch of G evaluation rows live in one buffer laid
// out [slot][plane][quad][row][4] (u64 words; plane 0 = Idle-or-Releasing
// fit, plane 1 = Idle fit; slot = node-axis shard of Wl 64-node words, quad
// = 4 consecutive words of it, kbg_slot_words(Wl) / 4 quads per row). A scan
// workgroup writes its rows' quad as one contiguous run, so no cache line is
// shared between workgroups (or XCDs). Unsharded, slot count 1 and Wl = W.
// Sharded, the per-shard slots are exactly an all-gather's receive layout, so
// the select kernel reads the same buffer whether the slots were written
// locally or gathered over RCCL.

struct ScanGeom {
  int32_t n_nodes;   // global node count N
  int32_t W;         // global 64-node words, ceil(N/64)
  int32_t Wl;        // words per shard slot
  int32_t chunk_lo;  // first global word this launch covers
  int32_t n_chunks;  // words this launch covers (Wl for one shard; slots*Wl for all local shards)
  int32_t tab_lo;    // first global node held by the node table (rows are node - tab_lo)
};

// `start`/`stop` (optional) are stamped at the kernel's own start and end
// (hipExtLaunchKernelGGL), so their elapsed time is the kernel duration.
// `out` points at the slot of chunk_lo.
hipError_t launch_scan(const NodeSoA& n, const ScanGeom& g, const uint64_t* class_mask, const TaskRec* tasks,
                       int32_t n_tasks, int32_t cap_check, int32_t int_mode, uint64_t* out, hipStream_t stream,
                       hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

// The fused scan + first-fit extraction (kbg_firstfit_kernel). Rows map to
// shapes: row g evaluates shape s = row_shape[g] & ~kRowWriter (grouped mode:
// row_shape null, s = g, every row a writer). A shape is a TaskRec whose
// flags carry kRowRelZeroFits and, from bit kRowWantShift, `want`: how many
// fits its list must hold before the walk may stop (EARLY_EXIT) and the
// output may end. The writer row of shape s writes, for the words [w_lo,
// w_lo + covered) in node order, the pair of 64-node masks {fits Idle or
// Releasing, fits Idle} (static predicate, pod cap and LessEqual applied)
// into masks[s * mw + (w - mask_w0)], and info[s * info_stride + part0 + part] = covered |
// kInfoAnyBit (some node of the part's walked words fits) |
// kCountIncompleteBit (covered < the part's words: the list is cut after the
// word holding its want-th fit; never with `complete`). Every fit of
// a covered word is in the masks, so the host reads the first-fit candidates
// in node order by scanning bits. The shape table is in the kernel arguments
// (n_shapes <= kInlineShapes: no PCIe read at launch) or host-mapped;
// row_shape, info, masks, avail may be host-mapped (zero-copy).
constexpr int kInlineShapes = 96;
constexpr int kFfRoundWords = 128;  // words per round of the fused walk (one round: no early exit)
constexpr int kFfMaxSplits = 8;
constexpr uint32_t kRowWriter = 0x80000000u;
constexpr int kRowWantShift = 1;
constexpr uint32_t kInfoAnyBit = 0x20000000u;
constexpr uint32_t kInfoWordsMask = 0x00ffffffu;
struct alignas(16) MaskPair {
  uint64_t f;  // fits Idle or Releasing
  uint64_t i;  // fits Idle
};
struct FirstFitArgs {
  const double* nodes;          // the node table as one block (NodeSoA of alloc_soa): rows of the nodes
                                // [tab_lo, tab_lo + tab_n), idle c/m/g, rel c/m/g f64[stride], ntasks,
                                // maxtasks i32[stride]
  const uint64_t* class_mask;   // [class][W]
  const TaskRec* shapes;        // host-mapped shape table, or null: inl[]
  const uint32_t* row_shape;    // [G] shape | kRowWriter, or null: row g is shape g and writes it
  uint32_t* info;               // [n_shapes]
  MaskPair* masks;              // [n_shapes][mw]
  uint32_t* avail;              // owner-resolve: [n_shapes] avail_bit when any node fits, else 0
  uint32_t avail_bit;
  int32_t stride, G, n_shapes, mw;
  int32_t n_nodes, W, w_lo, w_hi, tab_lo, tab_n;
  int32_t cap_check;            // the predicates plugin's pod cap is on
  int32_t early_exit;           // stop once every row's list is full (production mode)
  int32_t complete;             // every word's masks go out (want ignored): lists are never cut
  int32_t splits, split_words;  // the words [w_lo, w_hi) in `splits` parts of split_words, one workgroup
                                // each (a short batch's walk spread over more CUs); info is per (shape, part)
  int32_t rows;                 // rows per workgroup (firstfit_geometry; at most the kernel's ROWS)
  int32_t info_stride, part0;   // info[s * info_stride + part0 + part] (a single launch: splits, 0; a rank of
                                // the scan service: every rank's parts, this rank's first)
  int32_t mask_w0;              // the global word masks[s * mw] holds (w_lo; 0 under the scan service)
  int32_t runs;                 // full-scan with inline shapes: launch row l belongs to the slot s with
                                // run_end[s - 1] <= l < run_end[s] and the run's last row writes the slot
                                // (no row -> shape map to read: rows of a slot are identical evaluations)
  TaskRec inl[kInlineShapes];
  uint16_t run_end[kInlineShapes];
};
// Launch geometry of G rows: the kernel's rows-per-workgroup variant (16, 24
// or 32) and the rows each workgroup takes (<= that). Production (grouped)
// batches take whole 16/24/32-row blocks; full-scan batches spread their rows
// evenly over the 256 CUs (ceil(G / 256) rounded up to a pair), so a launch of
// 4.2k rows runs 17-18 rows on each CU instead of 24 on 174 of them.
struct FfGeometry {
  int32_t variant, rows;
};
FfGeometry firstfit_geometry(int32_t G, bool full_scan);
hipError_t launch_firstfit(const FirstFitArgs& a, int32_t int_mode, hipStream_t stream, hipEvent_t start = nullptr,
                           hipEvent_t stop = nullptr);


// Row g gets cap_off[g+1]-cap_off[g] candidate slots at out_cand[cap_off[g]],
// taken from the global words [w_lo, w_hi) in node order.
hipError_t launch_select(const uint64_t* bits, int32_t w_lo, int32_t w_hi, int32_t Wl, int32_t n_rows,
                         const uint32_t* cap_off, uint32_t* out_cand, uint32_t* out_count, hipStream_t stream,
                         hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

hipError_t launch_apply(const NodeSoA& n, const NodeDelta* deltas, int32_t n_deltas, hipStream_t stream);
// dst[0..n16) = src[0..n16), 16 B per lane (the node-table restore of kbg_session_reset)
hipError_t launch_copy16(void* dst, const void* src, size_t n16, hipStream_t stream);

// FitError counts of not-ready jobs (kbg_fitdelta_kernel).
struct FitQuery {
  int32_t cls, end, point, win;  // static class; nodes [0, end); decisions before `point` applied; the winner
  double req[3];                 // Resreq
};
struct FitArgs {
  const double* nodes;         // the final node table block (FirstFitArgs.nodes)
  int32_t stride, W;
  const uint64_t* class_mask;  // static predicate [class][W]
  const int32_t* hoff;         // [N + 1] each node's decisions
  const int32_t* hk;           // decision index | 0x80000000 for a Pipeline
  const double* hold;          // [3] per decision: the Idle (Allocate) / Releasing (Pipeline) before it
  const int32_t* na;           // per decision: the first Allocate at or after it on its node, -1 none
  const FitQuery* q;
  int32_t nq, cap_check;
  int32_t* out;                // [nq][4]: entries, negative cpu, memory, GPU deltas (host-mapped)
  int32_t tab_lo, tab_n;       // the global nodes the table holds (a shard of the scan service: its own)
};
hipError_t launch_fitdelta(const FitArgs& a, hipStream_t stream);
hipError_t launch_mask_apply(uint64_t* class_mask, const MaskDelta* deltas, int32_t n_deltas, hipStream_t stream);

// One victim scan evaluates every node of the range for one (preemptor,
// state) and writes two bitmaps of 32-node words, indexed by global node:
// stop[n] — the reference would stop at node n (validated victims, or a
// panic), panic[n] — that stop is a panic. The reference's answer is the
// lowest stop; the host keeps the maps and, as later tries of the same
// preemptor shape change the state, re-evaluates only the nodes those changes
// touched (kbg_session.cpp VictimCache). A workgroup (16 waves) covers 32
// consecutive nodes, two per wave, and writes its two words; sharded, each
// rank writes the words of its node range (64-node aligned) into zeroed
// arrays and an element-wise ncclAllReduce(max) of disjoint words is their OR.
constexpr int kVictimNodesPerBlock = 8;  // one node per wave; a workgroup writes one byte of stop bits
constexpr int kVictimBlockWaves = 8;
inline int32_t kbg_victim_words(int32_t n_nodes) { return (n_nodes + 31) / 32; }
hipError_t launch_victim_scan(const VictimScan& p, const VictimTables& t, uint32_t* stop_bits, uint32_t* panic_bits,
                              hipStream_t stream, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
// Nodes of the scanned range with more than 128 candidates (`rows`, table
// rows), evaluated after launch_victim_scan: ORed into its device words, or
// (row_out non-null) one byte per row, bit 0 stop and bit 1 panic.
hipError_t launch_victim_big(const VictimScan& p, const VictimTables& t, const int32_t* rows, int32_t n_rows,
                             uint32_t* stop_bits, uint32_t* panic_bits, uint8_t* row_out, hipStream_t stream);
// Host-side changes before a scan, read in place from host-mapped memory:
// node rows (NodeInfo.Tasks count / Idle / Releasing) and victim-table
// entries, in one launch.
hipError_t launch_victim_prep(const NodeSoA& n, const VictimTables& t, const NodeDelta* nd, int32_t n_nodes,
                              const StateDelta* sd, int32_t n_state, hipStream_t stream);
// The common case (a try evicted a few tasks) carried in the kernel arguments:
// no PCIe reads on the critical path.
constexpr int kArgNodeDeltas = 16;
constexpr int kArgStateDeltas = 48;
struct VictimPrepArgs {
  int32_t nn, ns;
  NodeDelta nd[kArgNodeDeltas];
  StateDelta sd[kArgStateDeltas];
};
hipError_t launch_victim_prep_inline(const NodeSoA& n, const VictimTables& t, const VictimPrepArgs& a,
                                     hipStream_t stream);

}  // namespace kbg
