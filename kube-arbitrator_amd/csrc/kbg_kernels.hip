// HIP kernels of the MI355X allocate path (gfx950, wave64).
//
// kbg_scan_kernel   — the hot kernel: for a batch of task evaluations, the
//                     feasibility of every (task, node) pair exactly as the
//                     reference's node loop decides it (allocate.go:119-162):
//                       PredicateFn == nil (predicates.go:121-201, resolved
//                       statically into class_mask + the dynamic pod-count cap
//                       predicates.go:125-127)
//                     && (Resreq.LessEqual(Idle) || Resreq.LessEqual(Releasing))
//                     (resource_info.go:142-146). One wave = 64 consecutive
//                     nodes held in registers; task rows are wave-uniform
//                     (scalar loads); results leave as 64-bit ballots.
// kbg_select_kernel — per task, the first M feasible node indices in
//                     ssn.Nodes order (first-fit = min index), with
//                     the Allocate/Pipeline kind of each.
// kbg_mask_kernel   — session-open static predicate masks (class x node bits).
// kbg_apply_kernel  — NodeInfo.AddTask deltas committed by the host.
//
// fp64 is compared with the reference's own expression; the file is compiled
// with -ffp-contract=off so nothing is fused.
#include <hip/hip_ext.h>

#include <algorithm>
#include <utility>

#include "kbg_device.hpp"

namespace kbg {

// Diagnostic build only (tools/libkbg_tools_stamps.so, -DKBG_FF_STAMPS): the
// fused kernel records the global 100 MHz clock at its phase boundaries, per
// workgroup, into a buffer nothing else reads. The shipped library has no
// stamps (FF_STAMP expands to nothing).
#ifdef KBG_FF_STAMPS
constexpr int kStampWG = 8192, kStampSlots = 8;
__device__ unsigned long long kbg_ff_stamps[kStampWG][kStampSlots];
#define FF_STAMP(slot)                                                                   \
  do {                                                                                   \
    unsigned long long t_;                                                               \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    if (threadIdx.x == 0 && blockIdx.x < kStampWG) kbg_ff_stamps[blockIdx.x][slot] = t_; \
  } while (0)
hipError_t read_ff_stamps(unsigned long long* out, int n_wg) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(kbg_ff_stamps), (size_t)n_wg * kStampSlots * 8, 0, hipMemcpyDeviceToHost);
}
#else
#define FF_STAMP(slot) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ bool le(double r, double a, double mn) {
  // (r < a || |a - r| < min)  — resource_info.go:142-146, one dimension
  return r < a || fabs(a - r) < mn;
}

// ------------------------------------------------------------------ scan
constexpr int kScanWaves = 4;          // waves per workgroup (256 threads)

// Lane mask of the nodes of this wave on which a row's request fits
// (Resource.LessEqual, one ballot per dimension, ANDed on the scalar unit).
// INT_MODE: the row carries thr = req - min and every value is an exact
// integer (kbg_device.hpp TaskRec), where `req <= a` is exactly `a > thr`.
template <bool INT_MODE>
__device__ __forceinline__ uint64_t fit_mask(double a0, double a1, double a2, double q0, double q1, double q2) {
  if (INT_MODE) return __ballot(a0 > q0) & __ballot(a1 > q1) & __ballot(a2 > q2);
  return __ballot(le(q0, a0, kMinMilliCPU)) & __ballot(le(q1, a1, kMinMemory)) & __ballot(le(q2, a2, kMinMilliGPU));
}

// One row J of the workgroup's 64: its request (q, read from LDS as a
// same-address broadcast by the caller) against this wave's 64 nodes. The raw
// fit ballots go to lane J (v_writelane_b32 with an inline-constant lane
// select: one scalar operand per VALU op on gfx9); the class mask, the pod
// cap and the Releasing-zero shortcut are applied by lane J itself once all
// rows are done, so a row costs its compares plus two lane moves (four when
// the wave holds Releasing resources).
template <bool INT_MODE, bool REL_ZERO, int J>
__device__ __forceinline__ void scan_row(double q0, double q1, double q2, double ic, double im, double ig, double rc,
                                         double rm, double rg, uint32_t (&keep)[4]) {
  const uint64_t mi = fit_mask<INT_MODE>(ic, im, ig, q0, q1, q2);
  asm("v_writelane_b32 %0, %2, %4\n\t"
      "v_writelane_b32 %1, %3, %4"
      : "+v"(keep[0]), "+v"(keep[1])
      : "s"((uint32_t)mi), "s"((uint32_t)(mi >> 32)), "i"(J));
  if constexpr (!REL_ZERO) {
    const uint64_t mr = fit_mask<INT_MODE>(rc, rm, rg, q0, q1, q2);
    asm("v_writelane_b32 %0, %2, %4\n\t"
        "v_writelane_b32 %1, %3, %4"
        : "+v"(keep[2]), "+v"(keep[3])
        : "s"((uint32_t)mr), "s"((uint32_t)(mr >> 32)), "i"(J));
  }
}

// All ROWS rows of the workgroup, unrolled at compile time in groups of
// kRowGroup whose LDS reads are issued together (one wave per SIMD is common
// in production launches, so the LDS latency must overlap within the wave).
// The host pads every batch to whole blocks with copies of a real row, so no
// row needs a bound check.
constexpr int kRowGroup = 8;
#ifndef KBG_SMALL_BATCH_ROWS
#define KBG_SMALL_BATCH_ROWS 1024
#endif
constexpr int kSmallBatchRows = KBG_SMALL_BATCH_ROWS;  // launch_scan: batches up to this many rows use 16-row workgroups
// Integer mode, no Releasing: rows J and J+1 together, their six compares
// issued back to back into six SGPR pairs before the first scalar AND reads
// one (a row's compares no longer wait on each other through VCC).
template <int J>
__device__ __forceinline__ void scan_row_pair(const double (&q)[2][3], double ic, double im, double ig,
                                              uint32_t (&keep)[4]) {
  uint64_t a0, a1, a2, b0, b1, b2;
  asm("v_cmp_gt_f64_e64 %0, %6, %9\n\t"
      "v_cmp_gt_f64_e64 %1, %7, %10\n\t"
      "v_cmp_gt_f64_e64 %2, %8, %11\n\t"
      "v_cmp_gt_f64_e64 %3, %6, %12\n\t"
      "v_cmp_gt_f64_e64 %4, %7, %13\n\t"
      "v_cmp_gt_f64_e64 %5, %8, %14"
      : "=&s"(a0), "=&s"(a1), "=&s"(a2), "=&s"(b0), "=&s"(b1), "=&s"(b2)
      : "v"(ic), "v"(im), "v"(ig), "v"(q[0][0]), "v"(q[0][1]), "v"(q[0][2]), "v"(q[1][0]), "v"(q[1][1]), "v"(q[1][2]));
  const uint64_t ma = a0 & a1 & a2, mb = b0 & b1 & b2;
  asm("v_writelane_b32 %0, %2, %6\n\t"
      "v_writelane_b32 %1, %3, %6\n\t"
      "v_writelane_b32 %0, %4, %7\n\t"
      "v_writelane_b32 %1, %5, %7"
      : "+v"(keep[0]), "+v"(keep[1])
      : "s"((uint32_t)ma), "s"((uint32_t)(ma >> 32)), "s"((uint32_t)mb), "s"((uint32_t)(mb >> 32)), "i"(J), "i"(J + 1));
}

// (integer mode, no Releasing: the next group's requests are read from LDS
// while this group's compares run)
template <int ROWS, int J, int GROUP>
__device__ __forceinline__ void scan_rows_int(const double (*s_req)[3], const double (&q)[GROUP][3], double ic,
                                              double im, double ig, uint32_t (&keep)[4], int nrows) {
  double qn[GROUP][3];
  if constexpr (J + GROUP < ROWS) {
#pragma unroll
    for (int u = 0; u < GROUP; ++u) {
      qn[u][0] = s_req[J + GROUP + u][0];
      qn[u][1] = s_req[J + GROUP + u][1];
      qn[u][2] = s_req[J + GROUP + u][2];
    }
  }
  [&]<int... U>(std::integer_sequence<int, U...>) {
    (scan_row_pair<J + 2 * U>(*reinterpret_cast<const double(*)[2][3]>(&q[2 * U][0]), ic, im, ig, keep), ...);
  }(std::make_integer_sequence<int, GROUP / 2>{});
  if constexpr (J + GROUP < ROWS)
    if (J + GROUP < nrows) scan_rows_int<ROWS, J + GROUP, GROUP>(s_req, qn, ic, im, ig, keep, nrows);
}

// `nrows` (wave-uniform, <= ROWS): the rows of the block that are real; the
// groups past it are skipped (a full-scan workgroup takes fewer rows than its
// variant holds, firstfit_geometry).
template <bool INT_MODE, bool REL_ZERO, int ROWS, int J = 0, int GROUP = kRowGroup>
__device__ __forceinline__ void scan_rows(const double (*s_req)[3], double ic, double im, double ig, double rc,
                                          double rm, double rg, uint32_t (&keep)[4], int nrows = ROWS) {
  double q[GROUP][3];
#pragma unroll
  for (int u = 0; u < GROUP; ++u) {
    q[u][0] = s_req[J + u][0];
    q[u][1] = s_req[J + u][1];
    q[u][2] = s_req[J + u][2];
  }
  if constexpr (INT_MODE && REL_ZERO && GROUP % 2 == 0 && J == 0) {
    scan_rows_int<ROWS, 0, GROUP>(s_req, q, ic, im, ig, keep, nrows);
    return;
  } else if constexpr (INT_MODE && REL_ZERO && GROUP % 2 == 0) {
    [&]<int... U>(std::integer_sequence<int, U...>) {
      (scan_row_pair<J + 2 * U>(*reinterpret_cast<const double(*)[2][3]>(&q[2 * U][0]), ic, im, ig, keep), ...);
    }(std::make_integer_sequence<int, GROUP / 2>{});
  } else {
    [&]<int... U>(std::integer_sequence<int, U...>) {
      (scan_row<INT_MODE, REL_ZERO, J + U>(q[U][0], q[U][1], q[U][2], ic, im, ig, rc, rm, rg, keep), ...);
    }(std::make_integer_sequence<int, GROUP>{});
  }
  if constexpr (J + GROUP < ROWS)
    if (J + GROUP < nrows) scan_rows<INT_MODE, REL_ZERO, ROWS, J + GROUP, GROUP>(s_req, ic, im, ig, rc, rm, rg, keep, nrows);
}

template <bool INT_MODE, int ROWS>
__global__ __launch_bounds__(256) void kbg_scan_kernel(NodeSoA nd, ScanGeom geo,
                                                       const uint64_t* __restrict__ class_mask,
                                                       const TaskRec* __restrict__ tasks, int32_t n_tasks,
                                                       int32_t cap_check, uint64_t* __restrict__ out) {
  __shared__ double s_req[ROWS][3];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rel = blockIdx.x * kScanWaves + wave;  // word relative to chunk_lo
  const int chunk = geo.chunk_lo + rel;            // global 64-node word
  const bool live = rel < geo.n_chunks && chunk < geo.W;  // words past W are never read
  const int t0 = blockIdx.y * ROWS;
  const int nt_blk = min(n_tasks - t0, ROWS);
  // Rows are padded to whole kScanRowsPerBlock blocks: every lane j < ROWS
  // has a real row t0 + j.
  const TaskRec tr = tasks[t0 + (lane & (ROWS - 1))];
  if (wave == 0 && lane < ROWS) {
    s_req[lane][0] = tr.req[0];
    s_req[lane][1] = tr.req[1];
    s_req[lane][2] = tr.req[2];
  }
  const uint64_t lane_mw = live ? class_mask[(size_t)tr.cls * geo.W + chunk] : 0ull;  // row `lane`, this chunk
  __syncthreads();
  if (!live) return;  // wave-uniform, after the barrier
  const int node = chunk * 64 + lane;
  const bool valid = node < geo.n_nodes;
  const int row = node - geo.tab_lo;
  double ic = 0, im = 0, ig = 0, rc = 0, rm = 0, rg = 0;
  int32_t nt = 0, mt = 0;
  if (valid) {
    ic = nd.idle_cpu[row];
    im = nd.idle_mem[row];
    ig = nd.idle_gpu[row];
    rc = nd.rel_cpu[row];
    rm = nd.rel_mem[row];
    rg = nd.rel_gpu[row];
    nt = nd.ntasks[row];
    mt = nd.maxtasks[row];
  }
  const uint64_t okm = __ballot(valid && (!cap_check || nt < mt));  // predicates.go:125-127 pod cap
  // Releasing is usually zero on every node of the wave; then a row's
  // Releasing fit is LessEqual(req, 0) on every lane (kRowRelZeroFits).
  const bool rel_zero_wave = __ballot(!(rc == 0.0 && rm == 0.0 && rg == 0.0)) == 0ull;
  uint32_t keep[4] = {0u, 0u, 0u, 0u};  // lane j: raw (idle-fit, releasing-fit) masks of row t0+j
  uint64_t mr;
  if (rel_zero_wave) {
    scan_rows<INT_MODE, true, ROWS>(s_req, ic, im, ig, rc, rm, rg, keep);
    mr = (tr.flags & kRowRelZeroFits) ? ~0ull : 0ull;
  } else {
    scan_rows<INT_MODE, false, ROWS>(s_req, ic, im, ig, rc, rm, rg, keep);
    mr = (uint64_t)keep[2] | ((uint64_t)keep[3] << 32);
  }
  if (lane < nt_blk) {
    const uint64_t mw = lane_mw & okm;  // static predicate and pod cap of row t0+lane on this wave's nodes
    const uint64_t mi = ((uint64_t)keep[0] | ((uint64_t)keep[1] << 32)) & mw;
    // [slot][plane][quad][row][4] (kbg_device.hpp ScanGeom): the workgroup's
    // four waves fill 32 contiguous bytes per row, its rows one 2-KB run
    const int slot = rel / geo.Wl, w = rel - slot * geo.Wl;
    const size_t plane = (size_t)n_tasks * kbg_slot_words(geo.Wl);
    uint64_t* o = out + (size_t)slot * 2 * plane + ((size_t)(w >> 2) * n_tasks + t0 + lane) * 4 + (w & 3);
    o[0] = mi | (mr & mw);
    o[plane] = mi;
  }
}

hipError_t launch_scan(const NodeSoA& n, const ScanGeom& g, const uint64_t* class_mask, const TaskRec* tasks,
                       int32_t n_tasks, int32_t cap_check, int32_t int_mode, uint64_t* out, hipStream_t stream,
                       hipEvent_t start, hipEvent_t stop) {
  if (n_tasks <= 0 || g.n_chunks <= 0) return hipSuccess;
  // Rows per workgroup: a wave's rows run back to back, so short batches
  // (grouped mode: tens of rows) get more, shorter waves.
  const int rows = (n_tasks <= kSmallBatchRows) ? 16 : 64;
  dim3 grid((g.n_chunks + kScanWaves - 1) / kScanWaves, (n_tasks + rows - 1) / rows);
  dim3 block(64 * kScanWaves);
  if (int_mode) {
    if (rows == 16)
      hipExtLaunchKernelGGL((kbg_scan_kernel<true, 16>), grid, block, 0, stream, start, stop, 0, n, g, class_mask, tasks,
                            n_tasks, cap_check, out);
    else
      hipExtLaunchKernelGGL((kbg_scan_kernel<true, 64>), grid, block, 0, stream, start, stop, 0, n, g, class_mask, tasks,
                            n_tasks, cap_check, out);
  } else {
    if (rows == 16)
      hipExtLaunchKernelGGL((kbg_scan_kernel<false, 16>), grid, block, 0, stream, start, stop, 0, n, g, class_mask,
                            tasks, n_tasks, cap_check, out);
    else
      hipExtLaunchKernelGGL((kbg_scan_kernel<false, 64>), grid, block, 0, stream, start, stop, 0, n, g, class_mask,
                            tasks, n_tasks, cap_check, out);
  }
  return hipGetLastError();
}

// ------------------------------------------------------ fused first-fit
// kbg_firstfit_kernel: the scan and the first-fit extraction in one launch.
// A workgroup of 16 waves owns ROWS rows (16, 24 or 32: the host picks the
// smallest that puts every row block on a CU at once, so no launch runs a
// second round of workgroups) and walks their words [w_lo, w_hi) in node
// order, up to kFfMaxRound words per round (C3's 79 in one): wave w evaluates
// words w, w + 16, ... of the round for every row (64 nodes in registers, the
// next word's loads in flight during the current one; rows read from LDS as
// same-address broadcasts; one v_cmp_f64 ballot per dimension ANDed on the
// scalar unit, the raw ballot moved to lane J with v_writelane_b32; class
// mask, pod cap and Releasing shortcut applied by lane J) and parks the masks
// in LDS. After the round's barrier the wave owning row j (rows w and w + 16)
// takes the row's words 64 at a time: a ballot prefix sum of their fit counts
// gives each word's first list position, and every word starting below the
// row's `want` is written to the output as its two masks (one 16-B store per
// word, 1 KB per wave instruction): no per-candidate writes, no second pass.
// Shapes come from the kernel arguments (no PCIe read at launch) or from
// host-mapped memory. `EARLY_EXIT` (production mode) ends the walk after a
// round in which every row's list is full (the rest of the table cannot
// change it); full-scan mode evaluates every node for every row (SURVEY
// §8(d)).
#ifndef KBG_FF_WAVES
#define KBG_FF_WAVES 16  // experiment builds (tools/build_variants.sh) try 8
#endif
constexpr int kFfWaves = KBG_FF_WAVES;
constexpr int kFfMaxRound = kFfRoundWords;  // words per round (LDS: 2 x 128 x ROWS x 8 B); a multiple of kFfWaves
// rows whose requests are read from LDS together
template <bool INT_MODE>
constexpr int kFfGroup = INT_MODE ? 4 : 2;
// (32-row workgroups: 2 rows per group keep the longer unrolled row walk within
// the register budget)
template <bool INT_MODE, int ROWS>
#ifdef KBG_FF_GROUP  // experiment builds (tools/build_variants.sh)
constexpr int kFfGroupR = ROWS > 24 ? 2 : KBG_FF_GROUP;
#else
constexpr int kFfGroupR = ROWS > 24 ? 2 : kFfGroup<INT_MODE>;
#endif
#ifndef KBG_FF_WGS_PER_CU
#define KBG_FF_WGS_PER_CU 1  // resident workgroups per CU the full-scan geometry plans for
#endif

// COMPLETE (a.complete: the walk is one round and every word's masks go out,
// so there is no list to cut): each wave stores a writer row's masks for its
// word right after the compares — lane j holds row j — and keeps an any-fit
// bit per row; no LDS staging of the masks, no round barrier, no prefix-sum
// extraction. One barrier at the end joins the any-fit bits for the info word.
template <bool INT_MODE, bool EARLY_EXIT, bool COMPLETE, int ROWS>
__global__ __launch_bounds__(64 * kFfWaves, kFfWaves / 4 * KBG_FF_WGS_PER_CU) void kbg_firstfit_kernel(FirstFitArgs a) {
  static_assert(ROWS % 8 == 0 && ROWS <= 4 * kFfWaves, "rows per workgroup");
  constexpr int RPW = (ROWS + kFfWaves - 1) / kFfWaves;  // rows a wave extracts (1 or 2)
  constexpr int SW = COMPLETE ? 1 : kFfMaxRound;           // (COMPLETE: no mask staging)
  __shared__ double s_req[ROWS][3];
  __shared__ int32_t s_cls[ROWS];
  __shared__ uint32_t s_flags[ROWS], s_map[ROWS];  // shape flags (want << 1 | rel-zero fit); shape | writer
  __shared__ uint64_t s_f[SW][ROWS];               // [word of the round][row]: fits (Idle or Releasing)
  __shared__ uint64_t s_i[SW][ROWS];               //                        fits in Idle
  __shared__ uint32_t s_done[ROWS];
  __shared__ uint16_t s_runs[kInlineShapes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rb = blockIdx.x / a.splits, part = blockIdx.x - rb * a.splits;  // row block, word part
  const int nrows = a.rows;  // rows of this block (<= ROWS; the rest of the variant's rows are skipped)
  const int g0 = rb * nrows;
  const int w_lo = a.w_lo + part * a.split_words, w_hi = min(a.w_hi, w_lo + a.split_words);
  FF_STAMP(0);
  if (wave == 0) {
    // runs: the slots' run ends (kernel arguments) into LDS, then each row
    // lane finds its slot by a binary search there — no row -> shape map
    if (a.runs)
      for (int i = lane; i < a.n_shapes; i += 64) s_runs[i] = a.run_end[i];
    // the search below reads entries other lanes wrote: their LDS writes are
    // issued before its reads (wave-local ordering, no workgroup barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < ROWS) {
      const bool real = lane < nrows && g0 + lane < a.G;
      const int g = min(g0 + min(lane, nrows - 1), a.G - 1);  // padding rows evaluate a copy of a real row
      uint32_t m;
      if (a.runs) {
        int lo = 0, hi = a.n_shapes - 1;  // the first slot whose run ends past g
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (s_runs[mid] > g) hi = mid;
          else lo = mid + 1;
        }
        m = (uint32_t)lo | (g + 1 == (int)s_runs[lo] ? kRowWriter : 0u);
      } else {
        m = a.row_shape ? a.row_shape[g] : ((uint32_t)g | kRowWriter);
      }
      const uint32_t sh = m & ~kRowWriter;
      const TaskRec tr = a.shapes ? a.shapes[sh] : a.inl[sh];
      s_req[lane][0] = tr.req[0];
      s_req[lane][1] = tr.req[1];
      s_req[lane][2] = tr.req[2];
      s_cls[lane] = tr.cls;
      s_flags[lane] = (uint32_t)tr.flags;
      s_map[lane] = real ? m : (m & ~kRowWriter);
      if (COMPLETE) s_done[lane] = 0u;  // the row's any-fit bit
    }
  }
  const int32_t tw = w_hi - w_lo;  // words this workgroup covers
  if (tw <= 0) {  // no words (a session without nodes): empty complete lists, no table or mask read
    __syncthreads();
    if (wave == 0 && lane < ROWS && (s_map[lane] & kRowWriter)) {
      const uint32_t sh = s_map[lane] & ~kRowWriter;
      a.info[sh * a.info_stride + a.part0 + part] = 0u;
      if (a.avail) a.avail[sh] = 0u;
    }
    return;
  }
  // A word's node rows (and, once the rows' classes are known, their class
  // mask words) are loaded one word ahead of its compares: the next word's
  // loads are in flight while this one is evaluated. The first word's loads
  // are issued before the rows arrive.
  struct Word {
    double ic = 0, im = 0, ig = 0, rc = 0, rm = 0, rg = 0;
    int32_t nt = 0, mt = 0;
    bool valid = false;
  };
  // Every load is unconditional, from a clamped (always legal) address, so
  // the compiler can wait for exactly the current word's loads and leave the
  // next word's in flight (a load under a branch makes it wait for all of
  // them, vmcnt(0), and the prefetch would buy nothing). Lanes past the table
  // read row 0 and are masked out by `valid` (okm).
  auto load_word = [&](int c, Word& w) {
    const int node = c * 64 + lane;
    const int row = node - a.tab_lo;
    w.valid = node < a.n_nodes && row >= 0 && row < a.tab_n;
    const int rr = w.valid ? row : 0;
    const double* p = a.nodes + rr;
    w.ic = p[0];
    w.im = p[a.stride];
    w.ig = p[2 * a.stride];
    w.rc = p[3 * a.stride];
    w.rm = p[4 * a.stride];
    w.rg = p[5 * a.stride];
    const int32_t* q = reinterpret_cast<const int32_t*>(a.nodes + 6 * (size_t)a.stride) + rr;
    w.nt = q[0];
    w.mt = q[a.stride];
  };
  const int w_last = w_hi - 1;
  Word cur;
  load_word(min(w_lo + wave, w_last), cur);
  __syncthreads();
  FF_STAMP(1);
  // the extraction state of the rows this wave owns (rows wave, wave + 16)
  uint32_t found[RPW], want[RPW], covered[RPW];
  bool done[RPW], writer[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int j = wave + i * kFfWaves;
    found[i] = 0u;
    covered[i] = 0u;
    writer[i] = j < ROWS && (s_map[j] & kRowWriter);
    want[i] = j >= ROWS ? 0u : a.complete ? 0xffffffffu : (s_flags[j] >> kRowWantShift);
    done[i] = !writer[i];
  }
  const int lrow = lane < ROWS ? lane : 0;
  const int cls_l = s_cls[lrow];
  const uint32_t flags_l = s_flags[lrow];
  // COMPLETE: lane j's output row (a writer row's masks from word mask_w0), or none
  MaskPair* const out_l =
      COMPLETE && lane < ROWS && (s_map[lrow] & kRowWriter)
          ? a.masks + (size_t)(s_map[lrow] & ~kRowWriter) * a.mw - a.mask_w0
          : nullptr;
  bool any_l = false;
  // rounds are kFfMaxRound (a multiple of kFfWaves) words apart, so a wave's
  // words are c, c + kFfWaves, ... across rounds too; lanes >= ROWS load a
  // row's mask word they never use
  uint64_t lane_mw = a.class_mask[(size_t)cls_l * a.W + min(w_lo + wave, w_last)];
#pragma unroll 1
  for (int r0 = w_lo; r0 < w_hi; r0 += kFfMaxRound) {
    const int nw = min(kFfMaxRound, w_hi - r0);  // words of this round
#pragma unroll 1
    for (int k = wave; k < nw; k += kFfWaves) {     // this wave's words of the round
      // the row requests are re-read from LDS per word (kept in registers
      // across the loop they would take 6 VGPRs per row)
      asm volatile("" ::: "memory");
      const int c = r0 + k;                           // global 64-node word
      const int cn = min(c + kFfWaves, w_last);       // this wave's next word (the last one again at the end)
      Word nxt;
      load_word(cn, nxt);
      const uint64_t nxt_mw = a.class_mask[(size_t)cls_l * a.W + cn];
      const uint64_t okm = __ballot(cur.valid && (!a.cap_check || cur.nt < cur.mt));  // predicates.go:125-127 pod cap
      const bool rel_zero_wave =
          __ballot(cur.valid && !(cur.rc == 0.0 && cur.rm == 0.0 && cur.rg == 0.0)) == 0ull;
      uint32_t keep[4] = {0u, 0u, 0u, 0u};
      uint64_t mr;
      if (rel_zero_wave) {
        scan_rows<INT_MODE, true, ROWS, 0, kFfGroupR<INT_MODE, ROWS>>(s_req, cur.ic, cur.im, cur.ig, cur.rc, cur.rm, cur.rg,
                                                               keep, nrows);
        mr = (flags_l & kRowRelZeroFits) ? ~0ull : 0ull;
      } else {
        scan_rows<INT_MODE, false, ROWS, 0, kFfGroupR<INT_MODE, ROWS>>(s_req, cur.ic, cur.im, cur.ig, cur.rc, cur.rm,
                                                                cur.rg, keep, nrows);
        mr = (uint64_t)keep[2] | ((uint64_t)keep[3] << 32);
      }
      if (COMPLETE) {
        const uint64_t mw = lane_mw & okm;
        const uint64_t fi = ((uint64_t)keep[0] | ((uint64_t)keep[1] << 32)) & mw;
        const uint64_t f = fi | (mr & mw);
        any_l |= f != 0ull;
        if (out_l) out_l[c] = MaskPair{f, fi};
      } else if (lane < ROWS) {
        const uint64_t mw = lane_mw & okm;
        const uint64_t fi = ((uint64_t)keep[0] | ((uint64_t)keep[1] << 32)) & mw;
        s_f[k][lane] = fi | (mr & mw);
        s_i[k][lane] = fi;
      }
      cur = nxt;
      lane_mw = nxt_mw;
    }
    if constexpr (COMPLETE) {  // one round; the rows' any-fit bits joined over the waves
      if (any_l && lane < ROWS) s_done[lane] = 1u;
      FF_STAMP(2);
      __syncthreads();
      FF_STAMP(3);
      if (wave == 0 && lane < ROWS && (s_map[lane] & kRowWriter)) {
        const uint32_t sh = s_map[lane] & ~kRowWriter;
        const bool any = s_done[lane] != 0u;
        a.info[sh * a.info_stride + a.part0 + part] = (uint32_t)tw | (any ? kInfoAnyBit : 0u);
        if (a.avail) a.avail[sh] = any ? a.avail_bit : 0u;
      }
      FF_STAMP(6);
      return;
    }
    if (r0 == w_lo) FF_STAMP(2);
    __syncthreads();
    if (r0 == w_lo) FF_STAMP(3);
    if (r0 == w_lo) FF_STAMP(4);
    // Extraction: the owner wave of row j takes its words 64 at a time. Lane
    // k holds word k's fit count; the exclusive prefix sum over lanes (one
    // ballot + mbcnt per bit of the count) is the list position of the word's
    // first node. A word starting below `want` goes out whole (its masks);
    // positions grow in node order, so the first word starting at or past
    // `want` ends the list.
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int j = wave + i * kFfWaves;
      if (j >= ROWS || done[i]) continue;  // wave-uniform
      MaskPair* out = a.masks + (size_t)(s_map[j] & ~kRowWriter) * a.mw + (r0 - a.mask_w0);
#pragma unroll 1
      for (int k0 = 0; k0 < nw; k0 += 64) {
        const int k = k0 + lane;
        const uint64_t f = k < nw ? s_f[k][j] : 0ull;
        const uint32_t pc = (uint32_t)__popcll(f);
        uint32_t excl = 0, tot = 0;
#pragma unroll
        for (int b = 0; b < 7; ++b) {  // pc <= 64
          const uint64_t bb = __ballot((pc >> b) & 1u);
          excl += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
          tot += (uint32_t)__popcll(bb) << b;
        }
        const bool put = k < nw && found[i] + excl < want[i];
        if (put) out[k] = MaskPair{f, s_i[k][j]};
        const uint32_t nput = (uint32_t)__popcll(__ballot(put));
        found[i] += tot;
        covered[i] = (uint32_t)(r0 - w_lo + k0) + nput;
        if (found[i] >= want[i]) {  // every later word starts at or past want
          done[i] = true;
          break;
        }
      }
    }
    if (r0 == w_lo) FF_STAMP(5);
    if (r0 + kFfMaxRound >= w_hi) break;  // the last round: no second barrier
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int j = wave + i * kFfWaves;
      if (j < ROWS && lane == 0) s_done[j] = done[i] ? 1u : 0u;
    }
    __syncthreads();  // the round's masks are read, the done flags written
    if (EARLY_EXIT) {  // every row's list is full: the same decision in every wave
      const uint32_t d = lane < ROWS ? s_done[lane] : 1u;
      if (__ballot(d == 0u) == 0ull) break;
    }
  }
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int j = wave + i * kFfWaves;
    if (!writer[i] || lane != 0) continue;
    const uint32_t sh = s_map[j] & ~kRowWriter;
    // covered: the words written; a row whose walk ended with its list not
    // full covered every word of the walk (EARLY_EXIT: the rounds walked)
    a.info[sh * a.info_stride + a.part0 + part] =
        covered[i] | (covered[i] < (uint32_t)tw ? kCountIncompleteBit : 0u) | (found[i] ? kInfoAnyBit : 0u);
    if (a.avail) a.avail[sh] = found[i] ? a.avail_bit : 0u;
  }
  FF_STAMP(6);
}

template <bool INT_MODE, bool EARLY_EXIT, bool COMPLETE>
hipError_t launch_firstfit_rows(const FirstFitArgs& a, int variant, hipStream_t stream, hipEvent_t start,
                                hipEvent_t stop) {
  const dim3 grid((a.G + a.rows - 1) / a.rows * a.splits), block(64 * kFfWaves);
  if (variant == 16)
    hipExtLaunchKernelGGL((kbg_firstfit_kernel<INT_MODE, EARLY_EXIT, COMPLETE, 16>), grid, block, 0, stream, start,
                          stop, 0, a);
  else if (variant == 24)
    hipExtLaunchKernelGGL((kbg_firstfit_kernel<INT_MODE, EARLY_EXIT, COMPLETE, 24>), grid, block, 0, stream, start,
                          stop, 0, a);
  else
    hipExtLaunchKernelGGL((kbg_firstfit_kernel<INT_MODE, EARLY_EXIT, COMPLETE, 32>), grid, block, 0, stream, start,
                          stop, 0, a);
  return hipGetLastError();
}

// One workgroup per CU at a time (16 waves, 80-128 VGPRs), so a launch of
// more than 256 workgroups runs a second, mostly idle round. Production
// batches take whole blocks of 16, 24 or 32 rows (short ones split their walk
// into word parts instead). Full-scan batches spread their rows evenly: every
// row costs the same walk of the whole table, so ceil(G / 256) rows (rounded
// up to a pair, the unit the scan's unrolled row walk skips by) on each CU
// gives the shortest launch — 4.2k rows: 17-18 rows per CU on ~232 CUs
// instead of 24 rows on 174.
FfGeometry firstfit_geometry(int32_t G, bool full_scan) {
  constexpr int kCUs = 256;
  if (!full_scan) {
    const int v = G <= 16 * kCUs ? 16 : G <= 24 * kCUs ? 24 : 32;
    return {v, v};
  }
  const int slots = kCUs * KBG_FF_WGS_PER_CU;
  int rows = (G + slots - 1) / slots;
  rows = std::min(32, std::max(2, (rows + 1) & ~1));
  return {rows <= 16 ? 16 : rows <= 24 ? 24 : 32, rows};
}

hipError_t launch_firstfit(const FirstFitArgs& a, int32_t int_mode, hipStream_t stream, hipEvent_t start,
                           hipEvent_t stop) {
  if (a.G <= 0) return hipSuccess;
  const FfGeometry geo = firstfit_geometry(a.G, !a.early_exit);
  if (a.rows <= 0 || a.rows > geo.variant) return hipErrorInvalidValue;  // the host sizes both (device_launch)
  // a complete walk (one round, every word out): the store-as-you-scan
  // variant; otherwise <.., false>: full-scan mode (every node of every row),
  // <.., true>: production
  if (a.complete) {
    if (a.w_hi - a.w_lo > kFfMaxRound) return hipErrorInvalidValue;
    return int_mode ? launch_firstfit_rows<true, false, true>(a, geo.variant, stream, start, stop)
                    : launch_firstfit_rows<false, false, true>(a, geo.variant, stream, start, stop);
  }
  if (int_mode)
    return a.early_exit ? launch_firstfit_rows<true, true, false>(a, geo.variant, stream, start, stop)
                        : launch_firstfit_rows<true, false, false>(a, geo.variant, stream, start, stop);
  return a.early_exit ? launch_firstfit_rows<false, true, false>(a, geo.variant, stream, start, stop)
                      : launch_firstfit_rows<false, false, false>(a, geo.variant, stream, start, stop);
}

// ------------------------------------------------------- FitError counts
// JobInfo.NodesFitDelta of a not-ready job's last evaluated task
// (allocate.go:116-144), summarised as JobInfo.FitError counts it
// (job_info.go:329-358), for every such job at once. A node's state at the
// task's evaluation point is the final table with the decisions at or after
// that point undone: the node's decisions in order (hk, hold), the first
// undone Allocate giving its Idle, the undone count its pod count.
// A workgroup of 16 waves takes kFitJobs jobs and walks the table 1024
// nodes at a time, a lane per node: the node's records (decision range, pod
// counts, Idle) are loaded once for all the group's jobs, whose static mask
// words are wave-uniform loads. A node's decisions are in log order, so the
// first one at or after a job's point is a binary search of its range, and
// the first undone Allocate from there one load of the host's next-Allocate
// index (na), then the Idle logged before it. Counts: per-wave ballots and
// popcounts, summed in LDS per job. Measured at C3 (937 jobs x 5120 nodes,
// profiles/r06/fitdelta_ab.txt): one workgroup per job walking each node's
// decisions a load at a time (round 5) 40 µs per launch — first-fit piles
// hundreds of decisions on the first nodes; one workgroup per job with
// binary searches 33 µs; 2 / 4 / 8 / 16 jobs per workgroup 19.9 / 23.4 / 41 /
// 119 µs (sharing the node loads against fewer workgroups, each a chain of
// dependent loads per pass); a grid over (node chunk, job) with
// cross-workgroup sums 540 µs (device-scope fences and atomics between XCDs).
constexpr int kFitBlock = 1024;
constexpr int kFitJobs = 2;
__global__ __launch_bounds__(kFitBlock) void kbg_fitdelta_kernel(FitArgs a) {
  __shared__ int32_t s_cnt[kFitJobs][4];
  const int q0 = blockIdx.x * kFitJobs;
  const int nj = min(kFitJobs, a.nq - q0);
  if (threadIdx.x < kFitJobs * 4) s_cnt[threadIdx.x >> 2][threadIdx.x & 3] = 0;
  __syncthreads();
  const int32_t* ni = reinterpret_cast<const int32_t*>(a.nodes + 6 * (size_t)a.stride);
  int n_end = 0;  // the furthest end of the group's jobs
  for (int jj = 0; jj < nj; ++jj) n_end = max(n_end, min(a.q[q0 + jj].end, a.tab_lo + a.tab_n));
  const int last = max(a.tab_lo, n_end - 1);  // a legal node for clamped loads
  int cnt[kFitJobs][4] = {};
  for (int base = a.tab_lo; base < n_end; base += kFitBlock) {
    const int n = base + (int)threadIdx.x;
    const int nc = min(n, last);
    const int r = nc - a.tab_lo;
    const int e0 = a.hoff[nc], e1 = a.hoff[nc + 1], nt = ni[r], mt = ni[a.stride + r];
    const double ic = a.nodes[r], im = a.nodes[a.stride + r], ig = a.nodes[2 * (size_t)a.stride + r];
#pragma unroll
    for (int jj = 0; jj < kFitJobs; ++jj) {
      if (jj >= nj) break;
      const FitQuery& fq = a.q[q0 + jj];
      const int end = min(fq.end, a.tab_lo + a.tab_n);
      if (__builtin_amdgcn_readfirstlane(base + (int)(threadIdx.x & ~63)) >= end) continue;  // the wave is past it
      const uint64_t mw = a.class_mask[(size_t)fq.cls * a.W + (nc >> 6)];
      bool hit = false, bc = false, bm = false, bg = false;
      if (n < end && ((mw >> (n & 63)) & 1ull)) {  // static predicate
        int lo = e0, hi = e1;  // decisions before the evaluation stay applied: the first at or after it
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((a.hk[mid] & 0x7fffffff) < fq.point) lo = mid + 1;
          else hi = mid;
        }
        double c = ic, m = im, g = ig;
        const int x = lo < e1 ? a.na[lo] : -1;  // the first undone Allocate: Idle before it
        if (x >= 0) {
          c = a.hold[3 * (size_t)x];
          m = a.hold[3 * (size_t)x + 1];
          g = a.hold[3 * (size_t)x + 2];
        }
        const bool capped = a.cap_check && nt - (e1 - lo) >= mt;  // pod cap then (predicates.go:125-127)
        const bool chosen = n != fq.win && le(fq.req[0], c, kMinMilliCPU) && le(fq.req[1], m, kMinMemory) &&
                            le(fq.req[2], g, kMinMilliGPU);
        if (!capped && !chosen) {  // Resource.FitDelta (resource_info.go:116-129)
          hit = true;
          bc = (fq.req[0] > 0 ? c - (fq.req[0] + kMinMilliCPU) : c) < 0;
          bm = (fq.req[1] > 0 ? m - (fq.req[1] + kMinMemory) : m) < 0;
          bg = (fq.req[2] > 0 ? g - (fq.req[2] + kMinMilliGPU) : g) < 0;
        }
      }
      cnt[jj][0] += __popcll(__ballot(hit));
      cnt[jj][1] += __popcll(__ballot(bc));
      cnt[jj][2] += __popcll(__ballot(bm));
      cnt[jj][3] += __popcll(__ballot(bg));
    }
  }
  if ((threadIdx.x & 63) == 0)  // (the counts are wave-uniform)
#pragma unroll
    for (int jj = 0; jj < kFitJobs; ++jj)
      if (cnt[jj][0]) {
        atomicAdd(&s_cnt[jj][0], cnt[jj][0]);
        atomicAdd(&s_cnt[jj][1], cnt[jj][1]);
        atomicAdd(&s_cnt[jj][2], cnt[jj][2]);
        atomicAdd(&s_cnt[jj][3], cnt[jj][3]);
      }
  __syncthreads();
  if (threadIdx.x < nj * 4) a.out[4 * (size_t)q0 + threadIdx.x] = s_cnt[threadIdx.x >> 2][threadIdx.x & 3];
}

hipError_t launch_fitdelta(const FitArgs& a, hipStream_t stream) {
  if (a.nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_fitdelta_kernel, dim3((a.nq + kFitJobs - 1) / kFitJobs), dim3(kFitBlock), 0, stream, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------- select
// One wave per row walks the row's words [w_lo, w_hi) in global node order
// (shard slots in rank order = ascending node index), so the candidates come
// out first-fit. An owner-resolve shard selects over its own words only.
__global__ __launch_bounds__(256) void kbg_select_kernel(const uint64_t* __restrict__ bits, int32_t w_lo, int32_t w_hi,
                                                         int32_t Wl, int32_t n_rows,
                                                         const uint32_t* __restrict__ cap_off,
                                                         uint32_t* __restrict__ out_cand,
                                                         uint32_t* __restrict__ out_count) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_rows) return;
  const size_t plane = (size_t)n_rows * kbg_slot_words(Wl);
  const int M = (int)(cap_off[t + 1] - cap_off[t]);
  uint32_t* cand = out_cand + cap_off[t];
  int found = 0;
  int base = w_lo;
  for (; base < w_hi && found < M; base += 64) {
    const int c = base + lane;
    uint64_t f = 0ull, iw = 0ull;
    if (c < w_hi) {
      const int slot = c / Wl, w = c - slot * Wl;
      const uint64_t* p = bits + (size_t)slot * 2 * plane + ((size_t)(w >> 2) * n_rows + t) * 4 + (w & 3);
      f = p[0];
      iw = p[plane];
    }
    const int pc = __popcll(f);
    int incl = pc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    const int total = __shfl(incl, 63, 64);
    int r = found + incl - pc;
    while (f != 0ull && r < M) {
      const int b = __ffsll((unsigned long long)f) - 1;
      f &= f - 1ull;
      const uint32_t kind = ((iw >> b) & 1ull) ? 0u : kCandPipelineBit;
      cand[r] = (uint32_t)(c * 64 + b) | kind;
      ++r;
    }
    found += total;
  }
  if (lane == 0) {
    const bool complete = base >= w_hi && found <= M;
    const uint32_t cnt = (uint32_t)(found < M ? found : M);
    out_count[t] = cnt | (complete ? 0u : kCountIncompleteBit);
  }
}

hipError_t launch_select(const uint64_t* bits, int32_t w_lo, int32_t w_hi, int32_t Wl, int32_t n_rows,
                         const uint32_t* cap_off, uint32_t* out_cand, uint32_t* out_count, hipStream_t stream,
                         hipEvent_t start, hipEvent_t stop) {
  if (n_rows <= 0) return hipSuccess;
  hipExtLaunchKernelGGL(kbg_select_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, stream, start, stop, 0, bits, w_lo,
                        w_hi, Wl, n_rows, cap_off, out_cand, out_count);
  return hipGetLastError();
}

// ----------------------------------------------------------------- apply
__global__ __launch_bounds__(256) void kbg_apply_kernel(NodeSoA nd, const NodeDelta* __restrict__ d, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int node = d[i].node;
  nd.idle_cpu[node] = d[i].idle[0];
  nd.idle_mem[node] = d[i].idle[1];
  nd.idle_gpu[node] = d[i].idle[2];
  nd.rel_cpu[node] = d[i].rel[0];
  nd.rel_mem[node] = d[i].rel[1];
  nd.rel_gpu[node] = d[i].rel[2];
  nd.ntasks[node] = d[i].ntasks;
  nd.maxtasks[node] = d[i].maxtasks;
}

hipError_t launch_apply(const NodeSoA& n, const NodeDelta* deltas, int32_t n_deltas, hipStream_t stream) {
  if (n_deltas <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_apply_kernel, dim3((n_deltas + 255) / 256), dim3(256), 0, stream, n, deltas, n_deltas);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void kbg_copy16_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                         size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

hipError_t launch_copy16(void* dst, const void* src, size_t n16, hipStream_t stream) {
  if (n16 == 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_copy16_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, stream, (uint4*)dst,
                     (const uint4*)src, n16);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void kbg_mask_apply_kernel(uint64_t* __restrict__ class_mask,
                                                             const MaskDelta* __restrict__ d, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) class_mask[d[i].index] = d[i].value;
}

hipError_t launch_mask_apply(uint64_t* class_mask, const MaskDelta* deltas, int32_t n_deltas, hipStream_t stream) {
  if (n_deltas <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_mask_apply_kernel, dim3((n_deltas + 255) / 256), dim3(256), 0, stream, class_mask, deltas,
                     n_deltas);
  return hipGetLastError();
}

// --------------------------------------------------------- victim scan
// resource_info.go:138-146 on [3] arrays
__device__ __forceinline__ bool res_le3(const double* r, const double* a) {
  return le(r[0], a[0], kMinMilliCPU) && le(r[1], a[1], kMinMemory) && le(r[2], a[2], kMinMilliGPU);
}
__device__ __forceinline__ bool res_less3(const double* r, const double* a) {
  return r[0] < a[0] && r[1] < a[1] && r[2] < a[2];
}
// drf.go:156-166 with helpers.Share
__device__ __forceinline__ double share3(const double* a, const double* tot) {
  double res = 0;
  for (int d = 0; d < 3; ++d) {
    const double s = tot[d] == 0 ? (a[d] == 0 ? 0.0 : 1.0) : a[d] / tot[d];
    if (s > res) res = s;
  }
  return res;
}

// One wave per node, in ssn.Nodes order; the lowest node where the reference
// stops (validated victims, or a panic inside PredicateFn or a victim fn)
// wins. The node's candidates — the session tasks Running on it at open, in
// NodeInfo.Tasks order — are taken in chunks of 64, one per lane
// (k = h * 64 + lane, h < kVictimChunks; the host checks the bound). The
// victim fns that accumulate per job (drf.go:87-100) or per queue
// (proportion.go:166-183) walk the preemptees in order as a wave-uniform
// loop: lane k applies preemptee k2 while k2 <= k, so each lane sees exactly
// the subtractions the reference has made when it reaches its candidate.
// Preemptees of the lane's own chunk come through v_readlane, those of
// earlier chunks through wave-uniform (scalar) loads.

__device__ __forceinline__ int32_t rl_i(int32_t v, int32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double rl_d(double v, int32_t l) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Candidate k of a node: its job, queue, request and preemptee filter.
struct VCand {
  int32_t job, queue;
  double r[3];
  bool f;
};
__device__ __forceinline__ VCand load_cand(const VictimScan& p, const VictimTables& t, int off, int L, int k) {
  VCand c{-1, -1, {0.0, 0.0, 0.0}, false};
  if (k < L) {
    const size_t pos = (size_t)off + k;  // candidate records in node order: a chunk is one contiguous read
    const int2 jq = t.c_jq[pos];
    c.job = jq.x;
    c.queue = jq.y;
    c.r[0] = t.c_req[3 * pos];
    c.r[1] = t.c_req[3 * pos + 1];
    c.r[2] = t.c_req[3 * pos + 2];
    if (t.c_run[pos]) {
      if (p.mode == VM_PREEMPT_JOBS) c.f = c.queue == p.queue && c.job != p.job;  // preempt.go:100-112
      else if (p.mode == VM_PREEMPT_TASKS) c.f = c.job == p.job;                // :146-154
      else c.f = c.queue != p.queue;                                            // reclaim.go:113-126
    }
  }
  return c;
}

// One preemptee k2 applied to this lane's running allocations (drf per job,
// proportion per queue) when k2 <= k; sets *panic on a Sub underflow, *vp at
// k2 == k (proportion's verdict is taken right after its own subtraction).
__device__ __forceinline__ void apply_preemptee(const VictimTables& t, int fns, int32_t j2, int32_t q2,
                                                const double (&r2)[3], bool self, int32_t jv, int32_t qv, double (&xd)[3],
                                                double (&xp)[3], bool& panic, bool& vp) {
  if ((fns & VP_DRF) && j2 == jv) {
    if (!res_le3(r2, xd)) panic = true;  // Resource.Sub (resource_info.go:100-110)
    xd[0] -= r2[0];
    xd[1] -= r2[1];
    xd[2] -= r2[2];
  }
  if ((fns & VP_PROP) && q2 == qv) {
    if (!res_less3(xp, r2)) {  // Less: skipped, allocation untouched
      if (!res_le3(r2, xp)) panic = true;
      xp[0] -= r2[0];
      xp[1] -= r2[1];
      xp[2] -= r2[2];
      if (self) vp = res_le3(t.q_deserved + 3 * (size_t)qv, xp);
    }
  }
}

// A wave-uniform 64-bit mask read back from LDS (every lane reads the same
// word; readfirstlane makes it scalar again).
__device__ __forceinline__ uint64_t lds_mask(const uint64_t* p) {
  const uint64_t v = *p;
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
}

// Per-chunk candidate masks of one node (preemptees, the tier's victims, the
// deciding tier's): in registers for the main scan (NCH <= 2), in this
// wave's LDS slice for the big-node kernel (16 chunks x 3 masks would not fit
// the register file: they spilled to scratch).
template <int NCH, bool LDS>
struct ChunkMasks {
  uint64_t pm[LDS ? 1 : NCH], tm[LDS ? 1 : NCH], vm[LDS ? 1 : NCH];
  uint64_t* lds;  // LDS: [3][NCH] of this wave
  int lane;
  __device__ uint64_t get(int which, int h) const {
    if constexpr (LDS) return lds_mask(lds + which * NCH + h);
    else return which == 0 ? pm[h] : which == 1 ? tm[h] : vm[h];
  }
  __device__ void set(int which, int h, uint64_t v) {
    if constexpr (LDS) {
      if (lane == 0) lds[which * NCH + h] = v;
      __builtin_amdgcn_wave_barrier();
    } else {
      (which == 0 ? pm : which == 1 ? tm : vm)[h] = v;
    }
  }
};

// The stop key of node n with its candidates in at most NCH chunks
// (wave-uniform), UINT32_MAX when the reference moves on to the next node.
// NCH is a compile-time bound so the per-chunk masks stay in registers
// (or, LDS, in the wave's LDS slice `lds_masks`).
template <int NCH, bool LDS = false>
__device__ uint32_t victim_candidates(const VictimScan& p, const VictimTables& t, int n, int off, int L, int lane,
                                      const VCand& c0, uint64_t* lds_masks = nullptr) {
  constexpr uint32_t kNone = 0xffffffffu;
  constexpr int PM = 0, TM = 1, VM = 2;
  const int nch = (L + 63) >> 6;  // <= NCH
  ChunkMasks<NCH, LDS> cm;
  cm.lds = lds_masks;
  cm.lane = lane;
  uint64_t any_pm = 0ull;
#pragma unroll
  for (int h = 0; h < NCH; ++h) {
    const uint64_t m = h < nch ? __ballot((h == 0 ? c0 : load_cand(p, t, off, L, h * 64 + lane)).f) : 0ull;
    cm.set(PM, h, m);
    any_pm |= m;
  }
  if (!any_pm) return kNone;  // no preemptee: every fn returns nil
  // the first chunk's gang inputs, requested before the tier walk needs them
  // (one dependent level less on the node's load chain)
  const bool g0 = c0.job >= 0 && t.j_min[c0.job] <= t.j_ready[c0.job] - 1;
  bool panic = false;
  bool victims = false;
  for (int ti = 0; ti < p.n_tiers && !victims && !panic; ++ti) {
    const int fns = p.tier_fns[ti];
    bool any = false;
#pragma unroll
    for (int h = 0; h < NCH; ++h) {
      if (h >= nch) {
        cm.set(TM, h, 0ull);
        continue;
      }
      const VCand c = h == 0 ? c0 : load_cand(p, t, off, L, h * 64 + lane);
      const uint64_t pmh = cm.get(PM, h);
      uint64_t m = pmh;
      if (fns & VP_GANG)  // gang.go:104-124
        m &= __ballot(h == 0 ? g0 : (c.job >= 0 && t.j_min[c.job] <= t.j_ready[c.job] - 1));
      if (fns & (VP_DRF | VP_PROP)) {
        const bool on = (pmh >> lane) & 1ull;
        double xd[3], xp[3];
        for (int d = 0; d < 3; ++d) {
          xd[d] = on && (fns & VP_DRF) ? t.j_alloc[3 * (size_t)c.job + d] : 0.0;
          xp[d] = on && (fns & VP_PROP) ? t.q_alloc[3 * (size_t)c.queue + d] : 0.0;
        }
        bool lpanic = false, vp = false;
        for (int h2 = 0; h2 < h; ++h2)  // preemptees of earlier chunks (all before this lane's k)
          for (uint64_t b = cm.get(PM, h2); b; b &= b - 1) {
            const size_t p2 = (size_t)off + h2 * 64 + __builtin_ctzll(b);  // wave-uniform
            const int2 jq2 = t.c_jq[p2];
            const int32_t j2 = jq2.x;
            const int32_t q2 = jq2.y;
            const double r2[3] = {t.c_req[3 * p2], t.c_req[3 * p2 + 1], t.c_req[3 * p2 + 2]};
            if (on) apply_preemptee(t, fns, j2, q2, r2, false, c.job, c.queue, xd, xp, lpanic, vp);
          }
        for (uint64_t b = pmh; b; b &= b - 1) {  // this chunk, in order, while k2 <= k
          const int l2 = __builtin_ctzll(b);
          const int32_t j2 = rl_i(c.job, l2);
          const int32_t q2 = rl_i(c.queue, l2);
          const double r2[3] = {rl_d(c.r[0], l2), rl_d(c.r[1], l2), rl_d(c.r[2], l2)};
          if (on && l2 <= lane) apply_preemptee(t, fns, j2, q2, r2, l2 == lane, c.job, c.queue, xd, xp, lpanic, vp);
        }
        bool vd = false;
        if ((fns & VP_DRF) && on) {
          const double rs = share3(xd, t.drf_total);
          vd = p.ls < rs || fabs(p.ls - rs) <= 0.000001;
        }
        if (fns & VP_DRF) m &= __ballot(vd);
        if (fns & VP_PROP) m &= __ballot(vp);
        if (__ballot(lpanic) != 0ull) panic = true;
      }
      cm.set(TM, h, m);
      any = any || m != 0ull;
    }
    if (!panic && any) {  // the host passes only the deciding tier (session_plugins.go:59-98)
#pragma unroll
      for (int h = 0; h < NCH; ++h) cm.set(VM, h, cm.get(TM, h));
      victims = true;
    }
  }
  if (panic) return ((uint32_t)n << 1) | 1u;
  if (!victims) return kNone;
  double all[3] = {0.0, 0.0, 0.0};  // validateVictims (preempt.go:242-253), in victims order
#pragma unroll
  for (int h = 0; h < NCH; ++h) {
    const uint64_t vmh = cm.get(VM, h);
    if (!vmh) continue;
    // each lane reads its own candidate's request (one coalesced load), the
    // wave-uniform sum takes them lane by lane in order
    const VCand c = h == 0 ? c0 : load_cand(p, t, off, L, h * 64 + lane);
    for (uint64_t b = vmh; b; b &= b - 1) {
      const int l2 = __builtin_ctzll(b);
      all[0] += rl_d(c.r[0], l2);
      all[1] += rl_d(c.r[1], l2);
      all[2] += rl_d(c.r[2], l2);
    }
  }
  if (res_less3(all, p.req)) return kNone;
  return (uint32_t)n << 1;
}

// NCH_MAX: the chunk bound of this kernel. The main scan takes nodes of up
// to 128 candidates; nodes holding more (rare: pod caps are ~110) are left to
// kbg_victim_big_kernel, whose larger per-chunk state would otherwise raise
// the register budget of every wave.
template <int NCH_MAX>
__device__ __forceinline__ uint32_t victim_node(const VictimScan& p, const VictimTables& t, int row, int lane,
                                uint64_t* lds_masks = nullptr) {
  constexpr uint32_t kNone = 0xffffffffu;
  const int n = p.node_lo + row;
  const int off = t.nt_off[n];
  const int L = t.nt_off[n + 1] - off;
  if (NCH_MAX <= 2 && L > 128) return kNone;  // evaluated by the big-node kernel
  // the first chunk's records are requested before the node's own tests
  // resolve, so the two loads overlap
  const VCand c0 = load_cand(p, t, off, L, lane);
  if (!((t.class_mask[(size_t)p.cls * p.W + (n >> 6)] >> (n & 63)) & 1ull)) return kNone;  // static predicate
  if (t.panic_node[n]) return ((uint32_t)n << 1) | 1u;  // SetNode(nil) inside PredicateFn (predicates.go:122-123)
  if (p.cap_check && t.ntasks[row] >= t.maxtasks[row]) return kNone;  // predicates.go:125-127
  if (NCH_MAX > 2) {  // inlined here: a call would pass the argument structs through scratch
    uint32_t key;
    [[clang::always_inline]] key = victim_candidates<NCH_MAX, true>(p, t, n, off, L, lane, c0, lds_masks);
    return key;
  }
  if (L <= 64) return victim_candidates<1>(p, t, n, off, L, lane, c0);
  return victim_candidates<2>(p, t, n, off, L, lane, c0);
}

// One node per wave, kVictimNodesPerBlock waves per workgroup: every node's
// dependent loads (header -> candidate records -> job tables) are in flight
// at once instead of two nodes back to back per wave. The workgroup writes
// its byte of stop bits and of panic bits (node_lo is 64-node aligned, so a
// shard starts on a byte).
__global__ __launch_bounds__(64 * kVictimBlockWaves) void kbg_victim_kernel(VictimScan p, VictimTables t,
                                                                           uint32_t* __restrict__ stop_bits,
                                                                           uint32_t* __restrict__ panic_bits) {
  __shared__ uint32_t s_stop, s_panic;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_stop = s_panic = 0u;
  __syncthreads();
  const int row = blockIdx.x * kVictimNodesPerBlock + w;
  if (row < p.node_n) {
    const uint32_t key = victim_node<2>(p, t, row, lane);  // wave-uniform
    if (key != 0xffffffffu && lane == 0) {
      atomicOr(&s_stop, 1u << w);
      if (key & 1u) atomicOr(&s_panic, 1u << w);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int byte = (p.node_lo >> 3) + blockIdx.x;
    reinterpret_cast<uint8_t*>(stop_bits)[byte] = (uint8_t)s_stop;
    reinterpret_cast<uint8_t*>(panic_bits)[byte] = (uint8_t)s_panic;
  }
}

// The nodes of the range holding more than 128 candidates, one wave each,
// after the main scan on the same stream: their bits are ORed into the words
// it wrote (several big nodes may share a word).
__global__ __launch_bounds__(256) void kbg_victim_big_kernel(VictimScan p, VictimTables t,
                                                             const int32_t* __restrict__ rows, int32_t n_rows,
                                                             uint32_t* __restrict__ stop_bits,
                                                             uint32_t* __restrict__ panic_bits,
                                                             uint8_t* __restrict__ row_out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n_rows) return;
  __shared__ uint64_t s_masks[4][3 * kVictimChunks];  // each wave's chunk masks (ChunkMasks)
  const int row = rows[i];
  const uint32_t key = victim_node<kVictimChunks>(p, t, row, lane, s_masks[threadIdx.x >> 6]);
  if (row_out) {  // one byte per big node (host-mapped; the host ORs them into its maps): bit 0 stop, bit 1 panic
    if (lane == 0) row_out[i] = key == 0xffffffffu ? 0u : (uint8_t)(1u | ((key & 1u) << 1));
    return;
  }
  if (key == 0xffffffffu || lane != 0) return;
  const int n = p.node_lo + row;
  atomicOr(stop_bits + (n >> 5), 1u << (n & 31));
  if (key & 1u) atomicOr(panic_bits + (n >> 5), 1u << (n & 31));
}

hipError_t launch_victim_big(const VictimScan& p, const VictimTables& t, const int32_t* rows, int32_t n_rows,
                             uint32_t* stop_bits, uint32_t* panic_bits, uint8_t* row_out, hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_victim_big_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, stream, p, t, rows, n_rows, stop_bits,
                     panic_bits, row_out);
  return hipGetLastError();
}

hipError_t launch_victim_scan(const VictimScan& p, const VictimTables& t, uint32_t* stop_bits, uint32_t* panic_bits,
                              hipStream_t stream, hipEvent_t start, hipEvent_t stop) {
  if (p.node_n <= 0) return hipSuccess;
  hipExtLaunchKernelGGL(kbg_victim_kernel, dim3((p.node_n + kVictimNodesPerBlock - 1) / kVictimNodesPerBlock),
                        dim3(64 * kVictimBlockWaves), 0, stream, start, stop, 0, p, t, stop_bits, panic_bits);
  return hipGetLastError();
}

__device__ __forceinline__ void apply_node_delta(const NodeSoA& nd, const NodeDelta& x) {
  nd.idle_cpu[x.node] = x.idle[0];
  nd.idle_mem[x.node] = x.idle[1];
  nd.idle_gpu[x.node] = x.idle[2];
  nd.rel_cpu[x.node] = x.rel[0];
  nd.rel_mem[x.node] = x.rel[1];
  nd.rel_gpu[x.node] = x.rel[2];
  nd.ntasks[x.node] = x.ntasks;
  nd.maxtasks[x.node] = x.maxtasks;
}

__device__ __forceinline__ void apply_state_delta(const VictimTables& t, const StateDelta& x) {
  switch (x.kind) {
    case 0: t.c_run[x.index] = (uint8_t)(x.v[0] != 0.0); break;
    case 1: t.j_ready[x.index] = (int32_t)x.v[0]; break;
    case 2:
      for (int k = 0; k < 3; ++k) t.j_alloc[3 * (size_t)x.index + k] = x.v[k];
      break;
    case 3:
      for (int k = 0; k < 3; ++k) t.q_alloc[3 * (size_t)x.index + k] = x.v[k];
      break;
  }
}

__global__ __launch_bounds__(256) void kbg_victim_prep_kernel(NodeSoA nd, VictimTables t,
                                                              const NodeDelta* __restrict__ d, int32_t nn,
                                                              const StateDelta* __restrict__ sd, int32_t ns) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nn) apply_node_delta(nd, d[i]);
  else if (i < nn + ns) apply_state_delta(t, sd[i - nn]);
}

__global__ __launch_bounds__(64) void kbg_victim_prep_inline_kernel(NodeSoA nd, VictimTables t, VictimPrepArgs a) {
  for (int i = threadIdx.x; i < a.nn + a.ns; i += 64) {
    if (i < a.nn) apply_node_delta(nd, a.nd[i]);
    else apply_state_delta(t, a.sd[i - a.nn]);
  }
}

hipError_t launch_victim_prep_inline(const NodeSoA& n, const VictimTables& t, const VictimPrepArgs& a,
                                     hipStream_t stream) {
  if (a.nn + a.ns <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_victim_prep_inline_kernel, dim3(1), dim3(64), 0, stream, n, t, a);
  return hipGetLastError();
}

hipError_t launch_victim_prep(const NodeSoA& n, const VictimTables& t, const NodeDelta* nd, int32_t n_nodes,
                              const StateDelta* sd, int32_t n_state, hipStream_t stream) {
  const int32_t tot = n_nodes + n_state;
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_victim_prep_kernel, dim3((tot + 255) / 256), dim3(256), 0, stream, n, t, nd, n_nodes, sd,
                     n_state);
  return hipGetLastError();
}

// ------------------------------------------------------------- static mask
// One lane = one (class, node) pair; vendor predicates.go:807-850 (selector +
// required node affinity), predicates.go:105-110 (unschedulable),
// predicates.go:1489-1517 (taints), with requirement validity already folded
// into the program on the host.
__device__ bool eval_req(const StaticTables& t, const ReqProg& r, int node) {
  switch (r.kind) {
    case REQ_FALSE: return false;
    case REQ_TRUE: return true;
    case REQ_ALL:
    case REQ_ANY:
    case REQ_NONE: {
      bool any = false, all = true;
      for (int w = 0; w < t.label_words; ++w) {
        const uint64_t m = t.mask_pool[r.mask_off + w];
        const uint64_t b = t.label_bits[(size_t)w * t.n_nodes + node] & m;
        any |= b != 0ull;
        all &= b == m;
      }
      return r.kind == REQ_ALL ? all : (r.kind == REQ_ANY ? any : !any);
    }
    case REQ_GT:
    case REQ_LT: {
      const size_t k = (size_t)r.col * t.n_nodes + node;
      if (!t.num_ok[k]) return false;
      return r.kind == REQ_GT ? t.num_vals[k] > r.value : t.num_vals[k] < r.value;
    }
    case REQ_NAME_EQ: return (int64_t)t.name_id[node] == r.value;
    case REQ_NAME_NE: return (int64_t)t.name_id[node] != r.value;
  }
  return false;
}

__global__ __launch_bounds__(256) void kbg_mask_kernel(StaticTables t, int32_t W, uint64_t* __restrict__ class_mask) {
  const int lane = threadIdx.x & 63;
  const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int cls = blockIdx.y;
  if (chunk >= W) return;
  const int node = chunk * 64 + lane;
  bool ok = false;
  if (node < t.n_nodes) {
    const ClassProg c = t.classes[cls];
    const uint8_t fl = t.node_flags[node];
    if (c.always) {
      ok = true;
    } else if (fl & NF_NIL) {
      ok = true;  // SetNode(nil) panics before any check: the host reports it when reached
    } else if (fl & (NF_UNSCHED | NF_DEAD)) {
      ok = false;
    } else {
      ok = true;
      if (c.sel_req >= 0) ok = eval_req(t, t.reqs[c.sel_req], node);
      if (ok && c.has_affinity) {
        bool any_term = false;
        for (int i = 0; i < c.term_len && !any_term; ++i) {
          const TermProg tp = t.terms[c.term_off + i];
          bool all = true;
          for (int j = 0; j < tp.req_len && all; ++j) all = eval_req(t, t.reqs[tp.req_off + j], node);
          any_term = all;
        }
        ok = any_term;
      }
      if (ok) {
        for (int w = 0; w < t.taint_words; ++w) {
          const uint64_t nb = t.taint_bits[(size_t)w * t.n_nodes + node];
          if (nb & ~t.tol_pool[c.tol_off + w]) { ok = false; break; }
        }
      }
    }
  }
  const uint64_t m = __ballot(ok);
  if (lane == 0) class_mask[(size_t)cls * W + chunk] = m;
}

hipError_t launch_build_class_mask(const StaticTables& t, int32_t n_classes, int32_t W, uint64_t* class_mask,
                                   hipStream_t stream) {
  if (n_classes <= 0 || W <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_mask_kernel, dim3((W + 3) / 4, n_classes), dim3(256), 0, stream, t, W, class_mask);
  return hipGetLastError();
}

}  // namespace kbg
