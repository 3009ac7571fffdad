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
//                     nodes held in registers; tasks are wave-uniform (scalar
//                     loads); results leave as 64-bit ballots.
// kbg_select_kernel — per task, the first M feasible node indices in
//                     ssn.Nodes order (first-fit = min index), with
//                     the Allocate/Pipeline kind of each.
// kbg_mask_kernel   — session-open static predicate masks (class x node bits).
// kbg_apply_kernel  — NodeInfo.AddTask deltas committed by the host.
//
// fp64 is compared with the reference's own expression; the file is compiled
// with -ffp-contract=off so nothing is fused.
#include <hip/hip_ext.h>

#include "kbg_device.hpp"

namespace kbg {

__device__ __forceinline__ bool le(double r, double a, double mn) {
  // (r < a || |a - r| < min)  — resource_info.go:142-146, one dimension
  return r < a || fabs(a - r) < mn;
}

// ------------------------------------------------------------------ scan
constexpr int kScanWaves = 4;          // waves per workgroup (256 threads)
constexpr int kScanTasksPerBlock = 64; // task evaluations per workgroup

// The row loop: lane = node, rows broadcast from LDS; REL_ZERO selects the
// per-row precomputed Releasing fit (all nodes of the wave have Releasing 0).
template <bool REL_ZERO>
__device__ __forceinline__ void scan_rows(const double (*s_req)[4], const uint64_t* s_mask, int nt_blk, int lane,
                                          int node_ok, double ic, double im, double ig, double rc, double rm,
                                          double rg, uint64_t rz_rows, uint64_t* keep_f, uint64_t* keep_i) {
  // Rows are processed 4 at a time with no remainder loop (ballots are
  // convergent, so a runtime-count remainder would block unrolling); rows past
  // nt_blk read stale LDS and their ballots are never stored.
  for (int j0 = 0; j0 < nt_blk; j0 += 4) {
#pragma unroll
  for (int j = j0; j < j0 + 4; ++j) {
    const double q0 = s_req[j][0];
    const double q1 = s_req[j][1];
    const double q2 = s_req[j][2];
    const uint64_t mw = s_mask[j];
    const int sbit = (int)((mw >> lane) & 1ull);
    const int ifit = (int)le(q0, ic, kMinMilliCPU) & (int)le(q1, im, kMinMemory) & (int)le(q2, ig, kMinMilliGPU);
    int rfit;
    if (REL_ZERO) {
      rfit = (int)((rz_rows >> j) & 1ull);
    } else {
      rfit = (int)le(q0, rc, kMinMilliCPU) & (int)le(q1, rm, kMinMemory) & (int)le(q2, rg, kMinMilliGPU);
    }
    const int ok = node_ok & sbit;
    const uint64_t fm = __ballot((ok & (ifit | rfit)) != 0);
    const uint64_t imk = __ballot((ok & ifit) != 0);
    if (lane == j) {
      *keep_f = fm;
      *keep_i = imk;
    }
  }
  }
}

__global__ __launch_bounds__(256) void kbg_scan_kernel(NodeSoA nd, ScanGeom geo,
                                                       const uint64_t* __restrict__ class_mask,
                                                       const TaskRec* __restrict__ tasks, int32_t n_tasks,
                                                       int32_t cap_check, uint64_t* __restrict__ out) {
  // Evaluation rows of this workgroup, staged once in LDS and read back as
  // same-address broadcasts; per wave, the class-mask word of each row for
  // the wave's 64-node chunk.
  __shared__ double s_req[kScanTasksPerBlock][4];
  __shared__ uint64_t s_mask[kScanWaves][kScanTasksPerBlock];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int rel = blockIdx.x * kScanWaves + wave;  // word relative to chunk_lo
  const int chunk = geo.chunk_lo + rel;            // global 64-node word
  const bool live = rel < geo.n_chunks && chunk < geo.W;
  const int t0 = blockIdx.y * kScanTasksPerBlock;
  const int nt_blk = min(n_tasks - t0, kScanTasksPerBlock);
  if (threadIdx.x < nt_blk) {
    const TaskRec tr = tasks[t0 + threadIdx.x];
    s_req[threadIdx.x][0] = tr.req[0];
    s_req[threadIdx.x][1] = tr.req[1];
    s_req[threadIdx.x][2] = tr.req[2];
  }
  if (lane < nt_blk && live) s_mask[wave][lane] = class_mask[(size_t)tasks[t0 + lane].cls * geo.W + chunk];
  __syncthreads();
  if (!live) return;  // wave-uniform exit (after the barrier); words past W are never read
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
  const int node_ok = (int)valid & ((int)!cap_check | (int)(nt < mt));
  // Releasing is usually zero on every node of the wave; then the Releasing
  // fit of a row is LessEqual(req, 0) for every lane — the same expression,
  // evaluated once per row (lane j for row j) instead of once per node.
  const bool rel_zero_wave = __ballot(!(rc == 0.0 && rm == 0.0 && rg == 0.0)) == 0ull;
  uint64_t rz_rows = 0;
  if (rel_zero_wave) {
    bool rz = false;
    if (lane < nt_blk) {
      const double q0 = s_req[lane][0], q1 = s_req[lane][1], q2 = s_req[lane][2];
      rz = ((int)le(q0, 0.0, kMinMilliCPU) & (int)le(q1, 0.0, kMinMemory) & (int)le(q2, 0.0, kMinMilliGPU)) != 0;
    }
    rz_rows = __ballot(rz);
  }
  uint64_t keep_f = 0, keep_i = 0;  // lane j keeps the ballots of row t0+j
  if (rel_zero_wave)
    scan_rows<true>(s_req, s_mask[wave], nt_blk, lane, node_ok, ic, im, ig, rc, rm, rg, rz_rows, &keep_f, &keep_i);
  else
    scan_rows<false>(s_req, s_mask[wave], nt_blk, lane, node_ok, ic, im, ig, rc, rm, rg, rz_rows, &keep_f, &keep_i);
  if (lane < nt_blk) {
    // [slot][plane][row][Wl] (kbg_device.hpp ScanGeom)
    const int slot = rel / geo.Wl, w = rel - slot * geo.Wl;
    const size_t plane = (size_t)n_tasks * geo.Wl;
    uint64_t* o = out + (size_t)slot * 2 * plane + (size_t)(t0 + lane) * geo.Wl + w;
    o[0] = keep_f;
    o[plane] = keep_i;
  }
}

hipError_t launch_scan(const NodeSoA& n, const ScanGeom& g, const uint64_t* class_mask, const TaskRec* tasks,
                       int32_t n_tasks, int32_t cap_check, uint64_t* out, hipStream_t stream, hipEvent_t start,
                       hipEvent_t stop) {
  if (n_tasks <= 0 || g.n_chunks <= 0) return hipSuccess;
  dim3 grid((g.n_chunks + kScanWaves - 1) / kScanWaves, (n_tasks + kScanTasksPerBlock - 1) / kScanTasksPerBlock);
  hipExtLaunchKernelGGL(kbg_scan_kernel, grid, dim3(64 * kScanWaves), 0, stream, start, stop, 0, n, g, class_mask,
                        tasks, n_tasks, cap_check, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- select
// One wave per row walks the row's words in global node order (shard slots in
// rank order = ascending node index), so the candidates come out first-fit.
__global__ __launch_bounds__(256) void kbg_select_kernel(const uint64_t* __restrict__ bits, int32_t W, int32_t Wl,
                                                         int32_t n_rows, const uint32_t* __restrict__ cap_off,
                                                         uint32_t* __restrict__ out_cand,
                                                         uint32_t* __restrict__ out_count) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_rows) return;
  const size_t plane = (size_t)n_rows * Wl;
  const uint64_t* row = bits + (size_t)t * Wl;
  const int M = (int)(cap_off[t + 1] - cap_off[t]);
  uint32_t* cand = out_cand + cap_off[t];
  int found = 0;
  int base = 0;
  for (; base < W && found < M; base += 64) {
    const int c = base + lane;
    uint64_t f = 0ull, iw = 0ull;
    if (c < W) {
      const int slot = c / Wl;
      const uint64_t* p = row + (size_t)slot * 2 * plane + (c - slot * Wl);
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
    const bool complete = base >= W && found <= M;
    const uint32_t cnt = (uint32_t)(found < M ? found : M);
    out_count[t] = cnt | (complete ? 0u : kCountIncompleteBit);
  }
}

hipError_t launch_select(const uint64_t* bits, int32_t W, int32_t Wl, int32_t n_rows, const uint32_t* cap_off,
                         uint32_t* out_cand, uint32_t* out_count, hipStream_t stream, hipEvent_t start,
                         hipEvent_t stop) {
  if (n_rows <= 0) return hipSuccess;
  hipExtLaunchKernelGGL(kbg_select_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, stream, start, stop, 0, bits, W, Wl,
                        n_rows, cap_off, out_cand, out_count);
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
}

hipError_t launch_apply(const NodeSoA& n, const NodeDelta* deltas, int32_t n_deltas, hipStream_t stream) {
  if (n_deltas <= 0) return hipSuccess;
  hipLaunchKernelGGL(kbg_apply_kernel, dim3((n_deltas + 255) / 256), dim3(256), 0, stream, n, deltas, n_deltas);
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
