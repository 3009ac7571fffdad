// The transports of a node-axis sharded session (kbg_comm.hpp) and the
// communicator part of the C ABI (kbgpu.h kbg_comm_*).
#include "kbg_comm.hpp"

#include <errno.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "kbg_session.hpp"

namespace kbg {
namespace {

using clk = std::chrono::steady_clock;

double comm_limit_ms() {
  static const double limit = [] {
    const char* e = getenv("KBG_COMM_TIMEOUT_MS");
    return e && atof(e) > 0 ? atof(e) : 300000.0;
  }();
  return limit;
}

// ------------------------------------------------------------------ RCCL
struct RcclColl final : Coll {
  ncclComm_t nccl = nullptr;
  std::atomic<bool> aborted{false};
  ~RcclColl() override {
    if (nccl && !aborted.load()) (void)ncclCommDestroy(nccl);  // (an aborted one is freed by the abort)
  }
  kbg_status rc(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return KBG_OK;
    err = std::string(what) + ": " + ncclGetErrorString(r);
    return KBG_E_RCCL;
  }
  kbg_status bcast(uint32_t* d, size_t n, hipStream_t s) override {
    return rc(ncclBroadcast(d, d, n, ncclUint32, 0, nccl, s), "ncclBroadcast");
  }
  kbg_status allreduce(const uint32_t* din, uint32_t* dout, size_t n, CollOp op, hipStream_t s) override {
    const ncclRedOp_t o = op == kCollSum ? ncclSum : op == kCollMin ? ncclMin : ncclMax;
    return rc(ncclAllReduce(din, dout, n, ncclUint32, o, nccl, s), "ncclAllReduce");
  }
  kbg_status allgather(const void* din, void* dout, size_t bytes, hipStream_t s) override {
    return rc(ncclAllGather(din, dout, bytes, ncclUint8, nccl, s), "ncclAllGather");
  }
  void group_start() override { (void)ncclGroupStart(); }
  kbg_status group_end() override { return rc(ncclGroupEnd(), "ncclGroupEnd"); }
  kbg_status health() override {
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      err = std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae);
      return KBG_E_RCCL;
    }
    return KBG_OK;
  }
  void abort() override {
    bool was = false;
    if (aborted.compare_exchange_strong(was, true)) (void)ncclCommAbort(nccl);
  }
  kbg_status ranks(int32_t* n, int32_t* r) override {
    int nn = 0, rr = 0;
    if (kbg_status st = rc(ncclCommCount(nccl, &nn), "ncclCommCount"); st != KBG_OK) return st;
    if (kbg_status st = rc(ncclCommUserRank(nccl, &rr), "ncclCommUserRank"); st != KBG_OK) return st;
    *n = nn;
    *r = rr;
    return KBG_OK;
  }
  const char* name() const override { return "rccl"; }
};

// ------------------------------------------------------- host shared memory
// One segment per clique: a header page, then one staging slot of kChunk
// bytes per rank. A collective moves its payload in chunks: each rank copies
// its part of a chunk from the device into its slot, a barrier, each rank
// reads what it needs from the slots (the root's, or all of them) into its
// own device buffer, a barrier before the slots are reused. Every wait polls
// the abort flag, the peers' liveness (a process that exited, or a rank that
// destroyed its communicator) and the time limit KBG_COMM_TIMEOUT_MS, so a
// failing rank cannot hang its peers.
constexpr size_t kHeaderBytes = 4096;
constexpr size_t kChunk = size_t(4) << 20;
constexpr uint32_t kAbsent = 0, kJoined = 1, kLeft = 2;

struct ShmHeader {
  std::atomic<int32_t> n_ranks;  // 0 until the first rank sets it
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> aborted;  // 1 + the rank that aborted it (0: live)
  std::atomic<uint32_t> bar_count;
  std::atomic<uint32_t> bar_gen;
  std::atomic<int32_t> pid[kHostCommMaxRanks];
  std::atomic<uint32_t> state[kHostCommMaxRanks];
  std::atomic<uint64_t> ops[kHostCommMaxRanks];  // collectives each rank entered (a failure names the lag)
};
static_assert(sizeof(ShmHeader) <= kHeaderBytes, "header page");
static_assert(std::atomic<uint32_t>::is_always_lock_free && std::atomic<uint64_t>::is_always_lock_free,
              "process-shared atomics");

// false once `pid` has exited (a zombie counts as exited: its parent may not
// have reaped it while it waits on this very rank)
bool pid_alive(int32_t pid) {
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[512];
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* p = strrchr(buf, ')');  // the state follows the command name
  if (!p || p[1] != ' ') return true;
  return p[2] != 'Z' && p[2] != 'X' && p[2] != 'x';
}

struct HostColl final : Coll {
  int32_t R = 1, me = 0;
  int fd = -1;
  void* base = nullptr;
  size_t bytes = 0;
  ShmHeader* hdr = nullptr;
  bool aborted_local = false;
  bool host_memory = false;  // developer tools: the "device" buffers are host memory (CPU self-test)
  int64_t exit_after = 0;  // KBG_HOST_COMM_EXIT_AFTER: fault injection (tests), exit at this collective
  int64_t ops = 0;
  std::vector<uint32_t> acc;  // allreduce result of one chunk

  ~HostColl() override {
    if (hdr) {
      hdr->state[me].store(kLeft, std::memory_order_release);
      munmap(base, bytes);
    }
    if (fd >= 0) close(fd);
  }
  char* slot(int32_t r) { return static_cast<char*>(base) + kHeaderBytes + (size_t)r * kChunk; }

  kbg_status failed(const std::string& m) {
    err = m;
    return KBG_E_RCCL;
  }
  // a peer that exited or left (-1: none)
  int32_t gone_peer() const {
    for (int32_t r = 0; r < R; ++r) {
      if (r == me) continue;
      const uint32_t s = hdr->state[r].load(std::memory_order_acquire);
      if (s == kLeft) return r;
      if (s == kJoined && !pid_alive(hdr->pid[r].load(std::memory_order_relaxed))) return r;
    }
    return -1;
  }
  // polls `done` until it holds; fails on abort, a gone peer or the time limit
  template <class F>
  kbg_status wait_for(F done, const char* what) {
    const auto t0 = clk::now();
    auto checked = t0;
    for (uint64_t spin = 0;; ++spin) {
      if (done()) return KBG_OK;
      if (const uint32_t by = hdr->aborted.load(std::memory_order_acquire)) {
        aborted_local = true;
        return failed("host communicator: rank " + std::to_string((int)by - 1) + " aborted it (rank " +
                      std::to_string(me) + " waited in " + what + ")");
      }
      if ((spin & 63) == 0) {
        const auto t = clk::now();
        if (t - checked > std::chrono::milliseconds(2)) {
          checked = t;
          const int32_t g = gone_peer();
          if (g >= 0 && !done()) {
            abort();
            char m[256];
            snprintf(m, sizeof m,
                     "host communicator: rank %d exited or left while rank %d waited in %s (collective %lld of rank "
                     "%d, %lld of rank %d)",
                     g, me, what, (long long)hdr->ops[me].load(), me, (long long)hdr->ops[g].load(), g);
            return failed(m);
          }
        }
        if (std::chrono::duration<double, std::milli>(t - t0).count() > comm_limit_ms()) {
          abort();
          return failed(std::string("host communicator: no progress for KBG_COMM_TIMEOUT_MS in ") + what);
        }
      }
      if (spin > 20000)
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      else if (spin > 200)
        sched_yield();
    }
  }
  kbg_status barrier(const char* what) {
    const uint32_t g = hdr->bar_gen.load(std::memory_order_acquire);
    if (hdr->bar_count.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)R - 1) {
      hdr->bar_count.store(0, std::memory_order_relaxed);
      hdr->bar_gen.fetch_add(1, std::memory_order_release);
      return KBG_OK;
    }
    return wait_for([&] { return hdr->bar_gen.load(std::memory_order_acquire) != g; }, what);
  }
  kbg_status enter() {
    if (const uint32_t by = hdr->aborted.load(std::memory_order_acquire))
      return failed("host communicator: rank " + std::to_string((int)by - 1) + " aborted it");
    if (aborted_local) return failed("host communicator: aborted");
    hdr->ops[me].fetch_add(1, std::memory_order_relaxed);
    if (exit_after > 0 && ++ops >= exit_after) _exit(3);  // fault injection: this rank dies mid-protocol
    return KBG_OK;
  }
  kbg_status hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return KBG_OK;
    abort();  // the peers are in (or about to enter) this collective
    err = std::string("host communicator: ") + what + ": " + hipGetErrorString(e);
    return KBG_E_HIP;
  }
  kbg_status sync(hipStream_t s) { return host_memory ? KBG_OK : hip(hipStreamSynchronize(s), "hipStreamSynchronize"); }
  kbg_status d2h(void* h, const void* d, size_t n, hipStream_t s) {
    if (host_memory) return std::memcpy(h, d, n), KBG_OK;
    if (kbg_status st = hip(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s), "hipMemcpyAsync"); st != KBG_OK)
      return st;
    return hip(hipStreamSynchronize(s), "hipStreamSynchronize");
  }
  kbg_status h2d(void* d, const void* h, size_t n, hipStream_t s) {
    if (host_memory) return std::memmove(d, h, n), KBG_OK;
    if (kbg_status st = hip(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s), "hipMemcpyAsync"); st != KBG_OK)
      return st;
    return hip(hipStreamSynchronize(s), "hipStreamSynchronize");
  }

  kbg_status bcast(uint32_t* d, size_t n, hipStream_t s) override {
    if (kbg_status st = enter(); st != KBG_OK) return st;
    if (kbg_status st = sync(s); st != KBG_OK) return st;
    char* p = reinterpret_cast<char*>(d);
    for (size_t o = 0, b = n * 4; o < b; o += kChunk) {
      const size_t c = std::min(kChunk, b - o);
      if (me == 0)
        if (kbg_status st = d2h(slot(0), p + o, c, s); st != KBG_OK) return st;
      if (kbg_status st = barrier("broadcast"); st != KBG_OK) return st;
      if (me != 0)
        if (kbg_status st = h2d(p + o, slot(0), c, s); st != KBG_OK) return st;
      if (kbg_status st = barrier("broadcast"); st != KBG_OK) return st;
    }
    return KBG_OK;
  }
  kbg_status allreduce(const uint32_t* din, uint32_t* dout, size_t n, CollOp op, hipStream_t s) override {
    if (kbg_status st = enter(); st != KBG_OK) return st;
    if (kbg_status st = sync(s); st != KBG_OK) return st;
    const size_t per = kChunk / 4;
    for (size_t o = 0; o < n; o += per) {
      const size_t c = std::min(per, n - o);
      if (kbg_status st = d2h(slot(me), din + o, c * 4, s); st != KBG_OK) return st;
      if (kbg_status st = barrier("all-reduce"); st != KBG_OK) return st;
      acc.assign(reinterpret_cast<const uint32_t*>(slot(0)), reinterpret_cast<const uint32_t*>(slot(0)) + c);
      for (int32_t r = 1; r < R; ++r) {
        const uint32_t* v = reinterpret_cast<const uint32_t*>(slot(r));
        if (op == kCollSum)
          for (size_t i = 0; i < c; ++i) acc[i] += v[i];
        else if (op == kCollMin)
          for (size_t i = 0; i < c; ++i) acc[i] = std::min(acc[i], v[i]);
        else
          for (size_t i = 0; i < c; ++i) acc[i] = std::max(acc[i], v[i]);
      }
      if (kbg_status st = barrier("all-reduce"); st != KBG_OK) return st;
      if (kbg_status st = h2d(dout + o, acc.data(), c * 4, s); st != KBG_OK) return st;
    }
    return KBG_OK;
  }
  kbg_status allgather(const void* din, void* dout, size_t bytes_per, hipStream_t s) override {
    if (kbg_status st = enter(); st != KBG_OK) return st;
    if (kbg_status st = sync(s); st != KBG_OK) return st;
    const char* in = static_cast<const char*>(din);
    char* out = static_cast<char*>(dout);
    for (size_t o = 0; o < bytes_per; o += kChunk) {
      const size_t c = std::min(kChunk, bytes_per - o);
      if (kbg_status st = d2h(slot(me), in + o, c, s); st != KBG_OK) return st;
      if (kbg_status st = barrier("all-gather"); st != KBG_OK) return st;
      for (int32_t r = 0; r < R; ++r)
        if (kbg_status st = h2d(out + (size_t)r * bytes_per + o, slot(r), c, s); st != KBG_OK) return st;
      if (kbg_status st = barrier("all-gather"); st != KBG_OK) return st;
    }
    return KBG_OK;
  }
  kbg_status health() override {
    if (aborted_local || hdr->aborted.load(std::memory_order_acquire))
      return failed("host communicator: a rank aborted it");
    return KBG_OK;
  }
  void abort() override {
    aborted_local = true;
    uint32_t live = 0;
    if (hdr) hdr->aborted.compare_exchange_strong(live, (uint32_t)me + 1, std::memory_order_acq_rel);
  }
  kbg_status ranks(int32_t* n, int32_t* r) override {
    *n = (int32_t)hdr->joined.load(std::memory_order_acquire);
    *r = me;
    return KBG_OK;
  }
  const char* name() const override { return "host"; }
};

}  // namespace

std::unique_ptr<Coll> make_rccl_coll(const uint8_t id[KBG_COMM_ID_BYTES], int32_t n_ranks, int32_t rank,
                                     kbg_status* st, std::string* err) {
  static_assert(sizeof(ncclUniqueId) == KBG_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  std::unique_ptr<RcclColl> c(new (std::nothrow) RcclColl());
  if (!c) {
    *st = KBG_E_NOMEM;
    *err = "comm";
    return nullptr;
  }
  const ncclResult_t r = ncclCommInitRank(&c->nccl, n_ranks, uid, rank);
  if (r != ncclSuccess) {
    c->nccl = nullptr;
    *st = KBG_E_RCCL;
    *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    return nullptr;
  }
  *st = KBG_OK;
  return c;
}

std::unique_ptr<Coll> make_host_coll(const char* name, int32_t n_ranks, int32_t rank, kbg_status* st,
                                     std::string* err, bool host_memory) {
  auto bad = [&](kbg_status code, const std::string& m) -> std::unique_ptr<Coll> {
    *st = code;
    *err = m;
    return nullptr;
  };
  const size_t len = strlen(name);
  if (len == 0 || len > 200) return bad(KBG_E_INVALID, "host communicator name: 1..200 characters");
  for (size_t i = 0; i < len; ++i) {
    const char ch = name[i];
    if (!(isalnum((unsigned char)ch) || ch == '.' || ch == '_' || ch == '-'))
      return bad(KBG_E_INVALID, "host communicator name: letters, digits, '.', '_', '-'");
  }
  if (n_ranks > kHostCommMaxRanks) return bad(KBG_E_INVALID, "host communicator: at most 16 ranks");
  const std::string path = std::string("/kbg.") + name;
  std::unique_ptr<HostColl> c(new (std::nothrow) HostColl());
  if (!c) return bad(KBG_E_NOMEM, "comm");
  c->R = n_ranks;
  c->me = rank;
  c->host_memory = host_memory;
  if (const char* e = getenv("KBG_HOST_COMM_EXIT_AFTER")) c->exit_after = atoll(e);
  c->fd = shm_open(path.c_str(), O_CREAT | O_RDWR, 0600);
  if (c->fd < 0) return bad(KBG_E_RCCL, "shm_open " + path + ": " + strerror(errno));
  c->bytes = kHeaderBytes + (size_t)kHostCommMaxRanks * kChunk;  // (pages are only backed once touched)
  struct stat sb;
  if (fstat(c->fd, &sb) != 0) return bad(KBG_E_RCCL, std::string("fstat: ") + strerror(errno));
  if ((size_t)sb.st_size < c->bytes && ftruncate(c->fd, (off_t)c->bytes) != 0)
    return bad(KBG_E_RCCL, std::string("ftruncate: ") + strerror(errno));
  c->base = mmap(nullptr, c->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, c->fd, 0);
  if (c->base == MAP_FAILED) {
    c->base = nullptr;
    return bad(KBG_E_RCCL, std::string("mmap: ") + strerror(errno));
  }
  ShmHeader* h = static_cast<ShmHeader*>(c->base);  // a new segment is zero: every field's initial state
  int32_t want = 0;
  if (!h->n_ranks.compare_exchange_strong(want, n_ranks) && want != n_ranks) {
    munmap(c->base, c->bytes);
    c->base = nullptr;
    return bad(KBG_E_INVALID, "host communicator: the ranks disagree on n_ranks");
  }
  uint32_t s0 = kAbsent;
  if (!h->state[rank].compare_exchange_strong(s0, kJoined)) {
    munmap(c->base, c->bytes);
    c->base = nullptr;
    return bad(KBG_E_INVALID, "host communicator: rank already joined (a stale segment of that name: use a fresh name)");
  }
  h->pid[rank].store((int32_t)getpid(), std::memory_order_relaxed);
  c->hdr = h;
  h->joined.fetch_add(1, std::memory_order_acq_rel);
  if (kbg_status s = c->wait_for([&] { return h->joined.load(std::memory_order_acquire) == (uint32_t)n_ranks; },
                                 "the join");
      s != KBG_OK)
    return bad(s, c->err);
  if (kbg_status s = c->barrier("the join"); s != KBG_OK) return bad(s, c->err);
  if (rank == 0) shm_unlink(path.c_str());  // every rank has it mapped: nothing is left behind in /dev/shm
  *st = KBG_OK;
  return c;
}

}  // namespace kbg

using kbg::fail_with;

extern "C" {

kbg_status kbg_comm_unique_id(uint8_t out[KBG_COMM_ID_BYTES]) {
  if (!out) return fail_with(KBG_E_INVALID, "null out");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail_with(KBG_E_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, sizeof(id));
  return KBG_OK;
}

static kbg_status comm_make(int32_t n_ranks, int32_t rank, int32_t device, kbg_comm** out,
                            std::unique_ptr<kbg::Coll> (*make)(const void*, int32_t, int32_t, kbg_status*, std::string*),
                            const void* arg) {
  if (!out) return fail_with(KBG_E_INVALID, "null argument");
  *out = nullptr;
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail_with(KBG_E_INVALID, "rank / n_ranks");
  if (hipSetDevice(device) != hipSuccess) return fail_with(KBG_E_HIP, "hipSetDevice failed");
  kbg_comm* c = new (std::nothrow) kbg_comm();
  if (!c) return fail_with(KBG_E_NOMEM, "comm");
  kbg_status st = KBG_OK;
  std::string err;
  c->coll = make(arg, n_ranks, rank, &st, &err);
  if (!c->coll) {
    delete c;
    return fail_with(st, err);
  }
  c->n_ranks = n_ranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return KBG_OK;
}

kbg_status kbg_comm_init(const uint8_t id[KBG_COMM_ID_BYTES], int32_t n_ranks, int32_t rank, int32_t device,
                         kbg_comm** out) {
  if (!id) return fail_with(KBG_E_INVALID, "null argument");
  return comm_make(n_ranks, rank, device, out,
                   [](const void* a, int32_t n, int32_t r, kbg_status* st, std::string* e) {
                     return kbg::make_rccl_coll(static_cast<const uint8_t*>(a), n, r, st, e);
                   },
                   id);
}

kbg_status kbg_comm_init_host(const char* name, int32_t n_ranks, int32_t rank, int32_t device, kbg_comm** out) {
  if (!name) return fail_with(KBG_E_INVALID, "null argument");
  return comm_make(n_ranks, rank, device, out,
                   [](const void* a, int32_t n, int32_t r, kbg_status* st, std::string* e) {
                     return kbg::make_host_coll(static_cast<const char*>(a), n, r, st, e);
                   },
                   name);
}

kbg_status kbg_comm_ranks(const kbg_comm* c, int32_t* n_ranks, int32_t* rank) {
  if (!c || !n_ranks || !rank) return fail_with(KBG_E_INVALID, "null argument");
  if (!c->coll || c->aborted.load()) return fail_with(KBG_E_RCCL, "the communicator is not live");
  if (kbg_status st = c->coll->ranks(n_ranks, rank); st != KBG_OK) return fail_with(st, c->coll->err);
  return KBG_OK;
}

int32_t kbg_comm_transport(const kbg_comm* c) {
  if (!c || !c->coll) return -1;
  return std::strcmp(c->coll->name(), "rccl") == 0 ? KBG_COMM_RCCL : KBG_COMM_HOST;
}

void kbg_comm_destroy(kbg_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  c->coll.reset();
  delete c;
}

}  // extern "C"
