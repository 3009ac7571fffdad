// Communicators of a node-axis sharded session: the clique of
// ranks a sharded session exchanges its scans over, and the collectives the
// protocols call. Two transports behind one interface:
//   RCCL  — one rank per GPU, every collective enqueued on the session's HIP
//           stream (kbg_comm_init; the multi-GPU path, xGMI between GPUs);
//   host  — ranks are processes of one host, the collectives run through a
//           POSIX shared-memory segment with a device<->host copy on each side
//           (kbg_comm_init_host). The ranks may share one GPU, so the
//           multi-rank protocols run across real processes on a one-GPU box.
// Every rank calls the same collectives in the same order; a protocol never
// knows which transport it is on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <string>

#include "../../include/kbgpu.h"

namespace kbg {

enum CollOp : int32_t { kCollSum = 0, kCollMin = 1, kCollMax = 2 };

struct Coll {
  virtual ~Coll() = default;
  // in place from rank 0: n 32-bit words at device address d
  virtual kbg_status bcast(uint32_t* d, size_t n, hipStream_t s) = 0;
  // element-wise over the ranks: n 32-bit unsigned words, din -> dout (may alias)
  virtual kbg_status allreduce(const uint32_t* din, uint32_t* dout, size_t n, CollOp op, hipStream_t s) = 0;
  // rank r's `bytes` at din land at dout + r * bytes on every rank (din may be that slice)
  virtual kbg_status allgather(const void* din, void* dout, size_t bytes, hipStream_t s) = 0;
  // a group of collectives issued together (RCCL fuses them; the host transport runs them in order)
  virtual void group_start() {}
  virtual kbg_status group_end() { return KBG_OK; }
  // KBG_OK while the clique is healthy; polled by a rank waiting on its stream
  virtual kbg_status health() = 0;
  // stop every rank's collectives: the peers' pending and later calls fail
  virtual void abort() = 0;
  // the clique as the transport itself counts it
  virtual kbg_status ranks(int32_t* n, int32_t* r) = 0;
  virtual const char* name() const = 0;
  std::string err;  // the message of the last failure
};

// RCCL communicator (kbg_comm.cpp)
std::unique_ptr<Coll> make_rccl_coll(const uint8_t id[KBG_COMM_ID_BYTES], int32_t n_ranks, int32_t rank,
                                     kbg_status* st, std::string* err);
// shared-memory communicator of processes on one host (kbg_comm.cpp);
// host_memory: the buffers handed to the collectives are host memory
// (developer tools' CPU self-test; the library always passes device memory)
std::unique_ptr<Coll> make_host_coll(const char* name, int32_t n_ranks, int32_t rank, kbg_status* st,
                                     std::string* err, bool host_memory = false);
constexpr int32_t kHostCommMaxRanks = 16;

}  // namespace kbg

// A clique of node-axis shards (kbgpu.h). `coll` is null for a communicator
// made by a developer tool whose ranks are threads of one process with their
// own transport (tools/engine_bench.cpp).
struct kbg_comm {
  std::unique_ptr<kbg::Coll> coll;
  int32_t n_ranks = 1, rank = 0, device = 0;
  // abort ran (a local failure inside a collective protocol, an asynchronous
  // transport error, or a peer that stopped answering): every later call on a
  // session of this communicator fails with KBG_E_RCCL
  std::atomic<bool> aborted{false};
};
