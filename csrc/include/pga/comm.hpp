// comm.hpp — inter-island communication of the C API island model.
//
// The reference claims "CUDA GPUs+MPI" (README.md:4) but ships no
// communication code; its migration entry points are empty
// (src/pga.cu:368-374, :393-395).  Here migration is a
// list of row transfers (a *plan*) executed by one of three transports:
//
//   RCCL, one process per GPU     ncclCommInitRank; every process posts the
//                                 transfers of its own rank (grouped
//                                 ncclSend/ncclRecv over xGMI)
//   RCCL, one process, n GPUs     ncclCommInitAll; the driver posts the
//                                 transfers of all ranks in ONE group
//   loopback                      in-process ranks (CPU or GPU islands),
//                                 plain copies; the test transport, with
//                                 fault injection (drop / corrupt)
//
// Plans are computed identically on every rank from (topology, epoch, seed),
// so no rank ever has to tell another whom it talks to.  Transfers are
// asynchronous.  RCCL posts them on a dedicated communication stream per
// rank that first waits for the emigrants packed on the compute stream;
// Comm::wait() then either makes the compute stream wait for the transfer
// (success) or, on a timeout / asynchronous error, calls ncclCommAbort at
// once and leaves the compute stream untouched, so a dead peer can never
// stall the generations that follow (the islands continue degraded).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#define PGA_COMM_HIP(expr)                                                                     \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace pga {

enum Topology : int32_t {
  TOPO_RING = 0,        // rank r -> r+1
  TOPO_RANDOM = 1,      // a fresh random ring per epoch (shared Philox draw)
  TOPO_ALL_TO_ALL = 2,  // every rank sends k/(n-1) emigrants to every other rank
};

// rows [src_off, src_off+n) of src's send buffer -> rows [dst_off, ...) of dst's receive buffer
struct Xfer {
  int src, dst;
  uint32_t src_off, dst_off, n;
};

// migrants per rank actually exchanged for k requested (all-to-all rounds to a multiple of n-1)
uint32_t plan_migrants(int topology, int nranks, uint32_t k);
std::vector<Xfer> migration_plan(int topology, int nranks, uint32_t k, uint64_t seed, uint32_t epoch);

// one rank's staging buffers (device memory for GPU islands, host for CPU ones)
struct LocalRank {
  int rank = 0;
  int device = -1;
  hipStream_t stream = nullptr;
  size_t row_bytes = 0;
  void* send_rows = nullptr;
  float* send_scores = nullptr;
  void* recv_rows = nullptr;
  float* recv_scores = nullptr;
};

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int size() const = 0;
  virtual const char* name() const = 0;
  // true when the caller drives every rank (InitAll / loopback)
  virtual bool drives_all_ranks() const = 0;
  // enqueue the plan's transfers that touch `local`
  virtual void exchange(const std::vector<Xfer>& plan, std::vector<LocalRank>& local) = 0;
  // host-side completion check of the last exchange; false: failed or timed
  // out (the communicator is then unusable and the islands run on alone)
  virtual bool wait(std::vector<LocalRank>& local, double timeout_s) = 0;
  // All-gather of `count` 32-bit words per rank (count <= kGatherMaxWords):
  // local[i] contributes mine[i * count ..]; `all` receives every rank's words
  // in rank order.  Bounded like wait(): with timeout_s > 0 the host polls the
  // completion against the deadline and on expiry or an asynchronous error
  // aborts the communicator and returns false (the caller degrades); with
  // timeout_s <= 0 it blocks until the collective completes.  Persistent
  // staging: no allocation or free per call.
  static constexpr uint32_t kGatherMaxWords = 16;
  virtual bool allgather(const std::vector<LocalRank>& local, const std::vector<uint32_t>& mine, uint32_t count,
                         std::vector<uint32_t>& all, double timeout_s) = 0;
  // `bytes` of rank `root`'s bufs[i] (the local rank's buffer: device memory
  // for GPU ranks, host for CPU ones) copied to every rank's buffer; the
  // buffers are written on the local ranks' compute streams beforehand and
  // read there afterwards.  Same deadline semantics as allgather.
  virtual bool broadcast(const std::vector<LocalRank>& local, const std::vector<void*>& bufs, size_t bytes, int root,
                         double timeout_s) = 0;
  // test-only fault injection (pga_comm_set_fault): loopback drops (1) or
  // corrupts (2) every `every`-th exchange; RCCL withholds this process's
  // sends (3) of every `every`-th exchange, so its receives can never
  // complete, or stalls (4) every `every`-th all-gather behind a receive
  // that never completes.  Mode 0 disarms it.
  virtual void set_fault(int every, int mode) = 0;
  // the stream this communicator moves `l`'s data on (RCCL: the rank's own
  // communication stream, concurrent with the compute stream), or nullptr
  // when the transport has none.  Work enqueued there runs in order with the
  // transfers: the engine island model packs its emigrants and re-scores its
  // immigrants on it, beside the generation kernel.
  virtual hipStream_t transport_stream(const LocalRank& l) {
    (void)l;
    return nullptr;
  }
  // test-only (pga_comm_set_self_exchange): a 1-rank communicator normally
  // skips migration; with this set it exchanges with itself, which runs the
  // real transport (and the fault injection) on one GPU
  bool self_exchange = false;
  uint64_t bytes_sent = 0;
};

// ---- RCCL ----
int rccl_unique_id(char out[128]);
std::shared_ptr<Comm> rccl_comm_rank(int nranks, int rank, const char id[128], int device);
std::shared_ptr<Comm> rccl_comm_all(const std::vector<int>& devices);

// ---- loopback ----
// fault injection: every `every`-th exchange (1-based count) is dropped
// (mode 1: nothing arrives and wait() reports the failure) or corrupted
// (mode 2: the received scores are overwritten with +3e38, which re-scoring
// must undo)
std::shared_ptr<Comm> loopback_comm(int nranks);

}  // namespace pga
