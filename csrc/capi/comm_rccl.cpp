// comm_rccl.cpp — RCCL transports of the C API island model (pga/comm.hpp).
//
// MI355X shape: the 8 GPUs of a node are fully connected by xGMI (7
// point-to-point links per GPU).  A ring migration moves k rows over ONE link
// per direction; all-to-all spreads k/(n-1) rows over all 7, which is what a
// large migration wants.  Every transfer of an epoch is posted inside one
// ncclGroupStart/End, so RCCL schedules the sends and receives of all peers
// (and, in the one-process ncclCommInitAll mode, of all local GPUs) together.
// The python layer uses torch.distributed (backend "nccl" = RCCL) instead and
// speaks the same protocol (libpga_amd/parallel/islands.py).
//
// Reference: the original claims "CUDA GPUs+MPI" (README.md:4) but contains no
// communication code at all.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <thread>

#include "pga/comm.hpp"

namespace pga {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

struct Group {
  Group() { nccl_check(ncclGroupStart(), "ncclGroupStart"); }
  ~Group() noexcept(false) {
    const ncclResult_t r = ncclGroupEnd();
    if (!std::uncaught_exceptions()) nccl_check(r, "ncclGroupEnd");  // never throw while unwinding
  }
};

class RcclComm final : public Comm {
 public:
  // comms_[i] is the communicator of local rank ranks_[i] (one entry per process
  // in InitRank mode, one per GPU in InitAll mode)
  RcclComm(std::vector<ncclComm_t> comms, std::vector<int> ranks, int nranks, bool all)
      : comms_(std::move(comms)), ranks_(std::move(ranks)), n_(nranks), all_(all) {
    ready_.resize(comms_.size(), nullptr);
    done_.resize(comms_.size(), nullptr);
    ag_done_.resize(comms_.size(), nullptr);
    streams_.resize(comms_.size(), nullptr);
    ag_dev_.resize(comms_.size(), nullptr);
    ag_host_.resize(comms_.size(), nullptr);
  }
  ~RcclComm() override {
    for (auto* v : {&ready_, &done_, &ag_done_})
      for (hipEvent_t e : *v)
        if (e) (void)hipEventDestroy(e);
    for (uint32_t* b : ag_dev_)
      if (b) (void)hipFree(b);
    for (uint32_t* b : ag_host_)
      if (b) (void)hipHostFree(b);
    if (!aborted_)
      for (ncclComm_t c : comms_)
        if (c) (void)ncclCommDestroy(c);
    // after an abort the communication streams may still hold the aborted
    // kernels' completions; they are released with the device context
    if (!aborted_)
      for (hipStream_t st : streams_)
        if (st) (void)hipStreamDestroy(st);
  }
  int size() const override { return n_; }
  const char* name() const override { return all_ ? "rccl-all" : "rccl"; }
  bool drives_all_ranks() const override { return all_; }
  hipStream_t transport_stream(const LocalRank& l) override { return streams_[ensure_stream(l)]; }

  void set_fault(int every, int mode) override {
    if (mode != 0 && mode != 3 && mode != 4)
      throw std::invalid_argument("RCCL fault mode must be 0 (none), 3 (withhold sends) or 4 (stall all-gathers)");
    every_ = every;
    mode_ = mode;
  }

  // The emigrants are packed on each rank's compute stream; the transfers
  // run on the rank's own communication stream, which waits for them.  The
  // compute stream is NOT ordered after the transfer here: wait() decides.
  void exchange(const std::vector<Xfer>& plan, std::vector<LocalRank>& local) override {
    if (aborted_) throw std::runtime_error("RCCL communicator was aborted");
    ++count_;
    const bool withhold = mode_ == 3 && every_ > 0 && count_ % (uint64_t)every_ == 0;
    for (LocalRank& l : local) {
      const size_t j = ensure_stream(l);
      PGA_COMM_HIP(hipEventRecord(ready_[j], l.stream));
      PGA_COMM_HIP(hipStreamWaitEvent(streams_[j], ready_[j], 0));
    }
    {
      Group g;
      for (LocalRank& l : local) {
        ncclComm_t c = comm_of(l.rank);
        hipStream_t cs = streams_[slot_of(l.rank)];
        const size_t rb = l.row_bytes;
        for (const Xfer& x : plan) {
          if (x.src == l.rank && !withhold) {
            nccl_check(ncclSend((const char*)l.send_rows + rb * x.src_off, rb * x.n, ncclUint8, x.dst, c, cs),
                       "ncclSend");
            nccl_check(ncclSend(l.send_scores + x.src_off, x.n, ncclFloat32, x.dst, c, cs), "ncclSend");
            bytes_sent += (rb + 4) * x.n;
          }
          if (x.dst == l.rank) {
            nccl_check(ncclRecv((char*)l.recv_rows + rb * x.dst_off, rb * x.n, ncclUint8, x.src, c, cs), "ncclRecv");
            nccl_check(ncclRecv(l.recv_scores + x.dst_off, x.n, ncclFloat32, x.src, c, cs), "ncclRecv");
          }
        }
      }
    }
    for (LocalRank& l : local) {
      const size_t j = slot_of(l.rank);
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipEventRecord(done_[j], streams_[j]));
    }
  }

  // timeout_s > 0: poll the transfers' completion events and RCCL's
  // asynchronous error state on the host until the deadline.  Success: the
  // compute streams wait for the transfers (the received rows are consumed
  // there).  Failure or expiry: ncclCommAbort now — it releases RCCL kernels
  // blocked on a dead peer — and the compute streams are left alone.
  // timeout_s <= 0: no host wait at all; only errors RCCL already reported
  // are seen, and the compute streams are ordered after the transfers.
  bool wait(std::vector<LocalRank>& local, double timeout_s) override {
    if (aborted_) return false;
    if (timeout_s > 0) {
      if (!poll(local, done_, timeout_s)) return abort_all();
    } else if (async_error()) {
      return abort_all();
    }
    for (LocalRank& l : local) {
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipStreamWaitEvent(l.stream, done_[slot_of(l.rank)], 0));
    }
    return true;
  }

  // The words travel host -> pinned staging -> device -> ncclAllGather ->
  // device -> pinned staging, all on the rank's communication stream (nothing
  // waits for the compute stream, so a gather never queues behind the
  // generation kernels), then the host polls the completion like wait().
  bool allgather(const std::vector<LocalRank>& local, const std::vector<uint32_t>& mine, uint32_t count,
                 std::vector<uint32_t>& all, double timeout_s) override {
    if (count == 0 || count > kGatherMaxWords) throw std::invalid_argument("allgather: bad word count");
    if (aborted_) return false;
    const size_t words = (size_t)n_ * count;
    ++ag_count_;
    const bool stall = mode_ == 4 && every_ > 0 && ag_count_ % (uint64_t)every_ == 0;
    for (size_t i = 0; i < local.size(); ++i) {
      const size_t j = ensure_stream(local[i]);
      if (!ag_dev_[j]) {
        PGA_COMM_HIP(hipMalloc(&ag_dev_[j], 4ull * (n_ + 2) * kGatherMaxWords));
        PGA_COMM_HIP(hipHostMalloc(&ag_host_[j], 4ull * (n_ + 1) * kGatherMaxWords, hipHostMallocDefault));
      }
      std::memcpy(ag_host_[j] + words, &mine[i * count], 4ull * count);
      PGA_COMM_HIP(hipMemcpyAsync(ag_dev_[j] + words, ag_host_[j] + words, 4ull * count, hipMemcpyHostToDevice,
                                  streams_[j]));
    }
    if (stall) {
      // test fault: a receive nobody sends, ahead of the all-gather on the
      // communication stream -- a peer that died between two check points
      Group g;
      for (const LocalRank& l : local) {
        const size_t j = slot_of(l.rank);
        nccl_check(ncclRecv(ag_dev_[j] + (n_ + 1) * kGatherMaxWords, 1, ncclUint32, ranks_[j], comms_[j], streams_[j]),
                   "ncclRecv");
      }
    }
    {
      Group g;
      for (const LocalRank& l : local) {
        const size_t j = slot_of(l.rank);
        nccl_check(ncclAllGather(ag_dev_[j] + words, ag_dev_[j], count, ncclUint32, comms_[j], streams_[j]),
                   "ncclAllGather");
      }
    }
    for (const LocalRank& l : local) {
      const size_t j = slot_of(l.rank);
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipMemcpyAsync(ag_host_[j], ag_dev_[j], 4ull * words, hipMemcpyDeviceToHost, streams_[j]));
      PGA_COMM_HIP(hipEventRecord(ag_done_[j], streams_[j]));
    }
    if (!poll(local, ag_done_, timeout_s)) return abort_all();
    all.assign(ag_host_[slot_of(local[0].rank)], ag_host_[slot_of(local[0].rank)] + words);
    return true;
  }

  bool broadcast(const std::vector<LocalRank>& local, const std::vector<void*>& bufs, size_t bytes, int root,
                 double timeout_s) override {
    if (aborted_) return false;
    for (const LocalRank& l : local) {
      const size_t j = ensure_stream(l);
      PGA_COMM_HIP(hipEventRecord(ready_[j], l.stream));
      PGA_COMM_HIP(hipStreamWaitEvent(streams_[j], ready_[j], 0));
    }
    {
      Group g;
      for (size_t i = 0; i < local.size(); ++i) {
        const size_t j = slot_of(local[i].rank);
        nccl_check(ncclBroadcast(bufs[i], bufs[i], bytes, ncclUint8, root, comms_[j], streams_[j]), "ncclBroadcast");
      }
    }
    for (const LocalRank& l : local) {
      const size_t j = slot_of(l.rank);
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipEventRecord(done_[j], streams_[j]));
    }
    if (!poll(local, done_, timeout_s)) return abort_all();
    for (const LocalRank& l : local) {
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipStreamWaitEvent(l.stream, done_[slot_of(l.rank)], 0));
    }
    return true;
  }

 private:
  // the local rank's communication stream and events (created on first use)
  size_t ensure_stream(const LocalRank& l) {
    const size_t j = slot_of(l.rank);
    PGA_COMM_HIP(hipSetDevice(l.device));
    if (!streams_[j]) {
      PGA_COMM_HIP(hipStreamCreateWithFlags(&streams_[j], hipStreamNonBlocking));
      PGA_COMM_HIP(hipEventCreateWithFlags(&ready_[j], hipEventDisableTiming));
      PGA_COMM_HIP(hipEventCreateWithFlags(&done_[j], hipEventDisableTiming));
      PGA_COMM_HIP(hipEventCreateWithFlags(&ag_done_[j], hipEventDisableTiming));
    }
    return j;
  }
  // completion of ev[slot] for every local rank.  timeout_s > 0: host poll
  // with the deadline, RCCL's asynchronous error state checked every round;
  // otherwise a blocking wait.  false: failed or expired (caller aborts).
  bool poll(const std::vector<LocalRank>& local, const std::vector<hipEvent_t>& ev, double timeout_s) {
    if (timeout_s <= 0) {
      for (const LocalRank& l : local)
        if (hipEventSynchronize(ev[slot_of(l.rank)]) != hipSuccess) return false;
      return !async_error();
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      bool done = true;
      for (const LocalRank& l : local) {
        const hipError_t q = hipEventQuery(ev[slot_of(l.rank)]);
        if (q == hipErrorNotReady) done = false;
        else if (q != hipSuccess) return false;
      }
      if (async_error()) return false;
      if (done) return true;
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (dt > timeout_s) return false;
      // spin the first 2 ms (a transfer usually lands within a generation:
      // the next launch should follow it within microseconds, and a sleep
      // costs a scheduler tick), then back off
      if (dt > 2e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  size_t slot_of(int rank) const {
    for (size_t i = 0; i < ranks_.size(); ++i)
      if (ranks_[i] == rank) return i;
    throw std::runtime_error("rank " + std::to_string(rank) + " is not local to this communicator");
  }
  ncclComm_t comm_of(int rank) const { return comms_[slot_of(rank)]; }
  bool async_error() const {
    for (ncclComm_t c : comms_) {
      ncclResult_t st = ncclSuccess;
      if (ncclCommGetAsyncError(c, &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) return true;
    }
    return false;
  }
  bool abort_all() {
    if (!aborted_)
      for (ncclComm_t c : comms_)
        if (c) (void)ncclCommAbort(c);
    aborted_ = true;
    return false;
  }

  std::vector<ncclComm_t> comms_;
  std::vector<int> ranks_;
  std::vector<hipEvent_t> ready_, done_, ag_done_;
  std::vector<hipStream_t> streams_;  // one communication stream per local rank
  std::vector<uint32_t*> ag_dev_, ag_host_;  // all-gather staging: (n + 1) x kGatherMaxWords words
  int n_;
  bool all_;
  bool aborted_ = false;
  uint64_t count_ = 0, ag_count_ = 0;
  int every_ = 0, mode_ = 0;
};

}  // namespace

int rccl_unique_id(char out[128]) {
  static_assert(sizeof(ncclUniqueId) <= 128, "unique id too large");
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memset(out, 0, 128);
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

std::shared_ptr<Comm> rccl_comm_rank(int nranks, int rank, const char id[128], int device) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("bad rank / nranks");
  PGA_COMM_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  nccl_check(ncclCommInitRank(&c, nranks, uid, rank), "ncclCommInitRank");
  return std::make_shared<RcclComm>(std::vector<ncclComm_t>{c}, std::vector<int>{rank}, nranks, false);
}

std::shared_ptr<Comm> rccl_comm_all(const std::vector<int>& devices) {
  const int n = (int)devices.size();
  if (n < 1) throw std::invalid_argument("rccl_comm_all: no devices");
  std::vector<ncclComm_t> comms(n, nullptr);
  nccl_check(ncclCommInitAll(comms.data(), n, devices.data()), "ncclCommInitAll");
  std::vector<int> ranks(n);
  for (int i = 0; i < n; ++i) ranks[i] = i;
  return std::make_shared<RcclComm>(std::move(comms), std::move(ranks), n, true);
}

}  // namespace pga
