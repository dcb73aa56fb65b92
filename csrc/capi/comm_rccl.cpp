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
    streams_.resize(comms_.size(), nullptr);
  }
  ~RcclComm() override {
    for (auto* v : {&ready_, &done_})
      for (hipEvent_t e : *v)
        if (e) (void)hipEventDestroy(e);
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

  void set_fault(int every, int mode) override {
    if (mode != 0 && mode != 3) throw std::invalid_argument("RCCL fault mode must be 0 (none) or 3 (withhold sends)");
    every_ = every;
    mode_ = mode;
    self_exchange = true;
  }

  // The emigrants are packed on each rank's compute stream; the transfers
  // run on the rank's own communication stream, which waits for them.  The
  // compute stream is NOT ordered after the transfer here: wait() decides.
  void exchange(const std::vector<Xfer>& plan, std::vector<LocalRank>& local) override {
    if (aborted_) throw std::runtime_error("RCCL communicator was aborted");
    ++count_;
    const bool withhold = mode_ == 3 && every_ > 0 && count_ % (uint64_t)every_ == 0;
    for (LocalRank& l : local) {
      const size_t j = slot_of(l.rank);
      PGA_COMM_HIP(hipSetDevice(l.device));
      if (!streams_[j]) {
        PGA_COMM_HIP(hipStreamCreateWithFlags(&streams_[j], hipStreamNonBlocking));
        PGA_COMM_HIP(hipEventCreateWithFlags(&ready_[j], hipEventDisableTiming));
        PGA_COMM_HIP(hipEventCreateWithFlags(&done_[j], hipEventDisableTiming));
      }
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
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        bool done = true;
        for (const LocalRank& l : local) {
          const hipError_t q = hipEventQuery(done_[slot_of(l.rank)]);
          if (q == hipErrorNotReady) done = false;
          else if (q != hipSuccess) return abort_all();
        }
        if (async_error()) return abort_all();
        if (done) break;
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > timeout_s) return abort_all();
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    } else if (async_error()) {
      return abort_all();
    }
    for (LocalRank& l : local) {
      PGA_COMM_HIP(hipSetDevice(l.device));
      PGA_COMM_HIP(hipStreamWaitEvent(l.stream, done_[slot_of(l.rank)], 0));
    }
    return true;
  }

  std::vector<float> allgather(const std::vector<LocalRank>& local, const std::vector<float>& mine) override {
    std::vector<float> all(n_, 0.f);
    std::vector<float*> dbuf(local.size(), nullptr);
    for (size_t i = 0; i < local.size(); ++i) {
      PGA_COMM_HIP(hipSetDevice(local[i].device));
      PGA_COMM_HIP(hipMalloc(&dbuf[i], sizeof(float) * (n_ + 1)));
      PGA_COMM_HIP(hipMemcpyAsync(dbuf[i] + n_, &mine[i], sizeof(float), hipMemcpyHostToDevice, local[i].stream));
    }
    {
      Group g;
      for (size_t i = 0; i < local.size(); ++i)
        nccl_check(ncclAllGather(dbuf[i] + n_, dbuf[i], 1, ncclFloat32, comm_of(local[i].rank), local[i].stream),
                   "ncclAllGather");
    }
    for (size_t i = 0; i < local.size(); ++i) {
      PGA_COMM_HIP(hipSetDevice(local[i].device));
      PGA_COMM_HIP(hipMemcpyAsync(all.data(), dbuf[i], sizeof(float) * n_, hipMemcpyDeviceToHost, local[i].stream));
      PGA_COMM_HIP(hipStreamSynchronize(local[i].stream));
      PGA_COMM_HIP(hipFree(dbuf[i]));
    }
    return all;
  }

 private:
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
  std::vector<hipEvent_t> ready_, done_;
  std::vector<hipStream_t> streams_;  // one communication stream per local rank
  int n_;
  bool all_;
  bool aborted_ = false;
  uint64_t count_ = 0;
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
