// comm_rccl.cpp — RCCL backend of the C API island model (one process per
// GPU, xGMI point-to-point links).  The python layer uses torch.distributed
// (backend "nccl" = RCCL) instead; both speak the same migration protocol:
// a ring of ranks, top-k emigrants out, worst-k replaced.
//
// Reference: the original claims "CUDA GPUs+MPI" (README.md:4) but contains no
// communication code at all.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "pga/comm.hpp"

namespace pga {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
}  // namespace

struct RcclComm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  float* dscratch = nullptr;
};

int rccl_unique_id(char out[128]) {
  static_assert(sizeof(ncclUniqueId) <= 128, "unique id too large");
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memset(out, 0, 128);
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

RcclComm* rccl_init(int nranks, int rank, const char id[128], int device) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("bad rank / nranks");
  PGA_COMM_HIP(hipSetDevice(device));
  auto* c = new RcclComm;
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  try {
    nccl_check(ncclCommInitRank(&c->comm, nranks, uid, rank), "ncclCommInitRank");
    PGA_COMM_HIP(hipMalloc(&c->dscratch, 64));
  } catch (...) {
    delete c;
    throw;
  }
  return c;
}

void rccl_destroy(RcclComm* c) {
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->dscratch) (void)hipFree(c->dscratch);
  delete c;
}

int rccl_rank(const RcclComm* c) { return c ? c->rank : 0; }
int rccl_size(const RcclComm* c) { return c ? c->nranks : 1; }

// send `bytes` to rank+1, receive the same from rank-1 (grouped, one link each way)
void rccl_ring_exchange(RcclComm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
  if (!c || c->nranks == 1) return;
  const int to = (c->rank + 1) % c->nranks, from = (c->rank + c->nranks - 1) % c->nranks;
  nccl_check(ncclGroupStart(), "ncclGroupStart");
  nccl_check(ncclSend(send, bytes, ncclUint8, to, c->comm, s), "ncclSend");
  nccl_check(ncclRecv(recv, bytes, ncclUint8, from, c->comm, s), "ncclRecv");
  nccl_check(ncclGroupEnd(), "ncclGroupEnd");
}

// all-gather one float per rank (host in/out, synchronises the stream)
void rccl_allgather_f32(RcclComm* c, float v, float* out, hipStream_t s) {
  if (!c || c->nranks == 1) {
    out[0] = v;
    return;
  }
  float* d = nullptr;
  PGA_COMM_HIP(hipMalloc(&d, sizeof(float) * (c->nranks + 1)));
  PGA_COMM_HIP(hipMemcpyAsync(d + c->nranks, &v, sizeof(float), hipMemcpyHostToDevice, s));
  nccl_check(ncclAllGather(d + c->nranks, d, 1, ncclFloat32, c->comm, s), "ncclAllGather");
  PGA_COMM_HIP(hipMemcpyAsync(out, d, sizeof(float) * c->nranks, hipMemcpyDeviceToHost, s));
  PGA_COMM_HIP(hipStreamSynchronize(s));
  PGA_COMM_HIP(hipFree(d));
}

}  // namespace pga
