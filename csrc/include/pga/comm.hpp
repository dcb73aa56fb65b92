// comm.hpp — inter-rank communication used by the C API island model.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#define PGA_COMM_HIP(expr)                                                                     \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace pga {

struct RcclComm;
int rccl_unique_id(char out[128]);
RcclComm* rccl_init(int nranks, int rank, const char id[128], int device);
void rccl_destroy(RcclComm* c);
int rccl_rank(const RcclComm* c);
int rccl_size(const RcclComm* c);
void rccl_ring_exchange(RcclComm* c, const void* send, void* recv, size_t bytes, hipStream_t s);
void rccl_allgather_f32(RcclComm* c, float v, float* out, hipStream_t s);

}  // namespace pga
