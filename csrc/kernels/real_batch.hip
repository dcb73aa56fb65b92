// real_batch.hip — batched-island launches of the REAL two-phase generation
// kernel (real_gen_tp_batch, real_dev.hpp): up to kRealMaxBatch islands of the
// same shape, operators and built-in objective on one device, island =
// blockIdx.y, ONE launch per generation for all of them — small islands are
// launch-bound on separate streams and share the process's hardware queues.
// Rotated objectives run their islands on streams.
//
// Reference: MAX_POPULATIONS = 10 islands per solver (include/pga.h:44), whose
// *_all loops run one after another (src/pga.cu:272-276, :327-331).
#include <hip/hip_runtime.h>

#include "pga/ops.hpp"
#include "pga/real_dev.hpp"

namespace pga {
namespace {

template <int GS, int OBJ>
uint32_t batch_go(RealBatch& b, uint32_t n, uint64_t S, hipStream_t s) {
  const void* k = (const void*)real_gen_tp_batch<GS, OBJ>;
  const TpGeom t = tp_geometry(S, n, k, 64 / GS, 7);  // the device split between the islands
  for (uint32_t i = 0; i < n; ++i) b.a[i].tp_unit = t.unit;
  hipLaunchKernelGGL((real_gen_tp_batch<GS, OBJ>), dim3(t.grid, n), t.block, t.lds, s, b);
  PGA_HIP_CHECK(hipGetLastError());
  return t.grid;
}

template <int GS>
uint32_t batch_obj(RealBatch& b, uint32_t n, uint64_t S, hipStream_t s) {
  switch (b.a[0].objective) {
    case OBJ_SPHERE: return batch_go<GS, OBJ_SPHERE>(b, n, S, s);
    case OBJ_RASTRIGIN: return batch_go<GS, OBJ_RASTRIGIN>(b, n, S, s);
    case OBJ_ROSENBROCK: return batch_go<GS, OBJ_ROSENBROCK>(b, n, S, s);
    case OBJ_ACKLEY: return batch_go<GS, OBJ_ACKLEY>(b, n, S, s);
    case OBJ_GRIEWANK: return batch_go<GS, OBJ_GRIEWANK>(b, n, S, s);
    case OBJ_SCHWEFEL: return batch_go<GS, OBJ_SCHWEFEL>(b, n, S, s);
    case OBJ_LINEAR: return batch_go<GS, OBJ_LINEAR>(b, n, S, s);
    case OBJ_KNAPSACK_REAL: return batch_go<GS, OBJ_KNAPSACK_REAL>(b, n, S, s);
    default: return 0;
  }
}

}  // namespace

uint32_t real_max_batch() { return kRealMaxBatch; }

uint32_t real_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s) {
  if (n == 0 || n > kRealMaxBatch) return 0;
  const GenArgs& a0 = args[0];
  RealBatch b;
  for (uint32_t i = 0; i < n; ++i) {
    const GenArgs& a = args[i];
    // every island: the two-phase kernel's conditions (for the whole batch's
    // population), the same shape, objective and parameters
    if (!real_tp_batchable(a, n) || a.S != a0.S || a.chunks != a0.chunks || a.objective != a0.objective ||
        a.obj_i != a0.obj_i)
      return 0;
    b.a[i] = a;
    b.parts[i] = parts[i];
  }
  switch (group_size(a0.chunks)) {
    case 1: return batch_obj<1>(b, n, a0.S, s);
    case 2: return batch_obj<2>(b, n, a0.S, s);
    case 4: return batch_obj<4>(b, n, a0.S, s);
    case 8: return batch_obj<8>(b, n, a0.S, s);
    case 16: return batch_obj<16>(b, n, a0.S, s);
    case 32: return batch_obj<32>(b, n, a0.S, s);
    default: return batch_obj<64>(b, n, a0.S, s);
  }
}

}  // namespace pga
