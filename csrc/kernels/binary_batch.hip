// binary_batch.hip — batched-island launches of the hot BINARY generation
// kernel (binary_gen_tp_batch, binary_dev.hpp): up to kMaxBatch islands of the
// same shape and operators on one device, island = blockIdx.y, ONE launch per
// generation for all of them.  Instantiated for the integer objectives the
// two-phase kernel tournaments on exact u16 keys (ONEMAX, LEADING_ONES, TRAP);
// other objectives and shapes run their islands on concurrent streams.
//
// Reference: MAX_POPULATIONS = 10 islands per solver (include/pga.h:44),
// *_all loops run them one after another (src/pga.cu:272-276, :327-331).
#include <hip/hip_runtime.h>

#include "pga/binary_dev.hpp"
#include "pga/ops.hpp"

namespace pga {
namespace {

template <int GS, int OBJ>
uint32_t batch_go(GenBatch& b, uint32_t n, uint64_t S, bool full, bool dense, hipStream_t s) {
  const void* k = full ? (dense ? (const void*)binary_gen_tp_batch<GS, OBJ, true, true>
                                : (const void*)binary_gen_tp_batch<GS, OBJ, true, false>)
                       : (dense ? (const void*)binary_gen_tp_batch<GS, OBJ, false, true>
                                : (const void*)binary_gen_tp_batch<GS, OBJ, false, false>);
  // the device split between the islands (tp_geometry)
  const TpGeom t = tp_geometry(S, n, k, 64 / GS);
  for (uint32_t i = 0; i < n; ++i) {
    b.a[i].tp_unit = t.unit;
    b.a[i].tp_pool_units = b.a[i].tp_pool ? tp_pool_units(t, S) : 0u;
    b.a[i].key_hist = nullptr;  // no fused histogram in the batched launch (no LDS for it)
  }
  const dim3 grid(t.grid, n);
  if (full) {
    if (dense) hipLaunchKernelGGL((binary_gen_tp_batch<GS, OBJ, true, true>), grid, t.block, t.lds, s, b);
    else hipLaunchKernelGGL((binary_gen_tp_batch<GS, OBJ, true, false>), grid, t.block, t.lds, s, b);
  } else {
    if (dense) hipLaunchKernelGGL((binary_gen_tp_batch<GS, OBJ, false, true>), grid, t.block, t.lds, s, b);
    else hipLaunchKernelGGL((binary_gen_tp_batch<GS, OBJ, false, false>), grid, t.block, t.lds, s, b);
  }
  PGA_HIP_CHECK(hipGetLastError());
  return t.grid;
}

template <int GS>
uint32_t batch_obj(int obj, GenBatch& b, uint32_t n, uint64_t S, bool full, bool dense, hipStream_t s) {
  switch (obj) {
    case OBJ_ONEMAX: return batch_go<GS, OBJ_ONEMAX>(b, n, S, full, dense, s);
    case OBJ_LEADING_ONES: return batch_go<GS, OBJ_LEADING_ONES>(b, n, S, full, dense, s);
    default: return batch_go<GS, OBJ_TRAP>(b, n, S, full, dense, s);
  }
}

}  // namespace

uint32_t binary_max_batch() { return kMaxBatch; }

uint32_t binary_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s) {
  if (n == 0 || n > kMaxBatch) return 0;
  const GenArgs& a0 = args[0];
  if (a0.objective != OBJ_ONEMAX && a0.objective != OBJ_LEADING_ONES && a0.objective != OBJ_TRAP) return 0;
  uint32_t gs = 0;
  bool full = false, dense = false;
  GenBatch b;
  for (uint32_t i = 0; i < n; ++i) {
    const GenArgs& a = args[i];
    uint32_t g2 = 0;
    bool f2 = false, d2 = false;
    // every island: the hot kernel's conditions, the same variant, shape and objective
    if (!binary_tp_plan(a, g2, f2, d2) || a.key_cur == nullptr || a.S != a0.S || a.chunks != a0.chunks ||
        a.objective != a0.objective)
      return 0;
    if (i == 0) {
      gs = g2;
      full = f2;
      dense = d2;
    } else if (g2 != gs || f2 != full || d2 != dense) {
      return 0;
    }
    b.a[i] = a;
    b.parts[i] = parts[i];
  }
  switch (gs) {
    case 1: return batch_obj<1>(a0.objective, b, n, a0.S, full, dense, s);
    case 2: return batch_obj<2>(a0.objective, b, n, a0.S, full, dense, s);
    case 4: return batch_obj<4>(a0.objective, b, n, a0.S, full, dense, s);
    case 8: return batch_obj<8>(a0.objective, b, n, a0.S, full, dense, s);
    case 16: return batch_obj<16>(a0.objective, b, n, a0.S, full, dense, s);
    case 32: return batch_obj<32>(a0.objective, b, n, a0.S, full, dense, s);
    default: return batch_obj<64>(a0.objective, b, n, a0.S, full, dense, s);
  }
}

}  // namespace pga
