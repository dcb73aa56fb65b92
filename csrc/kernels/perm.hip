// perm.hip — PERMUTATION encoding (placeholder until the PERMUTATION kernels land).
#include "pga/ops.hpp"
namespace pga {
uint32_t perm_launch(int, const GenArgs&, unsigned long long*, hipStream_t) {
  throw std::runtime_error("PERMUTATION encoding: not built yet");
}
}  // namespace pga
