// real.hip — f32 REAL encoding (placeholder until the REAL kernels land).
#include "pga/ops.hpp"
namespace pga {
uint32_t real_launch(int, const GenArgs&, unsigned long long*, hipStream_t) {
  throw std::runtime_error("REAL encoding: not built yet");
}
}  // namespace pga
