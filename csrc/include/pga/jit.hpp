// jit.hpp — user objectives compiled at runtime with hipRTC (SURVEY.md §7.1
// src/jit, §7.4: "keep the compat path correct but make templated/JIT
// objectives the fast path").
//
// The user writes one device function over a decoded row,
//   BINARY       float NAME(const unsigned int* words, unsigned int nbits, const float* data)
//   REAL         float NAME(const float* genes, unsigned int n, const float* data)
//   PERMUTATION  float NAME(const unsigned short* perm, unsigned int n, const float* data)
// and the engine compiles it for gfx950 into a batched evaluation kernel
// (one work-item per individual, per-block best partials in the engine's
// packed format) that runs right after every fused generation kernel.  Unlike
// the reference's device function pointers (include/pga.h:46, src/pga.cu:
// 250-262) the call is direct and inlined: no indirect call, no scratch stack.
// hipRTC is loaded lazily (dlopen), so the engine has no link-time dependency.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace pga {

class JitKernel {
 public:
  ~JitKernel();
  int encoding = 0;
  std::string name, source, log;
  std::vector<char> code;  // gfx950 code object
  // per-device loaded module / function (lazily, on first launch)
  hipFunction_t function(int device);
  // returns the number of blocks launched (= best partials written), <= max_grid
  uint32_t eval(int device, const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const float* data,
                float* scores, unsigned long long* parts, uint32_t max_grid, hipStream_t s);

 private:
  std::vector<hipModule_t> modules_;
  std::vector<hipFunction_t> fns_;
};

// compile (throws std::runtime_error with the hipRTC log on failure)
std::shared_ptr<JitKernel> jit_compile(int encoding, const std::string& source, const std::string& name,
                                       const std::vector<std::string>& extra_options);
// full kernel source the engine hands to hipRTC (for inspection / tests)
std::string jit_kernel_source(int encoding, const std::string& source, const std::string& name);

}  // namespace pga
