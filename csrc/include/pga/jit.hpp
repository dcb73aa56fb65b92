// jit.hpp — user objectives compiled at runtime with hipRTC (SURVEY.md §7.1
// src/jit, §7.4: "keep the compat path correct but make templated/JIT
// objectives the fast path").
//
// The user writes one device function over a decoded row,
//   BINARY       float NAME(const unsigned int* words, unsigned int nbits, const float* data)
//   REAL         float NAME(const float* genes, unsigned int n, const float* data)
//   PERMUTATION  float NAME(const unsigned short* perm, unsigned int n, const float* data)
// and the engine compiles it for gfx950.  BINARY objectives are linked into
// the hot generation kernel itself (gen_function: one launch per generation,
// the child's row staged in LDS and handed to the user function by the
// group's first lane); otherwise, and for initial / explicit evaluations, a
// batched evaluation kernel (one work-item per individual, per-block best
// partials in the engine's packed format) runs after the generation kernel.  Unlike
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
  std::string user_source;  // the objective as the user wrote it
  std::vector<std::string> options;  // the user's extra compile options (hipRTC and the fused build alike)
  std::vector<char> code;  // gfx950 code object
  // per-device loaded module / function (lazily, on first launch)
  hipFunction_t function(int device);
  // returns the number of blocks launched (= best partials written), <= max_grid
  uint32_t eval(int device, const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const float* data,
                float* scores, unsigned long long* parts, uint32_t max_grid, hipStream_t s);

  // FUSED generation (BINARY): the hot generation kernel binary_gen_tp with
  // this objective linked in (jitgen.hip bitcode + the user's bitcode, LTO-
  // linked by the ROCm toolchain in a child process, cached on disk), one
  // variant per (group size, full groups, dense mutation).
  // nullptr when fusion is unavailable (another encoding, no kernel bitcode,
  // a link error: fused_error() says why) — the caller falls back to
  // generation + eval().
  // build = false: only an already loaded variant (nothing is compiled or
  // loaded, e.g. while a stream is being captured into a graph)
  hipFunction_t gen_function(int device, uint32_t gs, bool full, bool dense, uint32_t L, bool build = true);
  // the linked code object of one variant (compiled / LTO-linked on first use,
  // cached on disk; no GPU needed): its path.  Throws with the toolchain log.
  std::string build_gen_object(uint32_t gs, bool full, bool dense, uint32_t L);
  // launches one fused generation; returns the grid (= best partials written)
  uint32_t gen_launch(hipFunction_t f, const void* args, size_t args_bytes, uint64_t S, unsigned long long* parts,
                      uint32_t max_grid, hipStream_t s);
  const std::string& fused_error() const { return fused_error_; }

 private:
  std::vector<hipModule_t> modules_;
  std::vector<hipFunction_t> fns_;
  std::vector<char> user_bc_;  // the objective (+ pga_user_objective wrapper) as LLVM bitcode
  struct GenVariant {
    int device;
    uint64_t key;
    hipModule_t mod;
    hipFunction_t fn;
    uint32_t occ;  // resident blocks per CU
    std::shared_ptr<std::vector<char>> image;  // the linked code object (kept for the module's lifetime)
  };
  std::vector<GenVariant> gen_;
  std::string fused_error_;
  bool fused_failed_ = false;
};

// directory holding the jitgen bitcode (build/jit): $PGA_JIT_DIR, else found
// next to the loaded library
std::string jit_bitcode_dir();

// compile (throws std::runtime_error with the hipRTC log on failure)
std::shared_ptr<JitKernel> jit_compile(int encoding, const std::string& source, const std::string& name,
                                       const std::vector<std::string>& extra_options);
// full kernel source the engine hands to hipRTC (for inspection / tests)
std::string jit_kernel_source(int encoding, const std::string& source, const std::string& name);

}  // namespace pga
