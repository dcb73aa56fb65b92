// jitgen_real.hip — the REAL two-phase generation kernel (real_gen_tp, see
// real.hip / real_dev.hpp) with a user objective: built to LLVM bitcode, one
// file per group size (tools/build.py: build/jit/gen_real_<GS>.bc).  At run
// time jit.cpp compiles the user's float objective to bitcode defining
// pga_user_objective_f32 and LTO-links the two into a code object, so a
// float-gene objective written as source — the reference's whole user model,
// `float obj(gene*, unsigned)` with gene = float (include/pga.h:29,46), called
// per individual in src/pga.cu:250-262 — is evaluated inside the ONE
// generation launch instead of a separate pass that re-reads every row.
#ifndef PGA_JIT_GS
#error "build with -DPGA_JIT_GS=<group size>"
#endif
#define PGA_JIT_GEN 1
#include "pga/real_dev.hpp"

namespace pga {
namespace jitgen {
template __global__ void real_gen_tp<PGA_JIT_GS, kObjJit, false>(GenArgs, unsigned long long*);
}  // namespace jitgen
}  // namespace pga
