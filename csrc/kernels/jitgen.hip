// jitgen.hip — the hot BINARY generation kernel (binary_gen_tp, see
// binary.hip / binary_dev.hpp) with a user objective: built to LLVM bitcode,
// one file per (group size, full groups, dense mutation) variant
// (tools/build.py: build/jit/gen_<GS>_<FULL>_<DENSE>.bc).  At run time jit.cpp
// compiles the user's objective to bitcode defining pga_user_objective and
// LTO-links the two into a code object, so selection, crossover,
// mutation, evaluation and the child / score / key / best stores stay ONE
// launch per generation with the user's function inlined — instead of the
// generation kernel plus a separate evaluation pass that re-reads every row.
//
// Reference: the objective is called per individual through a device
// function pointer in src/pga.cu:250-262 (K2 in SURVEY.md §2.3).
#ifndef PGA_JIT_GS
#error "build with -DPGA_JIT_GS=<group size> -DPGA_JIT_FULL=<0|1> -DPGA_JIT_DENSE=<0|1>"
#endif
#define PGA_JIT_GEN 1
#include "pga/binary_dev.hpp"

namespace pga {
namespace jitgen {
template __global__ void binary_gen_tp<PGA_JIT_GS, kObjJit, (bool)PGA_JIT_FULL, (bool)PGA_JIT_DENSE>(GenArgs,
                                                                                                 unsigned long long*);
}  // namespace jitgen
}  // namespace pga
