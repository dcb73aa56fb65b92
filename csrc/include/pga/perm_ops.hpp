// perm_ops.hpp — PERMUTATION encoding semantics shared by the gfx950 kernel
// (csrc/kernels/perm.hip) and the CPU reference (csrc/cpu/cpu_perm.cpp).
// Genes are u16 city ids; a chunk is 8 genes (16 bytes).  Every operator is a
// deterministic function of the parents and the child's random words, so the
// GPU and CPU produce identical children.
#pragma once

#include "pga/core.hpp"

namespace pga {

// longest genome of the 4-individuals-per-block kernels (their LDS arrays);
// longer ones run one individual per 64-lane block (perm.hip go_long)
constexpr uint32_t kPermMaxL = 4096;

// child-word layout extension for permutations
//   W_CUT1, W_CUT2  segment [lo, hi) of parent A (PMX / OX)
//   W_MUTIND        per-individual mutation test
//   W_MUTPOS, W_SEL + sel_words   the two mutation positions
PGA_HD void perm_segment(uint32_t w1, uint32_t w2, uint32_t L, uint32_t& lo, uint32_t& hi) {
  uint32_t a = word_to_index(w1, L), b = word_to_index(w2, L + 1);  // hi may be L
  if (a > b) { uint32_t t = a; a = b; b = t; }
  lo = a;
  hi = b;
}

// Fisher-Yates (Durstenfeld) with j_i = index(word_i, i + 1), i = L-1 .. 1,
// word_i = register i%4 of ST_INIT block i/4
PGA_HD uint32_t perm_init_word(const RngKey& key, uint64_t child, uint32_t i) {
  return sel4(draw(key, ST_INIT, child, i / 4u), i % 4u);
}

PGA_HD void perm_mut_positions(uint32_t w1, uint32_t w2, uint32_t L, uint32_t& i, uint32_t& j) {
  i = word_to_index(w1, L);
  j = word_to_index(w2, L);
  if (i > j) { uint32_t t = i; i = j; j = t; }
}

}  // namespace pga
