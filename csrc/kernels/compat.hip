// compat.hip — reference-ABI path for user device function pointers.
//
// The reference hands user code raw device function pointers
//   obj_f(gene*, unsigned), mutate_f(gene*, float* rand, unsigned),
//   crossover_f(gene* p1, gene* p2, gene* child, float* rand, unsigned)
// (include/pga.h:46-48) and calls them one thread per individual
// (src/pga.cu:250-347).  Objectives alone go through the fused REAL kernel
// (OBJ_USER_FNPTR in real.hip); once a user crossover or mutation callback
// is installed, generations run here: one thread per child, tournament
// selection, then the callbacks on the child row in place, each with its own
// fresh rand slice of L uniforms in (0, 1] (materialised in a scratch buffer,
// the only place the engine materialises random numbers; the reference reused
// ONE slice for selection, crossover and mutation).
//
// Indirect calls force a dynamic stack and conservative registers (SURVEY.md
// C9 probe); this path trades speed for ABI compatibility by design.
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"
#include "pga/real_ops.hpp"

typedef float (*pga_obj_fn)(float*, unsigned);
typedef void (*pga_mutate_fn)(float*, float*, unsigned);
typedef void (*pga_crossover_fn)(float*, float*, float*, float*, unsigned);

// Reference default operators, exported as device symbols so callers can
// fetch them with hipMemcpyFromSymbol (the reference's __crossover/__mutate,
// src/pga.cu:127-146).
__device__ void pga_default_mutate_impl(float* g, float* rand, unsigned len) {
  if (rand[1] <= 0.01f) {
    unsigned i = (unsigned)(rand[0] * (float)len);
    if (i >= len) i = len - 1;  // rand is in (0, 1]: the reference could write g[len]
    g[i] = rand[2];
  }
}
__device__ void pga_default_crossover_impl(float* p1, float* p2, float* c, float* rand, unsigned len) {
  for (unsigned i = 0; i < len; ++i) c[i] = rand[i] > 0.5f ? p1[i] : p2[i];
}
__device__ pga_mutate_fn pga_default_mutate = pga_default_mutate_impl;
__device__ pga_crossover_fn pga_default_crossover = pga_default_crossover_impl;

namespace pga {
namespace {

using namespace dev;

__device__ __forceinline__ void fill_rand(const GenArgs& a, uint64_t child, uint32_t phase, float* r) {
  for (uint32_t i = 0; i < a.L; i += 4) {
    const u32x4 w = draw(a.key, ST_COMPAT, child, (phase << 20) | (i >> 2));
    r[i] = word_to_unit(w.x);
    if (i + 1 < a.L) r[i + 1] = word_to_unit(w.y);
    if (i + 2 < a.L) r[i + 2] = word_to_unit(w.z);
    if (i + 3 < a.L) r[i + 3] = word_to_unit(w.w);
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void compat_kernel(GenArgs a, unsigned long long* best_parts) {
  resolve_gen(a);
  __shared__ unsigned long long lds_red[kBlock / 64];
  __shared__ uint32_t lds_elite;
  const uint32_t L = a.L;
  const uint64_t rw = a.row_words;
  const float* cur = (const float*)a.cur;
  float* nxt = (float*)a.next;
  constexpr bool EVALS = MODE == MODE_GEN || MODE == MODE_EVAL || MODE == MODE_INIT;
  const bool evals = EVALS && a.objective == OBJ_USER_FNPTR && a.user_fn;
  if (MODE == MODE_GEN && a.n_elite > 0 && a.elite_idx == nullptr) {
    if (blockIdx.x == 0) {
      unsigned long long b = block_reduce_parts(a.best_cur, a.n_best_cur, lds_red);
      if (threadIdx.x == 0) lds_elite = (uint32_t)best_index(b);
    }
    __syncthreads();
  }
  unsigned long long my_best = 0;
  ScoreStats st;
  // grid-stride over children (the reference RUN_KERNEL loop serves any S,
  // src/pga.cu:62-70); the grid is sized to the device, not to S
  for (uint64_t child = (uint64_t)blockIdx.x * kBlock + threadIdx.x; child < a.S;
       child += (uint64_t)gridDim.x * kBlock) {
    float* c = nxt + child * rw;
    float* rand = a.compat_rand + child * L;
    float score = 0.f;
    bool elite = false;
    if (MODE == MODE_GEN && child < a.n_elite) {
      elite = true;
      const uint32_t src = a.elite_idx ? a.elite_idx[child] : lds_elite;
      for (uint32_t i = 0; i < L; ++i) c[i] = cur[(uint64_t)src * rw + i];
      score = a.score_cur[src];
    }
    if (!elite && (MODE == MODE_GEN || MODE == MODE_CROSS)) {
      uint32_t pa = 0, pb = 0;
      const uint32_t S = (uint32_t)a.S;
      for (uint32_t p = 0; p < 2; ++p) {  // k-tournament, first max wins
        uint32_t b = word_to_index(child_word(a.key, child, W_SEL + p * a.tour_k), S);
        float bs = a.score_cur[b];
        for (uint32_t j = 1; j < a.tour_k; ++j) {
          const uint32_t x = word_to_index(child_word(a.key, child, W_SEL + p * a.tour_k + j), S);
          const float xs = a.score_cur[x];
          if (bs < xs) { bs = xs; b = x; }
        }
        if (p == 0) pa = b; else pb = b;
      }
      fill_rand(a, child, 0, rand);
      float* p1 = (float*)cur + (uint64_t)pa * rw;
      float* p2 = (float*)cur + (uint64_t)pb * rw;
      if (a.user_xo_fn) ((pga_crossover_fn)a.user_xo_fn)(p1, p2, c, rand, L);
      else pga_default_crossover_impl(p1, p2, c, rand, L);
    }
    if (!elite && (MODE == MODE_GEN || MODE == MODE_MUTATE)) {
      fill_rand(a, child, 1, rand);
      if (MODE == MODE_MUTATE) c = (float*)cur + child * rw;  // in place
      if (a.user_mut_fn) ((pga_mutate_fn)a.user_mut_fn)(c, rand, L);
      else pga_default_mutate_impl(c, rand, L);
    }
    if (MODE == MODE_INIT) {
      fill_rand(a, child, 2, c);  // reference: initial genes are U(0, 1]
      for (uint32_t i = L; i < rw; ++i) c[i] = 0.f;
    }
    if (evals && !elite) {
      float* g = (MODE == MODE_EVAL) ? (float*)cur + child * rw : c;
      score = ((pga_obj_fn)a.user_fn)(g, L);
    }
    if (evals) {
      a.score_next[child] = score;
      const unsigned long long pb = pack_best(score, child);
      if (pb > my_best) my_best = pb;
      st.add(score);
    }
  }
  if (evals && best_parts) {
    unsigned long long b = block_max_u64(my_best, lds_red);
    if (threadIdx.x == 0) best_parts[blockIdx.x] = b;
    if (a.stats_parts) block_stats_store(st, a.stats_parts);
  }
}

}  // namespace

uint32_t compat_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  if (!a.compat_rand) throw std::runtime_error("compat path needs its rand scratch buffer");
  // indirect calls pin a dynamic stack, so residency (not S) sizes the grid:
  // a few blocks per CU keep every SIMD busy while the loop covers any S
  const uint64_t need = (a.S + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)device_cu_count() * 8;
  const uint32_t grid = (uint32_t)(need < cap ? (need ? need : 1) : cap);
  switch (mode) {
    case MODE_GEN: hipLaunchKernelGGL(compat_kernel<MODE_GEN>, grid, kBlock, 0, s, a, best_parts); break;
    case MODE_INIT: hipLaunchKernelGGL(compat_kernel<MODE_INIT>, grid, kBlock, 0, s, a, best_parts); break;
    case MODE_EVAL: hipLaunchKernelGGL(compat_kernel<MODE_EVAL>, grid, kBlock, 0, s, a, best_parts); break;
    case MODE_CROSS: hipLaunchKernelGGL(compat_kernel<MODE_CROSS>, grid, kBlock, 0, s, a, best_parts); break;
    default: hipLaunchKernelGGL(compat_kernel<MODE_MUTATE>, grid, kBlock, 0, s, a, best_parts); break;
  }
  PGA_HIP_CHECK(hipGetLastError());
  return grid;
}

}  // namespace pga
