// refsem.hip — the "reference-semantics" baseline of BASELINE.md.
//
// pbalcer/libpga publishes no numbers and cannot run the north-star configs
// as shipped (L=1024 needs 256 KiB LDS per block, src/pga.cu:69), so the
// comparison point is its EXECUTION STRUCTURE re-created on the same MI355X:
//   * AoS float genes, two S·L generations + S scores (src/pga.cu:37-46, :108-111);
//   * a materialised S·L uniform RNG buffer refilled every generation
//     (__fill_rand, :99-105) — here a Philox fill kernel stands in for the
//     cuRAND host generator;
//   * one thread per individual, 8 blocks per launch, a host loop of
//     ⌈S/(8·T)⌉ launches per stage (ITERATE_POP_START / RUN_KERNEL, :58-77,
//     :199-200) with T=64 + dynamic LDS 64·L·4 B when it fits (SHARED_MEM),
//     else T=512 without LDS staging;
//   * objective / crossover / mutation called through device function
//     pointers (:127-146, :206-216); binary tournament with rand-slice
//     contestants (:278-292), uniform crossover (:135-143), 1% single-gene
//     reset mutation (:127-133);
//   * a device-wide sync after every stage (pga_evaluate/crossover/mutate,
//     :264-270, :319-325, :349-354) and the generation order of pga_run
//     (fill → evaluate → crossover → mutate → swap, :376-391).
// Written from that description — no reference code — so numbers measure the
// reference's design on gfx950, not its compiler.  Only difference by intent:
// contestant / gene indices are clamped to n-1 (the reference can index
// score[S] when a uniform draw is exactly 1.0).
//
//   refsem --objective onemax|rastrigin|sum --pop S --length L --gens G [--global]
// prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

typedef float (*obj_fn)(float*, unsigned);
typedef void (*mut_fn)(float*, float*, unsigned);
typedef void (*xo_fn)(float*, float*, float*, float*, unsigned);

__device__ float f_onemax(float* g, unsigned L) {  // float-encoded bits: gene > 0.5 is a one
  float s = 0.f;
  for (unsigned i = 0; i < L; ++i) s += g[i] > 0.5f ? 1.f : 0.f;
  return s;
}
__device__ float f_sum(float* g, unsigned L) {  // reference E1 (test/test.cu)
  float s = 0.f;
  for (unsigned i = 0; i < L; ++i) s += g[i];
  return s;
}
__device__ float f_rastrigin(float* g, unsigned L) {  // genes in (0,1] mapped to [-5.12, 5.12], maximise -f
  float s = 10.f * L;
  for (unsigned i = 0; i < L; ++i) {
    const float x = g[i] * 10.24f - 5.12f;
    s += x * x - 10.f * cosf(6.2831853f * x);
  }
  return -s;
}
__device__ void m_reset(float* g, float* r, unsigned L) {
  if (r[1] <= 0.01f) g[min((unsigned)(r[0] * L), L - 1)] = r[2];
}
__device__ void x_uniform(float* a, float* b, float* c, float* r, unsigned L) {
  for (unsigned i = 0; i < L; ++i) c[i] = r[i] > 0.5f ? a[i] : b[i];
}
__device__ obj_fn p_onemax = f_onemax;
__device__ obj_fn p_sum = f_sum;
__device__ obj_fn p_rastrigin = f_rastrigin;
__device__ mut_fn p_reset = m_reset;
__device__ xo_fn p_uniform = x_uniform;

// --- RNG fill: S·L uniforms in (0, 1] (Philox-4x32-10, one counter per 4 floats)
__device__ inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)p1;
    c[2] = n2;
    c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
__global__ void fill_rand(float* __restrict__ out, size_t n, uint32_t seed, uint32_t gen) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * q < n; q += stride) {
    uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), gen, 0x5EED};
    philox(c, seed, 0xC0FFEEu);
    float4 v;
    v.x = ((c[0] >> 8) + 1) * (1.f / 16777216.f);
    v.y = ((c[1] >> 8) + 1) * (1.f / 16777216.f);
    v.z = ((c[2] >> 8) + 1) * (1.f / 16777216.f);
    v.w = ((c[3] >> 8) + 1) * (1.f / 16777216.f);
    if (4 * q + 3 < n) {
      *(float4*)(out + 4 * q) = v;
    } else {
      const float t[4] = {v.x, v.y, v.z, v.w};
      for (size_t j = 0; 4 * q + j < n; ++j) out[4 * q + j] = t[j];
    }
  }
}

// --- stages: one thread per individual, offset = launch index · 8 · T
template <bool LDS>
__global__ void k_evaluate(size_t off, obj_fn obj, float* genomes, float* score, size_t S, unsigned L) {
  extern __shared__ float sh[];
  const size_t i = off + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  float* g = genomes + i * L;
  if (LDS) {
    float* s = sh + (size_t)threadIdx.x * L;
    for (unsigned j = 0; j < L; ++j) s[j] = g[j];
    g = s;
  }
  score[i] = obj(g, L);
}

__device__ inline size_t tournament(const float* score, const float* r, size_t S) {
  size_t best = min((size_t)(r[0] * S), S - 1);
  const size_t c = min((size_t)(r[1] * S), S - 1);
  if (score[best] < score[c]) best = c;
  return best;
}

template <bool LDS>
__global__ void k_crossover(size_t off, xo_fn xo, float* newg, float* oldg, const float* score, float* rnd, unsigned L,
                            size_t S) {
  extern __shared__ float sh[];
  const size_t i = off + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  float* r = rnd + i * L;
  const size_t a = tournament(score, r, S), b = tournament(score, r + 2, S);
  float* child = LDS ? sh + (size_t)threadIdx.x * L : newg + i * L;
  xo(oldg + a * L, oldg + b * L, child, r, L);
  if (LDS)
    for (unsigned j = 0; j < L; ++j) newg[i * L + j] = child[j];
}

template <bool LDS>
__global__ void k_mutate(size_t off, mut_fn mut, float* genomes, float* rnd, size_t S, unsigned L) {
  extern __shared__ float sh[];
  const size_t i = off + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S) return;
  float* g = genomes + i * L;
  if (LDS) {
    float* s = sh + (size_t)threadIdx.x * L;
    for (unsigned j = 0; j < L; ++j) s[j] = g[j];
    mut(s, rnd + i * L, L);
    for (unsigned j = 0; j < L; ++j) g[j] = s[j];
  } else {
    mut(g, rnd + i * L, L);
  }
}

int main(int argc, char** argv) {
  std::string objective = "onemax";
  size_t S = 1 << 20;
  unsigned L = 1024, G = 3, warm = 1;
  bool force_global = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(argv[++i]); };
    if (a == "--objective") objective = next();
    else if (a == "--pop") S = std::stoull(next());
    else if (a == "--length") L = (unsigned)std::stoul(next());
    else if (a == "--gens") G = (unsigned)std::stoul(next());
    else if (a == "--warmup") warm = (unsigned)std::stoul(next());
    else if (a == "--global") force_global = true;
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (L < 4 || S < 2) return 2;
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const size_t lds_need = 64ull * L * sizeof(float);
  const bool lds = !force_global && lds_need <= (size_t)prop.sharedMemPerBlock;
  const unsigned T = lds ? 64 : 512, B = 8;  // src/pga.cu:66, :72, :200
  const size_t per_launch = (size_t)B * T, shmem = lds ? lds_need : 0;
  if (lds) {
    CK(hipFuncSetAttribute((const void*)k_evaluate<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
    CK(hipFuncSetAttribute((const void*)k_crossover<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
    CK(hipFuncSetAttribute((const void*)k_mutate<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  }

  obj_fn obj;
  mut_fn mut;
  xo_fn xo;
  if (objective == "onemax") CK(hipMemcpyFromSymbol(&obj, HIP_SYMBOL(p_onemax), sizeof(obj)));
  else if (objective == "sum") CK(hipMemcpyFromSymbol(&obj, HIP_SYMBOL(p_sum), sizeof(obj)));
  else if (objective == "rastrigin") CK(hipMemcpyFromSymbol(&obj, HIP_SYMBOL(p_rastrigin), sizeof(obj)));
  else return 2;
  CK(hipMemcpyFromSymbol(&mut, HIP_SYMBOL(p_reset), sizeof(mut)));
  CK(hipMemcpyFromSymbol(&xo, HIP_SYMBOL(p_uniform), sizeof(xo)));

  const size_t n = S * (size_t)L;
  float *cur, *nxt, *score, *rnd;
  CK(hipMalloc(&cur, n * 4));
  CK(hipMalloc(&nxt, n * 4));
  CK(hipMalloc(&rnd, n * 4));
  CK(hipMalloc(&score, S * 4));
  const unsigned fill_grid = 4 * prop.multiProcessorCount;
  unsigned gen = 0;
  // population init = a copy of a fresh uniform buffer (__g_random_generate, :81-97)
  hipLaunchKernelGGL(fill_rand, dim3(fill_grid), dim3(256), 0, 0, cur, n, 1234u, gen++);
  CK(hipDeviceSynchronize());

  auto generation = [&]() {
    hipLaunchKernelGGL(fill_rand, dim3(fill_grid), dim3(256), 0, 0, rnd, n, 1234u, gen++);
    CK(hipDeviceSynchronize());
    for (size_t off = 0; off < S; off += per_launch) {
      if (lds) hipLaunchKernelGGL(k_evaluate<true>, dim3(B), dim3(T), shmem, 0, off, obj, cur, score, S, L);
      else hipLaunchKernelGGL(k_evaluate<false>, dim3(B), dim3(T), 0, 0, off, obj, cur, score, S, L);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    for (size_t off = 0; off < S; off += per_launch) {
      if (lds) hipLaunchKernelGGL(k_crossover<true>, dim3(B), dim3(T), shmem, 0, off, xo, nxt, cur, score, rnd, L, S);
      else hipLaunchKernelGGL(k_crossover<false>, dim3(B), dim3(T), 0, 0, off, xo, nxt, cur, score, rnd, L, S);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    for (size_t off = 0; off < S; off += per_launch) {
      if (lds) hipLaunchKernelGGL(k_mutate<true>, dim3(B), dim3(T), shmem, 0, off, mut, nxt, rnd, S, L);
      else hipLaunchKernelGGL(k_mutate<false>, dim3(B), dim3(T), 0, 0, off, mut, nxt, rnd, S, L);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::swap(cur, nxt);
  };
  for (unsigned g = 0; g < warm; ++g) generation();
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned g = 0; g < G; ++g) generation();
  // final evaluate so the scores describe the current generation (:389-390) — not timed
  auto t1 = std::chrono::steady_clock::now();
  for (size_t off = 0; off < S; off += per_launch) {
    if (lds) hipLaunchKernelGGL(k_evaluate<true>, dim3(B), dim3(T), shmem, 0, off, obj, cur, score, S, L);
    else hipLaunchKernelGGL(k_evaluate<false>, dim3(B), dim3(T), 0, 0, off, obj, cur, score, S, L);
  }
  CK(hipDeviceSynchronize());
  float* hs = (float*)std::malloc(S * 4);
  CK(hipMemcpy(hs, score, S * 4, hipMemcpyDeviceToHost));
  float best = -INFINITY;
  for (size_t i = 0; i < S; ++i) best = hs[i] > best ? hs[i] : best;
  std::free(hs);
  const double dt = std::chrono::duration<double>(t1 - t0).count();
  std::printf(
      "{\"mode\": \"reference-semantics\", \"objective\": \"%s\", \"pop\": %zu, \"length\": %u, \"gens\": %u, "
      "\"lds_staging\": %s, \"threads_per_block\": %u, \"blocks\": %u, \"launches_per_stage\": %zu, "
      "\"gens_per_sec\": %.6g, \"evals_per_sec\": %.6g, \"ms_per_gen\": %.6g, \"best\": %.6g, \"device\": \"%s\"}\n",
      objective.c_str(), S, L, G, lds ? "true" : "false", T, B, (S + per_launch - 1) / per_launch, G / dt,
      G / dt * (double)S, dt / G * 1e3, best, prop.name);
  CK(hipFree(cur));
  CK(hipFree(nxt));
  CK(hipFree(rnd));
  CK(hipFree(score));
  return 0;
}
