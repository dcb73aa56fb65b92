// qubo.hip — quadratic binary objectives on the int8 matrix cores of gfx950.
//
//   f(x) = x^T Q x,  x in {0,1}^L,  Q integer in [-128, 127]  (QUBO; Max-Cut
//   is the QUBO Q = diag(deg) - W).  score = sign * f.
//
// A population tile of children is the A operand (bit -> int8 0/1), Q^T the
// B operand, v_mfma_i32_16x16x64_i8 accumulates Y = X Q exactly in i32, and
// f = rowsum(Y o X) is folded in per 16-column tile.  Integer arithmetic
// end to end, so the CPU backend (cpu_ops.cpp qubo_eval) agrees bit for bit.
//
// Tiling (one workgroup = 4 waves, grid-stride over tiles of 64*MT children):
//   * the tile's bit rows are staged once in LDS; each wave expands its MT
//     16-child M-tiles into int8 A fragments for ALL of K (Lp = 64*KS bits,
//     4 VGPRs per 64-bit k-step) and keeps them in registers;
//   * Q^T is streamed through LDS in 64-column n-blocks (64 x Lp bytes,
//     rows padded by 16 B against bank conflicts) shared by the 4 waves;
//   * per 16-column n-tile: KS x MT MFMAs over the whole K, then the
//     accumulator (C layout: col = lane & 15, row = 4 (lane >> 4) + i) is
//     masked by the children's bits at those columns and summed.
// The A/B element order inside a 64-deep k-step (element j of lane group g
// <-> k = 16 g + j) is the SAME convention for both operands, so the dot
// product is correct whatever k-permutation the hardware applies internally;
// row/column/C maps follow the standard 16x16 MFMA layout.
//
// Reference: the reference only evaluates user device function pointers one
// thread per individual (src/pga.cu:250-262); SURVEY.md C10 asks for MFMA on
// linear/quadratic objectives batched over population tiles.
#include <hip/hip_runtime.h>

#include "pga/device.hpp"
#include "pga/ops.hpp"

namespace pga {
namespace {

using namespace dev;
typedef int v4i __attribute__((ext_vector_type(4)));

// 16 bits -> 16 int8 {0,1}: byte j of the 16-byte result = bit j
__device__ __forceinline__ v4i expand16(uint32_t h) {
  v4i r;
  r[0] = (int)(((h & 0xFu) * 0x00204081u) & 0x01010101u);
  r[1] = (int)((((h >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
  r[2] = (int)((((h >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
  r[3] = (int)((((h >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
  return r;
}

template <int KS, int MT>
__global__ __launch_bounds__(kBlock, 2) void qubo_eval_kernel(const uint32_t* __restrict__ rows, uint32_t row_words,
                                                           uint64_t S, const int8_t* __restrict__ qt, float sign,
                                                           float* __restrict__ scores,
                                                           unsigned long long* __restrict__ parts) {
  constexpr uint32_t Lp = 64u * KS;           // padded genome bits
  constexpr uint32_t QROW = Lp + 16u;         // LDS row stride of the Q^T block (bytes)
  constexpr uint32_t BROW = Lp / 8u + 8u;     // LDS row stride of a child's bits (bytes)
  constexpr uint32_t TILE = 4u * 16u * MT;    // children per workgroup tile
  unsigned char* smem = pga_dyn_lds;
  unsigned char* qb = smem;                   // [64][QROW]
  unsigned char* bits = smem + 64u * QROW;    // [TILE][BROW]
  __shared__ unsigned long long lds_red[kBlock / 64];

  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  const uint32_t col = lane & 15u, g = lane >> 4;
  unsigned long long my_best = 0;

  for (uint64_t base = (uint64_t)blockIdx.x * TILE; base < S; base += (uint64_t)gridDim.x * TILE) {
    // ---- stage the tile's bit rows (zero beyond S) ----
    __syncthreads();
    constexpr uint32_t WPR = Lp / 32u;  // 32-bit words per staged row
    for (uint32_t i = threadIdx.x; i < TILE * WPR; i += kBlock) {
      const uint32_t c = i / WPR, w = i % WPR;
      const uint64_t child = base + c;
      const uint32_t v = (child < S && w < row_words) ? rows[child * row_words + w] : 0u;
      *(uint32_t*)(bits + c * BROW + 4u * w) = v;
    }
    __syncthreads();

    // ---- int8 A fragments for all of K, kept in registers ----
    v4i A[MT][KS];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const unsigned char* br = bits + (wave * 16u * MT + 16u * t + col) * BROW;
#pragma unroll
      for (int s = 0; s < KS; ++s) A[t][s] = expand16(*(const uint16_t*)(br + 8u * s + 2u * g));
    }

    int fsum[MT][4];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) fsum[t][i] = 0;

#pragma unroll 1
    for (uint32_t nb = 0; nb < (uint32_t)KS; ++nb) {  // 64-column n-blocks of Q^T
      __syncthreads();
      constexpr uint32_t C16 = Lp / 16u;  // 16-byte chunks per Q^T row
      for (uint32_t i = threadIdx.x; i < 64u * C16; i += kBlock) {
        const uint32_t r = i / C16, c = i % C16;
        const uint4 v = *(const uint4*)(qt + (uint64_t)(64u * nb + r) * Lp + 16u * c);
        *(uint4*)(qb + r * QROW + 16u * c) = v;
      }
      __syncthreads();
      // the children's bits at this n-block's 64 columns, in C-layout rows
      unsigned long long xb[MT][4];
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xb[t][i] = *(const unsigned long long*)(bits + (wave * 16u * MT + 16u * t + 4u * g + i) * BROW + 8u * nb);
#pragma unroll 2
      for (int jj = 0; jj < 4; ++jj) {  // 16-column n-tiles
        v4i acc[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = v4i{0, 0, 0, 0};
        const unsigned char* qr = qb + (16u * jj + col) * QROW + 16u * g;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const v4i B = *(const v4i*)(qr + 64u * s);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[t][s], B, acc[t], 0, 0, 0);
        }
        const uint32_t sh = 16u * jj + col;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) fsum[t][i] += ((xb[t][i] >> sh) & 1ull) ? acc[t][i] : 0;
      }
    }

    // ---- row sums over the 16 column lanes, one score per child ----
#pragma unroll
    for (int t = 0; t < MT; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int v = fsum[t][i];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        fsum[t][i] = v;
      }
      // lane col = i stores child 4g + i (static register index: no scratch)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t child = base + wave * 16u * MT + 16u * t + 4u * g + (uint32_t)i;
        if (col == (uint32_t)i && child < S) {
          const float sc = sign * (float)fsum[t][i];
          scores[child] = sc;
          const unsigned long long pb = pack_best(sc, child);
          my_best = pb > my_best ? pb : my_best;
        }
      }
    }
  }
  const unsigned long long b = block_max_u64(my_best, lds_red);
  if (threadIdx.x == 0) parts[blockIdx.x] = b;
}

// Q (row-major L x L floats, integers) -> int8 Q^T padded to Lp x Lp
__global__ __launch_bounds__(kBlock) void qubo_pack_kernel(const float* q, uint32_t L, uint32_t Lp, int8_t* qt) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < (uint64_t)Lp * Lp;
       i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t n = (uint32_t)(i / Lp), k = (uint32_t)(i % Lp);
    qt[i] = (n < L && k < L) ? (int8_t)qubo_coef(q[(uint64_t)k * L + n]) : (int8_t)0;
  }
}

template <int KS, int MT>
uint32_t go(const uint32_t* rows, uint32_t row_words, uint64_t S, const int8_t* qt, float sign, float* scores,
            unsigned long long* parts, hipStream_t s) {
  constexpr uint32_t Lp = 64u * KS;
  const size_t lds = 64u * (Lp + 16u) + (size_t)(4u * 16u * MT) * (Lp / 8u + 8u);
  const void* k = (const void*)qubo_eval_kernel<KS, MT>;
  static bool attr = false;
  if (!attr) {
    PGA_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  int per_cu = 0;
  PGA_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kBlock, lds));
  if (per_cu < 1) per_cu = 1;
  const uint64_t tiles = (S + 64u * MT - 1) / (64u * MT);
  uint64_t grid = (uint64_t)per_cu * device_cu_count();
  if (grid > tiles) grid = tiles;
  if (grid > kMaxGrid) grid = kMaxGrid;
  hipLaunchKernelGGL((qubo_eval_kernel<KS, MT>), (uint32_t)grid, kBlock, lds, s, rows, row_words, S, qt, sign, scores,
                     parts);
  PGA_HIP_CHECK(hipGetLastError());
  return (uint32_t)grid;
}

}  // namespace

uint32_t qubo_padded_length(uint32_t L) {
  uint32_t lp = 64;
  while (lp < L) lp <<= 1;
  return lp;
}

void qubo_pack_launch(const float* q, uint32_t L, int8_t* qt, hipStream_t s) {
  const uint32_t Lp = qubo_padded_length(L);
  if (Lp > kQuboMaxBits) throw std::invalid_argument("QUBO objective supports genomes of at most 1024 bits");
  hipLaunchKernelGGL(qubo_pack_kernel, 512, kBlock, 0, s, q, L, Lp, qt);
  PGA_HIP_CHECK(hipGetLastError());
}

uint32_t qubo_eval_launch(const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const int8_t* qt, float sign,
                          float* scores, unsigned long long* parts, hipStream_t s) {
  const uint32_t* r = (const uint32_t*)rows;  // words past row_words read as 0 (bits >= L are 0 already)
  switch (qubo_padded_length(L)) {
    case 64: return go<1, 4>(r, row_words, S, qt, sign, scores, parts, s);
    case 128: return go<2, 4>(r, row_words, S, qt, sign, scores, parts, s);
    case 256: return go<4, 4>(r, row_words, S, qt, sign, scores, parts, s);
    case 512: return go<8, 4>(r, row_words, S, qt, sign, scores, parts, s);
    case 1024: return go<16, 2>(r, row_words, S, qt, sign, scores, parts, s);
    default: throw std::invalid_argument("QUBO objective supports genomes of at most 1024 bits");
  }
}

}  // namespace pga
