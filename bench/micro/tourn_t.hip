// micro: transposed tournament. Each group of 8 lanes breeds a batch of 8
// consecutive children; lane q runs the tournament of batch child q one batch
// ahead (4 u16 key loads per lane per batch instead of 4 per child), winners are
// broadcast with __shfl, row gathers are issued D iterations ahead.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <utility>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ inline unsigned hash(unsigned x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }
__device__ inline unsigned idx(unsigned w, unsigned S) { unsigned r = __umulhi(w, S); asm("" : "+v"(r)); return r; }

template <int D, int WAVES>
__global__ __launch_bounds__(256, WAVES) void tourn_t(const v4u* __restrict__ cur, v4u* __restrict__ nxt, const unsigned short* __restrict__ kc,
                                               unsigned short* __restrict__ kn, unsigned S, unsigned salt) {
  const unsigned lane = threadIdx.x & 63, q = lane & 7, gbase = lane & ~7u;
  const unsigned ngroups = gridDim.x * 32;
  const unsigned g = blockIdx.x * 32 + threadIdx.x / 8;
  const unsigned nb = S / 8;  // batches
  // lane-held tournament state
  unsigned pa_cur = 0, pb_cur = 0, pa_nxt = 0, pb_nxt = 0;
  unsigned i0 = 0, i1 = 0, i2 = 0, i3 = 0; float t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  auto issue_keys = [&](unsigned bi) {
    unsigned c = (bi < nb ? bi : nb - 1) * 8 + q;
    i0 = idx(hash(c * 4 + 0 + salt), S); i1 = idx(hash(c * 4 + 1 + salt), S);
    i2 = idx(hash(c * 4 + 2 + salt), S); i3 = idx(hash(c * 4 + 3 + salt), S);
    t0 = kc[i0]; t1 = kc[i1]; t2 = kc[i2]; t3 = kc[i3];
  };
  auto resolve = [&](unsigned& pa, unsigned& pb) {
    pa = t0 < t1 ? i1 : i0; pb = t2 < t3 ? i3 : i2;
  };
  unsigned bi = g;
  if (bi >= nb) return;
  issue_keys(bi); resolve(pa_cur, pb_cur);
  issue_keys(bi + ngroups); resolve(pa_nxt, pb_nxt);
  issue_keys(bi + 2 * ngroups);
  v4u A[D + 1], B[D + 1];
  // prologue: rows for iterations 0..D-1 of batch bi
#pragma unroll
  for (int j = 0; j < D; ++j) {
    unsigned pa = __shfl(pa_cur, gbase + j, 64), pb = __shfl(pb_cur, gbase + j, 64);
    A[j] = cur[(size_t)pa * 8 + q]; B[j] = cur[(size_t)pb * 8 + q];
  }
  for (;;) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // issue rows of iteration i + D
      const int j = i + D;
      unsigned pa, pb;
      if (j < 8) { pa = __shfl(pa_cur, gbase + j, 64); pb = __shfl(pb_cur, gbase + j, 64); }
      else { pa = __shfl(pa_nxt, gbase + (j - 8), 64); pb = __shfl(pb_nxt, gbase + (j - 8), 64); }
      A[(i + D) % (D + 1)] = cur[(size_t)pa * 8 + q]; B[(i + D) % (D + 1)] = cur[(size_t)pb * 8 + q];
      // finish child i
      const unsigned c = bi * 8 + i;
      v4u r = A[i % (D + 1)] ^ B[i % (D + 1)];
      nxt[(size_t)c * 8 + q] = r;
      unsigned pc = __popc(r.x) + __popc(r.y) + __popc(r.z) + __popc(r.w);
      pc += __shfl_xor(pc, 1, 64); pc += __shfl_xor(pc, 2, 64); pc += __shfl_xor(pc, 4, 64);
      if (q == 0) kn[c] = (unsigned short)pc;
    }
    bi += ngroups;
    if (bi >= nb) break;
    pa_cur = pa_nxt; pb_cur = pb_nxt;
    resolve(pa_nxt, pb_nxt);
    issue_keys(bi + 2 * ngroups);
    // rotate: A/B sets continue with index (8 % (D+1)) offset -> re-index by copying (compile-time)
    if ((8 % (D + 1)) != 0) {
      v4u tA[D + 1], tB[D + 1];
#pragma unroll
      for (int k = 0; k < D + 1; ++k) { tA[k] = A[(k + 8) % (D + 1)]; tB[k] = B[(k + 8) % (D + 1)]; }
#pragma unroll
      for (int k = 0; k < D + 1; ++k) { A[k] = tA[k]; B[k] = tB[k]; }
    }
  }
}

template <int D, int W>
float run(unsigned S, int grid, int iters) {
  v4u *x, *y; unsigned short *k0, *k1;
  CK(hipMalloc(&x, (size_t)S * 128)); CK(hipMalloc(&y, (size_t)S * 128));
  CK(hipMalloc(&k0, S * 2)); CK(hipMalloc(&k1, S * 2));
  CK(hipMemset(x, 1, (size_t)S * 128)); CK(hipMemset(k0, 0, S * 2));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) { hipLaunchKernelGGL((tourn_t<D, W>), grid, 256, 0, 0, x, y, k0, k1, S, i); std::swap(x, y); std::swap(k0, k1); }
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) { hipLaunchKernelGGL((tourn_t<D, W>), grid, 256, 0, 0, x, y, k0, k1, S, i); std::swap(x, y); std::swap(k0, k1); }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(k0)); CK(hipFree(k1));
  return 1000.f * ms / iters;
}

int main() {
  const unsigned S = 1u << 20;
  for (int blocks_per_cu : {4, 6, 8}) {
    int grid = 256 * blocks_per_cu;
    printf("grid %d: D1 %.1f  D2 %.1f  D3 %.1f us/gen\n", grid, run<1, 2>(S, grid, 200), run<2, 2>(S, grid, 200), run<3, 2>(S, grid, 200));
  }
  return 0;
}
