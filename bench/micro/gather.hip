// gather.hip — roofline of the GEN kernel's memory pattern on MI355X:
// per child, gather 2 random R-byte rows, write 1 row (16 B per lane, R/16
// lanes per row), no other work.  Variants: cache policy and working set.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ inline unsigned hash(unsigned x) { x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16; return x; }

template <int LANES, int NT, int SEQ>
__global__ __launch_bounds__(256) void gather(const v4u* cur, v4u* nxt, unsigned S, unsigned salt) {
  const unsigned q = threadIdx.x % LANES;
  const unsigned gpb = 256 / LANES;
  for (unsigned c = blockIdx.x * gpb + threadIdx.x / LANES; c < S; c += gridDim.x * gpb) {
    unsigned pa = SEQ ? c : (unsigned)(((unsigned long long)hash(c * 2 + salt) * S) >> 32);
    unsigned pb = SEQ ? c : (unsigned)(((unsigned long long)hash(c * 2 + 1 + salt) * S) >> 32);
    v4u a, b;
    if (NT & 2) { a = __builtin_nontemporal_load(cur + (size_t)pa * LANES + q); b = __builtin_nontemporal_load(cur + (size_t)pb * LANES + q); }
    else { a = cur[(size_t)pa * LANES + q]; b = cur[(size_t)pb * LANES + q]; }
    v4u r = a ^ b;
    if (NT & 1) __builtin_nontemporal_store(r, nxt + (size_t)c * LANES + q);
    else nxt[(size_t)c * LANES + q] = r;
  }
}

// with dependent tournament: 4 random score loads -> 2 winners -> row gathers
template <int LANES, int UNROLL, int V = 0>
__global__ __launch_bounds__(256) void tourn(const v4u* cur, v4u* nxt, const float* sc, float* sn, unsigned S, unsigned salt) {
  const unsigned q = threadIdx.x % LANES;
  const unsigned gpb = 256 / LANES;
  for (unsigned c0 = blockIdx.x * gpb * UNROLL + threadIdx.x / LANES; c0 < S; c0 += gridDim.x * gpb * UNROLL) {
    unsigned pa[UNROLL], pb[UNROLL];
    float s[UNROLL][4];
    unsigned id[UNROLL][4];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      unsigned c = c0 + u * gpb;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        id[u][k] = (unsigned)(((unsigned long long)hash(c * 4 + k + salt) * S) >> 32);
        if ((V & 4) && (k == 0 || k == 2)) id[u][k] = (k == 0) ? (c < S ? c : 0) : ((c + S / 2) % S);
        if (V & 8) s[u][k] = (float)((const unsigned short*)sc)[id[u][k]];
        else s[u][k] = sc[id[u][k]];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      pa[u] = s[u][0] < s[u][1] ? id[u][1] : id[u][0];
      pb[u] = s[u][2] < s[u][3] ? id[u][3] : id[u][2];
    }
    v4u a[UNROLL], b[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (V & 2) { a[u] = __builtin_nontemporal_load(cur + (size_t)pa[u] * LANES + q); b[u] = __builtin_nontemporal_load(cur + (size_t)pb[u] * LANES + q); }
      else { a[u] = cur[(size_t)pa[u] * LANES + q]; b[u] = cur[(size_t)pb[u] * LANES + q]; }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      unsigned c = c0 + u * gpb;
      if (c < S) {
        v4u r = a[u] ^ b[u];
        if (V & 1) __builtin_nontemporal_store(r, nxt + (size_t)c * LANES + q); else nxt[(size_t)c * LANES + q] = r;
        unsigned pc = __popc(r.x) + __popc(r.y) + __popc(r.z) + __popc(r.w);
        for (int o = LANES / 2; o > 0; o >>= 1) pc += __shfl_xor(pc, o, 64);
        if (q == 0) sn[c] = (float)pc;
      }
    }
  }
}

template <int LANES, int UNROLL, int V = 0>
float run_t(unsigned S, int grid, int iters) {
  v4u *x, *y; float *s0, *s1;
  CK(hipMalloc(&x, (size_t)S * LANES * 16)); CK(hipMalloc(&y, (size_t)S * LANES * 16));
  CK(hipMalloc(&s0, S * 4)); CK(hipMalloc(&s1, S * 4));
  CK(hipMemset(x, 1, (size_t)S * LANES * 16)); CK(hipMemset(s0, 0, S * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) { hipLaunchKernelGGL((tourn<LANES, UNROLL, V>), grid, 256, 0, 0, x, y, s0, s1, S, i); std::swap(x, y); std::swap(s0, s1); }
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) { hipLaunchKernelGGL((tourn<LANES, UNROLL, V>), grid, 256, 0, 0, x, y, s0, s1, S, i); std::swap(x, y); std::swap(s0, s1); }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(s0)); CK(hipFree(s1));
  return 1000.f * ms / iters;
}

template <int LANES, int NT, int SEQ>
float run(unsigned S, int grid, int iters) {
  v4u *x, *y;
  CK(hipMalloc(&x, (size_t)S * LANES * 16));
  CK(hipMalloc(&y, (size_t)S * LANES * 16));
  CK(hipMemset(x, 1, (size_t)S * LANES * 16));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) { hipLaunchKernelGGL((gather<LANES, NT, SEQ>), grid, 256, 0, 0, x, y, S, i); std::swap(x, y); }
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) { hipLaunchKernelGGL((gather<LANES, NT, SEQ>), grid, 256, 0, 0, x, y, S, i); std::swap(x, y); }
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipFree(x)); CK(hipFree(y));
  return 1000.f * ms / iters;
}

int main() {
  const int grid = 256 * 8;
  for (unsigned S : {1u << 20, 1u << 18, 1u << 16}) {
    float t0 = run<8, 0, 0>(S, grid, 200), t1 = run<8, 1, 0>(S, grid, 200), t2 = run<8, 2, 0>(S, grid, 200),
          t3 = run<8, 3, 0>(S, grid, 200), ts = run<8, 0, 1>(S, grid, 200);
    double mb = (double)S * 128 * 3 / 1e6;
    printf("S=%u rows=128B  plain %.1f us  ntstore %.1f  ntload %.1f  ntboth %.1f  | sequential %.1f us  (%.0f MB/gen; random %.2f TB/s)\n",
           S, t0, t1, t2, t3, ts, mb, mb / t0 / 1e6 * 1e6 / 1e6);
  }
  {
    const unsigned S = 1u << 20; const int g = 2048;
    printf("tournament+gather S=1M: base %.1f | ntstore %.1f | ntload %.1f | ntboth %.1f | u16 scores %.1f | u16+ntboth %.1f | self-contestant %.1f | self+ntboth %.1f | self+u16+ntboth %.1f\n",
      run_t<8, 2, 0>(S, g, 200), run_t<8, 2, 1>(S, g, 200), run_t<8, 2, 2>(S, g, 200), run_t<8, 2, 3>(S, g, 200),
      run_t<8, 2, 8>(S, g, 200), run_t<8, 2, 11>(S, g, 200), run_t<8, 2, 4>(S, g, 200), run_t<8, 2, 7>(S, g, 200),
      run_t<8, 2, 15>(S, g, 200));
  }
  // bigger rows: 1024 B per row (L = 8192 bits), S = 128K (same bytes)
  {
    unsigned S = 1u << 17;
    float t0 = run<64, 0, 0>(S, grid, 200), t3 = run<64, 3, 0>(S, grid, 200), ts = run<64, 0, 1>(S, grid, 200);
    printf("S=%u rows=1KB  plain %.1f us  ntboth %.1f | sequential %.1f us\n", S, t0, t3, ts);
  }
  return 0;
}
