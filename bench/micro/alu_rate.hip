// alu_rate.hip — issue rate of the integer ops the RNGs are built from
// (v_mad_u64_u32, v_mul_hi_u32, v_mul_lo_u32, v_xor_b32, v_alignbit_b32,
// v_mul_u32_u24) on gfx950: 8 independent chains per lane, full occupancy.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int N = 512;
template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned s) {
  unsigned a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (j + 1) + s;
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) { unsigned long long p = (unsigned long long)a[j] * 0xD2511F53u; a[j] = (unsigned)(p >> 32) ^ (unsigned)p; }
      if (OP == 1) a[j] = __umulhi(a[j], 0xD2511F53u) ^ s;
      if (OP == 2) a[j] = a[j] * 0xD2511F53u ^ s;
      if (OP == 3) a[j] = (a[j] ^ s) + 0x9E3779B9u;
      if (OP == 4) a[j] = __builtin_amdgcn_alignbit(a[j], a[j], 13) + s;
      if (OP == 5) a[j] = __mul24(a[j], 0x1F53) ^ s;
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= a[j];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}
template <int OP>
float run(unsigned* d, int grid) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, grid, 256, 0, 0, d, 1u);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k<OP>, grid, 256, 0, 0, d, (unsigned)i);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}
int main() {
  const int grid = 256 * 8 * 4;
  unsigned* d; CK(hipMalloc(&d, grid * 256 * 4));
  const double ops = (double)grid * 256 * N * 8;  // chain steps
  const char* nm[] = {"mad_u64_u32+xor", "mul_hi+xor", "mul_lo+xor", "xor+add", "alignbit+add", "mul_u24+xor"};
  float t[6] = {run<0>(d, grid), run<1>(d, grid), run<2>(d, grid), run<3>(d, grid), run<4>(d, grid), run<5>(d, grid)};
  // wave64 instructions per SIMD per step pair; report ns and steps/clk/SIMD at 2.4 GHz
  for (int i = 0; i < 6; ++i)
    printf("%-18s %.3f ms  %.2f lane-steps/clk/CU\n", nm[i], t[i], ops / (t[i] * 1e-3) / 2.4e9 / 256);
  return 0;
}
