// lds_occupancy.hip — how many 256-thread workgroups with X bytes of dynamic
// LDS are co-resident per gfx950 CU: the runtime's occupancy answer vs a
// timing probe (blocks spin ~50 us; wall time / 50 us = waves of blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void spin(unsigned* out, long long cycles) {
  extern __shared__ unsigned lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0) out[blockIdx.x] = lds[5];
}
int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  printf("CUs %d sharedMemPerBlock %zu sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu\n",
         p.multiProcessorCount, p.sharedMemPerBlock, p.sharedMemPerMultiprocessor, p.maxSharedMemoryPerMultiProcessor);
  (void)hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  unsigned* d;
  (void)hipMalloc(&d, 1 << 20);
  const int cus = p.multiProcessorCount;
  for (int kb : {8, 16, 24, 32, 40, 52, 64, 80, 100, 128, 160}) {
    size_t lds = (size_t)kb * 1024;
    int occ = -1;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)spin, 256, lds);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = cus * 8;
    hipLaunchKernelGGL(spin, blocks, 256, lds, 0, d, 100000LL);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(spin, blocks, 256, lds, 0, d, 100000LL);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    // single wave of 1 block/CU as the unit
    hipLaunchKernelGGL(spin, cus, 256, lds, 0, d, 100000LL);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(spin, cus, 256, lds, 0, d, 100000LL);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float unit = 0;
    (void)hipEventElapsedTime(&unit, a, b);
    printf("LDS %3d KiB: occupancy API %d blocks/CU; measured %.2f blocks/CU resident (8 blocks/CU in %.3f ms, unit %.3f ms)\n",
           kb, occ, 8.0 / (ms / unit), ms, unit);
  }
  return 0;
}
