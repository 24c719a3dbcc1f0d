// Workgroup launch-rate probe: empty / near-empty kernels with N blocks of 256
// threads and S bytes of dynamic LDS, timed with HIP events (10 launches each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void empty_k(int* out) {
  extern __shared__ int sm[];
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = sm[0];
}

int main() {
  int* d;
  hipMalloc(&d, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks[] = {4096, 16384, 32768, 65536};
  const int lds[] = {0, 16384, 40960, 53536};
  for (int b : blocks)
    for (int s : lds) {
      hipLaunchKernelGGL(empty_k, dim3(b), dim3(256), s, 0, d);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(empty_k, dim3(b), dim3(256), s, 0, d);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("blocks %6d lds %6d: %.4f ms per launch, %.1f ns per block\n", b, s, ms / 10, ms / 10 * 1e6 / b);
    }
  return 0;
}
