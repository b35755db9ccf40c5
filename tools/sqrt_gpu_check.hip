// tools/sqrt_gpu_check.hip — device check behind obs_sqrt (csrc/flock_common.hpp): for every
// non-negative finite float32 x, the kernels' sqrtf(x) must equal (float)sqrt((double)x).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/sqrt_gpu_check.hip -o tools/build/sqrt_gpu_check
//   tools/build/sqrt_gpu_check      prints the number of mismatching inputs (expected 0)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void check(uint32_t begin, uint32_t end, unsigned long long* bad, uint32_t* first) {
  unsigned long long nb = 0;
  for (uint64_t u = begin + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < end;
       u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)u);
    const float a = sqrtf(x);
    const float b = (float)sqrt((double)x);
    if (__float_as_uint(a) != __float_as_uint(b)) {
      ++nb;
      atomicMin(first, (uint32_t)u);
    }
  }
  atomicAdd(bad, nb);
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
  (void)hipMemset(bad, 0, 8);
  (void)hipMemset(first, 0xff, 4);
  const uint32_t end = 0x7f800000u;  // +0 .. largest finite float32
  hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, 0u, end, bad, first);
  unsigned long long hb = 0;
  uint32_t hf = 0;
  (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("sqrtf vs (float)sqrt((double)x) over %u non-negative float32 inputs: %llu mismatches", end, hb);
  if (hb) printf(" (first at bits 0x%08x)", hf);
  printf("\n");
  return hb != 0;
}
