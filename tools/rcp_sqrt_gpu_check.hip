// tools/rcp_sqrt_gpu_check.hip — device check behind rcp_rn / sqrt_rn (csrc/flock_common.hpp):
// over every non-negative finite float32 x, counts
//   rcp:  rcp_rn(x) != 1.0f / x                for x in [2^-23, 2^64]   (expected 0)
//   sqrt: sqrt_rn(x) != sqrtf(x)               for x >= 2^-48           (expected 0)
//   sqrt: (sqrt_rn(x) < FLT_EPSILON) != (sqrtf(x) < FLT_EPSILON)  for every x (expected 0)
// and, for information, the mismatches outside those ranges.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I gym-macm_amd/csrc tools/rcp_sqrt_gpu_check.hip -o tools/build/rcp_sqrt_gpu_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "flock_common.hpp"

enum { kRcpIn, kRcpOut, kSqrtIn, kSqrtOut, kSqrtBranch, kNCount };

__global__ void check(uint32_t end, unsigned long long* bad, uint32_t* first) {
  unsigned long long nb[kNCount] = {};
  for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < end; u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)u);
    if (x > 0.0f) {
      const bool in = x >= 0x1p-23f && x <= 0x1p64f;
      const float a = macm::rcp_rn(x), b = 1.0f / x;
      if (__float_as_uint(a) != __float_as_uint(b)) {
        ++nb[in ? kRcpIn : kRcpOut];
        if (in) atomicMin(&first[kRcpIn], (uint32_t)u);
      }
    }
    const float a = macm::sqrt_rn(x), b = sqrtf(x);
    const bool in = x >= 0x1p-48f;
    if (__float_as_uint(a) != __float_as_uint(b)) {
      ++nb[in ? kSqrtIn : kSqrtOut];
      if (in) atomicMin(&first[kSqrtIn], (uint32_t)u);
    }
    if ((a < macm::kEps) != (b < macm::kEps)) ++nb[kSqrtBranch];
  }
  for (int i = 0; i < kNCount; ++i) atomicAdd(&bad[i], nb[i]);
}

int main() {
  unsigned long long* bad;
  uint32_t* first;
  if (hipMalloc(&bad, 8 * kNCount) != hipSuccess || hipMalloc(&first, 4 * kNCount) != hipSuccess) return 2;
  (void)hipMemset(bad, 0, 8 * kNCount);
  (void)hipMemset(first, 0xff, 4 * kNCount);
  const uint32_t end = 0x7f800000u;  // +0 .. largest finite float32
  hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, end, bad, first);
  unsigned long long hb[kNCount];
  uint32_t hf[kNCount];
  (void)hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("over %u non-negative float32 inputs:\n", end);
  printf("  rcp_rn  != 1.0f/x,  x in [2^-23, 2^64]: %llu (first 0x%08x); outside: %llu\n", hb[kRcpIn], hf[kRcpIn], hb[kRcpOut]);
  printf("  sqrt_rn != sqrtf,   x >= 2^-48:         %llu (first 0x%08x); below: %llu\n", hb[kSqrtIn], hf[kSqrtIn], hb[kSqrtOut]);
  printf("  sqrt_rn / sqrtf disagree on len < FLT_EPSILON: %llu\n", hb[kSqrtBranch]);
  return (hb[kRcpIn] | hb[kSqrtIn] | hb[kSqrtBranch]) != 0;
}
