// tools/rcp_sqrt_gpu_check.hip — device check behind rcp_rn / sqrt_rn / div_by_invariant (csrc/flock_common.hpp):
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

// div_by_invariant(n, K) == n / K for every float32 n in {-0, +0} u [2^-40, 0.2] (the position solve's
// -C: 0 or >= 2^-40, at most kMaxLinearCorrection) and K in Ks: the default config's K and random ones.
__global__ void check_div(const float* Ks, int nK, uint32_t end, unsigned long long* bad) {
  unsigned long long nb[2] = {};  // n = 0 or n >= 2^-40 (what the step can give it), below
  for (int k = 0; k < nK; ++k) {
    const float K = Ks[k];
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u <= end; u += (uint64_t)gridDim.x * blockDim.x) {
      const float n = __uint_as_float((uint32_t)u);
      const float a = macm::div_by_invariant(n, K), b = n / K;
      if (__float_as_uint(a) != __float_as_uint(b)) ++nb[(n == 0.0f || n >= 0x1p-40f) ? 0 : 1];
    }
    // n = -0.0 (the step gives it when C = +0: -C), compared bitwise like the rest
    if (blockIdx.x == 0 && threadIdx.x == 0 &&
        __float_as_uint(macm::div_by_invariant(-0.0f, K)) != __float_as_uint(-0.0f / K))
      ++nb[0];
  }
  atomicAdd(&bad[0], nb[0]);
  atomicAdd(&bad[1], nb[1]);
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
  // K = 2 / (density * pi * r^2) in float32 as the step derives it: default (r 0.5, density 1)
  // and 255 random radius / density pairs
  const int nK = 256;
  float hK[nK];
  uint64_t st = 0x9e3779b97f4a7c15ull;
  for (int k = 0; k < nK; ++k) {
    float r = 0.5f, d = 1.0f;
    if (k) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      r = 0.05f + (float)((st >> 40) & 0xffff) / 65536.0f * 2.0f;
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      d = 0.1f + (float)((st >> 40) & 0xffff) / 65536.0f * 10.0f;
    }
    const float m = 1.0f / (d * 3.14159265359f * r * r);
    hK[k] = m + m;
  }
  float* dK;
  unsigned long long* dbad;
  if (hipMalloc(&dK, sizeof hK) != hipSuccess || hipMalloc(&dbad, 16) != hipSuccess) return 2;
  (void)hipMemcpy(dK, hK, sizeof hK, hipMemcpyHostToDevice);
  (void)hipMemset(dbad, 0, 16);
  const uint32_t nend = 0x3e4ccccdu;  // 0.2f
  hipLaunchKernelGGL(check_div, dim3(8192), dim3(256), 0, 0, dK, nK, nend, dbad);
  unsigned long long hd[2] = {};
  (void)hipMemcpy(hd, dbad, 16, hipMemcpyDeviceToHost);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("  div_by_invariant != n / K, n in {0} u [2^-40, 0.2] x %d K values (default K = %.9g): %llu; "
         "n in (0, 2^-40): %llu\n", nK, hK[0], hd[0], hd[1]);
  return (hb[kRcpIn] | hb[kSqrtIn] | hb[kSqrtBranch] | hd[0]) != 0;
}
