// tools/trig_gpu_check.hip — the device half of the exhaustive action-trig check.
// For every float32 x with |x| < 2^19 (both signs) it evaluates the device libm
// (ocml) sincos at x and x + pi/2 and macm_action_trig (csrc/macm_math.h), exactly as
// the step does, and records the inputs whose float32 action outcomes (tools/trig_outcomes.h)
// differ between the two, with the ocml values. tools/trig_check.c --ocml FILE then
// decides, against glibc, which inputs the library path would get wrong, so both paths
// are characterised over the same complete input set. It also prints a digest of every
// macm_action_trig result bit; trig_check.c prints the host's, and they must be equal.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I gym-macm_amd/csrc -I tools \
//         tools/trig_gpu_check.hip -o tools/build/trig_gpu_check
//   tools/build/trig_gpu_check gpurun_out/trig/ocml_records.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "macm_math.h"
#include "trig_outcomes.h"

struct Rec {
  uint32_t xbits, pad;
  double s0, c0, s1, c1;
};

constexpr uint32_t kLim = 0x49000000u;  // 2^19 as float32 bits
constexpr unsigned kCap = 1u << 16;

__global__ void check(uint64_t begin, uint64_t end, Rec* out, unsigned* n_out, unsigned long long* n_f64,
                      unsigned long long* digest) {
  unsigned long long f64 = 0, dig = 0;
  for (uint64_t k = begin + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < end;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t u = (uint32_t)(k < kLim ? k : (k - kLim) | 0x80000000u);
    const float f = __uint_as_float(u);
    const double x = (double)f, x1 = x + M_PI / 2;
    double s0l, c0l, s1l, c1l, s0m, c0m, s1m, c1m;
    sincos(x, &s0l, &c0l);
    sincos(x1, &s1l, &c1l);
    macm_action_trig(f, &s0m, &c0m, &s1m, &c1m);
    const bool d = __double_as_longlong(s0l) != __double_as_longlong(s0m) ||
                   __double_as_longlong(c0l) != __double_as_longlong(c0m) ||
                   __double_as_longlong(s1l) != __double_as_longlong(s1m) ||
                   __double_as_longlong(c1l) != __double_as_longlong(c1m);
    f64 += d;
    dig += trig_digest(s0m, c0m, s1m, c1m);
    if (d && f32_outcomes_differ(c0l, s0l, c1l, s1l, c0m, s0m, c1m, s1m)) {
      const unsigned i = atomicAdd(n_out, 1u);
      if (i < kCap) out[i] = Rec{u, 0u, s0l, c0l, s1l, c1l};
    }
  }
  atomicAdd(n_f64, f64);
  atomicAdd(digest, dig);
}

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s OUT.bin\n", argv[0]);
    return 2;
  }
  Rec* d_out;
  unsigned* d_n;
  unsigned long long* d_f64;
  unsigned long long* d_dig;
  CK(hipMalloc(&d_out, sizeof(Rec) * kCap));
  CK(hipMalloc(&d_n, sizeof(unsigned)));
  CK(hipMalloc(&d_f64, sizeof(unsigned long long)));
  CK(hipMalloc(&d_dig, sizeof(unsigned long long)));
  CK(hipMemset(d_dig, 0, sizeof(unsigned long long)));
  CK(hipMemset(d_n, 0, sizeof(unsigned)));
  CK(hipMemset(d_f64, 0, sizeof(unsigned long long)));
  const uint64_t total = 2ull * kLim, chunk = 1ull << 28;
  for (uint64_t b = 0; b < total; b += chunk) {
    const uint64_t e = b + chunk < total ? b + chunk : total;
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, b, e, d_out, d_n, d_f64, d_dig);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  unsigned n = 0;
  unsigned long long f64 = 0, dig = 0;
  CK(hipMemcpy(&n, d_n, sizeof(n), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&dig, d_dig, sizeof(dig), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&f64, d_f64, sizeof(f64), hipMemcpyDeviceToHost));
  const unsigned kept = n < kCap ? n : kCap;
  Rec* h = new Rec[kept > 0 ? kept : 1];
  CK(hipMemcpy(h, d_out, sizeof(Rec) * kept, hipMemcpyDeviceToHost));
  FILE* fp = fopen(argv[1], "wb");
  if (!fp) {
    perror(argv[1]);
    return 1;
  }
  fwrite(&kept, sizeof(kept), 1, fp);
  fwrite(h, sizeof(Rec), kept, fp);
  fclose(fp);
  printf("inputs %llu  f64 ocml != macm_action_trig: %llu  float32 outcomes differ: %u (kept %u)\n",
         (unsigned long long)total, f64, n, kept);
  printf("device macm_action_trig digest %016llx\n", dig);
  delete[] h;
  return n > kCap;
}
