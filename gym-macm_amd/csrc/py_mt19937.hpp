// py_mt19937.hpp — CPython `random` generator (Modules/_randommodule.c) for
// reproducing the reference's initial state: gym_macm/envs/mvmnt.py:47-64 draws
// targets and agent poses from the global `random` module, so env e of a batch
// seeded with s is initialised exactly like Flock(...) after random.seed(s + e).
// (MT19937, init_by_array over the 32-bit words of abs(seed), random() = res53.)
#pragma once
#include <stdint.h>

namespace macm {

class PyMT19937 {
 public:
  explicit PyMT19937(uint64_t seed) {
    uint32_t key[2] = {(uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32)};
    init_by_array(key, key[1] ? 2 : 1);
  }

  uint32_t next_u32() {
    if (idx_ >= kN) twist();
    uint32_t y = mt_[idx_++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // random.random()
  double random() {
    const uint32_t a = next_u32() >> 5, b = next_u32() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }

  // random.uniform(a, b) = a + (b - a) * random()
  double uniform(double a, double b) { return a + (b - a) * random(); }

  // Generator state (624 words + position), as the device-side stream continues it
  // (csrc/env_reset.hip).
  static constexpr int kWords = 624;
  const uint32_t* state() const { return mt_; }
  int index() const { return idx_; }

 private:
  static constexpr int kN = 624, kM = 397;
  uint32_t mt_[kN];
  int idx_ = kN + 1;

  void init_genrand(uint32_t s) {
    mt_[0] = s;
    for (int i = 1; i < kN; i++) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
    idx_ = kN;
  }

  void init_by_array(const uint32_t* key, int n) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = kN > n ? kN : n; k; k--) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      if (++i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
      if (++j >= n) j = 0;
    }
    for (int k = kN - 1; k; k--) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      if (++i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
    }
    mt_[0] = 0x80000000u;
  }

  void twist() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    int kk = 0;
    uint32_t y;
    for (; kk < kN - kM; kk++) {
      y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
      mt_[kk] = mt_[kk + kM] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < kN - 1; kk++) {
      y = (mt_[kk] & 0x80000000u) | (mt_[kk + 1] & 0x7fffffffu);
      mt_[kk] = mt_[kk + (kM - kN)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    y = (mt_[kN - 1] & 0x80000000u) | (mt_[0] & 0x7fffffffu);
    mt_[kN - 1] = mt_[kM - 1] ^ (y >> 1) ^ mag01[y & 1u];
    idx_ = 0;
  }
};

}  // namespace macm
