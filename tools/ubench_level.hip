// Microbenchmark of one Gauss-Seidel level step (kernel B's velocity level loop; V14 / V15 its
// position level step, round 5) in isolation:
// cycles per level step for several instruction forms, one wave per block, 1 block (a wave alone on
// its SIMD) or 2048 blocks (2 waves per SIMD, the C5 shard's residency).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o tools/build/ubench_level tools/ubench_level.hip
#include <hip/hip_runtime.h>
#include "../gym-macm_amd/csrc/flock_common.hpp"  // sqrt_rn / rcp_rn / div_by_invariant of the product
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void gsv(float2& va, float2& vb, float nx, float ny, float& ln, float& ltg, float mA,
                                    float mB, float kmass, float friction) {
  const float tx = ny, ty = -nx;
  {
    const float dvx = vb.x - va.x, dvy = vb.y - va.y;
    const float vt = dvx * tx + dvy * ty;
    float lambda = kmass * (-vt);
    const float maxf = friction * ln;
    const float ni = __builtin_amdgcn_fmed3f(ltg + lambda, -maxf, maxf);
    lambda = ni - ltg;
    ltg = ni;
    const float Px = lambda * tx, Py = lambda * ty;
    va.x = va.x - mA * Px; va.y = va.y - mA * Py;
    vb.x = vb.x + mB * Px; vb.y = vb.y + mB * Py;
  }
  {
    const float dvx = vb.x - va.x, dvy = vb.y - va.y;
    const float vn = dvx * nx + dvy * ny;
    float lambda = -kmass * vn;
    const float ni = fmaxf(ln + lambda, 0.0f);
    lambda = ni - ln;
    ln = ni;
    const float Px = lambda * nx, Py = lambda * ny;
    va.x = va.x - mA * Px; va.y = va.y - mA * Py;
    vb.x = vb.x + mB * Px; vb.y = vb.y + mB * Py;
  }
}

// kernel B's position step (flock_step_wg.hip gs_position<true>): b2PositionSolverManifold (Normalize
// with the product's sqrt_rn / rcp_rn), the clamped correction and -C / K; returns the separation
__device__ __forceinline__ float gsp(float2& ca, float2& cb, float radius, float mA, float mB) {
  float nx = cb.x - ca.x, ny = cb.y - ca.y;
  const float len = macm::sqrt_rn(nx * nx + ny * ny);
  if (len >= macm::kEps) {
    const float inv = macm::rcp_rn(len);
    nx *= inv;
    ny *= inv;
  }
  const float sep = ((cb.x - ca.x) * nx + (cb.y - ca.y) * ny) - radius - radius;
  const float Cc = __builtin_amdgcn_fmed3f(macm::kBaumgarte * (sep + macm::kLinearSlop), -macm::kMaxLinearCorrection, 0.0f);
  const float imp = macm::div_by_invariant(-Cc, mA + mB);
  const float Px = imp * nx, Py = imp * ny;
  ca.x = ca.x - mA * Px; ca.y = ca.y - mA * Py;
  cb.x = cb.x + mB * Px; cb.y = cb.y + mB * Py;
  return sep;
}

// packed position step (flock_step_wg.hip gs_position with kWgPacked, round 5)
__device__ __forceinline__ float gsp_pk(f2v& ca, f2v& cb, float radius, float mA, float mB) {
  const f2v d = cb - ca, d2 = d * d;
  const float len = macm::sqrt_rn(d2.x + d2.y);
  const f2v n = len < macm::kEps ? d : d * macm::rcp_rn(len);
  const f2v pr = d * n;
  const float sep = (pr.x + pr.y) - radius - radius;
  const float Cc = __builtin_amdgcn_fmed3f(macm::kBaumgarte * (sep + macm::kLinearSlop), -macm::kMaxLinearCorrection, 0.0f);
  const float imp = macm::div_by_invariant(-Cc, mA + mB);
  const f2v P = imp * n;
  ca = ca - mA * P;
  cb = cb + mB * P;
  return sep;
}

// packed form: the same IEEE ops on (x, y) pairs
__device__ __forceinline__ void gsv_pk(f2v& va, f2v& vb, f2v n, f2v t, float& ln, float& ltg, float mA,
                                       float kmass, float friction) {
  {
    const f2v dv = vb - va;
    const f2v pr = dv * t;
    const float vt = pr.x + pr.y;
    float lambda = kmass * (-vt);
    const float maxf = friction * ln;
    const float ni = __builtin_amdgcn_fmed3f(ltg + lambda, -maxf, maxf);
    lambda = ni - ltg;
    ltg = ni;
    const f2v P = lambda * t;
    const f2v mP = mA * P;
    va = va - mP;
    vb = vb + mP;
  }
  {
    const f2v dv = vb - va;
    const f2v pr = dv * n;
    const float vn = pr.x + pr.y;
    float lambda = -kmass * vn;
    const float ni = fmaxf(ln + lambda, 0.0f);
    lambda = ni - ln;
    ln = ni;
    const f2v P = lambda * n;
    const f2v mP = mA * P;
    va = va - mP;
    vb = vb + mP;
  }
}

template <int VAR>
__global__ __launch_bounds__(64) void lvl(float2* out, long long* cyc, int nlev, int iters, float mA, float fr) {
  __shared__ float2 s_v[1024 + 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024 + 64; i += 64) s_v[i] = make_float2(0.01f * i, -0.02f * i);
  __syncthreads();
  // two contacts per level: lanes 2l, 2l+1 at level l (disjoint bodies)
  const int mylv = lane >> 1;
  const int a = (lane * 7) & 1023, b = (lane * 7 + 3) & 1023;
  const float nx = 0.6f, ny = 0.8f;
  const float kmass = 1.0f / (mA + mA);
  float ln = 0.1f * lane, lt = 0.01f;
  float2* const pa0 = s_v + a;
  float2* const pb0 = s_v + b;
  float2* const pd = s_v + 1024 + lane;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (VAR == 0 || VAR == 9) {  // kernel B's form: branch-free, dummy slots, addresses a step ahead
      bool on = mylv == 0;
      float2* pa = on ? pa0 : pd;
      float2* pb = on ? pb0 : pd;
#pragma unroll VAR == 9 ? 2 : 1
      for (int lv = 0; lv < nlev; ++lv) {
        float2 va = *pa, vb = *pb;
        const bool onc = on;
        on = mylv == lv + 1;
        float2* const na = on ? pa0 : pd;
        float2* const nb = on ? pb0 : pd;
        float x = ln, y = lt;
        gsv(va, vb, nx, ny, x, y, mA, mA, kmass, fr);
        *pa = va;
        *pb = vb;
        ln = onc ? x : ln;
        lt = onc ? y : lt;
        pa = na;
        pb = nb;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 1) {  // exec-masked branch per level
      for (int lv = 0; lv < nlev; ++lv) {
        if (mylv == lv) {
          float2 va = *pa0, vb = *pb0;
          gsv(va, vb, nx, ny, ln, lt, mA, mA, kmass, fr);
          *pa0 = va;
          *pb0 = vb;
        }
        wave_lds_sync();
      }
    } else if constexpr (VAR == 2) {  // packed math, branch-free
      bool on = mylv == 0;
      f2v* pa = (f2v*)(on ? pa0 : pd);
      f2v* pb = (f2v*)(on ? pb0 : pd);
      const f2v n = {nx, ny}, t = {ny, -nx};
      for (int lv = 0; lv < nlev; ++lv) {
        f2v va = *pa, vb = *pb;
        const bool onc = on;
        on = mylv == lv + 1;
        f2v* const na = (f2v*)(on ? pa0 : pd);
        f2v* const nb = (f2v*)(on ? pb0 : pd);
        float x = ln, y = lt;
        gsv_pk(va, vb, n, t, x, y, mA, kmass, fr);
        *pa = va;
        *pb = vb;
        ln = onc ? x : ln;
        lt = onc ? y : lt;
        pa = na;
        pb = nb;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 3) {  // the VALU chain alone (bodies in registers, no LDS)
      float2 va = *pa0, vb = *pb0;
      for (int lv = 0; lv < nlev; ++lv) {
        const bool on = mylv == lv;
        float x = ln, y = lt;
        gsv(va, vb, nx, ny, x, y, mA, mA, kmass, fr);
        ln = on ? x : ln;
        lt = on ? y : lt;
      }
      *pa0 = va;
      *pb0 = vb;
    } else if constexpr (VAR == 4) {  // the LDS round trip alone (read, one add, write)
      bool on = mylv == 0;
      float2* pa = on ? pa0 : pd;
      float2* pb = on ? pb0 : pd;
      for (int lv = 0; lv < nlev; ++lv) {
        float2 va = *pa, vb = *pb;
        on = mylv == lv + 1;
        float2* const na = on ? pa0 : pd;
        float2* const nb = on ? pb0 : pd;
        va.x += vb.y;
        vb.x += va.y;
        *pa = va;
        *pb = vb;
        pa = na;
        pb = nb;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 6) {  // packed math under an exec-masked branch per level
      const f2v n = {nx, ny}, t = {ny, -nx};
      for (int lv = 0; lv < nlev; ++lv) {
        if (mylv == lv) {
          f2v va = *(f2v*)pa0, vb = *(f2v*)pb0;
          gsv_pk(va, vb, n, t, ln, lt, mA, kmass, fr);
          *(f2v*)pa0 = va;
          *(f2v*)pb0 = vb;
        }
        wave_lds_sync();
      }
    } else if constexpr (VAR == 7 || VAR == 8) {
      // chain lanes: lanes 0, 1 hold a chain each (one contact per level); body a is the chain's
      // (forwarded in registers from the lane's previous contact), body b comes from LDS: VAR 7
      // prefetched one level ahead (issued before this level's writes), VAR 8 read at the step's
      // start and waited for (an "X" level). Lanes >= 2 run the same instructions on dummy slots.
      const bool chain = lane < 2;
      float2* const pself = chain ? s_v + lane : pd;
      float2 va = *pself;
      const int cm = chain ? -1 : 0;  // branch-free: dummy lanes' b is their dummy slot
      auto bbody = [&](int l) -> float2* {
        const int idx = 2 + ((lane * 509 + l * 2 + (l & 1)) & 1021);
        return s_v + ((idx & cm) | ((1024 + lane) & ~cm));
      };
      float2 vbn = *bbody(0);
      __builtin_amdgcn_s_waitcnt(0);  // the loop's first step finds its operands in registers
      for (int lv = 0; lv < nlev; ++lv) {
        float2* const pb = bbody(lv);
        float2 vb;
        if constexpr (VAR == 7) {
          vb = vbn;
          vbn = *bbody(lv + 1);  // before this level's writes: valid for bodies not written now
          __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk to the step's end
        } else {
          vb = *pb;
        }
        float x = ln, y = lt;
        gsv(va, vb, nx, ny, x, y, mA, mA, kmass, fr);
        *pself = va;
        *pb = vb;
        ln = chain ? x : ln;
        lt = chain ? y : lt;
        if constexpr (VAR == 8) wave_lds_sync();
      }
    } else if constexpr (VAR == 12 || VAR == 13) {
      // V0 with ONE dummy slot shared by the lanes outside the level: their reads are an LDS
      // broadcast (no bank conflicts with the level's lanes). V12: only the level's lanes store
      // (exec-masked stores); V13: every lane stores (the dummy lanes all to the shared slot).
      float2* const ps = s_v + 1024;
      bool on = mylv == 0;
      float2* pa = on ? pa0 : ps;
      float2* pb = on ? pb0 : ps;
      for (int lv = 0; lv < nlev; ++lv) {
        float2 va = *pa, vb = *pb;
        const bool onc = on;
        on = mylv == lv + 1;
        float2* const na = on ? pa0 : ps;
        float2* const nb = on ? pb0 : ps;
        float x = ln, y = lt;
        gsv(va, vb, nx, ny, x, y, mA, mA, kmass, fr);
        if constexpr (VAR == 12) {
          if (onc) {
            *pa = va;
            *pb = vb;
          }
        } else {
          *pa = va;
          *pb = vb;
        }
        ln = onc ? x : ln;
        lt = onc ? y : lt;
        pa = na;
        pb = nb;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 10 || VAR == 11) {
      // uniform form (N <= 64): body b's velocity lives in lane b (vx, vy); the level's contact
      // (VAR 11: two disjoint contacts) has wave-uniform bodies, read by readlane, solved on
      // uniform values and written back by writelane; its normal and impulses live in lane
      // (level & 63) of per-lane registers. No LDS in the level loop.
      float vx = s_v[lane].x, vy = s_v[lane].y;
      float cnx = nx + 0.001f * lane, cny = ny - 0.001f * lane;
      auto rl = [](float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
      auto wl = [](float v, int l, float old) {  // as writelane_m0 in flock_step_w64.hip
        int o = __float_as_int(old);
        asm volatile("s_nop 1\n\tv_writelane_b32 %0, %1, m0"
                     : "+v"(o)
                     : "s"(__builtin_amdgcn_readfirstlane(__float_as_int(v))), "{m0}"(__builtin_amdgcn_readfirstlane(l)));
        return __int_as_float(o);
      };
      for (int lv = 0; lv < nlev; ++lv) {
        const int c = lv & 63;
        const int a0 = (lv * 7) & 63, b0 = (lv * 7 + 3) & 63;
        float2 va = make_float2(rl(vx, a0), rl(vy, a0)), vb = make_float2(rl(vx, b0), rl(vy, b0));
        float x = rl(ln, c), y = rl(lt, c);
        gsv(va, vb, rl(cnx, c), rl(cny, c), x, y, mA, mA, kmass, fr);
        if constexpr (VAR == 11) {
          const int c2 = (lv + 32) & 63;
          const int a1 = (lv * 7 + 5) & 63, b1 = (lv * 7 + 9) & 63;
          float2 va1 = make_float2(rl(vx, a1), rl(vy, a1)), vb1 = make_float2(rl(vx, b1), rl(vy, b1));
          float x1 = rl(ln, c2), y1 = rl(lt, c2);
          gsv(va1, vb1, rl(cnx, c2), rl(cny, c2), x1, y1, mA, mA, kmass, fr);
          vx = wl(va1.x, a1, vx);
          vy = wl(va1.y, a1, vy);
          vx = wl(vb1.x, b1, vx);
          vy = wl(vb1.y, b1, vy);
          ln = wl(x1, c2, ln);
          lt = wl(y1, c2, lt);
        }
        vx = wl(va.x, a0, vx);
        vy = wl(va.y, a0, vy);
        vx = wl(vb.x, b0, vx);
        vy = wl(vb.y, b0, vy);
        ln = wl(x, c, ln);
        lt = wl(y, c, lt);
      }
      s_v[lane] = make_float2(vx, vy);
    } else if constexpr (VAR == 14) {  // the position step's VALU chain alone (bodies in registers)
      float2 ca = *pa0, cb = make_float2(pa0->x + 0.9f, pa0->y + 0.1f);
      float mn = 0.0f;
      for (int lv = 0; lv < nlev; ++lv) {
        const float sep = gsp(ca, cb, 0.5f, mA, mA);
        mn = fminf(mn, sep);
      }
      *pa0 = ca;
      *pb0 = cb;
      ln += mn;
    } else if constexpr (VAR == 15) {  // kernel B's position level step: branch-free, LDS, atomic min
      float* const s_min = reinterpret_cast<float*>(s_v + 1024 + 32);  // per-lane words, never read here
      float* const pmi = reinterpret_cast<float*>(s_v + 1024) + (lane & 1);
      float* const pmd = s_min + lane;
      bool on = mylv == 0;
      float2* pa = on ? pa0 : pd;
      float2* pb = on ? pb0 : pd;
      float* pm = on ? pmi : pmd;
      for (int lv = 0; lv < nlev; ++lv) {
        float2 ca = *pa, cb = *pb;
        on = mylv == lv + 1;
        float2* const na = on ? pa0 : pd;
        float2* const nb = on ? pb0 : pd;
        float* const nm = on ? pmi : pmd;
        const float sep = gsp(ca, cb, 0.5f, mA, mA);
        *pa = ca;
        *pb = cb;
        __hip_atomic_fetch_min(pm, sep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        pa = na;
        pb = nb;
        pm = nm;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 16) {  // the packed position step's VALU chain alone (round 5)
      f2v ca = *(f2v*)pa0, cb = {pa0->x + 0.9f, pa0->y + 0.1f};
      float mn = 0.0f;
      for (int lv = 0; lv < nlev; ++lv) {
        const float sep = gsp_pk(ca, cb, 0.5f, mA, mA);
        mn = fminf(mn, sep);
      }
      *(f2v*)pa0 = ca;
      *(f2v*)pb0 = cb;
      ln += mn;
    } else if constexpr (VAR == 17) {  // V15 on packed pairs: kernel B's position level step (round 5)
      float* const s_min = reinterpret_cast<float*>(s_v + 1024 + 32);
      float* const pmi = reinterpret_cast<float*>(s_v + 1024) + (lane & 1);
      float* const pmd = s_min + lane;
      bool on = mylv == 0;
      f2v* pa = (f2v*)(on ? pa0 : pd);
      f2v* pb = (f2v*)(on ? pb0 : pd);
      float* pm = on ? pmi : pmd;
      for (int lv = 0; lv < nlev; ++lv) {
        f2v ca = *pa, cb = *pb;
        on = mylv == lv + 1;
        f2v* const na = (f2v*)(on ? pa0 : pd);
        f2v* const nb = (f2v*)(on ? pb0 : pd);
        float* const nm = on ? pmi : pmd;
        const float sep = gsp_pk(ca, cb, 0.5f, mA, mA);
        *pa = ca;
        *pb = cb;
        __hip_atomic_fetch_min(pm, sep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        pa = na;
        pb = nb;
        pm = nm;
        wave_lds_sync();
      }
    } else if constexpr (VAR == 5) {  // packed VALU chain alone
      f2v va = *(f2v*)pa0, vb = *(f2v*)pb0;
      const f2v n = {nx, ny}, t = {ny, -nx};
      for (int lv = 0; lv < nlev; ++lv) {
        const bool on = mylv == lv;
        float x = ln, y = lt;
        gsv_pk(va, vb, n, t, x, y, mA, kmass, fr);
        ln = on ? x : ln;
        lt = on ? y : lt;
      }
      *(f2v*)pa0 = va;
      *(f2v*)pb0 = vb;
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + lane] = s_v[lane] + make_float2(ln, lt);
}

template <int VAR>
static void run(const char* name, int blocks, int nlev, int iters) {
  float2* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float2) * 64 * blocks);
  hipMalloc(&cyc, sizeof(long long) * blocks);
  lvl<VAR><<<blocks, 64>>>(out, cyc, nlev, iters, 1.2732395f, 0.3f);  // warm
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  lvl<VAR><<<blocks, 64>>>(out, cyc, nlev, iters, 1.2732395f, 0.3f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(blocks);
  hipMemcpy(h.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double steps = (double)nlev * iters;
  // s_memtime counts shader clocks; the event time gives the wall clock per step
  printf("%-28s blocks %5d: median %7.1f cyc/step, max %7.1f cyc/step, wall %7.1f ns/step\n", name, blocks,
         h[blocks / 2] / steps, h[blocks - 1] / steps, ms * 1e6 / steps);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int nlev = 32, iters = 400;
  for (int blocks : {1, 2048, 4096}) {
    run<0>("V0 branch-free (kernel B)", blocks, nlev, iters);
    run<1>("V1 exec-masked branch", blocks, nlev, iters);
    run<2>("V2 packed, branch-free", blocks, nlev, iters);
    run<6>("V6 packed, exec-masked branch", blocks, nlev, iters);
    run<9>("V9 = V0 unrolled x2", blocks, nlev, iters);
    run<7>("V7 chain lanes, prefetched b", blocks, nlev, iters);
    run<8>("V8 chain lanes, b read+wait", blocks, nlev, iters);
    run<12>("V12 shared dummy, masked st", blocks, nlev, iters);
    run<13>("V13 shared dummy, all store", blocks, nlev, iters);
    run<10>("V10 uniform, 1 contact/level", blocks, nlev, iters);
    run<11>("V11 uniform, 2 contacts/level", blocks, nlev, iters);
    run<3>("V3 VALU chain only", blocks, nlev, iters);
    run<14>("V14 position VALU chain only", blocks, nlev, iters);
    run<15>("V15 position, kernel B form", blocks, nlev, iters);
    run<5>("V5 packed VALU chain only", blocks, nlev, iters);
    run<16>("V16 packed position chain", blocks, nlev, iters);
    run<17>("V17 packed position, B form", blocks, nlev, iters);
    run<4>("V4 LDS round trip only", blocks, nlev, iters);
  }
  return 0;
}
