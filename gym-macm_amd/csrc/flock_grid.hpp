// flock_grid.hpp — per-env spatial cells for the workgroup path's pair sweep (64 < N <= 1024),
// rebuilt in LDS every step: x-strip cells swept by LDS tiles. It replaces the O(N^2) all-pairs
// sweep of SynchronizeFixtures' pair search (Box2D's dynamic tree, reached through world.Step,
// cm_framework.py:222-223) and of get_obs' nearest-neighbour loop (mvmnt.py:185-196).
//
// Cells. Bodies are binned by the x of their position c into strips of width w, counting-sorted
// into LDS (entry = c.x, c.y, body). Every fat AABB contains its body's position
// (SynchronizeFixtures builds it around the old and new circle), so with Dx = max(c.x - lo.x) +
// max(hi.x - c.x) over the env's bodies, two fat AABBs can overlap only if |c_i.x - c_j.x| <= Dx.
//
// Tiles. Thread t takes the body of sorted entry t, so a wave holds 64 bodies of neighbouring
// strips: an x-interval [x_lo, x_hi]. Every partner of every lane lies in the strips covering
// [x_lo - Dx, x_hi + Dx] — one contiguous range of the sorted entries. The wave walks that
// range once with the same entry read by every lane (an LDS broadcast, as in an all-pairs
// sweep, no per-lane divergence) and each lane tests each candidate exactly: the range only
// cuts what cannot overlap. This was measured against a 2-D hash (3 x 3 cells per body, each
// lane walking its own cells): the per-lane walks diverge and their indirection costs more
// than the cells save at N <= 1024.
//
// Nearest neighbour. Each lane's best d2 over the tile is certified when every body outside the
// tile's strips is farther: the lane's x-distance to the tile's outer strip edges, less the
// rounding margin, squared, exceeds best. Otherwise the wave walks the remaining strips for the
// uncertified lanes. Ties go to the lowest index, so the result equals the reference's
// ascending scan with strict '<' in any visiting order.
//
// Rounding. u = fl((c.x - x0) * inv) is monotone in c.x, so strip membership is consistent
// between bodies; the tile is widened by one strip each way beyond [x_lo - Dx, x_hi + Dx], which
// covers the rounding of u (|u| < 2^16 by construction of w) and of x_lo - Dx, x_hi + Dx;
// certification subtracts 1/32 strip. Non-finite positions or extents disable the cells for the
// env: the caller runs its all-pairs sweep.
#pragma once

#include "flock_common.hpp"

namespace macm {
namespace grid {

constexpr int kCellsMinAgents = 512;  // below: the all-pairs sweep (StepParams.sweep overrides)

__host__ __device__ inline int buckets(int N) {  // strips: a power of two >= N
  int h = 64;
  while (h < N) h <<= 1;
  return h;
}

struct Lds {
  float* red;        // [16 waves][4] reduction scratch
  float* par;        // [8]: x0, inv, w, Dx, ok
  uint32_t* start;   // [H + 1] strip starts
  float4* ent;       // [N] (c.x, c.y, body bits, 0), strip order
  int H;
};

// Build the strips (every thread of the block calls it; act = thread holds a body at c with
// fat AABB f). Returns false if the env must use the all-pairs sweep.
__device__ __forceinline__ bool build(const Lds& G, bool act, float2 c, float4 f) {
  const int tid = threadIdx.x, BS = blockDim.x, lane = tid & 63, wid = tid >> 6, nw = BS >> 6;
  for (int h = tid; h <= G.H; h += BS) G.start[h] = 0u;
  // v: max(c.x - lo.x), max(hi.x - c.x), max(c.x), max(-c.x)
  float v[4] = {0.0f, 0.0f, -__builtin_inff(), -__builtin_inff()};
  if (act) {
    v[0] = c.x - f.x;
    v[1] = f.z - c.x;
    v[2] = c.x;
    v[3] = -c.x;
    // NaN / inf anywhere (a NaN sum survives, fmaxf would drop it): disable the cells
    if (!__builtin_isfinite(v[0] + v[1] + c.x + c.y + f.y + f.w)) v[0] = __builtin_inff();
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] = fmaxf(v[k], __shfl_xor(v[k], o, 64));
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) G.red[wid * 4 + k] = v[k];
  }
  __syncthreads();
  if (tid == 0) {
    float m[4] = {0.0f, 0.0f, -__builtin_inff(), -__builtin_inff()};
    for (int w = 0; w < nw; ++w) {
#pragma unroll
      for (int k = 0; k < 4; ++k) m[k] = fmaxf(m[k], G.red[w * 4 + k]);
    }
    const float Dx = m[0] + m[1], x0 = -m[3], ext = m[2] - x0;
    // strip width: Dx / 2 (a tile then spans its own strips + ~2 on each side), at least the
    // extent / H so the strips cover the env, and |u| stays < 2^16
    float w = fmaxf(Dx * 0.5f, ext * (1.0f / (float)G.H) * (1.0f + 1.0f / 64.0f));
    w = fmaxf(w, fmaxf(fabsf(x0), fabsf(m[2])) * (1.0f / 32768.0f));
    w = fmaxf(w, 1e-6f);
    const bool ok = __builtin_isfinite(Dx) && __builtin_isfinite(ext) && fabsf(x0) < 1e15f && fabsf(m[2]) < 1e15f &&
                    w < 1e30f;
    G.par[0] = x0;
    G.par[1] = 1.0f / w;
    G.par[2] = w;
    G.par[3] = Dx;
    G.par[4] = ok ? 1.0f : 0.0f;
  }
  __syncthreads();
  if (G.par[4] == 0.0f) return false;
  const float x0 = G.par[0], inv = G.par[1];
  int slot = 0, h = 0;
  if (act) {
    h = min(G.H - 1, max(0, (int)floorf((c.x - x0) * inv)));
    slot = (int)atomicAdd(&G.start[h], 1u);
  }
  __syncthreads();
  // exclusive scan of the strip counts in place: thread t owns strips [t*per, (t+1)*per)
  {
    const int per = (G.H + BS - 1) / BS;
    const int b0 = tid * per, b1 = min(G.H, b0 + per);
    uint32_t s = 0;
    for (int b = b0; b < b1; ++b) s += G.start[b];
    uint32_t incl = s;  // block scan: wave shuffles + per-wave totals (red is free again)
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    if (lane == 63) ((uint32_t*)G.red)[wid] = incl;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int w = 0; w < nw; ++w) {
      const uint32_t t = ((uint32_t*)G.red)[w];
      if (w < wid) base += t;
      total += t;
    }
    uint32_t run = base + incl - s;
    for (int b = b0; b < b1; ++b) {
      const uint32_t cnt = G.start[b];
      G.start[b] = run;
      run += cnt;
    }
    if (tid == 0) G.start[G.H] = total;
  }
  __syncthreads();
  if (act) G.ent[G.start[h] + slot] = make_float4(c.x, c.y, __int_as_float(tid), 0.0f);
  __syncthreads();
  return true;
}

// The strip of an x (clamped to the env's strips).
__device__ __forceinline__ int strip_of(const Lds& G, float x) {
  const float u = floorf((x - G.par[0]) * G.par[1]);
  return (int)fminf(fmaxf(u, 0.0f), (float)(G.H - 1));
}

// The tile of the wave (lanes with has = true hold a body at x): the strips [s0, s1] that can
// hold a partner of any of them. Wave-uniform.
__device__ __forceinline__ void tile(const Lds& G, bool has, float x, int& s0, int& s1) {
  float lo = has ? x : __builtin_inff(), hi = has ? -x : __builtin_inff();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fminf(hi, __shfl_xor(hi, o, 64));
  }
  lo = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(lo)));
  hi = -__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(hi)));
  if (!(lo <= hi)) {  // no bodies in this wave
    s0 = 1;
    s1 = 0;
    return;
  }
  const float Dx = G.par[3];
  s0 = max(0, strip_of(G, lo - Dx) - 1);
  s1 = min(G.H - 1, strip_of(G, hi + Dx) + 1);
}

// Is best below the squared distance of every body outside strips [s0, s1]?
__device__ __forceinline__ bool certified(const Lds& G, float x, int s0, int s1, float best) {
  const float x0 = G.par[0], w = G.par[2], inv = G.par[1];
  const float u = (x - x0) * inv;
  float g = __builtin_inff();
  if (s0 > 0) g = fminf(g, u - (float)s0);
  if (s1 < G.H - 1) g = fminf(g, (float)(s1 + 1) - u);
  if (g == __builtin_inff()) return true;
  g -= 1.0f / 32.0f;
  if (!(g > 0.0f)) return false;
  const float gw = g * w * (1.0f - 1e-5f);
  return best < gw * gw;
}

// nearest other body: d2 < best, ties to the lowest index (mvmnt.py:194's strict '<' in
// ascending order)
__device__ __forceinline__ void nn_take(int j, float d2, float& best, int& bj) {
  if (d2 < best || (d2 == best && j < bj)) {
    best = d2;
    bj = j;
  }
}

}  // namespace grid
}  // namespace macm
