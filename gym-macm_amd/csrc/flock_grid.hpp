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

constexpr int kCellsMinAgents = 256;  // below: the all-pairs sweep (StepParams.sweep overrides)

__host__ __device__ inline int buckets(int N) {  // strips: a power of two >= N / 4, at least 64
  int h = 64;
  while (4 * h < N) h <<= 1;
  return h;
}

struct Lds {
  float* red;        // [16 waves][4] reduction scratch
  float* par;        // [8]: x0, inv, w, Dx, ok, margin
  uint32_t* start;   // [H + 1] strip starts
  float4* ent;       // [N] (c.x, c.y, body bits, 0), strip order
  uint32_t* sext;    // [H] per strip: the largest x-extent max(c.x - lo.x, hi.x - c.x) of its bodies (float bits)
  int H;
};

// Build the strips (every thread of the block calls it; act = thread holds a body at c with
// fat AABB f). Returns false if the env must use the all-pairs sweep.
__device__ __forceinline__ bool build(const Lds& G, bool act, float2 c, float4 f) {
  const int tid = threadIdx.x, BS = blockDim.x, lane = tid & 63, wid = tid >> 6, nw = BS >> 6;
  for (int h = tid; h <= G.H; h += BS) G.start[h] = 0u;
  for (int h = tid; h < G.H; h += BS) G.sext[h] = 0u;
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
    // strip width: the extent / H (the strips just cover the env: narrow strips, so the per-strip
    // extents prune finely, tile()), and |u| stays < 2^16
    float w = ext * (1.0f / (float)G.H) * (1.0f + 1.0f / 64.0f);
    w = fmaxf(w, fmaxf(fabsf(x0), fabsf(m[2])) * (1.0f / 32768.0f));
    w = fmaxf(w, 1e-6f);
    const bool ok = __builtin_isfinite(Dx) && __builtin_isfinite(ext) && fabsf(x0) < 1e15f && fabsf(m[2]) < 1e15f &&
                    w < 1e30f;
    G.par[0] = x0;
    G.par[1] = 1.0f / w;
    G.par[2] = w;
    G.par[3] = Dx;
    G.par[4] = ok ? 1.0f : 0.0f;
    // absolute margin of the strip pruning: a strip edge x0 + s w and its sums with extents are
    // float expressions of magnitude <= |x0| + ext + Dx + H w; 2^-20 of that covers their rounding
    // and a body's strip (u rounded to the strip below or above) is covered by one strip of slack
    G.par[5] = (fabsf(x0) + ext + Dx + (float)G.H * w) * (1.0f / 1048576.0f);
  }
  __syncthreads();
  if (G.par[4] == 0.0f) return false;
  const float x0 = G.par[0], inv = G.par[1];
  int slot = 0, h = 0;
  if (act) {
    h = min(G.H - 1, max(0, (int)floorf((c.x - x0) * inv)));
    slot = (int)atomicAdd(&G.start[h], 1u);
    // extents are >= +0 (the fat AABB contains c), so their float bits order as the floats
    atomicMax(&G.sext[h], __float_as_uint(fmaxf(fmaxf(c.x - f.x, f.z - c.x), 0.0f)));
  }
  __syncthreads();
  // exclusive scan of the strip counts in place: thread t owns strips [t*per, (t+1)*per)
  {
    const int per = (G.H + BS - 1) / BS;
    const int b0 = tid * per, b1 = min(G.H, b0 + per);
    uint32_t s = 0;
    for (int b = b0; b < b1; ++b) s += G.start[b];
    const uint32_t incl = (uint32_t)wave_prefix_sum((int)s);  // block scan: wave DPP scan + per-wave totals (red is free again)
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

// The tile of the wave (lanes with has = true hold a body at x with x-extent e): the strips
// [s0, s1] that can hold a partner of any of them by the env-wide Dx (wave-uniform), and within
// them the strips worth walking: a non-empty strip s whose bodies all lie farther in x from the
// wave's [lo, hi] than E_W + E_s (the wave's and the strip's largest extents) holds no body whose
// fat AABB can overlap one of the wave's (|c_i.x - c_j.x| <= e_i + e_j for an overlap), so it is
// skipped. At C5 a wave's x-range is ~1.4 m, Dx ~3.3 m but a typical extent ~0.75 m: the walked
// strips hold ~40% fewer candidates than [s0, s1]. [c0, c1]: the strips around the wave's own that
// are walked or empty (the nearest-neighbour certification covers the strips outside it,
// certified()). Batches of 64 strips: batch(b) returns the walked-strip mask of strips
// s0 + 64 b + k and updates [c0, c1].
struct Tile {
  float lo, hi, ew;
  int s0, s1, c0, c1, o0, o1;
  bool gap_lo, gap_hi;
};
__device__ __forceinline__ void tile(const Lds& G, bool has, float x, float e, Tile& T) {
  float lo = has ? x : __builtin_inff(), hi = has ? -x : __builtin_inff(), ew = has ? e : 0.0f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fminf(hi, __shfl_xor(hi, o, 64));
    ew = fmaxf(ew, __shfl_xor(ew, o, 64));
  }
  T.lo = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(lo)));
  T.hi = -__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(hi)));
  T.ew = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ew)));
  T.gap_lo = T.gap_hi = false;
  if (!(T.lo <= T.hi)) {  // no bodies in this wave
    T.s0 = T.c0 = T.o0 = 1;
    T.s1 = T.c1 = T.o1 = 0;
    return;
  }
  const float Dx = G.par[3];
  T.s0 = max(0, strip_of(G, T.lo - Dx) - 1);
  T.s1 = min(G.H - 1, strip_of(G, T.hi + Dx) + 1);
  T.o0 = strip_of(G, T.lo);  // the wave's own strips
  T.o1 = strip_of(G, T.hi);
  T.c0 = T.s0;
  T.c1 = T.s1;
}
__device__ __forceinline__ unsigned long long batch(const Lds& G, Tile& T, int b) {
  const float x0 = G.par[0], w = G.par[2], mg = G.par[5];
  const int s = T.s0 + 64 * b + (int)(threadIdx.x & 63);
  bool walk = false, skip = false;
  if (s <= T.s1) {
    const bool empty = G.start[s + 1] == G.start[s];
    const float es = __uint_as_float(G.sext[s]);
    const float left = x0 + (float)s * w, right = left + w;
    // one strip of slack each way for the binning's rounding, mg for these sums'
    skip = !empty && (right + w + es + T.ew + mg < T.lo || left - w - es - T.ew - mg > T.hi);
    walk = !empty && !skip;
  }
  const unsigned long long sk = __ballot(skip);
  const int base = T.s0 + 64 * b;
  // skipped strips below the wave's own: the highest one bounds the core from below
  const int nlo = min(64, max(0, T.o0 - base));  // bits k < nlo are strips below o0
  const unsigned long long mlo = nlo == 64 ? sk : (sk & ((1ull << nlo) - 1ull));
  if (mlo) {
    T.c0 = base + (63 - __clzll(mlo)) + 1;
    T.gap_lo = true;
  }
  // skipped strips above: the lowest one (the first batch that has one) bounds it from above
  const int nhi = min(64, max(0, T.o1 + 1 - base));  // bits k >= nhi are strips above o1
  const unsigned long long mhi = nhi == 64 ? 0ull : (sk & ~((1ull << nhi) - 1ull));
  if (mhi && !T.gap_hi) {
    T.c1 = base + __ffsll((long long)mhi) - 2;
    T.gap_hi = true;
  }
  return __ballot(walk);
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
