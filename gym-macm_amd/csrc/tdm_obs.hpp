// tdm_obs.hpp — TDM.get_obs (gym_macm/envs/combat.py:206-227) as fixed [N, N-1, 4] slots, written
// by one 64-lane wave (tdm_obs_block: by a workgroup, any N): shared by the wave kernel
// (flock_step_w64.hip), the workgroup TDM step (tdm_step_wg.hip) and the spill step
// (flock_spill.hpp), which steps TDM envs beyond the wave kernel's contact capacities.
#pragma once

#include "flock_common.hpp"

namespace macm {

__device__ __forceinline__ double sgn(double x) { return (double)((x > 0.0) - (x < 0.0)); }

// t = t - np.sign(t) * 2 * np.pi if np.abs(t) > np.pi else t      (mvmnt.py:199,214)
// |t| > pi implies t != 0, so sign(t) * 2 * pi is copysign(2 pi, t) (2 pi exact in double)
__device__ __forceinline__ double wrap_pi(double t) {
  return fabs(t) > M_PI ? t - copysign(2.0 * M_PI, t) : t;
}


// team of agent x without a loop: team_end[t] = N for every t >= n_teams - 1
__device__ __forceinline__ int tdm_team_nb(const TdmParams& T, int x) {
  return (x >= T.team_end[0]) + (x >= T.team_end[1]) + (x >= T.team_end[2]);
}

template <typename OT>
__device__ __forceinline__ void store4(OT* o, double a, double b, double c, double d) {
  if constexpr (sizeof(OT) == 4) {
    *reinterpret_cast<float4*>(o) = make_float4((float)a, (float)b, (float)c, (float)d);
  } else {
    reinterpret_cast<double2*>(o)[0] = make_double2(a, b);
    reinterpret_cast<double2*>(o)[1] = make_double2(c, d);
  }
}

// TDM.get_obs (combat.py:206-227) as fixed slots: slot k of agent i is the other
// agent j = k < i ? k : k + 1, holding (r, t, p, is_ally) with rel = other - agent
// (float32), r = sqrt(b2DistanceSquared), t = atan2(rel) - angle_i and
// p = angle_j - angle_i each wrapped once; mask = both alive, masked slots zero.
// One unordered pair {i, j} (i < j) per lane: the lane writes slot (i, j) and slot (j, i).
// Both directions share r (|rel| is the same), the ally flag, the mask and atan2's
// reduction and polynomial (obs_atan2_core of |rel.x|, |rel.y|); each keeps its own
// rel = other - agent (float32), quadrant, "- angle" and wrap, so every value is bit-identical
// to evaluating the two slots separately, with half the f64 atan2 work.
// m: both agents alive.
template <typename OT>
__device__ __forceinline__ void tdm_obs_pair_m(OT* __restrict__ obs, uint8_t* __restrict__ mask, int S, int i, int j,
                                               bool m, const TdmParams& TP, const float2* sc, const float* sa) {
  double r = 0.0, t1 = 0.0, t2 = 0.0, p1 = 0.0, p2 = 0.0, ty = 0.0;
  if (m) {
    const float2 ci = sc[i], cj = sc[j];
    const float xi = ci.x, yi = ci.y, xj = cj.x, yj = cj.y, ai = sa[i], aj = sa[j];
    const float rx = xj - xi, ry = yj - yi;  // row i: other.position - agent.position
    const float qx = xi - xj, qy = yi - yj;  // row j
    const float d2 = rx * rx + ry * ry;      // b2DistanceSquared (the same for row j)
    r = obs_sqrt<OT>(d2);
    const double core = obs_atan2_core(fabs((double)rx), fabs((double)ry));
    t1 = wrap_pi(obs_atan2_finish(core, (double)ry, (double)rx) - (double)ai);
    t2 = wrap_pi(obs_atan2_finish(core, (double)qy, (double)qx) - (double)aj);
    p1 = wrap_pi((double)aj - (double)ai);
    p2 = -p1;  // = wrap_pi(ai - aj) exactly: a - b == -(b - a) and the wrap is odd in IEEE arithmetic
    ty = tdm_team_nb(TP, j) == tdm_team_nb(TP, i) ? 1.0 : 0.0;
  }
  const size_t s1 = (size_t)i * S + (j - 1), s2 = (size_t)j * S + i;
  if (obs) {
    store4<OT>(obs + s1 * 4, r, t1, p1, ty);
    store4<OT>(obs + s2 * 4, r, t2, p2, ty);
  }
  if (mask) {
    mask[s1] = m ? 1 : 0;
    mask[s2] = m ? 1 : 0;
  }
}

template <typename OT>
__device__ __forceinline__ void tdm_obs_pair(OT* __restrict__ obs, uint8_t* __restrict__ mask, int S, int i, int j,
                                             unsigned long long livem, const TdmParams& TP, const float2* sc,
                                             const float* sa) {
  tdm_obs_pair_m<OT>(obs, mask, S, i, j, ((livem >> i) & (livem >> j) & 1ull) != 0ull, TP, sc, sa);
}

// Any N, by a whole workgroup (the workgroup TDM step, N > 64; alive agents as an LDS bitmap): the
// N(N-1)/2 unordered pairs as a round robin. Thread i takes {i, (i + d) mod N} for d = 1 ..
// (N-1)/2, and for even N also d = N/2 when i < N/2: every pair exactly once, (N-1)/2 or N/2 pairs
// per thread. Each pair is evaluated as tdm_obs_pair (both directions, one shared atan2 core).
template <typename OT>
__device__ __forceinline__ void tdm_obs_block(OT* __restrict__ obs, uint8_t* __restrict__ mask, int N, int tid,
                                              const uint32_t* alivew, const TdmParams& TP, const float2* sc,
                                              const float* sa) {
  if (tid >= N) return;
  const int D = (N - 1) / 2 + ((N % 2) == 0 && tid < N / 2 ? 1 : 0);
  const bool li = ((alivew[tid >> 5] >> (tid & 31)) & 1u) != 0u;
  for (int d = 1; d <= D; ++d) {
    const int k = tid + d < N ? tid + d : tid + d - N;
    const bool m = li && ((alivew[k >> 5] >> (k & 31)) & 1u) != 0u;
    tdm_obs_pair_m<OT>(obs, mask, N - 1, tid < k ? tid : k, tid < k ? k : tid, m, TP, sc, sa);
  }
}

// Any N, by a whole workgroup, in memory order: thread t of the block writes slots t, t + BS, ... of
// the env's [N, N-1] block, so each store instruction covers 64 consecutive 16-B slots (whole 128-B
// lines) and the mask 64 consecutive bytes; each slot evaluates its own atan2 (tdm_obs_linear's
// arithmetic, bit-identical to the pair form).
template <typename OT>
__device__ __forceinline__ void tdm_obs_block_linear(OT* __restrict__ obs, uint8_t* __restrict__ mask, int N, int tid,
                                                     int BS, const uint32_t* alivew, const TdmParams& TP,
                                                     const float2* sc, const float* sa) {
  const int S = N - 1, ns = N * S;
  int i = tid / S, k = tid - i * S;  // slot q = i * S + k, advanced by BS per pass
  const int di = BS / S, dk = BS - di * S;
  for (int q = tid; q < ns; q += BS) {
    const int j = k < i ? k : k + 1;
    const bool m = ((alivew[i >> 5] >> (i & 31)) & (alivew[j >> 5] >> (j & 31)) & 1u) != 0u;
    double r = 0.0, t = 0.0, p = 0.0, ty = 0.0;
    if (m) {
      const float2 ci = sc[i], cj = sc[j];
      const float rx = cj.x - ci.x, ry = cj.y - ci.y;  // other.position - agent.position
      r = obs_sqrt<OT>(rx * rx + ry * ry);
      t = wrap_pi(obs_atan2((double)ry, (double)rx) - (double)sa[i]);
      p = wrap_pi((double)sa[j] - (double)sa[i]);
      ty = tdm_team_nb(TP, j) == tdm_team_nb(TP, i) ? 1.0 : 0.0;
    }
    if (obs) store4<OT>(obs + (size_t)q * 4, r, t, p, ty);
    if (mask) mask[q] = m ? 1 : 0;
    i += di;
    k += dk;
    if (k >= S) {
      k -= S;
      ++i;
    }
  }
}

// The pairs in 8 x 8 tiles (agent blocks I < J), one tile per pass: lane (a, b) = (lane / 8,
// lane % 8) takes pair (8I + a, 8J + b). A store instruction then writes 8 runs of 8
// consecutive slots for both directions (rows 8I + a, and rows 8J + b), so whole L2 lines fill
// within one instruction; the row-major pair order left the (j, i) half as a column walk of
// single 16-B slots, and lines left L2 partly written (+37% HBM writes). The diagonal tiles'
// 28 pairs (a < b) go two tiles per pass.
template <typename OT>
__device__ __forceinline__ void tdm_obs_pairs(OT* __restrict__ obs, uint8_t* __restrict__ mask, int N, int lane,
                                              unsigned long long livem, const TdmParams& TP, const float2* sc,
                                              const float* sa) {
  const int S = N - 1;
  const int nb = (N + 7) >> 3;
  const int a = lane >> 3, b = lane & 7;
  for (int I = 0; I < nb; ++I) {
    const int i = 8 * I + a;
    for (int J = I + 1; J < nb; ++J) {
      const int j = 8 * J + b;
      if (i < N && j < N) tdm_obs_pair<OT>(obs, mask, S, i, j, livem, TP, sc, sa);
    }
  }
  // diagonal tiles: pair k < 28 of tile D (row-major over r < c) on lane 32 (D & 1) + k
  const int k = lane & 31;
  int r = 0, rem = k;
  while (r < 7 && rem >= 7 - r) {
    rem -= 7 - r;
    ++r;
  }
  const int c = r + 1 + rem;
  for (int D0 = 0; D0 < nb; D0 += 2) {
    const int D = D0 + (lane >> 5);
    const int i = 8 * D + r, j = 8 * D + c;
    if (k < 28 && D < nb && j < N) tdm_obs_pair<OT>(obs, mask, S, i, j, livem, TP, sc, sa);
  }
}

// Row-block order (round 4): the pair tiles of tdm_obs_pairs (each unordered pair once, both
// directions from one atan2 core), but taken row block by row block so that every 128-B line of
// the env's [N, N-1, 4] block is written within one short stretch. Row block R (rows 8R .. 8R+7,
// 8 x 496 B = 31 whole lines at N = 32) gets its tiles (R, J > R) in the pair's own direction
// (row i, slot j - 1), its diagonal tile, and its slots i < 8R, which the tiles (I < R, R)
// computed in earlier blocks and left in an LDS stage as the finished float32 slot (the same bits
// the pair form stores). The pair tiles wrote that direction into rows of later blocks as 8-slot
// runs spread over the whole obs phase, whose lines left L2 partly written (PMC: ~150 B per
// agent-step of HBM writes above the algorithmic bytes). float32 obs; stage:
// 512 nb (nb - 1) bytes, nb = N / 8 rounded up (6 KB at N = 32: the wave kernel's dead contact
// arrays).
__host__ __device__ constexpr int tdm_obs_rb_stage_bytes(int N) { return 512 * ((N + 7) >> 3) * (((N + 7) >> 3) - 1); }

template <typename OT>
__device__ __forceinline__ void tdm_obs_rowblocks(OT* __restrict__ obs, uint8_t* __restrict__ mask, int N, int lane,
                                                  unsigned long long livem, const TdmParams& TP, const float2* sc,
                                                  const float* sa, float4* stage, bool mask_pieces = false) {
  static_assert(sizeof(OT) == 4, "the stage keeps the finished float32 slots");
  const int S = N - 1, nb = (N + 7) >> 3;
  const int a = lane >> 3, b = lane & 7;
  // mask_pieces: the mask in 16-B pieces after the slots (each byte alive(i) & alive(j), from livem
  // alone) when the env's [N, N-1] mask block is a whole number of aligned pieces (N = 32: 62 lanes, one
  // store each) instead of a byte store per slot beside each slot's store (the byte stores are 3% of
  // C4's step). Measured (profiles/r06/abtests/mask_pieces/): the 512-env shard -2.1%, 4096 envs
  // +0.5 / +1.3% (window / steady), so the tail observation's rows take it and the fused step does not.
  const bool mfast = mask_pieces && mask && ((N * S) & 15) == 0 && (reinterpret_cast<uintptr_t>(mask) & 15) == 0;
  uint8_t* const mk = mfast ? nullptr : mask;
  int dr = 0, rem = lane & 31;  // diagonal pair `lane & 31` (< 28) of a block: row-major over dr < dc
  while (dr < 7 && rem >= 7 - dr) {
    rem -= 7 - dr;
    ++dr;
  }
  const int dc = dr + 1 + rem;
  auto soff = [](int J) { return 32 * J * (J - 1); };  // stage entries of the blocks before J: 8J' slots x 8 rows
  for (int R = 0; R < nb; ++R) {
    const int i = 8 * R + a;
    for (int J = R + 1; J < nb; ++J) {
      const int j = 8 * J + b;
      if (i < N && j < N) {
        const bool m = ((livem >> i) & (livem >> j) & 1ull) != 0ull;
        double r = 0.0, t1 = 0.0, t2 = 0.0, p1 = 0.0, ty = 0.0;
        if (m) {  // tdm_obs_pair_m's arithmetic
          const float2 ci = sc[i], cj = sc[j];
          const float xi = ci.x, yi = ci.y, xj = cj.x, yj = cj.y, ai = sa[i], aj = sa[j];
          const float rx = xj - xi, ry = yj - yi;
          const float qx = xi - xj, qy = yi - yj;
          const float d2 = rx * rx + ry * ry;
          r = obs_sqrt<OT>(d2);
          const double core = obs_atan2_core(fabs((double)rx), fabs((double)ry));
          t1 = wrap_pi(obs_atan2_finish(core, (double)ry, (double)rx) - (double)ai);
          t2 = wrap_pi(obs_atan2_finish(core, (double)qy, (double)qx) - (double)aj);
          p1 = wrap_pi((double)aj - (double)ai);
          ty = tdm_team_nb(TP, j) == tdm_team_nb(TP, i) ? 1.0 : 0.0;
        }
        const size_t s1 = (size_t)i * S + (j - 1);
        if (obs) store4<OT>(obs + s1 * 4, r, t1, p1, ty);
        if (mk) mk[s1] = m ? 1 : 0;
        // row j = 8J + b, slot i, as store4 would write it (p2 = -p1 exactly); lanes contiguous
        stage[soff(J) + 8 * i + b] = make_float4((float)r, (float)t2, (float)(-p1), (float)ty);
      }
    }
    // the diagonal tiles two at a time (lanes 0-27 block R, lanes 32-59 block R + 1, as the pair
    // tiles do): block R + 1's own pairs are written one block early
    if ((R & 1) == 0) {
      const int D = R + (lane >> 5), k = lane & 31;
      if (k < 28 && D < nb && 8 * D + dc < N) tdm_obs_pair<OT>(obs, mk, S, 8 * D + dr, 8 * D + dc, livem, TP, sc, sa);
    }
    if (R > 0) {
      wave_lds_sync();  // the stage entries of block R (other lanes, earlier blocks)
      // rows 8R .. 8R + 7, slots o < 8R: 64 R entries, one per lane, entry e = 8 o + rb (each store
      // instruction: 8 rows x 8 consecutive slots); masked slots were staged as zeros
      for (int e = lane; e < 64 * R; e += 64) {
        const int o = e >> 3, rb = e & 7;
        const int j = 8 * R + rb;
        if (j < N) {
          const size_t s2 = (size_t)j * S + o;
          if (obs) *reinterpret_cast<float4*>(obs + s2 * 4) = stage[soff(R) + e];
          if (mk) mk[s2] = ((livem >> o) & (livem >> j) & 1ull) ? 1 : 0;
        }
      }
    }
  }
  if (mfast) {
    for (int q = 16 * lane; q < N * S; q += 16 * 64) {
      int i = q / S, k = q - i * S;  // byte q: row i, slot k (the other agent k < i ? k : k + 1)
      uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int j = k < i ? k : k + 1;
        w[t >> 2] |= (uint32_t)((livem >> i) & (livem >> j) & 1ull) << (8 * (t & 3));
        if (++k == S) {
          k = 0;
          ++i;
        }
      }
      *reinterpret_cast<uint4*>(mask + q) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}


}  // namespace macm
