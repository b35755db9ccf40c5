/* TEST / MEASUREMENT INFRASTRUCTURE ONLY (built into liboracle_flock.so; never the product).
 * Gauss-Seidel level structure of a batch of envs, for the chain floor (bench.py's cpu_baseline
 * leg, tools/chain_floor.py): for each env, the touching contacts of its ordered contact list (b2CollideCircles:
 * touching iff |pB - pA|^2 <= (2r)^2 in float32), Box2D's island order of them (seeds from the
 * highest body with edges, each body's edges in list order, as b2World::Solve's DFS over the
 * prepend-ordered edge lists) and the level of each contact in that order
 * (1 + the level of the last earlier contact sharing a body): what the step kernels' level-parallel
 * solvers step through once per velocity / position pass. Sleeping bodies are not modelled (an
 * early window from reset has none).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* out[e*4 + 0] touching contacts, [1] levels (the deepest island's depth), [2] islands,
 * [3] contacts of the largest island */
void gs_levels(int E, int N, int C, const float* pos, const int32_t* cnt, const uint32_t* ab, float rr,
               int32_t* out) {
#pragma omp parallel
  {
    int* deg = malloc(sizeof(int) * (N + 1));
    int* off = malloc(sizeof(int) * (N + 1));
    int* last = malloc(sizeof(int) * N);
    char* vis = malloc(N);
    int* stk = malloc(sizeof(int) * N);
    int cap = 0;
    int *ta = NULL, *tb = NULL, *adj = NULL;
    char* cvis = NULL;
#pragma omp for schedule(dynamic, 4)
    for (int e = 0; e < E; ++e) {
      const float* p = pos + (size_t)e * N * 2;
      const uint32_t* l = ab + (size_t)e * C;
      const int M = cnt[e];
      if (M > cap) {
        cap = M;
        ta = realloc(ta, sizeof(int) * cap);
        tb = realloc(tb, sizeof(int) * cap);
        adj = realloc(adj, sizeof(int) * 2 * cap);
        cvis = realloc(cvis, cap);
      }
      int T = 0;
      for (int k = 0; k < M; ++k) {
        const int a = l[k] & 0xffff, b = l[k] >> 16;
        const float dx = p[2 * b] - p[2 * a], dy = p[2 * b + 1] - p[2 * a + 1];
        if (!(dx * dx + dy * dy > rr)) {
          ta[T] = a;
          tb[T] = b;
          ++T;
        }
      }
      memset(deg, 0, sizeof(int) * (N + 1));
      for (int t = 0; t < T; ++t) {
        deg[ta[t]]++;
        deg[tb[t]]++;
      }
      off[0] = 0;
      for (int i = 0; i < N; ++i) off[i + 1] = off[i] + deg[i];
      memset(deg, 0, sizeof(int) * (N + 1));
      for (int t = 0; t < T; ++t) {  /* list order within each body's segment */
        adj[off[ta[t]] + deg[ta[t]]++] = t;
        adj[off[tb[t]] + deg[tb[t]]++] = t;
      }
      memset(vis, 0, N);
      memset(cvis, 0, T > 0 ? T : 1);
      for (int i = 0; i < N; ++i) last[i] = 0;
      int maxlv = 0, nisl = 0, bigisl = 0;
      for (int s = N - 1; s >= 0; --s) {
        if (vis[s] || off[s + 1] == off[s]) continue;
        ++nisl;
        int ic = 0, sp = 0;
        vis[s] = 1;
        stk[sp++] = s;
        while (sp > 0) {
          const int bd = stk[--sp];
          for (int q = off[bd]; q < off[bd + 1]; ++q) {
            const int t = adj[q];
            if (cvis[t]) continue;
            cvis[t] = 1;
            ++ic;
            const int a = ta[t], b = tb[t];
            const int lv = (last[a] > last[b] ? last[a] : last[b]) + 1;
            last[a] = last[b] = lv;
            if (lv > maxlv) maxlv = lv;
            const int o = a == bd ? b : a;
            if (!vis[o]) {
              vis[o] = 1;
              stk[sp++] = o;
            }
          }
        }
        if (ic > bigisl) bigisl = ic;
      }
      out[(size_t)e * 4 + 0] = T;
      out[(size_t)e * 4 + 1] = maxlv;
      out[(size_t)e * 4 + 2] = nisl;
      out[(size_t)e * 4 + 3] = bigisl;
    }
    free(deg);
    free(off);
    free(last);
    free(vis);
    free(stk);
    free(ta);
    free(tb);
    free(adj);
    free(cvis);
  }
}
