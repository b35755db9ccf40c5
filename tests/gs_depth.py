"""Gauss-Seidel dependency depth of the velocity passes (a measurement script, not a test).

Runs one env of the CPU oracle from reset, takes its touching contacts after `steps` steps, orders
them as Box2D's island DFS does (seeds from the highest body, each body's edges in list order) and
prints: contacts T; the depth of one pass (the levels the solvers step through); 9 passes done
level by level (warm start + 8 velocity passes); and the depth of the 9 passes as one dataflow
(pass p + 1 of a contact may start once both bodies took every earlier update), which is what
overlapping passes could at best reach. DESIGN.md §7 quotes its output:

    python tests/gs_depth.py 1024 8     # C5 shape, step 8
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "oracle"), HERE, os.path.join(HERE, "..", "gym-macm_amd")]

from parity import oracle_for  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402


def main():
    N, steps = int(sys.argv[1]), int(sys.argv[2])
    cfg = to_config(flockSettings(), N, 1, obs_f64=True)
    orc = oracle_for(cfg, np.zeros(N, np.int32), 1, 56, 0)
    rng = np.random.default_rng(1)
    for _ in range(steps):
        orc.step(rng.integers(0, 3, size=(1, N, 3)).astype(np.uint8))
    st = orc.get_state(32 * N)
    pos, cnt = st["pos"][0], st["contact_count"][0]
    ab = st["contact_ab"][0][:cnt]
    a, b = ab & 0xFFFF, ab >> 16
    touch = ((pos[b] - pos[a]) ** 2).sum(-1) <= 1.0
    ta, tb = a[touch], b[touch]
    adj = [[] for _ in range(N)]
    for t in range(len(ta)):
        adj[ta[t]].append(t)
        adj[tb[t]].append(t)
    vis, cvis, order = np.zeros(N, bool), np.zeros(len(ta), bool), []
    for s in range(N - 1, -1, -1):
        if vis[s] or not adj[s]:
            continue
        vis[s] = True
        stk = [s]
        while stk:
            bd = stk.pop()
            for t in adj[bd]:
                if cvis[t]:
                    continue
                cvis[t] = True
                order.append(t)
                o = tb[t] if ta[t] == bd else ta[t]
                if not vis[o]:
                    vis[o] = True
                    stk.append(o)

    def depth(passes):
        last, mx = np.zeros(N, int), 0
        for _ in range(passes):
            for t in order:
                lv = max(last[ta[t]], last[tb[t]]) + 1
                last[ta[t]] = last[tb[t]] = lv
                mx = max(mx, lv)
        return mx

    d1 = depth(1)
    print(f"N={N} step={steps} T={len(ta)} depth/pass={d1} 9 passes level by level={9 * d1} "
          f"as one dataflow={depth(9)}")


if __name__ == "__main__":
    main()
