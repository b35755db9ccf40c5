"""Island structure of the C3 closed loop (bots.flock) from the CPU oracle (a measurement script,
not a test): what bounds kernel A's islands-first walks.

    python tools/c3_islands.py [N] [steps] [flocks] [envs]      # default 256 200 4 4

After `steps` closed-loop steps (tests/parity.flock_bot on the oracle's own obs) it prints per env
the touching contacts, whether kernel A takes the wave-parallel DFS kernel (2T >= 4N), and the
islands: contacts and bodies of each, the ones walked by a whole wave (> kBigIsland = 48 contacts)
and the longest serial walk (the thread that walks the largest of the other islands).
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), os.path.join(REPO, "gym-macm_amd"),
                os.path.join(REPO, "tools")]

from c5_structure import island_order, levels  # noqa: E402
from parity import flock_bot, oracle_for  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402

BIG = 48


def islands(N, ta, tb):
    par = list(range(N))

    def find(x):
        while par[x] != x:
            par[x] = par[par[x]]
            x = par[x]
        return x

    for a, b in zip(ta, tb):
        ra, rb = find(a), find(b)
        if ra != rb:
            par[min(ra, rb)] = max(ra, rb)
    nc, nb = {}, {}
    for a, b in zip(ta, tb):
        r = find(a)
        nc[r] = nc.get(r, 0) + 1
    for x in set(ta.tolist()) | set(tb.tolist()):
        r = find(x)
        nb[r] = nb.get(r, 0) + 1
    return sorted(((nc[r], nb[r]) for r in nc), reverse=True)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    flocks = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    E = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    tidx = np.array([i * flocks // N for i in range(N)], np.int32)
    orc = oracle_for(to_config(flockSettings(), N, flocks, obs_f64=True), tidx, E, 0x6D61636D, 0)
    obs, _ = orc.observe()
    for _ in range(steps):
        obs = orc.step(flock_bot(obs))["obs"]
    st = orc.get_state(64 * N)
    for e in range(E):
        pos, cnt = st["pos"][e], st["contact_count"][e]
        ab = st["contact_ab"][e][:cnt]
        a, b = ab & 0xFFFF, ab >> 16
        touch = ((pos[b] - pos[a]) ** 2).sum(-1) <= 1.0
        ta, tb = a[touch], b[touch]
        T = len(ta)
        isl = islands(N, ta, tb)
        big = [c for c, _ in isl if c > BIG]
        small = [c for c, _ in isl if c <= BIG]
        order, _ = island_order(N, ta, tb)
        D, width, _ = levels(N, ta, tb, order)
        print(f"env {e}: list {cnt}, touching {T} ({'DFS kernel' if 2 * T >= 4 * N else 'islands first'}), "
              f"{len(isl)} islands, {D} levels per pass (width mean {width.mean():.2f})")
        print(f"   wave-walked (> {BIG} contacts): {[(c, bd) for c, bd in isl if c > BIG]}")
        print(f"   serial: {len(small)} islands, largest {small[:6]}, contacts {sum(small)}")
        _ = big


if __name__ == "__main__":
    main()
