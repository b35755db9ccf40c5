"""Structure of a dense workgroup-path env from the CPU oracle (a measurement script, not a test):
what bounds kernels B and C at C5.

    python tools/c5_structure.py [N] [steps] [flocks]      # default 1024 12 1 (the C5 window)

Per step (after `steps` random-action steps from reset, seed 56) it prints
  - the Gauss-Seidel dependency structure of Box2D's island order: touching contacts, islands,
    levels per pass and their widths (contacts per level), and how many levels a greedy
    assignment of contacts to lanes ("chain lanes": a contact takes the lane of its level - 1
    predecessor) would leave with a cross-lane dependency;
  - the pair sweep's new pairs: how many bodies get one, and how many get more than two (kernel
    C keeps two per body in a register and re-walks only for the rest);
  - the strip cells' candidates per body: with the env-wide Dx band (round 3) and with the
    per-strip extent pruning (round 4).
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"), os.path.join(REPO, "gym-macm_amd")]

from parity import oracle_for  # noqa: E402
from gym_macm.settings import flockSettings, to_config  # noqa: E402


def island_order(N, ta, tb):
    adj = [[] for _ in range(N)]
    for t in range(len(ta)):
        adj[ta[t]].append(t)
        adj[tb[t]].append(t)
    vis, cvis, order, nisl = np.zeros(N, bool), np.zeros(len(ta), bool), [], 0
    for s in range(N - 1, -1, -1):
        if vis[s] or not adj[s]:
            continue
        nisl += 1
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
    return order, nisl


def levels(N, ta, tb, order):
    last, lastc = np.full(N, -1), np.full(N, -1)
    lvl, preds = {}, {}
    for t in order:
        la, lb = last[ta[t]], last[tb[t]]
        lv = max(la, lb) + 1
        preds[t] = ((lastc[ta[t]], la), (lastc[tb[t]], lb))
        lvl[t] = lv
        last[ta[t]] = last[tb[t]] = lv
        lastc[ta[t]] = lastc[tb[t]] = t
    D = max(lvl.values()) + 1 if lvl else 0
    bylv = [[] for _ in range(D)]
    for t in order:
        bylv[lvl[t]].append(t)
    lane, cross = {}, np.zeros(D, int)
    for l in range(D):
        used = set()
        for t in bylv[l]:
            imm = [c for (c, lp) in preds[t] if c >= 0 and lp == l - 1]
            chosen = next((lane[c] for c in imm if lane[c] not in used), None)
            if chosen is None:
                chosen = 0
                while chosen in used:
                    chosen += 1
            used.add(chosen)
            lane[t] = chosen
            cross[l] += sum(1 for c in imm if lane[c] != chosen)
    return D, np.array([len(x) for x in bylv]), cross


def strip_candidates(c, f, N, H):
    L, R = c[:, 0] - f[:, 0], f[:, 2] - c[:, 0]
    E = np.maximum(L, R)
    Dx = L.max() + R.max()
    order = np.argsort(c[:, 0], kind="stable")
    xs, Es = c[order, 0], E[order]
    w = (xs[-1] - xs[0]) / H * (1 + 1 / 64)
    strip = np.clip(np.floor((xs - xs[0]) / w).astype(int), 0, H - 1)
    Estrip = np.zeros(H)
    np.maximum.at(Estrip, strip, Es)
    cur = new = 0
    for w0 in range(0, N, 64):
        lo, hi, EW = xs[w0], xs[min(N, w0 + 64) - 1], Es[w0:w0 + 64].max()
        cur += min(64, N - w0) * ((xs >= lo - 1.5 * Dx) & (xs <= hi + 1.5 * Dx)).sum()
        left = xs[0] + np.arange(H) * w
        keep = ~((left + 2 * w + Estrip + EW < lo) | (left - w - Estrip - EW > hi)) & (Estrip > 0)
        new += min(64, N - w0) * np.isin(strip, np.nonzero(keep)[0]).sum()
    return Dx, np.median(E), E.max(), cur / N, new / N


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    flocks = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    tidx = np.array([i * flocks // N for i in range(N)], np.int32)
    orc = oracle_for(to_config(flockSettings(), N, flocks, obs_f64=True), tidx, 1, 56, 0)
    rng = np.random.default_rng(1)
    prev = None
    H = max(64, 1 << int(np.ceil(np.log2(max(1, N / 4)))))
    for t in range(steps):
        orc.step(rng.integers(0, 3, size=(1, N, 3)).astype(np.uint8))
        st = orc.get_state(64 * N)
        pos, cnt = st["pos"][0], st["contact_count"][0]
        ab = st["contact_ab"][0][:cnt]
        pairs = set(ab.tolist())
        if t >= steps - 3:
            a, b = ab & 0xFFFF, ab >> 16
            touch = ((pos[b] - pos[a]) ** 2).sum(-1) <= 1.0
            ta, tb = a[touch], b[touch]
            order, nisl = island_order(N, ta, tb)
            D, width, cross = levels(N, ta, tb, order)
            new = [x for x in pairs if prev is not None and x not in prev]
            per = np.bincount(np.array([x & 0xFFFF for x in new], np.int64), minlength=N) if new else np.zeros(N, int)
            Dx, Emed, Emax, cur, pruned = strip_candidates(pos, st["fat"][0], N, H)
            print(f"step {t + 1}: touching {len(order)} in {nisl} islands, {D} levels per pass "
                  f"(width mean {width.mean():.2f}, max {width.max()}); levels with a cross-lane dependency "
                  f"under chain lanes {(cross > 0).mean():.0%}")
            print(f"   new pairs {len(new)}: bodies with one or more {(per > 0).sum()}, with more than two "
                  f"{(per > 2).sum()}")
            print(f"   strips (H={H}): Dx {Dx:.2f} m, extent median {Emed:.2f} max {Emax:.2f}; candidates per body "
                  f"with the Dx band ~{cur:.0f}, with per-strip pruning ~{pruned:.0f}")
        prev = pairs


if __name__ == "__main__":
    main()
