"""Host simulation of the tail observation's row claims (flock_step_w64.hip tdm_tail_row, TailObs):
nq = min(kTailQ, blocks) sub-queues by env range, wave b claims kTailChunk rows at a time from
sub-queue b % nq only (step-major inside a sub-queue, a counter load before each claim). Checks that
every (step, env) row of a launch is observed exactly once and that no row index leaves the launch,
for launch shapes (envs, observe-only waves, tail steps). Run before a GPU session that changes the
claim logic; tests/test_tail_rows.py runs it in the CPU suite.
    python tools/tail_rows_sim.py"""
K_TAIL_Q, K_TAIL_CHUNK = 64, 2  # = kTailQ (flock_common.hpp), kTailChunk (flock_step_w64.hip)


def simulate(E, X, K, kTailQ=K_TAIL_Q, C=K_TAIL_CHUNK):
    G = E + X
    nq = min(G, kTailQ)
    env0 = lambda q: (E * q) // nq  # noqa: E731
    ctr = [0] * nq
    seen = set()
    waves = [dict(q=b % nq, left=1, r=0, r_end=0, more=True) for b in range(G)]
    active = True
    while active:  # the waves' calls interleaved one row at a time
        active = False
        for w in waves:
            if not w["more"]:
                continue
            active = True
            while w["r"] >= w["r_end"]:
                if w["left"] == 0:
                    w["more"] = False
                    break
                ne = env0(w["q"] + 1) - env0(w["q"])
                nrows = K * ne
                c = 0
                if ne > 0:
                    c = ctr[w["q"]]
                    if c * C < nrows:
                        ctr[w["q"]] += 1
                if ne == 0 or c * C >= nrows:
                    w["q"] = 0 if w["q"] + 1 == nq else w["q"] + 1
                    w["left"] -= 1
                    continue
                w["r"], w["r_end"] = c * C, min(c * C + C, nrows)
            if not w["more"]:
                continue
            e0 = env0(w["q"])
            ne = env0(w["q"] + 1) - e0
            i = w["r"]
            w["r"] += 1
            k, e = i // ne, e0 + i % ne
            assert 0 <= k < K and 0 <= e < E, (E, X, K, k, e)
            assert (k, e) not in seen, (E, X, K, k, e)
            seen.add((k, e))
    assert len(seen) == K * E, (E, X, K, len(seen))
    return len(seen)


SHAPES = [(512, 512, 20), (4096, 0, 20), (12, 12, 7), (37, 3, 19), (24, 24, 9), (64, 64, 33), (16, 16, 25),
          (1536, 1536, 20), (1, 0, 3), (65, 0, 2), (4096, 0, 5), (63, 1, 4)]

if __name__ == "__main__":
    for s in SHAPES:
        simulate(*s)
    print(f"every row exactly once for {len(SHAPES)} launch shapes")
