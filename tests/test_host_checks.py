"""Host-side argument checks that guard the C-ABI (no GPU needed): the trajectory buffers a caller
hands to rollout_traj are checked for dtype and per-step shape before any kernel writes K rows into
them (a wrong buffer would be overrun on the device)."""
import pytest
import torch

from gym_macm.world import check_traj

KEYS = ("obs", "nbr_id", "done")
SPEC = dict(obs=(torch.float32, (4, 8, 6)), nbr_id=(torch.int32, (4, 8)), done=(torch.uint8, (4,)))
DEV = torch.device("cpu")


def bufs(K=3):
    return dict(obs=torch.zeros((K, 4, 8, 6)), nbr_id=torch.zeros((K, 4, 8), dtype=torch.int32),
                done=torch.zeros((K, 4), dtype=torch.uint8))


def test_good_buffers_pass_in_key_order():
    b = bufs()
    out = check_traj(b, SPEC, 3, DEV, KEYS)
    assert [t.data_ptr() for t in out] == [b[k].data_ptr() for k in KEYS]
    b.pop("nbr_id")
    assert check_traj(b, SPEC, 2, DEV, KEYS)[1] is None  # absent outputs are skipped; more rows than K is fine


@pytest.mark.parametrize("key,t", [
    ("obs", torch.zeros((3, 4, 8, 6), dtype=torch.float64)),        # wrong dtype (an f64-obs buffer)
    ("obs", torch.zeros((3, 5, 8, 6))),                             # more envs than the world
    ("nbr_id", torch.zeros((3, 4, 7), dtype=torch.int32)),          # fewer agents
    ("done", torch.zeros((2, 4), dtype=torch.uint8)),               # fewer than K rows
    ("obs", torch.zeros((3, 4, 8, 12))[..., ::2]),                  # not contiguous
    ("extra", torch.zeros(3)),                                      # an unknown buffer
])
def test_bad_buffers_raise(key, t):
    b = bufs()
    b[key] = t
    with pytest.raises(ValueError):
        check_traj(b, SPEC, 3, DEV, KEYS)


def test_pairwise_reward_sum_order():
    """gym_macm.dist.pairwise_reward_sum: the device's order (flock_common.hpp block_pairwise_sum) —
    float32 rewards as float64, pairwise over P = 64 * 2^ceil(log2(waves)) slots with +0.0 past N —
    against a recursive restatement, at N that fill 1, 2, 3 -> 4 and 5 -> 8 waves."""
    import numpy as np
    from gym_macm.dist import env_order_sum, pairwise_reward_sum

    def rec(x):
        return x[0] if len(x) == 1 else rec(x[:len(x) // 2]) + rec(x[len(x) // 2:])

    rng = np.random.default_rng(0)
    for N, P in ((2, 64), (64, 64), (65, 128), (150, 256), (300, 512), (1024, 1024)):
        r = (1.0 - rng.uniform(0, 60, size=(3, N)) / 35).astype(np.float32)
        got = pairwise_reward_sum(r)
        for e in range(3):
            x = [float(v) for v in r[e]] + [0.0] * (P - N)
            assert got[e] == rec(x), (N, e)
    assert env_order_sum([0.1, 0.2, 0.3]) == (0.1 + 0.2) + 0.3
