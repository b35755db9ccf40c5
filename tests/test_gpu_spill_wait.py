"""An env left unstepped by a full spill pool (MACM_ST_SPILL_WAIT) keeps its whole state.

A dense env takes a working-set slot for its spill step (csrc/flock_spill.hpp, spill::acquire_slot);
when a pooled world's slots stay taken for ~1 s the env is not stepped and SPILL_WAIT is reported.
ADVICE r04: the early return left the next list buffer unwritten, so the following step (or step
k + 1 of a rollout) read a contact list two steps old beside the un-advanced bodies. The test hook
MACM_DEBUG_SPILL_FAIL makes every slot request fail; with MACM_DEBUG_FORCE_SPILL every env takes
that path, in every caller: the Flock wave kernel (N <= 64) and kernel A (N > 64), the TDM wave
kernel's hand-over and the workgroup TDM step, one launch per step and the multi-step launch.
Bar: the full state after the call — contact order and warm-start impulses included — equals the
state before it, the status word says SPILL_WAIT, and the next call refuses (MACM_E_OVERFLOW)."""
import numpy as np
import pytest
import torch

from parity import assert_state_equal
from test_gpu_parity import rand_actions
from test_gpu_tdm import assert_tdm_state_equal, make_pair as tdm_pair, random_actions

pytestmark = pytest.mark.gpu

from gym_macm import _abi  # noqa: E402
from gym_macm.vec import FlockVec  # noqa: E402


@pytest.mark.parametrize("N,spread,form", [(64, 6, "step"), (64, 6, "rollout"), (100, 9, "step"),
                                           (100, 9, "rollout")])
def test_flock_spill_wait_leaves_the_env_wholly_unstepped(N, spread, form):
    E = 4
    v = FlockVec(E, n_agents=[N], seed=N + spread, device="cuda:0", start_spread=spread)
    rng = np.random.default_rng(N)
    for _ in range(4):  # non-trivial lists and impulses first
        v.step(torch.from_numpy(rand_actions(rng, E, N)).cuda())
    before = v.get_state()
    assert before["contact_count"].min() > 0 and np.abs(before["contact_imp"]).max() > 0
    v.world.set_debug(_abi.DEBUG_FORCE_SPILL | _abi.DEBUG_SPILL_FAIL)
    if form == "step":
        v.step(torch.from_numpy(rand_actions(rng, E, N)).cuda())
    else:
        v.rollout(torch.from_numpy(np.stack([rand_actions(rng, E, N) for _ in range(3)])).cuda())
    torch.cuda.synchronize()
    assert v.status() & _abi.ST_SPILL_WAIT
    assert_state_equal(v.get_state(), before, f"after a SPILL_WAIT {form}")
    with pytest.raises(_abi.MacmOverflowError):
        v.step(torch.from_numpy(rand_actions(rng, E, N)).cuda())


@pytest.mark.parametrize("teams,form", [([16, 16], "step"), ([16, 16], "rollout"), ([40, 40], "step")])
def test_tdm_spill_wait_leaves_the_env_wholly_unstepped(teams, form):
    E, N = 4, sum(teams)
    w, _ = tdm_pair(E, teams, seed=N, world_width=8.0, world_height=8.0)
    rng = np.random.default_rng(N)
    for _ in range(4):
        w.step(torch.from_numpy(random_actions(rng, E, N, p_attack=0.3)).cuda())
    before = w.get_state()
    assert before["contact_count"].min() > 0
    w.set_debug(_abi.DEBUG_FORCE_SPILL | _abi.DEBUG_SPILL_FAIL)
    if form == "step":
        w.step(torch.from_numpy(random_actions(rng, E, N, p_attack=0.5)).cuda())
    else:
        w.rollout(torch.from_numpy(np.stack([random_actions(rng, E, N, p_attack=0.5) for _ in range(3)])).cuda())
    torch.cuda.synchronize()
    assert w.status() & _abi.ST_SPILL_WAIT
    after = w.get_state()
    assert_tdm_state_equal(after, before, f"after a SPILL_WAIT {form}")
    for k in ("health", "alive", "cd_atk", "cd_mov", "listener", "done", "winner"):
        np.testing.assert_array_equal(after[k], before[k], err_msg=k)


def test_spill_fail_and_pool_flags_exclude_each_other():
    v = FlockVec(2, n_agents=[16], seed=1, device="cuda:0")
    with pytest.raises(_abi.MacmLibraryError):
        v.world.set_debug(_abi.DEBUG_SPILL_FAIL | _abi.DEBUG_SPILL_POOL | (1 << 8))
