"""CPU check of the tail observation's row claims (tools/tail_rows_sim.py restates
flock_step_w64.hip tdm_tail_row): every (step, env) row of a launch is observed exactly once and no
row index leaves the launch, for the launch shapes the GPU tests use."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import tail_rows_sim  # noqa: E402


@pytest.mark.parametrize("shape", tail_rows_sim.SHAPES)
def test_every_row_once(shape):
    E, X, K = shape
    assert tail_rows_sim.simulate(E, X, K) == E * K
