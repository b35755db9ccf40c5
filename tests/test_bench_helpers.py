"""CPU checks of bench.py's measurement helpers (no GPU): the Gauss-Seidel chain floor, the CPU
baseline's level replay of the GPU leg's window, the TDM algorithmic bytes, and the PMC summary's
per-kernel counter means (the rollout kernel's name with its fifth template parameter)."""
import csv
import importlib.util
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def bench():
    return load("bench_mod", "bench.py")


def test_chain_floor_per_launch_and_pipelined(bench):
    # 3 steps x 2 envs: per launch the deepest env of each step, pipelined the deepest env's sum
    L = np.array([[10, 4], [2, 9], [7, 7]])
    cyc = 9 * bench.C_VEL_LEVEL + 3 * bench.C_POS_LEVEL
    ms, d = bench.chain_floor(L, rollout=False)
    assert d["sum_k_max_e"] == 10 + 9 + 7 and d["max_e_sum_k"] == max(19, 20)
    assert ms == pytest.approx(26 * cyc / (bench.SHADER_GHZ * 1e9) * 1e3 / 3)
    ms_r, _ = bench.chain_floor(L, rollout=True)
    assert ms_r == pytest.approx(20 * cyc / (bench.SHADER_GHZ * 1e9) * 1e3 / 3)
    assert d["levels_per_step_deepest"] == [10, 9, 7] and d["steps_sampled"] == 3


def test_cpu_baseline_replays_the_gpu_window_levels(bench):
    """The baseline times the oracle on the GPU leg's own actions, and the untimed replay records
    each timed step's level structure ([steps, envs], the deepest island's levels per pass)."""
    E, N, W, K = 4, 24, 2, 3
    rng = np.random.default_rng(5)
    acts = rng.integers(0, 3, size=(W + K, E, N, 3)).astype(np.uint8)
    base, lv = bench.cpu_baseline(N, 7, budget_s=30.0, n_envs=E, warmup=W, steps=K, acts_host=acts,
                                  levels_budget_s=30.0)
    assert base["kind"] == "port" and base["value"] > 0 and f"steps {W + 1}..{W + K}" in base["sample"]
    assert lv is not None and lv.shape == (K, E) and (lv >= 0).all()
    base2, lv2 = bench.cpu_baseline(N, 7, budget_s=30.0, n_envs=E, warmup=W, steps=K, acts_host=acts,
                                    levels_budget_s=30.0)
    np.testing.assert_array_equal(lv, lv2)  # a function of the seed and the actions


def test_tdm_algorithmic_bytes(bench):
    assert bench.b_alg_tdm(32) == 670
    assert bench.b_alg_tdm(32, obs_f64=True) == 670 + 31 * 16


def test_pmc_summary_matches_the_rollout_kernel(tmp_path):
    pmc = load("pmc_summary_mod", "tools/pmc_summary.py")
    p = tmp_path / "run_counter_collection.csv"
    rows = [("void macm::env_rollout_w64<0, 64, float, true>(macm::RolloutArgs<float>)", "1", "FETCH_SIZE", "10"),
            ("void macm::env_rollout_w64<0, 64, float, true>(macm::RolloutArgs<float>)", "2", "FETCH_SIZE", "30"),
            ("void macm::env_rollout_w64<0, 64, float, false>(macm::RolloutArgs<float>)", "3", "FETCH_SIZE", "99")]
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        w.writerows(rows)
    k = "env_rollout_w64<0, 64, float, true>"
    assert pmc.kernel_means(str(p), k)["FETCH_SIZE"] == 20.0
    assert pmc.kernel_means(str(p), k, last=True)["FETCH_SIZE"] == 30.0
