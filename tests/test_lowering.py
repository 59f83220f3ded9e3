"""Product host lowering (distilp_amd/solver/lower.py) vs the reference's MILP arrays.

The CSR, bounds, objective and row bounds built by `lower_fleet(...).instance(k)`
must be bit-identical to what the reference passed to scipy.optimize.milp
(tests/golden/lowered.npz) and to the oracle's independent dense lowering.
"""

import numpy as np
import pytest

from distilp_amd.solver.lower import kv_bits_to_factor, lower_fleet
from oracle import milp_oracle as mo

from .conftest import GOLDEN
from .helpers import fixture_fleet, golden_lowered_keys, load_golden_lowered, synth_devices


def _check(fl, k, ref):
    c, lb, ub, row_lb, row_ub, integ, W = fl.instance(k)
    A = fl.dense()
    m_ub = ref["A_ub"].shape[0]
    assert A.shape == (m_ub + 1, len(ref["c"]))
    assert np.array_equal(A[:m_ub], ref["A_ub"])
    assert np.array_equal(A[m_ub:], ref["A_eq"])
    assert np.array_equal(c, ref["c"])
    assert np.array_equal(lb, ref["lb"]) and np.array_equal(ub, ref["ub"])
    assert np.array_equal(integ, ref["integrality"])
    assert np.array_equal(row_ub[:-1], ref["b_ub"]) and row_ub[-1] == ref["b_eq"][0] == row_lb[-1] == W
    assert np.all(np.isneginf(row_lb[:-1]))
    # CSR invariants: sorted columns, no explicit zeros
    for r in range(fl.n_rows):
        cols = fl.col_idx[fl.row_ptr[r]:fl.row_ptr[r + 1]]
        assert np.all(np.diff(cols) > 0)
    assert np.all(fl.val != 0)


def test_lowering_matches_reference_golden_arrays(llama_online_model):
    z = np.load(GOLDEN / "lowered.npz")
    for key, (M, seed, k) in golden_lowered_keys(z).items():
        fl = lower_fleet(synth_devices(M, seed), llama_online_model, "4bit")
        _check(fl, k, load_golden_lowered(z, key))


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16, 32, 64])
def test_lowering_matches_oracle(llama_online_model, M):
    for seed in range(4):
        devs = synth_devices(M, seed)
        fl = lower_fleet(devs, llama_online_model, "4bit")
        for k in (1, 2, 5, 80, 3):
            _check(fl, k, mo.lower_dense(devs, llama_online_model, k, 0.5))


@pytest.mark.parametrize("kv", ["4bit", "8bit", "fp16", " BF16 "])
def test_lowering_fixtures_all_kv(kv):
    for folder in ["hermes_70b", "llama_3_70b/4bit", "llama_3_70b/online", "qwen3_32b/bf16"]:
        devs, model = fixture_fleet(folder)
        fl = lower_fleet(devs, model, kv)
        for k in (1, 2, 4, 16):
            _check(fl, k, mo.lower_dense(devs, model, k, kv_bits_to_factor(kv)))


def test_kv_bits_error_message():
    with pytest.raises(ValueError, match="Unsupported kv_bits 'int3'"):
        kv_bits_to_factor("int3")


def test_objective_constant_matches_reference(fixtures_golden):
    """obj_value = c.x + sum t_comm + sum xi + kappa, using HiGHS's own x from the golden."""
    for fx in fixtures_golden["fixtures"].values():
        devs, model = fixture_fleet(fx["folder"])
        fl = lower_fleet(devs, model, fx["kv_bits"])
        for rec in fx["per_k"]:
            if rec["success"]:
                c = fl.instance(rec["k"])[0]
                assert fl.objective_value(c, np.array(rec["x"])) == rec["obj_value"]
