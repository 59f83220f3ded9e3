"""The oracle, pinned against the reference's own outputs (tests/golden, made by gen_golden.py).

CPU only. Checks:
  * the oracle's dense lowering is bit-identical to the arrays the reference
    passed to scipy.optimize.milp (lowered.npz);
  * the oracle's HiGHS sweep reproduces the reference's HALDAResult bit-exactly
    on every profile fixture x kv_bits x mip_gap;
  * the exact C solver (oracle/halda_exact.c) agrees with the reference's HiGHS
    answers on every seeded synthetic instance: same status, same (w, n) where
    the optimum is unique, objective within 1e-12 relative.
"""

import json

import numpy as np
import pytest

from oracle import milp_oracle as mo

from .conftest import GOLDEN
from .helpers import fixture_fleet, golden_lowered_keys, load_golden_lowered, synth_devices


def test_oracle_lowering_matches_reference_arrays(llama_online_model):
    z = np.load(GOLDEN / "lowered.npz")
    keys = golden_lowered_keys(z)
    assert len(keys) >= 10
    for key, (M, seed, k) in keys.items():
        devs = synth_devices(M, seed)
        p = mo.lower_dense(devs, llama_online_model, k, 0.5)
        ref = load_golden_lowered(z, key)
        for name in ("c", "lb", "ub", "integrality", "b_ub", "A_eq"):
            assert np.array_equal(p[name], ref[name]), (key, name)
        assert np.array_equal(p["A_ub"], ref["A_ub"]), key


@pytest.mark.parametrize("solver", ["highs", "exact"])
def test_oracle_sweep_matches_reference_on_fixtures(fixtures_golden, solver):
    for key, fx in fixtures_golden["fixtures"].items():
        devs, model = fixture_fleet(fx["folder"])
        best, per_k = mo.halda_solve_oracle(devs, model, mip_gap=fx["mip_gap"], kv_bits=fx["kv_bits"], solver=solver)
        ref = fx["result"]
        assert (best["k"], best["w"], best["n"], best["sets"]) == (ref["k"], ref["w"], ref["n"], ref["sets"]), key
        if solver == "highs":
            assert best["obj_value"] == ref["obj_value"], key
        else:
            assert best["obj_value"] == pytest.approx(ref["obj_value"], rel=1e-12, abs=1e-12), key
        ref_k = {r["k"]: r for r in fx["per_k"]}
        for rec in per_k:
            assert rec["success"] == ref_k[rec["k"]]["success"], (key, rec["k"])


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16, 32, 64])
def test_exact_oracle_matches_reference_synthetic(synth_golden, llama_online_model, M):
    G = synth_golden[M]
    for fleet in G["fleets"]:
        devs = synth_devices(M, fleet["seed"], fleet["devices"])
        sets = mo.sets_of(devs)
        for rec in fleet["per_k"]:
            p = mo.lower_dense(devs, llama_online_model, rec["k"], 0.5, sets)
            st, x, best, second, _ = mo.exact_solve(p)
            if not rec["success"]:
                assert st == 2, (M, fleet["seed"], rec["k"], st)
                continue
            assert st == 0
            obj = mo.objective_value(p, x)
            assert obj == pytest.approx(rec["obj_value"], rel=1e-12, abs=1e-12)
            w = [int(round(v)) for v in x[:M]]
            n = [int(round(v)) for v in x[M:2 * M]]
            if mo.uniqueness_margin_ok(best, second):
                assert (w, n) == (rec["w"], rec["n"]), (M, fleet["seed"], rec["k"])


def test_exact_oracle_infeasible_bounds():
    """k > L makes W = 0 < lb(w) = 1; the reference gets a non-success status from HiGHS."""
    from distilp_amd.common import ModelProfileSplit
    from distilp_amd.synth import load_model_dict

    model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    devs = synth_devices(2, 0)
    p = mo.lower_dense(devs, model, 81, 0.5)
    st, *_ = mo.exact_solve(p)
    assert st == 2
    assert not mo.highs_solve(p).success


def test_golden_files_are_data_only():
    """Goldens hold inputs/outputs only (no reference source text)."""
    for p in GOLDEN.glob("*.json"):
        json.loads(p.read_text())


def test_exact_oracle_matches_highs_on_tied_fleets(llama_online_model):
    """Fleets of repeated devices (tests/ties.py; the reference's own "same device twice",
    test/test_integration.py:88): the exact C solver and the reference's arithmetic (dense lowering +
    scipy HiGHS) agree on status and objective per k, so the GPU tie test (test_gpu_ties.py) checks
    against a pinned oracle there too. Ties make the optimum non-unique, so (w, n) is not compared."""
    from .ties import FIXTURE_FOLDERS, fixture_twice, tied_fleets

    cases = [fixture_twice(f) for f in FIXTURE_FOLDERS]
    cases += [(devs, llama_online_model) for _, devs in tied_fleets(2)]
    for devs, model in cases:
        hi, hk = mo.halda_solve_oracle(devs, model, kv_bits="4bit", solver="highs")
        ex, ek = mo.halda_solve_oracle(devs, model, kv_bits="4bit", solver="exact")
        assert hi["k"] == ex["k"]
        assert abs(hi["obj_value"] - ex["obj_value"]) <= 1e-9 * max(1.0, abs(ex["obj_value"]))
        for a, b in zip(hk, ek):
            assert a["k"] == b["k"] and a["success"] == b["success"]
            if a["success"]:
                assert abs(a["obj_value"] - b["obj_value"]) <= 1e-9 * max(1.0, abs(b["obj_value"]))


def test_exact_oracle_matches_highs_with_zero_w_bounds(llama_online_model):
    """Outside the reference's own instances (it always sets lb(w) = 1): w lower bounds of 0 on some
    devices (the screen's bound-prefix test, test_gpu_parity.py). The exact solver's DP and its
    bound-infeasibility check follow the bounds, not w >= 1: the same status and objective as HiGHS."""
    from .helpers import synth_devices  # noqa: F401
    from distilp_amd.common import DeviceProfile
    from distilp_amd.synth import synth_fleet

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(77, 16)]
    for k, nz in ((8, 11), (8, 4), (1, 11), (5, 16), (16, 16)):
        p = mo.lower_dense(devs, llama_online_model, k, 0.5)
        p["lb"] = p["lb"].copy()
        p["lb"][:nz] = 0.0
        st, _, b1, _, _ = mo.exact_solve(p)
        r = mo.highs_solve(p)
        assert (st == 0) == (r.status == 0), (k, nz, st, r.status)
        if st == 0:
            assert abs(b1 - r.fun) <= 1e-9 * max(1.0, abs(r.fun)), (k, nz, b1, r.fun)


def test_oracle_matches_reference_tie_goldens():
    """tests/golden/ties.json -- the reference itself run on fleets of repeated devices (the "same device
    twice" shape of test/test_integration.py:88 for every folder x kv_bits x mip_gap, and tied synthetic
    fleets under two models): the oracle's HiGHS path returns the reference's HALDAResult bit for bit
    (the same lowering, scipy and HiGHS), and the exact C solver's sweep lies inside what HiGHS proved
    per k (check_sweep_against_golden). This pins the oracle on ties, where test_gpu_ties.py checks the GPU."""
    from .ties import TIE_MODELS, check_sweep_against_golden, tie_golden, tie_model, tied_fleets, twice_cases

    for key, devs, model, kv, gap, g in twice_cases():
        hi, _ = mo.halda_solve_oracle(devs, model, mip_gap=gap, kv_bits=kv, solver="highs")
        assert hi == g["result"], key
        ex, ek = mo.halda_solve_oracle(devs, model, mip_gap=gap, kv_bits=kv, solver="exact")
        check_sweep_against_golden(g, {r["k"]: (r["obj_value"] if r["success"] else None) for r in ek}, ex["k"],
                                   ex["obj_value"])
    gold = tie_golden()
    fleets = tied_fleets(gold["n_each"], gold["seed0"])
    for name in TIE_MODELS:
        model = tie_model(name)
        rows = gold["tied"][name]["fleets"]
        assert len(rows) == len(fleets)
        for i in range(0, len(fleets), 3):  # every third fleet through HiGHS (time), all through the exact solver
            hi, _ = mo.halda_solve_oracle(fleets[i][1], model, mip_gap=1e-4, kv_bits="4bit", solver="highs")
            assert hi == rows[i]["result"], (name, i)
        for (kind, devs), row in zip(fleets, rows):
            assert kind == row["kind"]
            ex, ek = mo.halda_solve_oracle(devs, model, mip_gap=1e-4, kv_bits="4bit", solver="exact")
            check_sweep_against_golden(row, {r["k"]: (r["obj_value"] if r["success"] else None) for r in ek},
                                       ex["k"], ex["obj_value"])
