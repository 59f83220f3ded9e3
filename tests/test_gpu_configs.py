"""GPU parity on the benchmark configurations themselves, the k > 1 DP-per-candidate fallback and
the INTEGRATION.md path-B stub.

  * C3: 1,024 of the bench's own fleets (seeds 0..1023, M = 64, L = 80, all 9 k) through the
    production launch sequence (two-pass screen + persistent k = 1 kernel + general kernel) and
    through the GPU-lowered k-sweep (halda_solve_fleets), against the exact oracle;
  * C5: the perturbed stream of SURVEY.md §8(d) (base fleet seed 0, every numeric DeviceProfile
    field x LU(0.9, 1.1), seed stream 10_000 + i), 256 instances through halda_solve_fleets, against
    the exact oracle and, on a sample, the reference's own arithmetic (scipy HiGHS);
  * the general kernel's DP-per-candidate threshold scan (halda.hip dp_pass, taken when a leaf's
    cycle time is not monotone so the incremental scan does not apply);
  * the reference's captured milp() arguments (tests/golden/lowered.npz) through the ctypes stub a
    maintainer would add to the reference (integration/halda_milp.py, INTEGRATION.md path B).
Reference call surface: halda_p_solver.py:340-357 (milp -> success, x -> w, n, obj_value).
"""

import os

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver._libhalda import LIB_PATH, STATUS_INFEASIBLE, STATUS_OPTIMAL, get_context
from distilp_amd.solver.batch import assemble
from distilp_amd.solver.fleets import fleet_table, halda_solve_fleets, solve_table
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.synth import load_templates, perturbed_fleet, synth_fleet
from oracle import milp_oracle as mo

from .conftest import GOLDEN
from .helpers import golden_lowered_keys, load_golden_lowered, synth_devices

pytestmark = pytest.mark.gpu

KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]
OBJ_REL = 1e-9


def _close(a, b):
    return abs(a - b) <= OBJ_REL * max(1.0, abs(b))


def _oracle_k1(devs, model):
    p = mo.lower_dense(devs, model, 1, 0.5)
    st, xo, b1, b2, _ = mo.exact_solve(p)
    return p, st, xo, b1, b2


def test_c3_bench_fleets_vs_exact_oracle(llama_online_model):
    """C3 seeds 0..1023 (the bench's first quarter): every k > 1 infeasible (M = 64 > W), every k = 1
    optimal with the exact oracle's objective and, where the optimum is unique, its (w, n); the
    k-sweep through halda_solve_fleets returns the same k, w, n and obj_value."""
    tpl = load_templates()
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, 64, tpl)] for s in range(1024)]
    model = llama_online_model
    lowered = [lower_fleet(devs, model, "4bit") for devs in fleets]
    batch, refs = assemble(lowered, [KS] * len(lowered))
    res = get_context(0).solve(batch)
    sweep = solve_table(fleet_table(fleets, model), model, KS, 0.5)
    assert np.array_equal(sweep.status.reshape(-1), res.status)
    n_unique = 0
    for f, devs in enumerate(fleets):
        for j, k in enumerate(KS):
            idx = f * len(KS) + j
            if k > 1:
                assert res.status[idx] == STATUS_INFEASIBLE
                continue
            p, st, xo, b1, b2 = _oracle_k1(devs, model)
            assert st == 0 and res.status[idx] == STATUS_OPTIMAL, (f, st, res.status[idx])
            x = res.x[refs[idx].col_off:refs[idx].col_off + refs[idx].n_cols]
            assert _close(float(res.obj_lin[idx]), b1), (f, float(res.obj_lin[idx]), b1)
            obj = mo.objective_value(p, x)
            assert sweep.best_k[f] == 1 and _close(float(sweep.obj_value[f]), obj)
            w, n = x[:64], x[64:128]
            assert np.array_equal(sweep.w[64 * f:64 * f + 64], np.rint(w)) and np.array_equal(
                sweep.n[64 * f:64 * f + 64], np.rint(n))
            if mo.uniqueness_margin_ok(b1, b2):
                n_unique += 1
                assert np.array_equal(x[:128], xo[:128]), f
    assert n_unique >= 900
    # the register launch's exact DP fallback (forced for every k = 1 solve) on the same fleets
    ctx = get_context(0)
    ctx.set_fleets_path("dp")
    try:
        dp = solve_table(fleet_table(fleets, model), model, KS, 0.5)
    finally:
        ctx.set_fleets_path(True)
    assert np.array_equal(dp.best_k, sweep.best_k)
    assert np.allclose(dp.obj_value, sweep.obj_value, rtol=1e-12, atol=0.0)
    # the oracle agrees that k > 1 is infeasible (a sample: every k of the first fleets)
    for devs in fleets[:4]:
        for k in KS[1:]:
            assert mo.exact_solve(mo.lower_dense(devs, model, k, 0.5))[0] == 2


def test_c5_perturbed_stream_vs_oracle(llama_online_model):
    """C5 stream instances 0..255: halda_solve_fleets k-sweep == exact oracle
    sweep (k, w, n, obj); the first 6 also against scipy HiGHS (the reference's arithmetic)."""
    base = synth_fleet(0, 64)
    fleets = [[DeviceProfile.model_validate(d) for d in perturbed_fleet(base, i)] for i in range(256)]
    model = llama_online_model
    got = halda_solve_fleets(fleets, model, kv_bits="4bit")
    for i, (devs, r) in enumerate(zip(fleets, got)):
        want, per_k = mo.halda_solve_oracle(devs, model, kv_bits="4bit", solver="exact")
        assert r is not None and want is not None
        assert r.k == want["k"] and r.sets == want["sets"], i
        assert _close(r.obj_value, want["obj_value"]), (i, r.obj_value, want["obj_value"])
        rec = next(q for q in per_k if q["k"] == want["k"])
        if rec["margin"] > 1e-7 * max(1.0, abs(rec["obj_value"])):
            assert (r.w, r.n) == (want["w"], want["n"]), i
        if i < 6:
            hi, _ = mo.halda_solve_oracle(devs, model, kv_bits="4bit", solver="highs")
            assert (r.k, r.w, r.n) == (hi["k"], hi["w"], hi["n"]), i
            assert _close(r.obj_value, hi["obj_value"])


def _steepen_cycle_rows(batch, refs, M, dev, L):
    """One fleet: rewrite device `dev`'s two cycle rows so that its least cycle time strictly
    DEcreases in w (w coefficient -big, right-hand side lowered by big * W / 2 so it crosses the
    other devices' times near w = W / 2): the incremental threshold scan needs it nondecreasing, the DP-per-candidate scan does
    not. Its objective price of w goes up by (k - 1) big / 2 per instance, so that cost and cycle
    time pull w_dev in opposite directions and the threshold scan has work to do."""
    batch.val, batch.row_ub, batch.c = batch.val.copy(), batch.row_ub.copy(), batch.c.copy()
    m = int(batch.n_rows[0])
    rp = batch.row_ptr
    for r in range(m - 1 - 2 * M, m - 1):
        cols = batch.col_idx[rp[r]:rp[r + 1]]
        if cols[-2] != 6 * M + dev:  # z column of another device
            continue
        vals = batch.val[rp[r]:rp[r + 1]]
        assert cols[0] == dev  # the w entry leads the row
        big = 2.0 * float(np.abs(vals[1:-2]).sum()) + 1.0
        batch.val[rp[r]] = -big
        for j in range(len(refs)):
            batch.row_ub[int(batch.row_off[j]) + r] -= big * (L // refs[j].k) / 2
            if vals[-2] > 0:  # once per device (first cycle row)
                batch.c[int(batch.col_off[j]) + dev] += 0.5 * (refs[j].k - 1) * big
    return batch


@pytest.mark.parametrize("M,seed", [(3, 0), (6, 1), (12, 2)])
def test_dp_per_candidate_fallback(llama_online_model, M, seed):
    """k > 1 with a non-monotone leaf: the general kernel's DP-per-candidate scan (phase-0 pass, one
    DP pass per candidate threshold, final pass) must give the exact oracle's optimum."""
    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    ks = [2, 4, 5]
    batch, refs = assemble([fl], [ks])
    batch = _steepen_cycle_rows(batch, refs, M, 0, llama_online_model.L)
    res = get_context(0).solve(batch)
    A = np.zeros((int(batch.n_rows[0]), int(batch.n_cols[0])))
    for r in range(A.shape[0]):
        a, b = batch.row_ptr[r], batch.row_ptr[r + 1]
        A[r, batch.col_idx[a:b]] = batch.val[a:b]
    ran_scan = False
    for j, ref in enumerate(refs):
        p = mo.lower_dense(devs, llama_online_model, ref.k, 0.5)
        p["A_ub"] = A[:-1].copy()
        p["b_ub"] = batch.row_ub[int(batch.row_off[j]):int(batch.row_off[j]) + A.shape[0] - 1].copy()
        p["c"] = batch.c[int(batch.col_off[j]):int(batch.col_off[j]) + int(batch.n_cols[j])].copy()
        st, xo, b1, b2, _ = mo.exact_solve(p)
        if st == 2:
            assert res.status[j] == STATUS_INFEASIBLE
            continue
        assert res.status[j] == STATUS_OPTIMAL, (M, ref.k, res.status[j])
        assert _close(float(res.obj_lin[j]), b1), (M, ref.k, float(res.obj_lin[j]), b1)
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        assert _close(float(np.dot(p["c"], x)), b1)
        if mo.uniqueness_margin_ok(b1, b2):
            assert np.array_equal(x[:2 * M], xo[:2 * M])
        ran_scan |= int(res.nodes[j]) >= 3  # phase 0 + >= 1 candidate pass + final pass
    assert ran_scan


def test_path_b_stub_on_reference_arrays(synth_golden, llama_online_model):
    """The reference's own milp() arguments (captured by spying on halda_p_solver.milp,
    tests/golden/lowered.npz) through integration/halda_milp.py: success / w / n as HiGHS gave them
    (tests/golden/synthetic_M*.json), obj_value equal within 1e-9."""
    from scipy.optimize import Bounds, LinearConstraint

    os.environ["HALDA_LIB"] = str(LIB_PATH)
    from integration.halda_milp import halda_milp

    z = np.load(GOLDEN / "lowered.npz")
    for key, (M, seed, k) in golden_lowered_keys(z).items():
        ref = load_golden_lowered(z, key)
        cons = [LinearConstraint(ref["A_ub"], -np.inf, ref["b_ub"]),
                LinearConstraint(ref["A_eq"], ref["b_eq"], ref["b_eq"])]
        res = halda_milp(ref["c"], ref["integrality"], Bounds(ref["lb"], ref["ub"]), cons,
                         {"time_limit": 3600, "mip_rel_gap": 1e-4})
        gold = next(r for r in synth_golden[M]["fleets"][seed]["per_k"] if r["k"] == k)
        assert res.success == gold["success"], key
        if not gold["success"]:
            continue
        w = [int(round(v)) for v in res.x[:M]]
        n = [int(round(v)) for v in res.x[M:2 * M]]
        fl = lower_fleet(synth_devices(M, seed), llama_online_model, "4bit")
        obj = fl.objective_value(ref["c"], res.x)
        assert _close(obj, gold["obj_value"]), (key, obj, gold["obj_value"])
        assert (w, n) == (gold["w"], gold["n"]), key


def test_c2_fleets_vs_exact_oracle(llama_online_model):
    """C2 (BASELINE configs[1]): 256 synthetic 16-device fleets (seeds 0..255), every k of L = 80,
    through halda_solve_fleets (the fused sweep: k = 1, 2, 4, 5 feasible) against the exact oracle
    per (fleet, k) -- status, objective, (w, n) where unique -- and its k-sweep."""
    tpl = load_templates()
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, 16, tpl)] for s in range(256)]
    model = llama_online_model
    res = solve_table(fleet_table(fleets, model), model, KS, 0.5, want_x=True)
    n_unique = 0
    for f, devs in enumerate(fleets):
        best = None
        for j, k in enumerate(KS):
            p = mo.lower_dense(devs, model, k, 0.5)
            st, xo, b1, b2, _ = mo.exact_solve(p)
            if st == 2:
                assert res.status[f, j] == STATUS_INFEASIBLE, (f, k)
                continue
            assert res.status[f, j] == STATUS_OPTIMAL, (f, k, res.status[f, j])
            x = res.x[f, j, :p["c"].shape[0]]
            assert _close(float(np.dot(p["c"], x)), b1), (f, k)
            obj = mo.objective_value(p, x)
            assert _close(float(res.obj_by_k[f, j]), obj)
            if mo.uniqueness_margin_ok(b1, b2):
                n_unique += 1
                assert np.array_equal(x[:32], xo[:32]), (f, k)
            if best is None or obj < best[0]:
                best = (obj, k)
        assert res.best_k[f] == best[1], f
    assert n_unique >= 900
