"""Shapes the reference accepts without limit (halda_p_solver.py:72: W = L // k, any L, any M).

libhalda sizes its on-chip scratch from a per-batch shape summary; tables beyond the LDS budget
go to a global-memory launch of the same general kernel, and DP nodes wider than 128 states are
evaluated in chunks. Every (fleet, k) is checked against the exact CPU oracle (status, objective,
and (w, n) wherever the optimum is unique); the whole k-sweep against the oracle's sweep.
Parity here is against the exact oracle only: no reference fixture has L != 64/80 (parity of
these shapes with HiGHS is covered by the oracle's own pinning on the goldens).
"""

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver import halda_solve
from distilp_amd.solver._libhalda import STATUS_INFEASIBLE, STATUS_OPTIMAL, get_context
from distilp_amd.solver.batch import assemble
from distilp_amd.solver.fleets import halda_solve_fleets
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.synth import synth_fleet
from oracle import milp_oracle as mo

pytestmark = pytest.mark.gpu

OBJ_REL = 1e-9


def _close(a, b):
    return abs(a - b) <= OBJ_REL * max(1.0, abs(b))


def _factors(L):
    return [d for d in range(1, L) if L % d == 0]


def _check_batch(fleets, model, ks):
    """CSR path (halda_solve_batch) for every (fleet, k) vs the exact oracle; returns oracle sweeps."""
    lowered = [lower_fleet(devs, model, "4bit") for devs in fleets]
    batch, refs = assemble(lowered, [ks] * len(lowered))
    res = get_context(0).solve(batch)
    for idx, ref in enumerate(refs):
        devs = fleets[ref.fleet]
        M = len(devs)
        p = mo.lower_dense(devs, model, ref.k, 0.5)
        st, xo, b1, b2, _ = mo.exact_solve(p)
        gst = int(res.status[idx])
        if st == 2:
            assert gst == STATUS_INFEASIBLE, (M, model.L, ref.k, gst)
            continue
        assert gst == STATUS_OPTIMAL, (M, model.L, ref.k, gst)
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        assert _close(float(res.obj_lin[idx]), b1), (M, model.L, ref.k, float(res.obj_lin[idx]), b1)
        assert _close(float(np.dot(p["c"], x)), b1)
        assert int(round(x[:M].sum())) == p["W"]
        if mo.uniqueness_margin_ok(b1, b2):
            assert np.array_equal(x[:2 * M], xo[:2 * M]), (M, model.L, ref.k)


@pytest.mark.parametrize("L", [96, 160, 256])
@pytest.mark.parametrize("M", [1, 2, 3, 8])
def test_large_L_every_factor_k(llama_online_model, L, M):
    """L in {96, 160, 256} (R + 1 up to 256 > the old 128 cap), M in {1, 2, 3, 8}, every factor k:
    per-instance CSR path and the GPU-lowered k-sweep (halda_solve / halda_solve_fleets)."""
    model = llama_online_model.model_copy(update={"L": L})
    ks = _factors(L)
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)] for s in (11, 12)]
    _check_batch(fleets, model, ks)
    got = halda_solve_fleets(fleets, model, k_candidates=ks, kv_bits="4bit")
    for devs, r in zip(fleets, got):
        want, per_k = mo.halda_solve_oracle(devs, model, k_candidates=ks, kv_bits="4bit", solver="exact")
        if want is None:
            assert r is None
            continue
        assert r is not None and r.k == want["k"], (L, M, r, want)
        assert _close(r.obj_value, want["obj_value"])
        rec = next(q for q in per_k if q["k"] == want["k"])
        p = mo.lower_dense(devs, model, want["k"], 0.5)
        _, _, b1, b2, _ = mo.exact_solve(p)
        if mo.uniqueness_margin_ok(b1, b2):
            assert (r.w, r.n) == (rec["w"], rec["n"])
        one = halda_solve(devs, model, k_candidates=ks, plot=False, kv_bits="4bit")
        assert (one.k, one.w, one.n) == (r.k, r.w, r.n) and _close(one.obj_value, want["obj_value"])


def test_wide_fleet_and_big_tables(llama_online_model):
    """One batch mixing a 100-device fleet (M > 64: no k = 1 fast path, tables beyond the LDS budget)
    with a 48-device and an 8-device fleet at L = 256: the batch's shape summary exceeds the LDS
    budget, so the general kernel runs capped LDS slices plus the global-table launch (k > 1
    threshold scan and k = 1 tables on HBM)."""
    model = llama_online_model.model_copy(update={"L": 256})
    lib = get_context(0).lib
    assert lib.halda_lds_bytes(7 * 100 + 1, 157, 100 * 157, 100 * 29) > 160 * 1024
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)] for s, M in ((0, 100), (1, 48), (2, 8))]
    _check_batch(fleets, model, [1, 2, 4])
    got = halda_solve_fleets(fleets, model, k_candidates=[1, 2, 4], kv_bits="4bit")
    for devs, r in zip(fleets, got):
        want, _ = mo.halda_solve_oracle(devs, model, k_candidates=[1, 2, 4], kv_bits="4bit", solver="exact")
        assert r.k == want["k"] and _close(r.obj_value, want["obj_value"]), (len(devs), r, want)


def test_big_table_launches_on_two_streams(llama_online_model):
    """Batches whose tables exceed the LDS budget share the context's global-memory tables
    (halda_sweep_big_kernel / halda_solve_big_kernel): two such fused-sweep batches alternating over two
    streams, with a CSR-pipeline batch on global tables in between, must each give the results of one
    synchronous call, bit for bit (the big launches are ordered after the previous one on another
    stream; without that they would write the same table slices concurrently)."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table, solve_table

    model = llama_online_model.model_copy(update={"L": 256})
    ks = [1, 2, 4]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    tables = [fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)]
                           for s, M in zip(range(b * 8, b * 8 + 8), (100, 80, 72, 96, 66, 100, 90, 70))], model)
              for b in range(2)]
    want = [solve_table(t, model, ks, 0.5, want_x=False) for t in tables]
    dts = [DeviceFleetTable(t, model, ks, 0.5, dev, want_per_k=True) for t in tables]
    mid_fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, 100)] for s in (40, 41)]
    lowered = [lower_fleet(devs, model, "4bit") for devs in mid_fleets]
    batch, _ = assemble(lowered, [ks] * len(lowered))
    mid_want = ctx.solve(batch)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for i in range(6):
        dts[i % 2].launch(ctx, streams[i % 2].cuda_stream)
        if i == 3:
            mid = ctx.solve(batch)
            assert np.array_equal(mid.status, mid_want.status) and np.array_equal(mid.x, mid_want.x)
    torch.cuda.synchronize(dev)
    for d, w in zip(dts, want):
        assert np.array_equal(d.out["best_k"].cpu().numpy(), w.best_k)
        assert np.array_equal(d.out["w"].cpu().numpy(), w.w) and np.array_equal(d.out["n"].cpu().numpy(), w.n)
        assert np.array_equal(d.out["obj_value"].cpu().numpy(), w.obj_value)
        assert np.array_equal(d.out["status"].cpu().numpy(), w.status.ravel())
        assert np.array_equal(d.out["obj_by_k"].cpu().numpy(), w.obj_by_k.ravel())


@pytest.mark.parametrize("L,M", [(96, 12), (96, 16), (120, 16), (48, 8)])
def test_kslot_kernel_other_L(llama_online_model, L, M):
    """The k-slot kernel (more than 64 fleets of at most 16 devices, one wave per open k) on other layer
    counts than C2's L = 80: other open k's, another split slot / helper / leaf-check wave (the split
    slot is the largest table, the checker the smallest other one), default path and the split in
    sequential order against the one-fleet-per-wave sweep bit for bit, and 4 fleets' sweeps against the
    exact oracle."""
    from distilp_amd.solver.fleets import fleet_table, solve_table

    model = llama_online_model.model_copy(update={"L": L})
    ks = _factors(L)
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(31000 + s, M)] for s in range(72)]
    table = fleet_table(fleets, model)
    ctx = get_context(0)
    runs = {}
    try:
        ctx.set_timing(True)
        for path in ("fused", "kslot_sequential", "wave"):
            ctx.set_fleets_path(path)
            runs[path] = solve_table(table, model, ks, 0.5, want_x=True)
            if path != "wave":
                assert "halda_sweep_kslot_kernel" in ctx.last_fleet_ms(), (path, ctx.last_fleet_ms())
    finally:
        ctx.set_fleets_path("fused")
        ctx.set_timing(False)
    for path in ("fused", "kslot_sequential"):
        for f in ("status", "obj_by_k", "best_k", "obj_value", "w", "n"):
            assert np.array_equal(getattr(runs[path], f), getattr(runs["wave"], f)), (path, f)
        N = 7 * M + 1
        assert np.array_equal(runs[path].x[:, :, :N], runs["wave"].x[:, :, :N]), path
    res = runs["fused"]
    for fi in range(4):
        want, _ = mo.halda_solve_oracle(fleets[fi], model, k_candidates=ks, kv_bits="4bit", solver="exact")
        assert res.best_k[fi] == want["k"] and _close(float(res.obj_value[fi]), want["obj_value"]), (fi, want)
