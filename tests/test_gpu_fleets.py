"""GPU k-sweeps from a device-field table (libhalda halda_solve_fleets): the GPU lowering of the
CSR pipeline is bit-identical to the host lowering (itself pinned to the reference's arrays by
test_lowering), and the per-fleet results of the default fused sweep equal the host-lowered
path's and the reference goldens."""

import ctypes

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver import halda_solve_batch
from distilp_amd.solver._libhalda import HaldaBatchC, HaldaResultC, get_context
from distilp_amd.solver.fleets import _bind, fleet_table, halda_solve_fleets, solve_table
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.synth import synth_fleet

from .helpers import fixture_fleet, synth_devices

pytestmark = pytest.mark.gpu

KS80 = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def _hip():
    return ctypes.CDLL("libamdhip64.so")


def _d2h(ptr, count, dtype):
    out = np.empty(count, dtype)
    if count:
        rc = _hip().hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(out.nbytes), 2)
        assert rc == 0
    return out


def _lowered():
    ctx = get_context(0)
    lib = _bind(ctx.lib)
    b, r = HaldaBatchC(), HaldaResultC()
    assert lib.halda_last_lowered(ctx.ctx, ctypes.byref(b), ctypes.byref(r)) == 0
    return b


@pytest.mark.parametrize("M,seeds", [(1, range(6)), (3, range(6)), (7, range(4)), (16, range(3)), (64, range(2))])
def test_gpu_lowering_is_bit_identical(llama_online_model, M, seeds):
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)] for s in seeds]
    ks = KS80 + [3, 7]
    ks = sorted(set(ks))
    ctx = get_context(0)
    ctx.set_fleets_path(False)  # the CSR pipeline keeps the lowered batch (the fused sweep has none)
    try:
        solve_table(fleet_table(fleets, llama_online_model), llama_online_model, ks, 0.5)
        b = _lowered()
    finally:
        ctx.set_fleets_path(True)
    n = b.n_inst
    n_cols, n_rows = _d2h(b.n_cols, n, np.int32), _d2h(b.n_rows, n, np.int32)
    csr_off, col_off, row_off = (_d2h(getattr(b, f), n, np.int64) for f in ("csr_off", "col_off", "row_off"))
    for fi, devs in enumerate(fleets):
        fl = lower_fleet(devs, llama_online_model, "4bit")
        for j, k in enumerate(ks):
            i = fi * len(ks) + j
            m = int(n_rows[i])
            assert (n_cols[i], m) == (fl.n_cols, fl.n_rows)
            rp = _d2h(b.row_ptr + 4 * int(csr_off[i]), m + 1, np.int32)
            assert np.array_equal(np.diff(rp), np.diff(fl.row_ptr))
            cols = _d2h(b.col_idx + 4 * int(rp[0]), int(rp[-1] - rp[0]), np.int32)
            vals = _d2h(b.val + 8 * int(rp[0]), int(rp[-1] - rp[0]), np.float64)
            assert np.array_equal(cols, fl.col_idx) and np.array_equal(vals, fl.val), (M, fi, k)
            c, lb, ub, rlb, rub, integ, W = fl.instance(k)
            co, ro = int(col_off[i]), int(row_off[i])
            if W < M:  # bound-infeasible: only what the screen reads is lowered
                assert np.array_equal(_d2h(b.col_lb + 8 * co, M, np.float64), lb[:M])
                assert np.array_equal(_d2h(b.col_ub + 8 * co, M, np.float64), ub[:M])
                assert _d2h(b.c + 8 * (co + 7 * M), 1, np.float64)[0] == c[7 * M]
                assert np.array_equal(_d2h(b.row_ub + 8 * (ro + m - 1), 1, np.float64), rub[-1:])
                assert np.array_equal(_d2h(b.row_lb + 8 * (ro + m - 1), 1, np.float64), rlb[-1:])
                continue
            assert np.array_equal(_d2h(b.c + 8 * co, fl.n_cols, np.float64), c)
            assert np.array_equal(_d2h(b.col_lb + 8 * co, fl.n_cols, np.float64), lb)
            assert np.array_equal(_d2h(b.col_ub + 8 * co, fl.n_cols, np.float64), ub)
            assert np.array_equal(_d2h(b.integrality + co, fl.n_cols, np.uint8), integ)
            assert np.array_equal(_d2h(b.row_lb + 8 * ro, m, np.float64), rlb)
            assert np.array_equal(_d2h(b.row_ub + 8 * ro, m, np.float64), rub)


@pytest.mark.parametrize("M,seeds", [(2, range(40)), (5, range(20)), (16, range(12)), (64, range(8))])
def test_fleet_sweep_matches_host_lowered_path(llama_online_model, M, seeds):
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s + 900, M)] for s in seeds]
    host = halda_solve_batch(fleets, llama_online_model, mip_gap=1e-4, kv_bits="4bit")
    gpu = halda_solve_fleets(fleets, llama_online_model, mip_gap=1e-4, kv_bits="4bit")
    for h, g in zip(host, gpu):
        if h is None:
            assert g is None
            continue
        assert (g.k, g.w, g.n, g.sets) == (h.k, h.w, h.n, h.sets)
        assert abs(g.obj_value - h.obj_value) <= 1e-12 * max(1.0, abs(h.obj_value))


def test_fleet_sweep_matches_reference_goldens(synth_golden, fixtures_golden, llama_online_model):
    for M in (1, 2, 3, 4, 8, 16, 32, 64):
        G = synth_golden[M]
        fleets = [synth_devices(M, f["seed"], f["devices"]) for f in G["fleets"]]
        out = halda_solve_fleets(fleets, llama_online_model, mip_gap=1e-4, kv_bits="4bit")
        for r, f in zip(out, G["fleets"]):
            ref = f["result"]
            assert (r.k, r.w, r.n, r.sets) == (ref["k"], ref["w"], ref["n"], ref["sets"]), (M, f["seed"])
            assert abs(r.obj_value - ref["obj_value"]) <= 1e-9 * max(1.0, abs(ref["obj_value"]))
    for key, fx in fixtures_golden["fixtures"].items():
        devs, model = fixture_fleet(fx["folder"])
        r = halda_solve_fleets([devs], model, mip_gap=fx["mip_gap"], kv_bits=fx["kv_bits"])[0]
        ref = fx["result"]
        assert (r.k, r.w, r.n, r.sets) == (ref["k"], ref["w"], ref["n"], ref["sets"]), key
        assert abs(r.obj_value - ref["obj_value"]) <= 1e-9 * max(1.0, abs(ref["obj_value"]))


def test_fleet_sweep_per_k_objectives(llama_online_model):
    """obj_by_k equals the host path's per-k objective; infeasible k -> +inf, status 2."""
    from distilp_amd.solver._libhalda import STATUS_INFEASIBLE
    from distilp_amd.solver.batch import assemble

    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, 12)] for s in range(6)]
    res = solve_table(fleet_table(fleets, llama_online_model), llama_online_model, KS80, 0.5)
    lowered = [lower_fleet(d, llama_online_model, "4bit") for d in fleets]
    batch, refs = assemble(lowered, [KS80] * len(lowered))
    host = get_context(0).solve(batch)
    for idx, ref in enumerate(refs):
        j = KS80.index(ref.k)
        if host.status[idx] == STATUS_INFEASIBLE:
            assert res.status[ref.fleet, j] == STATUS_INFEASIBLE and np.isinf(res.obj_by_k[ref.fleet, j])
            continue
        x = host.x[ref.col_off:ref.col_off + ref.n_cols]
        want = lowered[ref.fleet].objective_value(ref.c, x)
        assert abs(res.obj_by_k[ref.fleet, j] - want) <= 1e-12 * max(1.0, abs(want))


def test_host_zero_copy_x_of_infeasible_k_are_zero(llama_online_model):
    """The host zero-copy path (small synchronous calls): the fused sweep leaves the x / c of
    non-optimal (fleet, k) instances unwritten in the pinned buffer and the copy-out zero-fills
    them. Two different batches in a row (the second would see the first's x / c if the fill were
    missing): non-optimal rows all zero, optimal rows equal to a large call's (device staging)."""
    ctx = get_context(0)
    for seeds, M in (([500, 501], 64), ([502, 503, 504], 12)):
        fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)] for s in seeds]
        table = fleet_table(fleets, llama_online_model)
        small = solve_table(table, llama_online_model, KS80, 0.5, want_x=True)
        N = 7 * M + 1
        for f in range(len(seeds)):
            for j in range(len(KS80)):
                if small.status[f, j] != 0:
                    assert not small.x[f, j].any() and not small.c[f, j].any(), (f, KS80[j])
        assert (small.status == 0).any() and (small.status != 0).any()
        # the same fleets inside a batch too large for the zero-copy path: same statuses and x / c
        big_fleets = fleets + [[DeviceProfile.model_validate(d) for d in synth_fleet(600 + i, M)] for i in range(300)]
        big = solve_table(fleet_table(big_fleets, llama_online_model), llama_online_model, KS80, 0.5, want_x=True)
        n = len(seeds)
        assert np.array_equal(big.status[:n], small.status)
        assert np.array_equal(big.x[:n, :, :N], small.x[:, :, :N]) and np.array_equal(big.c[:n, :, :N], small.c[:, :, :N])
    assert ctx is not None


def test_batch_api_equals_halda_solve_bits(llama_online_model):
    """halda_solve_batch (ONE fused k-sweep over all fleets, the objectives formed on the host from the
    compact x / c of the open instances) returns exactly what halda_solve returns fleet by fleet --
    k, w, n, sets and obj_value to the bit (the reference's own formula, halda_p_solver.py:347-357) --
    on a ragged batch (1..64 devices, incl. the C2 shape's four feasible k) and on a uniform one."""
    import contextlib
    import io

    from distilp_amd.solver import halda_solve

    sizes = [1, 2, 5, 16, 16, 64, 3, 40, 16, 7] * 3
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(4200 + s, M)] for s, M in enumerate(sizes)]
    for batch in (fleets, fleets[3:5] * 40):
        out = halda_solve_batch(batch, llama_online_model, mip_gap=1e-4, kv_bits="4bit")
        for devs, r in zip(batch, out):
            with contextlib.redirect_stdout(io.StringIO()):
                want = halda_solve(devs, llama_online_model, mip_gap=1e-4, plot=False, kv_bits="4bit")
            assert r is not None
            assert (r.k, r.w, r.n, r.sets, r.obj_value) == (want.k, want.w, want.n, want.sets, want.obj_value)
    # user k lists: a negative k is infeasible, k = 0 raises like the reference's W = L // k
    out = halda_solve_batch(fleets[:4], llama_online_model, k_candidates=[-2, 1, 3], kv_bits="4bit")
    assert all(r is not None and r.k in (1, 3) for r in out)
    with pytest.raises(ZeroDivisionError):
        halda_solve_batch(fleets[:2], llama_online_model, k_candidates=[0, 1], kv_bits="4bit")


def test_torch_still_sees_the_gpu_after_libhalda():
    """PyTorch-ROCm bundles its own HIP runtime: libhalda initialises torch's first when torch is
    imported (tools/probe_runtime_order.py shows the failure the other way round), so a process that
    imported torch, then solved with libhalda, can still use torch's device (a fresh subprocess, so
    that nothing initialised either runtime before)."""
    import subprocess
    import sys

    from .conftest import REPO

    code = ("import sys; sys.path.insert(0, '.'); import torch; "
            "from distilp_amd.solver._libhalda import get_context; get_context(0); "
            "x = torch.ones(8, device='cuda'); print(float(x.sum()))")
    r = subprocess.run([sys.executable, "-c", code], cwd=str(REPO), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and r.stdout.strip().endswith("8.0"), r.stderr[-2000:]


def test_c_abi_objective_against_halda_solve(fixtures_golden, llama_online_model):
    """What a C / C++ caller of halda_solve_fleets gets ("objective"): obj_value formed on
    the GPU (c.x in a fixed tree order), the best k picked with it. Against halda_solve (the reference's
    formula, halda_p_solver.py:356-357, c.x by NumPy on the host): obj_value within 1e-12 relative and the
    same best k wherever the best two k's objectives are more than 1e-12 apart (the documented near-tie
    caveat), on the 24 fixture cases and 1,024 C3 fleets."""
    import contextlib
    import io

    from distilp_amd.solver import halda_solve
    from distilp_amd.solver.lower import kv_bits_to_factor

    cases = []
    for fx in fixtures_golden["fixtures"].values():
        devs, model = fixture_fleet(fx["folder"])
        cases.append(([devs], model, fx["kv_bits"]))
    cases.append(([[DeviceProfile.model_validate(d) for d in synth_fleet(s, 64)] for s in range(1024)],
                  llama_online_model, "4bit"))
    n_cmp = n_bits = 0
    for fleets, model, kv in cases:
        with contextlib.redirect_stdout(io.StringIO()):
            from distilp_amd.solver.coefficients import valid_factors_of_L
            ks = sorted(valid_factors_of_L(model.L))
        res = solve_table(fleet_table(fleets, model), model, ks, kv_bits_to_factor(kv))
        for f, devs in enumerate(fleets):
            with contextlib.redirect_stdout(io.StringIO()):
                want = halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits=kv)
            got = float(res.obj_value[f])
            assert abs(got - want.obj_value) <= 1e-12 * max(1.0, abs(want.obj_value)), (f, got, want.obj_value)
            obk = np.sort(res.obj_by_k[f][np.isfinite(res.obj_by_k[f])])
            near = len(obk) > 1 and obk[1] - obk[0] <= 1e-12 * max(1.0, abs(obk[0]))
            if not near:
                assert int(res.best_k[f]) == want.k, (f, int(res.best_k[f]), want.k)
            n_cmp += 1
            n_bits += got == want.obj_value
    assert n_cmp == 24 + 1024
    print(f"C ABI obj_value bit-equal to halda_solve's on {n_bits} of {n_cmp}")


@pytest.mark.parametrize("want_x", ["open", True])
def test_page_locked_workspaces_equal_staged_copies(llama_online_model, want_x):
    """halda_solve_fleets_host with every array in halda_host_alloc blocks (the batch API's workspaces) DMAs
    straight from and to them; with pageable arrays it stages through the context's own buffer. Both give
    the same best k, obj_value, w, n, per-k objectives, statuses and x / c, bit for bit, on a batch above
    the zero-copy size (300 C3 fleets) -- compact ("open") and dense x / c layouts."""
    from distilp_amd.solver import fleets as FL

    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(9100 + s, 64)] for s in range(300)]
    pageable = fleet_table(fleets, llama_online_model)
    want = solve_table(pageable, llama_online_model, KS80, 0.5, want_x=want_x)
    pinned = fleet_table(fleets, llama_online_model, _reuse=True)
    assert FL._PINNED_OK, "halda_host_alloc failed on a GPU box"
    got = solve_table(pinned, llama_online_model, KS80, 0.5, want_x=want_x, _reuse=True)
    for f in ("best_k", "obj_value", "w", "n", "obj_by_k", "status", "x", "c"):
        assert np.array_equal(getattr(got, f), getattr(want, f)), f
    if want_x == "open":
        assert np.array_equal(got.x_off, want.x_off)
