"""GPU parity: libhalda (HIP, gfx950) vs the reference goldens and the CPU oracle.

Rule (north star): k, w, n and sets identical wherever the optimum is unique
(uniqueness from the exact oracle's second-best margin, rel 1e-7); the objective
within 1e-9 relative otherwise. Infeasible (fleet, k) pairs must match exactly.
All calls go through the C ABI (distilp_amd/libhalda.so via ctypes).
"""

import numpy as np
import pytest

from distilp_amd.solver import halda_solve, halda_solve_batch
from distilp_amd.solver._libhalda import STATUS_INFEASIBLE, STATUS_OPTIMAL, get_context
from distilp_amd.solver.batch import assemble
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.synth import synth_fleet
from oracle import milp_oracle as mo

from .helpers import fixture_fleet, synth_devices

pytestmark = pytest.mark.gpu

OBJ_REL = 1e-9


def _obj_close(a, b):
    return abs(a - b) <= OBJ_REL * max(1.0, abs(b))


def test_fixture_profiles_match_reference(fixtures_golden, capsys):
    for key, fx in fixtures_golden["fixtures"].items():
        devs, model = fixture_fleet(fx["folder"])
        r = halda_solve(devs, model, mip_gap=fx["mip_gap"], plot=False, kv_bits=fx["kv_bits"])
        ref = fx["result"]
        assert (r.k, r.w, r.n, r.sets) == (ref["k"], ref["w"], ref["n"], ref["sets"]), key
        assert _obj_close(r.obj_value, ref["obj_value"]), (key, r.obj_value, ref["obj_value"])
        out = capsys.readouterr().out
        assert out == fx["stdout"], key  # the "L [factors]" line, nothing else


def _solve_fleets(fleets, model, ks):
    lowered = [lower_fleet(devs, model, "4bit") for devs in fleets]
    batch, refs = assemble(lowered, [ks] * len(lowered))
    res = get_context(0).solve(batch)
    return lowered, refs, res


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16, 32, 64])
def test_synthetic_goldens_per_instance(synth_golden, llama_online_model, M):
    G = synth_golden[M]
    fleets = [synth_devices(M, f["seed"], f["devices"]) for f in G["fleets"]]
    ks = [r["k"] for r in G["fleets"][0]["per_k"]]
    lowered, refs, res = _solve_fleets(fleets, llama_online_model, ks)
    n_unique = 0
    for idx, ref in enumerate(refs):
        gold = G["fleets"][ref.fleet]["per_k"][ks.index(ref.k)]
        st = int(res.status[idx])
        if not gold["success"]:
            assert st == STATUS_INFEASIBLE, (M, ref.fleet, ref.k, st)
            continue
        assert st == STATUS_OPTIMAL, (M, ref.fleet, ref.k, st)
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        fl = lowered[ref.fleet]
        obj = fl.objective_value(ref.c, x)
        assert _obj_close(obj, gold["obj_value"]), (M, ref.fleet, ref.k, obj, gold["obj_value"])
        w = [int(round(v)) for v in x[:M]]
        n = [int(round(v)) for v in x[M:2 * M]]
        p = mo.lower_dense(fleets[ref.fleet], llama_online_model, ref.k, 0.5)
        _, _, b1, b2, _ = mo.exact_solve(p)
        if mo.uniqueness_margin_ok(b1, b2):
            n_unique += 1
            assert (w, n) == (gold["w"], gold["n"]), (M, ref.fleet, ref.k)
        # the GPU objective equals the proven optimum
        assert _obj_close(float(res.obj_lin[idx]), b1)
        assert res.dual_bound[idx] == res.obj_lin[idx] and res.gap[idx] == 0.0
    assert n_unique > 0


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16, 32, 64])
def test_batch_api_matches_reference(synth_golden, llama_online_model, M):
    G = synth_golden[M]
    fleets = [synth_devices(M, f["seed"], f["devices"]) for f in G["fleets"]]
    out = halda_solve_batch(fleets, llama_online_model, mip_gap=1e-4, kv_bits="4bit")
    for r, f in zip(out, G["fleets"]):
        ref = f["result"]
        assert (r.k, r.w, r.n, r.sets) == (ref["k"], ref["w"], ref["n"], ref["sets"])
        assert _obj_close(r.obj_value, ref["obj_value"])


@pytest.mark.parametrize("M,seeds", [(2, range(100, 140)), (5, range(100, 130)), (12, range(100, 120)),
                                     (24, range(100, 110)), (40, range(100, 104))])
def test_fresh_seeds_vs_exact_oracle(llama_online_model, M, seeds):
    """Unseen fleets (incl. M not in the goldens): GPU == exact CPU oracle."""
    from distilp_amd.common import DeviceProfile

    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)] for s in seeds]
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40, 3, 7]
    lowered, refs, res = _solve_fleets(fleets, llama_online_model, ks)
    for idx, ref in enumerate(refs):
        p = mo.lower_dense(fleets[ref.fleet], llama_online_model, ref.k, 0.5)
        st, xo, b1, b2, _ = mo.exact_solve(p)
        gst = int(res.status[idx])
        if st == 2:
            assert gst == STATUS_INFEASIBLE
            continue
        assert gst == STATUS_OPTIMAL
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        assert _obj_close(float(res.obj_lin[idx]), b1), (M, ref.fleet, ref.k)
        assert _obj_close(float(np.dot(p["c"], x)), b1)
        if mo.uniqueness_margin_ok(b1, b2):
            assert np.array_equal(x[:2 * M], xo[:2 * M]), (M, ref.fleet, ref.k)


def test_solution_is_feasible_and_deterministic(llama_online_model):
    """Full-size property check (config C3 shape): feasibility of x in the MILP, Sum w = W, determinism."""
    from distilp_amd.common import DeviceProfile

    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(s, 64)] for s in range(500, 756)]
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    lowered, refs, res = _solve_fleets(fleets, llama_online_model, ks)
    _, _, res2 = _solve_fleets(fleets, llama_online_model, ks)
    assert np.array_equal(res.status, res2.status) and np.array_equal(res.x, res2.x)
    for idx, ref in enumerate(refs):
        fl = lowered[ref.fleet]
        if ref.k > 1:
            assert res.status[idx] == STATUS_INFEASIBLE  # M = 64 > W
            continue
        assert res.status[idx] == STATUS_OPTIMAL
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        A = fl.dense()
        act = A @ x
        c, lb, ub, row_lb, row_ub, integ, W = fl.instance(ref.k)
        slack_tol = 1e-6 * np.maximum(1.0, np.abs(row_ub))
        assert np.all(act <= row_ub + slack_tol)
        assert np.all(act >= row_lb - slack_tol)
        assert np.all(x >= lb) and np.all(x <= ub)
        assert int(x[:fl.M].sum()) == W
        xi = x[integ.astype(bool)]
        assert np.array_equal(xi, np.round(xi))


def test_edge_k_candidates(llama_online_model, capsys):
    devs = synth_devices(2, 0)
    # k > L: W = 0 < lb(w) -> infeasible; non-divisor k: W = L // k; duplicates removed
    r = halda_solve(devs, llama_online_model, k_candidates=[3, 3, 81, 7], plot=False, kv_bits="4bit")
    best, per_k = mo.halda_solve_oracle(devs, llama_online_model, k_candidates=[3, 81, 7], kv_bits="4bit",
                                        solver="highs")
    assert (r.k, r.w, r.n) == (best["k"], best["w"], best["n"])
    assert capsys.readouterr().out == ""  # explicit k list: no factor print
    with pytest.raises(RuntimeError, match="No feasible MILP found for any k this round."):
        halda_solve(devs, llama_online_model, k_candidates=[81, 100], plot=False)
    with pytest.raises(ZeroDivisionError):
        halda_solve(devs, llama_online_model, k_candidates=[0, 1], plot=False)
    with pytest.raises(ValueError, match="Unsupported kv_bits"):
        halda_solve(devs, llama_online_model, kv_bits="2bit", plot=False)


def test_unsupported_structure_is_rejected(llama_online_model):
    devs = synth_devices(3, 1)
    fl = lower_fleet(devs, llama_online_model, "4bit")
    batch, refs = assemble([fl], [[1, 2]])
    batch.val = batch.val.copy()
    batch.val[0] = 0.5  # link row n - w <= 0 becomes n - 0.5 w <= 0: not a HALDA row
    res = get_context(0).solve(batch)
    assert list(res.status) == [-1, -1]


def test_debug_output_format(llama_online_model, capsys):
    devs, model = fixture_fleet("llama_3_70b/online")
    halda_solve(devs, model, plot=False, debug=True, kv_bits="4bit", k_candidates=[1, 2, 80])
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "Objectives by k"
    assert out[1] == "k: 1" and out[2].startswith("  k=1     obj=")
    assert out[-1] == "  k=80    obj=infeasible"


def test_host_api_computes_shape_summary_itself(llama_online_model):
    """INTEGRATION.md path B: one scipy-style MILP, shape summary left at 0."""
    import dataclasses

    devs = synth_devices(8, 3)
    fl = lower_fleet(devs, llama_online_model, "4bit")
    batch, refs = assemble([fl], [[1, 2, 4, 5]])
    auto = dataclasses.replace(batch, max_cols=0, max_R1=0, max_tab=0, max_tab_kc=0)
    a = get_context(0).solve(batch)
    b = get_context(0).solve(auto)
    assert np.array_equal(a.status, b.status) and np.array_equal(a.x, b.x)


@pytest.mark.parametrize("M,seed", [(6, 3), (16, 1), (64, 2)])
def test_k1_hand_back_path(llama_online_model, M, seed):
    """A k = 1 leaf that does not start at w = lb(w) (here lb(n_i) = 3 with n_i <= w_i, so w_i >= 3):
    the fast path hands the instance to the general path (tables in global scratch). GPU == exact
    oracle on the same modified MILP."""
    from distilp_amd.common import DeviceProfile

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    batch, refs = assemble([fl], [[1]])
    p = mo.lower_dense(devs, llama_online_model, 1, 0.5)
    gpu_dev = [i for i in range(M) if p["ub"][M + i] > 0]
    assert gpu_dev, "fleet needs a device with a GPU split"
    i = gpu_dev[0]
    batch.col_lb = batch.col_lb.copy()
    batch.col_lb[refs[0].col_off + M + i] = 3.0
    p["lb"] = p["lb"].copy()
    p["lb"][M + i] = 3.0
    res = get_context(0).solve(batch)
    st, xo, b1, b2, _ = mo.exact_solve(p)
    if st == 2:
        assert res.status[0] == STATUS_INFEASIBLE
        return
    assert res.status[0] == STATUS_OPTIMAL
    x = res.x[:refs[0].n_cols]
    assert x[M + i] >= 3.0 and x[i] >= 3.0
    assert _obj_close(float(res.obj_lin[0]), b1)
    assert _obj_close(float(np.dot(p["c"], x)), b1)
    if mo.uniqueness_margin_ok(b1, b2):
        assert np.array_equal(x[:2 * M], xo[:2 * M])


@pytest.mark.parametrize("M,seed", [(5, 0), (64, 1)])
def test_row_order_does_not_matter(llama_online_model, M, seed):
    """The k = 1 fast path decodes rows in the reference's order (capacity rows, then cycle rows);
    a CSR with its ub rows permuted takes the generic decode and gives the same solution."""
    import dataclasses

    from distilp_amd.common import DeviceProfile

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    batch, refs = assemble([fl], [[1, 2]])
    base = get_context(0).solve(batch)
    m = int(batch.n_rows[0])
    rp = batch.row_ptr[batch.csr_off[0]:batch.csr_off[0] + m + 1]
    perm = np.random.default_rng(seed).permutation(m - 1)
    perm = np.append(perm, m - 1)  # the equality row stays last
    cols, vals, ptr = [], [], [0]
    for r in perm:
        cols.append(batch.col_idx[rp[r]:rp[r + 1]])
        vals.append(batch.val[rp[r]:rp[r + 1]])
        ptr.append(ptr[-1] + rp[r + 1] - rp[r])
    row_lb, row_ub = batch.row_lb.copy(), batch.row_ub.copy()
    for ro in batch.row_off:
        row_lb[ro:ro + m] = batch.row_lb[ro + perm]
        row_ub[ro:ro + m] = batch.row_ub[ro + perm]
    shuffled = dataclasses.replace(batch, row_ptr=np.asarray(ptr, np.int32), col_idx=np.concatenate(cols),
                                   val=np.concatenate(vals), csr_off=np.zeros_like(batch.csr_off),
                                   row_lb=row_lb, row_ub=row_ub)
    res = get_context(0).solve(shuffled)
    assert np.array_equal(res.status, base.status)
    assert np.array_equal(res.x, base.x)


@pytest.mark.parametrize("M,seed,how", [(3, 0, "coef"), (64, 1, "coef"), (16, 2, "cols"), (6, 3, "hand_back")])
def test_bad_equality_row_is_rejected(llama_online_model, M, seed, how):
    """The equality row must read sum_i w_i = W. The fused k = 1 screen defers that check to the
    k = 1 decode; the general kernel repeats it for instances handed back to it. A corrupted row
    is UNSUPPORTED on every path (k = 1 fast path, k > 1, hand-back)."""
    from distilp_amd.common import DeviceProfile

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    batch, refs = assemble([fl], [[1, 2]])
    batch.col_idx, batch.val, batch.col_lb = batch.col_idx.copy(), batch.val.copy(), batch.col_lb.copy()
    seen = set()  # instances of one fleet may share their CSR
    for j, ref in enumerate(refs):
        m = int(batch.n_rows[j])
        rp = batch.row_ptr[batch.csr_off[j]:]
        eq = int(rp[m - 1])
        if eq in seen:
            continue
        seen.add(eq)
        if how == "cols":
            batch.col_idx[eq], batch.col_idx[eq + 1] = batch.col_idx[eq + 1], batch.col_idx[eq]
        else:
            batch.val[eq + 1] = 2.0
    for ref in refs:
        if how == "hand_back":
            p = mo.lower_dense(devs, llama_online_model, ref.k, 0.5)
            i = [d for d in range(M) if p["ub"][M + d] > 0][0]
            batch.col_lb[ref.col_off + M + i] = 3.0
    res = get_context(0).solve(batch)
    assert list(res.status) == [-1, -1], (how, list(res.status))


@pytest.mark.parametrize("M,seed,case", [(5, 0, "empty"), (64, 1, "empty"), (6, 2, "fixed"), (64, 3, "fixed"),
                                         (16, 4, "capped")])
def test_w_upper_bounds_are_honoured(llama_online_model, M, seed, case):
    """The screen reads only the w lower bounds; the w upper bounds are the solve's business. A
    device with an empty w range (lb 3 > ub 2) makes every k infeasible; a fixed w (lb = ub) or a
    tight cap must give the exact oracle's optimum. k = 1 (fast path) and k = 2 (general kernel)."""
    from distilp_amd.common import DeviceProfile

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(seed, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    ks = [1, 2]
    batch, refs = assemble([fl], [ks])
    batch.col_lb, batch.col_ub = batch.col_lb.copy(), batch.col_ub.copy()
    lo, hi = {"empty": (3.0, 2.0), "fixed": (1.0, 1.0), "capped": (1.0, 2.0)}[case]  # lb never below the lowering's (shape summary)
    probs = []
    for ref in refs:
        p = mo.lower_dense(devs, llama_online_model, ref.k, 0.5)
        p["lb"], p["ub"] = p["lb"].copy(), p["ub"].copy()
        for i in (0, M // 2):
            batch.col_lb[ref.col_off + i], batch.col_ub[ref.col_off + i] = lo, hi
            p["lb"][i], p["ub"][i] = lo, hi
        probs.append(p)
    res = get_context(0).solve(batch)
    for j, (ref, p) in enumerate(zip(refs, probs)):
        st, xo, b1, b2, _ = mo.exact_solve(p)
        if st == 2:
            assert res.status[j] == STATUS_INFEASIBLE, (case, ref.k, res.status[j])
            continue
        assert res.status[j] == STATUS_OPTIMAL, (case, ref.k, res.status[j])
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        assert _obj_close(float(res.obj_lin[j]), b1)
        assert lo <= x[0] <= hi and lo <= x[M // 2] <= hi
        if mo.uniqueness_margin_ok(b1, b2):
            assert np.array_equal(x[:2 * M], xo[:2 * M])


@pytest.mark.parametrize("n_streams", [2, 9])
def test_csr_batches_on_several_streams(llama_online_model, n_streams):
    """The milp() replacement (halda_solve_batch_device) with its verdict bytes and hand-back flag in
    the stream's scratch slot: batches alternating over 2 and 9 streams (more streams than slots: a
    slot is handed over after the launches of the stream it leaves), k > 1 instances included (16-
    device fleets), give the results of one synchronous call each, bit for bit."""
    import torch

    from distilp_amd.common import DeviceProfile

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    batches = []
    for b, M in enumerate([16, 64, 12]):
        fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(900 + 40 * b + s, M)] for s in range(40)]
        lowered = [lower_fleet(devs, llama_online_model, "4bit") for devs in fleets]
        batch, _ = assemble(lowered, [ks] * len(lowered))
        batches.append((batch, ctx.solve(batch)))
    fields = ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr", "col_idx", "val", "c", "col_lb",
              "col_ub", "row_lb", "row_ub", "integrality")
    runs = []
    for batch, _ in batches:
        keep = {f: torch.from_numpy(np.ascontiguousarray(getattr(batch, f))).to(dev) for f in fields}
        n = batch.n_inst
        out = {"status": torch.empty(n, dtype=torch.int32, device=dev),
               "x": torch.zeros(batch.total_cols, dtype=torch.float64, device=dev),
               "obj_lin": torch.empty(n, dtype=torch.float64, device=dev),
               "dual_bound": torch.empty(n, dtype=torch.float64, device=dev),
               "gap": torch.empty(n, dtype=torch.float64, device=dev),
               "nodes": torch.empty(n, dtype=torch.int64, device=dev)}
        runs.append((keep, out))
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    ctx.set_timing(False)
    try:
        for i in range(3 * n_streams):
            j = i % len(batches)
            keep, out = runs[j]
            ctx.solve_device({f: t.data_ptr() for f, t in keep.items()}, batches[j][0],
                             {f: t.data_ptr() for f, t in out.items()}, stream=streams[i % n_streams].cuda_stream)
        torch.cuda.synchronize(dev)
    finally:
        ctx.set_timing(True)
    for (batch, want), (_, out) in zip(batches, runs):
        assert np.array_equal(out["status"].cpu().numpy(), want.status)
        assert np.array_equal(out["x"].cpu().numpy(), want.x)
        assert np.array_equal(out["obj_lin"].cpu().numpy(), want.obj_lin)


@pytest.mark.parametrize("case", ["lowered", "zero_prefix", "neg_tail", "nan_tail"])
def test_screen_bound_infeasibility_from_a_prefix(llama_online_model, case):
    """The screen proves bound infeasibility (sum_i ceil(lb(w_i)) > W, HiGHS's presolve verdict) from the
    first min(M, W + 1) w lower bounds when they already exceed W (every bound is >= 0 or infeasible by
    itself), reading the others only when they do not. M = 16 at k = 8 (W = 10 < M): as lowered it is
    infeasible from the prefix; with the first 11 bounds 0 the rest decide (sum 5 <= 10: solved, against
    the exact oracle); a negative or NaN bound past the prefix does not change the verdict. k = 1 (W = 80:
    the prefix is every bound) is solved as usual."""
    from distilp_amd.common import DeviceProfile

    M = 16
    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(77, M)]
    fl = lower_fleet(devs, llama_online_model, "4bit")
    ks = [1, 8]
    batch, refs = assemble([fl], [ks])
    batch.col_lb = batch.col_lb.copy()
    probs = []
    for ref in refs:
        p = mo.lower_dense(devs, llama_online_model, ref.k, 0.5)
        p["lb"] = p["lb"].copy()
        if ref.k == 8:
            if case == "zero_prefix":
                for i in range(11):
                    batch.col_lb[ref.col_off + i] = p["lb"][i] = 0.0
            elif case == "neg_tail":
                batch.col_lb[ref.col_off + 15] = p["lb"][15] = -1.0
            elif case == "nan_tail":
                batch.col_lb[ref.col_off + 15] = np.nan
        probs.append(p)
    batch.max_cols = batch.max_R1 = batch.max_tab = batch.max_tab_kc = 0  # summary from the bounds (host API)
    res = get_context(0).solve(batch)
    for j, (ref, p) in enumerate(zip(refs, probs)):
        if ref.k == 8 and case != "zero_prefix":
            assert res.status[j] == STATUS_INFEASIBLE, (case, res.status[j])
            continue
        st, xo, b1, b2, _ = mo.exact_solve(p)
        assert st == 0 and res.status[j] == STATUS_OPTIMAL, (case, ref.k, st, res.status[j])
        assert _obj_close(float(res.obj_lin[j]), b1), (case, ref.k)
        x = res.x[ref.col_off:ref.col_off + ref.n_cols]
        if mo.uniqueness_margin_ok(b1, b2):
            assert np.array_equal(x[:2 * M], xo[:2 * M])
