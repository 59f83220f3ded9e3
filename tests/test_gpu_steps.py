"""Group launches (halda_fleets_group_create / _launch, `PlanGroup`): `steps` batches over resident
tables in ONE launch (halda_sweep_steps_kernel) -- the bench's C3 headline and a streaming caller's
loop over re-profiled fleets (halda_p_solver.py:369-436 once per fleet and batch). Every batch must
leave in its own table's result arrays exactly the bits its own halda_solve_fleets call writes."""

from dataclasses import replace

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver._libhalda import HaldaContext, get_context
from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS, fleet_table, solve_table
from distilp_amd.synth import synth_fleet

pytestmark = pytest.mark.gpu

KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def _tiled(model, M, n_base, nf, seed):
    """nf fleets of M devices: n_base synthetic fleets tiled to nf, every numeric field perturbed
    (LU(0.9, 1.1)) so that no two fleets are the same."""
    base = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(seed + s, M)] for s in range(n_base)],
                       model)
    reps = -(-nf // n_base)
    big = replace(base, dev_off=np.arange(n_base * reps + 1, dtype=np.int64) * M,
                  **{f: np.tile(getattr(base, f), reps) for f in ("os_class", "flags") + F64_FIELDS + BYTE_FIELDS})
    big = replace(big, dev_off=big.dev_off[:nf + 1],
                  **{f: getattr(big, f)[:nf * M] for f in ("os_class", "flags") + F64_FIELDS + BYTE_FIELDS})
    return big.perturbed(np.random.default_rng(seed))


def _check(dt, want, per_k):
    assert np.array_equal(dt.out["best_k"].cpu().numpy(), want.best_k)
    assert np.array_equal(dt.out["obj_value"].cpu().numpy(), want.obj_value)
    assert np.array_equal(dt.out["w"].cpu().numpy(), want.w) and np.array_equal(dt.out["n"].cpu().numpy(), want.n)
    if per_k:
        assert np.array_equal(dt.out["status"].cpu().numpy(), want.status.ravel())
        assert np.array_equal(dt.out["obj_by_k"].cpu().numpy(), want.obj_by_k.ravel())


@pytest.mark.parametrize("nf,n_tab,first,steps,per_k", [(300, 3, 2, 7, True), (4096 + 77, 4, 5, 13, False),
                                                         (64, 5, 0, 20, False), (1, 2, 1, 3, True)])
def test_group_launch_equals_per_table_solves(llama_online_model, nf, n_tab, first, steps, per_k):
    """C3-shaped tables (M = 64, every k of L = 80): the group runs as ONE launch (one wave per (batch,
    fleet) item); every batch (table (first + t) % n_tab) leaves the bits of its own synchronous solve --
    a fleet count that is not a multiple of the four-wave workgroups, 4,173 fleets, a batch count that is
    not a multiple of the tables and one fleet alone. The outputs are zeroed first, so every table must be
    written by the launch."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    tabs, wants = [], []
    for t in range(n_tab):
        table = _tiled(llama_online_model, 64, min(nf, 24), nf, 31000 + 97 * t)
        wants.append(solve_table(table, llama_online_model, KS, 0.5))
        tabs.append(DeviceFleetTable(table, llama_online_model, KS, 0.5, dev, want_per_k=per_k))
    group = PlanGroup(tabs, ctx)
    assert group.persistent
    for t in tabs:
        for v in t.out.values():
            v.zero_()
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    with pytest.raises(RuntimeError):  # one launch carries at most 65,535 batches (the grid's y extent)
        group.launch(first, 65536, stream.cuda_stream)
    group.launch(first, steps, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    for t in range(n_tab):
        if any((first + s) % n_tab == t for s in range(steps)):
            _check(tabs[t], wants[t], per_k)
        else:
            assert not tabs[t].out["best_k"].any()
    group.close()


def test_group_batches_see_in_place_rewrites(llama_online_model):
    """A streaming caller rewrites a resident table between group launches (re-profiled fleets, C5): the
    next launch solves the new contents; plans freed after the group was made do not matter to it."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    table = _tiled(llama_online_model, 64, 16, 500, 32000)
    dts = [DeviceFleetTable(table, llama_online_model, KS, 0.5, dev) for _ in range(2)]
    group = PlanGroup(dts, ctx)
    for d in dts:
        d.replan()  # the group keeps its own copy of the plans
    stream = torch.cuda.Stream(dev)
    group.launch(0, 2, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    want = solve_table(table, llama_online_model, KS, 0.5)
    for d in dts:
        _check(d, want, False)
    moved = table.perturbed(np.random.default_rng(9))
    for f in F64_FIELDS + BYTE_FIELDS:
        dts[1].arrs[f].copy_(torch.from_numpy(np.ascontiguousarray(getattr(moved, f))))
    group.launch(1, 1, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    _check(dts[1], solve_table(moved, llama_online_model, KS, 0.5), False)
    group.close()


@pytest.mark.parametrize("M,persistent", [(16, True), (70, False), (12, True)])
def test_group_other_shapes(llama_online_model, M, persistent):
    """C2's k > 1 tables (16 devices) run as the k-slot form of the steps launch
    (halda_sweep_kslot_steps_kernel); fleets wider than 64 devices batch by batch; M = 12 at L = 12 opens
    only k = 1 and W = M, so it is a register sweep. Either way every batch's results equal its own solve."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup

    model = llama_online_model if M != 12 else llama_online_model.model_copy(update={"L": 12})
    ks = KS if M != 12 else [1, 2, 3, 4, 6]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    tabs, wants = [], []
    for t in range(2):
        table = _tiled(model, M, 8, 90, 33000 + 11 * t)
        wants.append(solve_table(table, model, ks, 0.5))
        tabs.append(DeviceFleetTable(table, model, ks, 0.5, dev, want_per_k=True))
    group = PlanGroup(tabs, ctx)
    assert group.persistent == persistent
    stream = torch.cuda.Stream(dev)
    group.launch(0, 3, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    for d, w in zip(tabs, wants):
        _check(d, w, True)
    group.close()


def test_plans_and_groups_fail_cleanly_after_the_context_is_freed(llama_online_model):
    """halda_free detaches the context's plans and groups: launching through them afterwards is a
    HALDA_E_ARG (RuntimeError here), not a use of freed memory; freeing them afterwards is harmless."""
    import ctypes

    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup, PlanRotation, _bind

    dev = torch.device("cuda", 0)
    ctx = HaldaContext(0)
    table = _tiled(llama_online_model, 64, 4, 40, 34000)
    dt = DeviceFleetTable(table, llama_online_model, KS, 0.5, dev)
    stream = torch.cuda.Stream(dev)
    dt.launch(ctx, stream.cuda_stream)
    group = PlanGroup([dt], ctx)
    rot = PlanRotation([dt], ctx, [stream.cuda_stream])
    torch.cuda.synchronize(dev)
    _, h, fn = dt._plans[id(ctx)]
    ctx.close()
    lib = _bind(ctx.lib)
    assert fn(h, ctypes.c_void_p(stream.cuda_stream)) != 0  # the raw C call on the stale plan
    with pytest.raises(RuntimeError):
        dt.launch(ctx, stream.cuda_stream)
    with pytest.raises(RuntimeError):
        group.launch(0, 1, stream.cuda_stream)
    with pytest.raises(RuntimeError):
        rot.launch(0, 1)
    rc = lib.halda_fleets_group_launch(group.group, 0, 1, ctypes.c_void_p(stream.cuda_stream))
    assert rc != 0
    group.close()
    dt.replan()


@pytest.mark.parametrize("first,steps", [(0, 7), (2, 20)])
def test_kslot_group_launch_with_hand_backs(llama_online_model, first, steps):
    """The k-slot form of the group launch on fleets of 1..16 devices (one-device fleets and k = 1
    fast-path fallbacks are flagged by the k-slot items and redone per batch by the gated
    halda_sweep_tables_steps_kernel): three tables (the same layout, perturbed values), more batches than
    tables; every table's statuses, per-k objectives, best k, obj_value, w, n equal its own solve."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    sizes = [1 + (s * 7) % 16 for s in range(300)]
    base = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(35000 + s, M)]
                        for s, M in enumerate(sizes)], llama_online_model)
    tabs, wants = [], []
    for t in range(3):
        table = base.perturbed(np.random.default_rng(70 + t)) if t else base
        wants.append(solve_table(table, llama_online_model, KS, 0.5))
        tabs.append(DeviceFleetTable(table, llama_online_model, KS, 0.5, dev, want_per_k=True))
    group = PlanGroup(tabs, ctx)
    assert group.persistent
    for t in tabs:
        for v in t.out.values():
            v.zero_()
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    try:
        group.launch(first, steps, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ms = ctx.last_fleet_ms()
    finally:
        ctx.set_timing(False)
    assert "halda_sweep_kslot_kernel" in ms and "halda_sweep_tables_kernel" in ms, ms
    for d, w in zip(tabs, wants):
        _check(d, w, True)
    group.close()


def test_rotation_over_kslot_tables_of_different_lds(llama_online_model):
    """Prepared k-slot launches whose dynamic LDS differs (C2's 16-device fleets at L = 80, about 40 KiB,
    and at L = 160, above 64 KiB for the k = 2 slot's tables) in one rotation: the kernel's LDS attribute
    only ever grows (Ctx::ensure_lds), so the larger plan's launches are not refused or mis-sized after
    the smaller one ran, and every table's results equal its own solve."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanRotation

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    models = [llama_online_model, llama_online_model.model_copy(update={"L": 160})]
    tabs, wants = [], []
    for i, model in enumerate(models):
        ks = [d for d in range(1, model.L) if model.L % d == 0 and d <= 40]
        table = _tiled(model, 16, 8, 200, 36000 + 7 * i)
        wants.append(solve_table(table, model, ks, 0.5))
        tabs.append(DeviceFleetTable(table, model, ks, 0.5, dev, want_per_k=True))
    stream = torch.cuda.Stream(dev)
    rot = PlanRotation(tabs, ctx, [stream.cuda_stream])
    for t in tabs:
        for v in t.out.values():
            v.zero_()
    torch.cuda.synchronize(dev)
    rot.launch(0, 5)
    torch.cuda.synchronize(dev)
    for d, w in zip(tabs, wants):
        _check(d, w, True)
