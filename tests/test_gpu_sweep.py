"""The fused k-sweep (halda_sweep_kernel, the default halda_solve_fleets path) against the CSR
pipeline (GPU lowering -> screen / k = 1 / general kernels -> pick) on the same fleet tables.

The sweep builds each device's record from the fleet table with the coefficient code the lowering
kernel writes into the CSR, so the two paths must agree on every status, on (w, n) of every
optimal instance up to exact ties of the objective, on best k / w / n, and on obj_value within
1e-12 (the fused path sums c.x in another fixed order). Reference: halda_p_solver.py:59-436."""

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver._libhalda import STATUS_INFEASIBLE, STATUS_OPTIMAL, STATUS_UNSUPPORTED, get_context
from distilp_amd.solver.fleets import fleet_table, solve_table
from distilp_amd.synth import synth_fleet

pytestmark = pytest.mark.gpu


def _both(table, model, ks):
    ctx = get_context(0)
    fused = solve_table(table, model, ks, 0.5, want_x=True)
    ctx.set_fleets_path(False)
    try:
        csr = solve_table(table, model, ks, 0.5, want_x=True)
    finally:
        ctx.set_fleets_path(True)
    return fused, csr


def _compare(table, fused, csr, ks):
    assert np.array_equal(fused.status, csr.status)
    assert np.array_equal(fused.best_k, csr.best_k)
    for f in range(table.n_fleets):
        M = int(table.dev_off[f + 1] - table.dev_off[f])
        N = 7 * M + 1
        for j in range(len(ks)):
            if csr.status[f, j] != STATUS_OPTIMAL:
                assert np.isinf(fused.obj_by_k[f, j])
                continue
            a, b = fused.obj_by_k[f, j], csr.obj_by_k[f, j]
            assert abs(a - b) <= 1e-12 * max(1.0, abs(b)), (f, ks[j], a, b)
            assert np.array_equal(fused.c[f, j, :N], csr.c[f, j, :N])
            xa, xb = fused.x[f, j, :N], csr.x[f, j, :N]
            if not np.array_equal(xa[:2 * M], xb[:2 * M]):  # only an exact tie may pick another optimum
                ca = float(np.dot(csr.c[f, j, :N], xa))
                cb = float(np.dot(csr.c[f, j, :N], xb))
                assert abs(ca - cb) <= 1e-12 * max(1.0, abs(cb)), (f, ks[j])
    assert np.array_equal(fused.w, csr.w) and np.array_equal(fused.n, csr.n)
    ok = fused.best_k > 0
    assert np.allclose(fused.obj_value[ok], csr.obj_value[ok], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("L,M,n", [(80, 1, 24), (80, 2, 24), (80, 3, 16), (80, 5, 16), (80, 16, 16),
                                   (80, 64, 64), (256, 8, 6), (160, 100, 2), (64, 24, 8)])
def test_fused_sweep_equals_csr_pipeline(llama_online_model, L, M, n):
    model = llama_online_model.model_copy(update={"L": L})
    ks = [d for d in range(1, L) if L % d == 0][:12]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(7000 + s, M)] for s in range(n)]
    table = fleet_table(fleets, model)
    fused, csr = _both(table, model, ks)
    _compare(table, fused, csr, ks)


def test_fused_sweep_mixed_fleet_sizes(llama_online_model):
    """One table with fleets of 1..70 devices (tables for k > 1 and for the 70-device fleet)."""
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(8000 + s, M)]
              for s, M in enumerate([1, 70, 2, 33, 64, 5, 12, 3])]
    table = fleet_table(fleets, llama_online_model)
    fused, csr = _both(table, llama_online_model, ks)
    _compare(table, fused, csr, ks)


def test_fused_sweep_rejects_what_decode_rejects(llama_online_model):
    """A capacity row whose least slack is beyond 1e8 layers is not decoded by the CSR path
    (UNSUPPORTED); the fused sweep rejects the same instances, bound-infeasible k stay INFEASIBLE."""
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(3, 6)]
    devs[1] = devs[1].model_copy(update={"d_avail_ram": -(10 ** 18)})  # a linux (M3) device
    table = fleet_table([devs], llama_online_model)
    fused, csr = _both(table, llama_online_model, ks)
    assert np.array_equal(fused.status, csr.status)
    W = [80 // k for k in ks]
    assert [int(s) for s in fused.status[0]] == [STATUS_UNSUPPORTED if w >= 6 else STATUS_INFEASIBLE for w in W]


def test_multi_device_context_equals_single(llama_online_model):
    """halda_init_multi / halda_solve_fleets_multi: fleets dealt over several contexts (here three on
    GPU 0) give exactly the single-context answers, x and per-k results included."""
    from distilp_amd.solver.fleets import MultiDeviceContext

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(9000 + s, M)]
              for s, M in enumerate([3, 16, 64, 5, 70, 12, 2, 33, 8, 64, 1])]
    table = fleet_table(fleets, llama_online_model)
    one = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
    multi = MultiDeviceContext([0, 0, 0])
    try:
        many = multi.solve(table, llama_online_model, ks, 0.5, want_x=True)
    finally:
        multi.close()
    for f in ("best_k", "obj_value", "w", "n", "obj_by_k", "status"):
        assert np.array_equal(getattr(one, f), getattr(many, f)), f
    for fi, devs in enumerate(fleets):  # x / c are defined on each fleet's 7 M + 1 columns
        N = 7 * len(devs) + 1
        assert np.array_equal(one.x[fi, :, :N], many.x[fi, :, :N]) and np.array_equal(one.c[fi, :, :N], many.c[fi, :, :N])


@pytest.mark.parametrize("path,kernel,sizes", [
    ("fused", "halda_sweep_kslot_kernel", [1 + (s * 7) % 16 for s in range(300)]),
    ("fused", "halda_sweep_kslot_kernel", [16] * 200 + [12] * 57),
    # the k = 2 threshold scan unsplit (the default splits it in two)
    ("kslot_unsplit", "halda_sweep_kslot_kernel", [1 + (s * 7) % 16 for s in range(300)]),
    ("kslot_unsplit", "halda_sweep_kslot_kernel", [16] * 200 + [12] * 57),
    # the split scan in sequential order (part 1 makes its own leaf checks and phase 0; the default
    # leaves them to other waves of the workgroup for rows finite at both ends)
    ("kslot_sequential", "halda_sweep_kslot_kernel", [1 + (s * 7) % 16 for s in range(300)]),
    ("kslot_sequential", "halda_sweep_kslot_kernel", [16] * 200 + [12] * 57),
    ("seg", "halda_sweep_seg_kernel", [1 + (s * 7) % 16 for s in range(300)]),
])
def test_segment_sweep_equals_one_fleet_per_wave(llama_online_model, path, kernel, sizes):
    """The two kernels for fleets of <= 16 devices -- halda_sweep_kslot_kernel (four fleets per wave,
    one wave per open k, the best k picked in the workgroup; the default) and halda_sweep_seg_kernel
    (four fleets per wave, every k in turn) -- against the one-fleet-per-wave sweep on fleets of 1..16
    devices (and a C2-like batch of 16- and 12-device fleets): the same bits everywhere (statuses,
    obj_by_k, x, c, best k, obj_value, w, n). One-device fleets and k = 1 fast-path fallbacks are
    flagged and redone by the gated table launch; the CSR pipeline agrees too."""
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(11000 + s, M)] for s, M in enumerate(sizes)]
    table = fleet_table(fleets, llama_online_model)
    ctx = get_context(0)
    ctx.set_timing(True)
    try:
        ctx.set_fleets_path(path)
        seg = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
        solve_table(table, llama_online_model, ks, 0.5)
        assert kernel in ctx.last_fleet_ms()  # the segment / k-slot launch ran
        ctx.set_fleets_path("wave")
        wave = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
        solve_table(table, llama_online_model, ks, 0.5)
        assert kernel not in ctx.last_fleet_ms()
    finally:
        ctx.set_fleets_path("fused")
        ctx.set_timing(False)
    for f in ("status", "obj_by_k", "best_k", "obj_value", "w", "n"):
        assert np.array_equal(getattr(seg, f), getattr(wave, f)), f
    for fi, M in enumerate(sizes):
        N = 7 * M + 1
        assert np.array_equal(seg.x[fi, :, :N], wave.x[fi, :, :N]) and np.array_equal(seg.c[fi, :, :N], wave.c[fi, :, :N])
    ctx.set_fleets_path(path)
    try:  # the compact x / c layout (x_off) gives the same x / c of every open instance
        op = solve_table(table, llama_online_model, ks, 0.5, want_x="open")
    finally:
        ctx.set_fleets_path("fused")
    xo = op.x_off.reshape(len(sizes), len(ks))
    for fi, M in enumerate(sizes):
        N = 7 * M + 1
        for j in range(len(ks)):
            if xo[fi, j] >= 0:
                a = xo[fi, j]
                assert np.array_equal(op.x[a:a + N], wave.x[fi, j, :N]) and np.array_equal(op.c[a:a + N], wave.c[fi, j, :N])
            else:
                assert wave.status[fi, j] != 0
    ctx.set_fleets_path("csr")
    try:
        csr = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
    finally:
        ctx.set_fleets_path("fused")
    _compare(table, seg, csr, ks)


@pytest.mark.parametrize("sizes", [[64] * 160, [48, 64] * 80])
def test_k1_dp_fallback_path_equals_greedy(llama_online_model, sizes):
    """The register launch's own fallback for the k = 1 greedy (k1_dp, an exact min-plus DP over the
    devices; it is why that launch needs no table launch behind it), forced for every k = 1 instance
    by the "dp" path: the same statuses, best k and obj_value as the greedy exchange, and (w, n)
    equal up to exact ties of the objective (fleets repeat device templates: swapping identical
    devices ties). Uniform fleet sizes (dev_off from dev_off[0]) and mixed ones (dev_off[f])."""
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(9000 + s, M)] for s, M in enumerate(sizes)]
    table = fleet_table(fleets, llama_online_model)
    ctx = get_context(0)
    greedy = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
    ctx.set_fleets_path("dp")
    try:
        dp = solve_table(table, llama_online_model, ks, 0.5, want_x=True)
    finally:
        ctx.set_fleets_path(True)
    assert np.array_equal(dp.status, greedy.status)
    assert np.array_equal(dp.best_k, greedy.best_k)
    assert (greedy.best_k == 1).all()
    assert np.allclose(dp.obj_value, greedy.obj_value, rtol=1e-12, atol=1e-12)
    n_same = 0
    for f in range(table.n_fleets):
        M = int(table.dev_off[f + 1] - table.dev_off[f])
        N = 7 * M + 1
        assert np.array_equal(dp.c[f, 0, :N], greedy.c[f, 0, :N])
        xa, xb = dp.x[f, 0, :N], greedy.x[f, 0, :N]
        ca, cb = float(np.dot(xa, greedy.c[f, 0, :N])), float(np.dot(xb, greedy.c[f, 0, :N]))
        assert abs(ca - cb) <= 1e-12 * max(1.0, abs(cb)), f
        n_same += bool(np.array_equal(xa[:2 * M], xb[:2 * M]))
    assert n_same >= table.n_fleets // 4  # most fleets have a unique optimum


def test_register_launches_overlap_on_two_streams(llama_online_model):
    """The register launch of a C3-shaped batch touches no context scratch, so launches on two
    streams do not wait for each other (bench: one batch's loads overlap the previous batch's
    compute). Batches alternating over two streams, with a CSR-pipeline call (which does use the
    scratch) between them, give the results of one synchronous call each."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    tables = [fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(s, 64)]
                           for s in range(b * 160, b * 160 + 160)], llama_online_model) for b in range(2)]
    want = [solve_table(t, llama_online_model, ks, 0.5) for t in tables]
    dts = [DeviceFleetTable(t, llama_online_model, ks, 0.5, dev) for t in tables]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for i in range(8):
        dts[i % 2].launch(ctx, streams[i % 2].cuda_stream)
        if i == 4:
            ctx.set_fleets_path("csr")
            try:
                mid = solve_table(tables[1], llama_online_model, ks, 0.5)
            finally:
                ctx.set_fleets_path(True)
            assert np.array_equal(mid.best_k, want[1].best_k) and np.array_equal(mid.w, want[1].w)
    torch.cuda.synchronize(dev)
    for d, w in zip(dts, want):
        assert np.array_equal(d.out["best_k"].cpu().numpy(), w.best_k)
        assert np.array_equal(d.out["w"].cpu().numpy(), w.w) and np.array_equal(d.out["n"].cpu().numpy(), w.n)
        assert np.array_equal(d.out["obj_value"].cpu().numpy(), w.obj_value)


@pytest.mark.parametrize("n_streams", [3, 10])
def test_table_launches_on_many_streams(llama_online_model, n_streams):
    """Launches that use the fused sweep's scratch (per-fleet flags, hand-back flag: the k-slot launch
    of C2-shaped batches and its gated table launch) take a scratch slot per stream, so batches on
    different streams need no ordering between them; more streams than slots hand a slot over after
    the launches of the stream it leaves. Batches of 16- and 10-device fleets (every k of L = 80)
    alternating over the streams give the results of one synchronous call each, per-k outputs
    included."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    shapes = [16, 10, 16]
    tables = [fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(s, M)]
                           for s in range(b * 130, b * 130 + 130)], llama_online_model) for b, M in enumerate(shapes)]
    want = [solve_table(t, llama_online_model, ks, 0.5) for t in tables]
    dts = [DeviceFleetTable(t, llama_online_model, ks, 0.5, dev, want_per_k=True) for t in tables]
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    for i in range(3 * n_streams):
        dts[i % len(dts)].launch(ctx, streams[i % n_streams].cuda_stream)
    torch.cuda.synchronize(dev)
    for d, w in zip(dts, want):
        assert np.array_equal(d.out["best_k"].cpu().numpy(), w.best_k)
        assert np.array_equal(d.out["w"].cpu().numpy(), w.w) and np.array_equal(d.out["n"].cpu().numpy(), w.n)
        assert np.array_equal(d.out["obj_value"].cpu().numpy(), w.obj_value)
        assert np.array_equal(d.out["status"].cpu().numpy(), w.status.ravel())
        assert np.array_equal(d.out["obj_by_k"].cpu().numpy(), w.obj_by_k.ravel())


@pytest.mark.parametrize("M", [64, 12])
def test_uniform_fleets_viewed_from_an_offset_dev_off(llama_online_model, M):
    """A device-resident table viewed from fleet 7 on (dev_off pointing into the middle, so dev_off[0]
    != 0, the field arrays unchanged): with one fleet size the sweep issues the field loads from
    dev_off[0] = 0 and reloads when the read of dev_off[0] says otherwise. Results equal the whole
    table's for those fleets (w / n at the same absolute device indices)."""
    import ctypes

    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, HaldaFleetResultC, HaldaFleetsC, _bind

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(700 + s, M)] for s in range(40)],
                        llama_online_model)
    dt = DeviceFleetTable(table, llama_online_model, ks, 0.5, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    dt.launch(ctx, stream)
    torch.cuda.synchronize(dev)
    full = {k: v.cpu().numpy() for k, v in dt.out.items()}
    skip = 7
    fs = HaldaFleetsC.from_buffer_copy(dt.fs)
    fs.n_fleets = table.n_fleets - skip
    fs.dev_off = dt.arrs["dev_off"].data_ptr() + 8 * skip
    out = {"best_k": torch.zeros(fs.n_fleets, dtype=torch.int32, device=dev),
           "obj_value": torch.zeros(fs.n_fleets, dtype=torch.float64, device=dev),
           "w": torch.full((table.n_devices,), -1, dtype=torch.int32, device=dev),
           "n": torch.full((table.n_devices,), -1, dtype=torch.int32, device=dev)}
    res = HaldaFleetResultC(out["best_k"].data_ptr(), out["obj_value"].data_ptr(), out["w"].data_ptr(),
                            out["n"].data_ptr(), None, None, None, None)
    lib = _bind(ctx.lib)
    with ctx._lock:
        rc = lib.halda_solve_fleets(ctx.ctx, ctypes.byref(dt.model), ctypes.byref(fs), dt.ks.ctypes.data,
                                    len(dt.ks), ctypes.byref(res), ctypes.c_void_p(stream))
    assert rc == 0
    torch.cuda.synchronize(dev)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    assert np.array_equal(got["best_k"], full["best_k"][skip:])
    assert np.array_equal(got["obj_value"], full["obj_value"][skip:])
    d0 = skip * M
    assert np.array_equal(got["w"][d0:], full["w"][d0:]) and np.array_equal(got["n"][d0:], full["n"][d0:])
    assert (got["w"][:d0] == -1).all()  # devices of the fleets outside the view are untouched


@pytest.mark.parametrize("sizes", [[64] * 100, [16] * 100, [5, 16, 9] * 30, [3] * 10, [70, 40] * 3])
def test_prepared_plan_equals_solve_fleets(llama_online_model, sizes):
    """halda_fleets_plan_create / _launch (the bench's and a streaming caller's launch) against
    halda_solve_fleets on the same resident buffers: register, k-slot, table-alone and wide (gated table)
    launch sequences give the same bits; the plan reads the buffers' CURRENT contents, so a table
    rewritten in place between launches (a re-profiled fleet stream, config C5) is solved as rewritten."""
    import torch

    from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS, DeviceFleetTable

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(23000 + s, M)] for s, M in enumerate(sizes)]
    table = fleet_table(fleets, llama_online_model)
    want = solve_table(table, llama_online_model, ks, 0.5)
    dt = DeviceFleetTable(table, llama_online_model, ks, 0.5, dev, want_per_k=True)
    stream = torch.cuda.Stream(dev)
    for _ in range(2):
        dt.launch(ctx, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        assert np.array_equal(dt.out["best_k"].cpu().numpy(), want.best_k)
        assert np.array_equal(dt.out["obj_value"].cpu().numpy(), want.obj_value)
        assert np.array_equal(dt.out["w"].cpu().numpy(), want.w) and np.array_equal(dt.out["n"].cpu().numpy(), want.n)
        assert np.array_equal(dt.out["status"].cpu().numpy(), want.status.ravel())
        assert np.array_equal(dt.out["obj_by_k"].cpu().numpy(), want.obj_by_k.ravel())
    rng = np.random.default_rng(5)
    moved = table.perturbed(rng)
    for f in F64_FIELDS + BYTE_FIELDS:  # rewrite the resident table in place
        dt.arrs[f].copy_(torch.from_numpy(np.ascontiguousarray(getattr(moved, f))))
    want2 = solve_table(moved, llama_online_model, ks, 0.5)
    dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    assert np.array_equal(dt.out["best_k"].cpu().numpy(), want2.best_k)
    assert np.array_equal(dt.out["obj_value"].cpu().numpy(), want2.obj_value)
    assert np.array_equal(dt.out["w"].cpu().numpy(), want2.w)
    dt.replan()


def test_plan_launch_many_rotates_tables_and_streams(llama_online_model):
    """halda_fleets_plan_launch_many (the bench's timed k-sweep steps): step i runs table i % T on
    stream i % S; three differently seeded C2-shaped tables over two streams, 7 steps from an odd first
    index, give each table the results of its own synchronous halda_solve_fleets, bit for bit."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable, PlanRotation

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    tabs, wants = [], []
    for t in range(3):
        fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(26000 + 100 * t + s, 16)] for s in range(80)]
        table = fleet_table(fleets, llama_online_model)
        wants.append(solve_table(table, llama_online_model, ks, 0.5))
        tabs.append(DeviceFleetTable(table, llama_online_model, ks, 0.5, dev, want_per_k=True))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    rot = PlanRotation(tabs, ctx, [s.cuda_stream for s in streams])
    for t in tabs:
        for f in ("best_k", "obj_value", "w", "n", "status", "obj_by_k"):
            t.out[f].zero_()
    torch.cuda.synchronize(dev)
    rot.launch(5, 7)
    torch.cuda.synchronize(dev)
    for t, want in zip(tabs, wants):
        assert np.array_equal(t.out["best_k"].cpu().numpy(), want.best_k)
        assert np.array_equal(t.out["obj_value"].cpu().numpy(), want.obj_value)
        assert np.array_equal(t.out["w"].cpu().numpy(), want.w) and np.array_equal(t.out["n"].cpu().numpy(), want.n)
        assert np.array_equal(t.out["status"].cpu().numpy(), want.status.ravel())
        assert np.array_equal(t.out["obj_by_k"].cpu().numpy(), want.obj_by_k.ravel())
    with pytest.raises(RuntimeError):
        PlanRotation(tabs, ctx, []).launch(0, 1)


def test_prepared_plan_follows_the_context_path(llama_online_model):
    """A prepared plan re-plans when the context's path changes (halda_set_fleets_path): C2-shaped batch,
    planned on the k-slot path, then launched on the one-fleet-per-wave and CSR paths -- each runs its
    own kernels and gives the same statuses, best k and (w, n)."""
    import torch

    from distilp_amd.solver.fleets import DeviceFleetTable

    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(24000 + s, 16)] for s in range(100)]
    table = fleet_table(fleets, llama_online_model)
    dt = DeviceFleetTable(table, llama_online_model, ks, 0.5, dev, want_per_k=True)
    stream = torch.cuda.Stream(dev)
    outs = {}
    try:
        ctx.set_timing(True)
        for path, kernel in (("fused", "halda_sweep_kslot_kernel"), ("wave", "halda_sweep_tables_kernel"),
                             ("csr", "halda_solve_kernel"), ("fused", "halda_sweep_kslot_kernel")):
            ctx.set_fleets_path(path)
            dt.launch(ctx, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            ms = ctx.last_fleet_ms()
            assert kernel in ms and (path == "fused") == ("halda_sweep_kslot_kernel" in ms), (path, ms)
            outs[path] = {k: v.cpu().numpy().copy() for k, v in dt.out.items()}
    finally:
        ctx.set_fleets_path("fused")
        ctx.set_timing(False)
    for path in ("wave", "csr"):
        for f in ("status", "best_k", "w", "n"):
            assert np.array_equal(outs[path][f], outs["fused"][f]), (path, f)
        assert np.allclose(outs[path]["obj_value"], outs["fused"]["obj_value"], rtol=1e-12, atol=0.0)
