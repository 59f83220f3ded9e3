"""halda_solve_batch_device_settled: the milp() replacement told which instances the caller has already
proved bound-infeasible (batch.settled_instances) reads none of their rows and writes for them the
screen's own INFEASIBLE verdict; every other instance is solved as before. The results -- status, x,
obj_lin, dual_bound, gap, nodes -- equal the synchronous halda_solve_batch's bit for bit, on C3- and
C2-shaped batches, ragged tails, waves of settled instances alone, and instances that are infeasible
but not marked (a zero flag is always allowed). Reference: halda_p_solver.py:369-436 (one milp() per k)."""

import numpy as np
import pytest

from distilp_amd.solver._libhalda import get_context
from distilp_amd.solver.batch import assemble, settled_instances
from distilp_amd.solver.lower import lower_fleet
from distilp_amd.synth import synth_fleet

pytestmark = pytest.mark.gpu

FIELDS = ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr", "col_idx", "val", "c", "col_lb", "col_ub",
          "row_lb", "row_ub", "integrality")


def _device_solve(ctx, batch, settled, dev, stream):
    import torch

    keep = {f: torch.from_numpy(np.ascontiguousarray(getattr(batch, f))).to(dev) for f in FIELDS}
    n = batch.n_inst
    out = {"status": torch.full((n,), 7, dtype=torch.int32, device=dev),
           "x": torch.full((batch.total_cols,), -3.0, dtype=torch.float64, device=dev),
           "obj_lin": torch.full((n,), -5.0, dtype=torch.float64, device=dev),
           "dual_bound": torch.full((n,), -5.0, dtype=torch.float64, device=dev),
           "gap": torch.full((n,), -5.0, dtype=torch.float64, device=dev),
           "nodes": torch.full((n,), -9, dtype=torch.int64, device=dev)}
    hint = torch.from_numpy(settled).to(dev)
    torch.cuda.synchronize(dev)
    ctx.solve_device({f: t.data_ptr() for f, t in keep.items()}, batch, {f: t.data_ptr() for f, t in out.items()},
                     stream=stream.cuda_stream, settled=hint.data_ptr())
    torch.cuda.synchronize(dev)
    return {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("M,nf,ks,mask", [
    (64, 37, [1, 2, 4, 5, 8, 10, 16, 20, 40], "proved"),  # C3: 8 of 9 settled, 333 instances (ragged tail)
    (16, 40, [1, 2, 4, 5, 8, 10, 16, 20, 40], "proved"),  # C2: k > 1 instances solved beside settled ones
    (64, 9, [2, 4, 5, 8, 10, 16, 20, 40], "proved"),     # every instance settled: waves that read nothing
    (64, 11, [1, 2, 4, 5, 8, 10, 16, 20, 40], "half"),   # some infeasible instances left to the screen
    (12, 23, [1, 2, 4, 5, 8, 10, 16], "proved"),
])
def test_settled_batch_equals_synchronous_solve(llama_online_model, M, nf, ks, mask):
    import torch

    from distilp_amd.common import DeviceProfile

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(5000 + 13 * M + s, M)] for s in range(nf)]
    batch, refs = assemble([lower_fleet(devs, llama_online_model, "4bit") for devs in fleets], [ks] * nf)
    settled = settled_instances(batch)
    assert settled.any()
    if mask == "half":
        settled = settled.copy()
        settled[::2] = 0
    want = ctx.solve(batch)
    got = _device_solve(ctx, batch, settled, dev, torch.cuda.Stream(dev))
    assert np.array_equal(got["status"], want.status)
    assert np.array_equal(got["obj_lin"], want.obj_lin)
    assert np.array_equal(got["dual_bound"], want.dual_bound)
    assert np.array_equal(got["gap"], want.gap)
    assert np.array_equal(got["nodes"], want.nodes)
    opt = want.status == 0
    for i in np.flatnonzero(opt):  # x is written for OPTIMAL instances only
        a, b = int(batch.col_off[i]), int(batch.col_off[i] + batch.n_cols[i])
        assert np.array_equal(got["x"][a:b], want.x[a:b])
    if not opt.any():
        assert (got["x"] == -3.0).all()


@pytest.mark.parametrize("flags", ["none", "proved"])
def test_fused_screen_equals_screen_launch_on_hostile_batches(llama_online_model, flags):
    """A settled batch is screened inside its k = 1 kernel (halda_solve_k1_settled_kernel: no screen launch).
    Every instance the caller leaves unflagged gets the screen's own verdict there -- on fleets of 1 to 80
    devices (the k = 1 fast path's shapes, the small ones it hands back, a wide fleet for the general
    launch), k > 1 instances for the k > 1 launch, and corrupted instances: an equality-row coefficient 2,
    swapped equality-row columns, row_lb != row_ub and a fractional W on the equality row, a negative and
    a NaN w lower bound. Flags "none" screens every instance in the k = 1 kernel, "proved" the ones the
    caller's own proof leaves. Status, obj_lin, dual_bound, gap, nodes and x equal the screen launch's."""
    import torch

    from distilp_amd.common import DeviceProfile

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ks = [1, 2, 4, 5]
    sizes = [1, 2, 3, 5, 16, 64, 64, 64, 64, 64, 64, 16, 80]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(7100 + s, M)] for s, M in enumerate(sizes)]
    batch, refs = assemble([lower_fleet(devs, llama_online_model, "4bit") for devs in fleets], [ks] * len(fleets))
    for f in ("col_idx", "val", "col_lb", "row_lb", "row_ub"):
        setattr(batch, f, getattr(batch, f).copy())

    def inst(fleet, k):
        return next(j for j, r in enumerate(refs) if r.fleet == fleet and r.k == k)

    def eq_start(j):
        m = int(batch.n_rows[j])
        return int(batch.row_ptr[batch.csr_off[j] + m - 1])

    batch.val[eq_start(inst(6, 1)) + 1] = 2.0                      # a coefficient 2 (every k of fleet 6)
    e = eq_start(inst(7, 1))
    batch.col_idx[e], batch.col_idx[e + 1] = batch.col_idx[e + 1], batch.col_idx[e]  # swapped columns
    j = inst(8, 1)
    batch.row_lb[batch.row_off[j] + batch.n_rows[j] - 1] -= 1.0    # row_lb != row_ub
    j = inst(9, 1)
    batch.row_lb[batch.row_off[j] + batch.n_rows[j] - 1] = batch.row_ub[batch.row_off[j] + batch.n_rows[j] - 1] = 79.5
    batch.col_lb[batch.col_off[inst(10, 1)] + 3] = -1.0             # a negative w lower bound
    batch.col_lb[batch.col_off[inst(11, 2)] + 15] = np.nan          # a NaN w lower bound (counts 0)
    want = ctx.solve(batch)
    settled = np.zeros(batch.n_inst, np.uint8) if flags == "none" else settled_instances(batch)
    got = _device_solve(ctx, batch, settled, dev, torch.cuda.Stream(dev))
    assert np.array_equal(got["status"], want.status), (got["status"], want.status)
    for f in ("obj_lin", "dual_bound", "gap", "nodes"):
        assert np.array_equal(got[f], getattr(want, f)), f
    for i in np.flatnonzero(want.status == 0):
        a, b = int(batch.col_off[i]), int(batch.col_off[i] + batch.n_cols[i])
        assert np.array_equal(got["x"][a:b], want.x[a:b])
    # every verdict kind occurred
    assert {0, 2, -1} <= set(want.status.tolist())


@pytest.mark.parametrize("M,nf,G", [(64, 37, 7), (16, 40, 5)])
def test_replicated_settled_batch_equals_each_copy(llama_online_model, M, nf, G):
    """G batches handed over as ONE settled batch (helpers.replicate_batch: every array repeated, the offsets
    of copy g shifted past the copies before it), in which the settled k = 1 kernel's persistent waves take
    many open instances each (measured as a throughput form and not kept in the bench). Every copy's status, obj_lin,
    dual_bound, gap, nodes and x equal the synchronous solve of the one batch, bit for bit (C3 shape: k = 1
    fast path; C2 shape: k > 1 instances through the general launch behind it)."""
    import torch

    from distilp_amd.common import DeviceProfile

    from .helpers import replicate_batch

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(8100 + 7 * M + s, M)] for s in range(nf)]
    batch, _ = assemble([lower_fleet(devs, llama_online_model, "4bit") for devs in fleets], [ks] * nf)
    want = ctx.solve(batch)
    keep = {f: torch.from_numpy(np.ascontiguousarray(getattr(batch, f))).to(dev) for f in FIELDS}
    settled = torch.from_numpy(settled_instances(batch)).to(dev)
    big, out, hint, shape = replicate_batch(keep, batch, settled, G, torch)
    torch.cuda.synchronize(dev)
    ctx.solve_device({f: t.data_ptr() for f, t in big.items()}, shape, {f: t.data_ptr() for f, t in out.items()},
                     stream=torch.cuda.Stream(dev).cuda_stream, settled=hint.data_ptr())
    torch.cuda.synchronize(dev)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    n, nc = batch.n_inst, batch.total_cols
    for g in range(G):
        sl = slice(g * n, (g + 1) * n)
        assert np.array_equal(got["status"][sl], want.status), g
        for f in ("obj_lin", "dual_bound", "gap", "nodes"):
            assert np.array_equal(got[f][sl], getattr(want, f)), (g, f)
        xg = got["x"][g * nc:(g + 1) * nc]
        for i in np.flatnonzero(want.status == 0):
            a, b = int(batch.col_off[i]), int(batch.col_off[i] + batch.n_cols[i])
            assert np.array_equal(xg[a:b], want.x[a:b]), (g, i)
