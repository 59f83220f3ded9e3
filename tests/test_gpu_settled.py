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
