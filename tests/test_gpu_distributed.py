"""Multi-GPU engine on the GPU: two ranks (subprocesses, gloo collectives) sharing cuda:0 run
halda_solve_distributed (k-candidates dealt over ranks, all-reduce(min) of the objective, owner
broadcast of w / n) and halda_solve_batch_distributed (fleet shards, one halda_solve_fleets k-sweep
per rank, all_gather of the results) with the real libhalda engine -- no _solve injection. Both
ranks must return the reference's goldens (halda_p_solver.py:369-436 semantics)."""

import json
import os
import socket
import subprocess
import sys

import pytest

from .conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _close(a, b):
    return abs(a - b) <= 1e-9 * max(1.0, abs(b))


def test_two_ranks_on_one_gpu_match_goldens(tmp_path, fixtures_golden, synth_golden):
    port = str(_free_port())
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, str(REPO / "tests" / "dist_gpu_rank.py"), str(r), "2", port,
                               str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    logs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), logs
    outs = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(2)]
    assert outs[0] == outs[1]  # every rank returns the same answer
    got = outs[0]
    for fx in fixtures_golden["fixtures"].values():
        key = f"{fx['folder']}|{fx['kv_bits']}"
        if key not in got["single"] or fx["mip_gap"] != 1e-4:
            continue
        r, ref = got["single"][key], fx["result"]
        assert (r["k"], r["w"], r["n"], r["sets"]) == (ref["k"], ref["w"], ref["n"], ref["sets"]), key
        assert _close(r["obj_value"], ref["obj_value"])
    for M, res in got["batch"].items():
        G = synth_golden[int(M)]
        for r, f in zip(res, G["fleets"]):
            ref = f["result"]
            assert (r["k"], r["w"], r["n"], r["sets"]) == (ref["k"], ref["w"], ref["n"], ref["sets"]), (M, f["seed"])
            assert _close(r["obj_value"], ref["obj_value"])
        # throughput mode forms obj_value on the host like halda_solve does: the same bits
        assert res == got["single_of_batch"][M], M


def test_rccl_sharded_latency_mode_world_one():
    """The C ABI's latency mode over RCCL (halda_solve_fleets_sharded) on a one-rank communicator
    built by libhalda itself: the k-sharding bookkeeping, the three device-side all-reduces and the
    scatter / owner kernels between them leave exactly the single-GPU sweep's results (best k,
    obj_value, w, n, obj_by_k, status) on a C2-like and a ragged batch. (More ranks need more GPUs than
    this box has: RCCL does not put two ranks on one device.)"""
    import torch

    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, RcclComm, fleet_table, launch_sharded
    from distilp_amd.synth import load_model_dict, synth_fleet

    m2 = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    comm = RcclComm(1, 0, RcclComm.unique_id(), 0)
    try:
        for sizes in ([16] * 100, [1 + (s * 5) % 64 for s in range(80)]):
            fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(3100 + s, M)] for s, M in enumerate(sizes)]
            table = fleet_table(fleets, m2)
            a = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
            b = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
            a.launch(ctx, stream.cuda_stream)
            launch_sharded(b, ctx, comm, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            for f in ("best_k", "obj_value", "w", "n", "obj_by_k", "status"):
                assert torch.equal(a.out[f], b.out[f]), f
            assert (b.out["best_k"] > 0).all()
    finally:
        comm.close()


@pytest.mark.parametrize("world", [2, 3, 8, 10])
def test_sharded_latency_mode_emulated_ranks(world):
    """The C ABI's latency mode at world > 1 on one GPU (halda_solve_fleets_sharded_emulated): `world`
    virtual ranks each sweep ks[r], ks[r + world], ... into their own arrays, and each RCCL all-reduce of
    halda_solve_fleets_sharded is a device reduction over the ranks' arrays, in the same order -- so the
    k dealing, the owner / tie kernel modes 1 and 2 and (world 10 > 9 k) a rank with no k at all all run.
    Every virtual rank ends with exactly the single-GPU sweep's results (best k, obj_value, w, n,
    obj_by_k, status; halda_p_solver.py:407's tie rule) on a C2 batch and a ragged batch."""
    import torch

    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table, launch_sharded_emulated
    from distilp_amd.synth import load_model_dict, synth_fleet

    m2 = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    for sizes in ([16] * 100, [1 + (s * 5) % 64 for s in range(80)]):
        fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(3300 + s, M)] for s, M in enumerate(sizes)]
        table = fleet_table(fleets, m2)
        a = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
        a.launch(ctx, stream.cuda_stream)
        for rank in sorted({0, world - 1, world // 2}):
            b = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
            for t in b.out.values():
                t.fill_(-7)
            launch_sharded_emulated(b, ctx, world, rank, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            for f in ("best_k", "obj_value", "w", "n", "obj_by_k", "status"):
                assert torch.equal(a.out[f], b.out[f]), (world, rank, f)
        assert (a.out["best_k"] > 0).all()


def test_emulated_sharding_rejects_bad_k_lists_before_any_allocation():
    """halda_solve_fleets_sharded_emulated checks n_k (1..1024) and the k list (ascending, unique, > 0)
    before it sizes or reallocates its per-rank scratch: each bad call is HALDA_E_ARG (-22), not a HIP
    error from a wrapped size, and a good call afterwards still returns the single-GPU sweep's results."""
    import ctypes

    import numpy as np
    import torch

    from distilp_amd.common import DeviceProfile, ModelProfileSplit
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, _bind, fleet_table, launch_sharded_emulated
    from distilp_amd.synth import load_model_dict, synth_fleet

    m2 = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(3400 + s, 16)] for s in range(20)], m2)
    a = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
    a.launch(ctx, stream.cuda_stream)
    b = DeviceFleetTable(table, m2, ks, 0.5, dev, want_per_k=True)
    launch_sharded_emulated(b, ctx, 2, 0, stream.cuda_stream)  # the scratch exists before the bad calls
    lib = _bind(ctx.lib)
    bad = [(-1, ks), (0, ks), (2000, ks), (3, [2, 1, 4]), (2, [1, 1]), (2, [0, 1]), (2, [-2, 1])]
    for n_k, kl in bad:
        karr = np.zeros(max(len(kl), 1), np.int32)
        karr[:len(kl)] = kl
        with ctx._lock:
            rc = lib.halda_solve_fleets_sharded_emulated(ctx.ctx, 2, 0, ctypes.byref(b.model), ctypes.byref(b.fs),
                                                         karr.ctypes.data, n_k, ctypes.byref(b.res),
                                                         ctypes.c_void_p(stream.cuda_stream))
        assert rc == -22, (n_k, kl, rc)
    for t in b.out.values():
        t.fill_(-7)
    launch_sharded_emulated(b, ctx, 2, 1, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    for f in ("best_k", "obj_value", "w", "n", "obj_by_k", "status"):
        assert torch.equal(a.out[f], b.out[f]), f
