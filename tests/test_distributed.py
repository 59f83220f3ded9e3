"""Multi-process orchestration on CPU (gloo, world_size 2): fleet sharding and the
k-sharded all-reduce(min) pick. The per-rank engine is swapped for the CPU oracle
(test-only injection), so this runs without a GPU; tie-breaking and sharding are
what is under test."""

import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from .conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_solve(fleets, model, ks, kv_bits, mip_gap):
    from distilp_amd.solver.coefficients import ILPResult
    from oracle import milp_oracle as mo

    out = []
    for devs in fleets:
        _, per_k = mo.halda_solve_oracle(devs, model, k_candidates=list(ks), mip_gap=mip_gap, kv_bits=kv_bits,
                                         solver="exact")
        out.append([(r["k"], ILPResult(k=r["k"], w=r["w"], n=r["n"], obj_value=r["obj_value"]) if r["success"]
                     else None) for r in per_k])
    return out


def _worker(rank, world, port, outdir):
    import sys

    sys.path.insert(0, str(REPO))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from distilp_amd.distributed import halda_solve_batch_distributed, halda_solve_distributed
    from tests.helpers import fixture_fleet, synth_devices

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        devs, model = fixture_fleet("llama_3_70b/online")
        r = halda_solve_distributed(devs, model, mip_gap=1e-4, kv_bits="4bit", _solve=_oracle_solve)
        from distilp_amd.common import ModelProfileSplit
        from distilp_amd.synth import load_model_dict

        m2 = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
        fleets = [synth_devices(4, s) for s in range(5)]
        out = halda_solve_batch_distributed(fleets, m2, mip_gap=1e-4, kv_bits="4bit", _solve=_oracle_solve)
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump({"single": r.model_dump(), "batch": [o.model_dump() for o in out]}, f)
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_everything():
    from distilp_amd.distributed import shard_bounds

    for n in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            parts = [shard_bounds(n, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def test_two_rank_gloo_matches_single_process(tmp_path, fixtures_golden, synth_golden):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0 = json.loads((tmp_path / "r0.json").read_text())
    r1 = json.loads((tmp_path / "r1.json").read_text())
    assert r0 == r1  # every rank returns the same answer
    ref = fixtures_golden["fixtures"]["llama_3_70b/online|4bit|0.0001"]["result"]
    got = r0["single"]
    assert (got["k"], got["w"], got["n"], got["sets"]) == (ref["k"], ref["w"], ref["n"], ref["sets"])
    for got, fleet in zip(r0["batch"], synth_golden[4]["fleets"][:5]):
        ref = fleet["result"]
        assert (got["k"], got["w"], got["n"]) == (ref["k"], ref["w"], ref["n"])
