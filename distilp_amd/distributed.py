"""Multi-GPU HALDA: one process per GPU, torch.distributed (RCCL over xGMI on MI355X).

Two modes:

* throughput (`halda_solve_batch_distributed`, configs C3/C5): fleets are
  independent, so each rank solves a contiguous shard of them on its own GPU as
  one halda_solve_fleets k-sweep (device-field table, no host lowering; the
  objectives formed on the host in the reference's own arithmetic) — no
  collective on the data path; results are gathered once at the end.
* latency (`halda_solve_distributed`, one fleet, config C2 at 8 GPUs): the
  k-candidates are dealt round-robin over the ranks, each rank solves its k's
  exactly, then ONE all-reduce(min) of the objective (8 B) and one of the
  winning k (ties -> smallest k, the reference's strict "<" over ascending k,
  halda_p_solver.py:407) pick the answer; its owner broadcasts (w, n).

The per-rank engine is libhalda on the rank's GPU (tests/test_gpu_distributed.py
runs both modes with it: two gloo ranks on one GPU). `_solve` is an injection
point for tests of the orchestration on CPU (gloo); it is never an engine
fallback.
"""

from __future__ import annotations

import math
from typing import Callable, Iterable, List, Optional, Sequence, Tuple

from .common import DeviceProfile, ModelProfile
from .solver.coefficients import HALDAResult, ILPResult, assign_sets, valid_factors_of_L

PerK = List[Tuple[int, Optional[ILPResult]]]


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of n items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _default_solve(device: int) -> Callable:
    """Per-k results of each fleet on this rank's GPU: one halda_solve_fleets k-sweep per fleet with
    obj_value formed on the host exactly as the reference forms it (solver.halda._sweep_on_gpu)."""
    from .solver.coefficients import assign_sets as _sets
    from .solver.halda import _sweep_on_gpu
    from .solver.lower import kv_bits_to_factor

    def solve(fleets: Sequence[List[DeviceProfile]], model: ModelProfile, ks: Sequence[int], kv_bits: str,
              mip_gap: float) -> List[PerK]:
        kv = kv_bits_to_factor(kv_bits)
        return [_sweep_on_gpu(list(devs), model, _sets(list(devs)), list(ks), kv, device, False) for devs in fleets]

    return solve


def _dist():
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized():
        raise RuntimeError("torch.distributed is not initialised (launch with torch.distributed.run)")
    return dist


def _coll_device(dist, group):
    import torch

    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def halda_solve_distributed(devs: List[DeviceProfile], model: ModelProfile,
                            k_candidates: Optional[Iterable[int]] = None, mip_gap: Optional[float] = 1e-4,
                            kv_bits: str = "8bit", group=None, device: Optional[int] = None,
                            _solve: Optional[Callable] = None) -> HALDAResult:
    """Latency mode: k-candidates sharded over ranks; every rank returns the same HALDAResult."""
    import torch

    dist = _dist()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if k_candidates:
        Ks = sorted(set(k_candidates))
    elif rank == 0:
        Ks = valid_factors_of_L(model.L)  # prints "L [factors]" once, like the reference
    else:
        L = model.L
        Ks = sorted({d for d in range(1, L) if L % d == 0})
    mine = Ks[rank::world]
    solve = _solve or _default_solve(torch.cuda.current_device() if device is None else device)
    per_k = solve([devs], model, mine, kv_bits, mip_gap)[0] if mine else []
    best: Optional[ILPResult] = None
    for _, r in per_k:
        if r is not None and (best is None or r.obj_value < best.obj_value or
                              (r.obj_value == best.obj_value and r.k < best.k)):
            best = r
    dev = _coll_device(dist, group)
    obj = torch.tensor([best.obj_value if best else math.inf], dtype=torch.float64, device=dev)
    dist.all_reduce(obj, op=dist.ReduceOp.MIN, group=group)
    if not math.isfinite(obj.item()):
        raise RuntimeError("No feasible MILP found for any k this round.")
    kk = torch.tensor([best.k if best and best.obj_value == obj.item() else 2**62], dtype=torch.int64, device=dev)
    dist.all_reduce(kk, op=dist.ReduceOp.MIN, group=group)
    owner = torch.tensor([rank if best and best.k == kk.item() else world], dtype=torch.int64, device=dev)
    dist.all_reduce(owner, op=dist.ReduceOp.MIN, group=group)
    payload = [None]
    if rank == owner.item():
        payload = [(best.k, best.w, best.n, best.obj_value)]
    dist.broadcast_object_list(payload, src=dist.get_global_rank(group, int(owner.item())) if group else
                               int(owner.item()), group=group)
    k, w, n, objv = payload[0]
    sets = assign_sets(devs)
    return HALDAResult(w=list(w), n=list(n), k=k, obj_value=objv, sets={s: list(v) for s, v in sets.items()})


def halda_solve_batch_distributed(fleets: Sequence[List[DeviceProfile]], model: ModelProfile,
                                  k_candidates: Optional[Iterable[int]] = None, mip_gap: Optional[float] = 1e-4,
                                  kv_bits: str = "8bit", group=None, device: Optional[int] = None,
                                  gather: bool = True, _solve: Optional[Callable] = None):
    """Throughput mode: rank r solves fleets[shard_bounds(len, r, world)] on its GPU.

    Returns the full result list on every rank when gather=True (one all_gather
    at the end), else only this rank's (lo, results)."""
    import torch

    dist = _dist()
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if k_candidates:
        Ks = sorted(set(k_candidates))
    else:
        L = model.L
        Ks = sorted({d for d in range(1, L) if L % d == 0})
    lo, hi = shard_bounds(len(fleets), rank, world)
    results: List[Optional[HALDAResult]] = []
    if _solve is None and hi > lo:
        # the rank's shard as ONE GPU k-sweep (the fused sweep from the device-field table), objectives
        # formed on the host exactly as the reference forms them (solver.halda._batch_on_gpu): the same
        # obj_value, to the bit, as halda_solve of each fleet
        from .solver.halda import _batch_on_gpu
        from .solver.lower import kv_bits_to_factor

        dev = torch.cuda.current_device() if device is None else device
        kv = kv_bits_to_factor(kv_bits)
        results = _batch_on_gpu(list(fleets[lo:hi]), model, Ks, kv, dev) if Ks else [None] * (hi - lo)
    elif hi > lo:
        local = _solve(list(fleets[lo:hi]), model, Ks, kv_bits, mip_gap)
        for devs, per_k in zip(fleets[lo:hi], local):
            best: Optional[ILPResult] = None
            for _, r in per_k:
                if r is not None and (best is None or r.obj_value < best.obj_value):
                    best = r
            sets = assign_sets(devs)
            results.append(None if best is None else HALDAResult(w=list(best.w), n=list(best.n), k=best.k,
                                                                 obj_value=best.obj_value,
                                                                 sets={s: list(v) for s, v in sets.items()}))
    if not gather:
        return lo, results
    everything = [None] * world
    dist.all_gather_object(everything, (lo, results), group=group)
    out: List[Optional[HALDAResult]] = [None] * len(fleets)
    for part_lo, part in everything:
        for j, r in enumerate(part):
            out[part_lo + j] = r
    return out
