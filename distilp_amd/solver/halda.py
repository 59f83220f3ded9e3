"""halda_solve: the k-sweep behind the reference's public API, solved on MI355X.

Reference: `halda_solve` / `solve_fixed_k_milp` in
src/distilp/solver/halda_p_solver.py:59-436. The observable contract kept:

  * Ks = sorted(set(k_candidates)) if k_candidates else valid_factors_of_L(L)
    (the latter prints "L [factors]", dense_common.py:21);
  * kv_bits -> factor, ValueError on unknown strings (raised after that print);
  * every k is one fixed-k MILP; a k without a feasible MILP is skipped (the
    reference swallows its RuntimeError, :409-412); when no k is feasible
    RuntimeError("No feasible MILP found for any k this round.") (:413-414);
  * w, n = int(round(x)); obj_value = c.x + sum t_comm + sum xi + kappa (:350-357);
  * best k by strict "<" in ascending k (smallest k wins ties, :407);
  * debug prints and plot_k_curve(...) as in :389-435.

What changed: all k-candidates of the fleet are lowered once to a shared CSR
and solved in ONE libhalda batch on the GPU (exactly, gap 0), instead of one
scipy/HiGHS call per k.
"""

from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

from ..common import DeviceProfile, ModelProfile
from ._libhalda import STATUS_INFEASIBLE, STATUS_OPTIMAL, BatchResult, get_context
from .batch import assemble
from .coefficients import HALDAResult, ILPResult, assign_sets, valid_factors_of_L
from .lower import FleetMILP, kv_bits_to_factor, lower_fleet


def _k_list(model: ModelProfile, k_candidates: Optional[Iterable[int]]) -> List[int]:
    return sorted(set(k_candidates)) if k_candidates else valid_factors_of_L(model.L)


def _results_for(fleets: Sequence[FleetMILP], refs, res: BatchResult) -> List[List[Tuple[int, Optional[ILPResult]]]]:
    """Per fleet: [(k, ILPResult or None if infeasible)] in k order."""
    out: List[List[Tuple[int, Optional[ILPResult]]]] = [[] for _ in fleets]
    for idx, ref in enumerate(refs):
        fl = fleets[ref.fleet]
        st = int(res.status[idx])
        if st == STATUS_OPTIMAL:
            x = res.x[ref.col_off:ref.col_off + ref.n_cols]
            M = fl.M
            w = [int(round(v)) for v in x[:M]]
            n = [int(round(v)) for v in x[M:2 * M]]
            out[ref.fleet].append((ref.k, ILPResult(k=ref.k, w=w, n=n, obj_value=fl.objective_value(ref.c, x))))
        elif st == STATUS_INFEASIBLE:
            out[ref.fleet].append((ref.k, None))
        else:
            raise RuntimeError(f"libhalda rejected instance (fleet {ref.fleet}, k={ref.k}) with status {st}: "
                               "the lowered MILP does not have the HALDA structure")
    return out


def _pick(per_k: List[Tuple[int, Optional[ILPResult]]]) -> Optional[ILPResult]:
    best: Optional[ILPResult] = None
    for _, r in per_k:
        if r is not None and (best is None or r.obj_value < best.obj_value):
            best = r
    return best


def halda_solve(
    devs: List[DeviceProfile],
    model: ModelProfile,
    k_candidates: Optional[Iterable[int]] = None,
    mip_gap: Optional[float] = 1e-4,
    plot: bool = True,
    debug: bool = False,
    kv_bits: str = "8bit",
    device: int = 0,
) -> HALDAResult:
    """HALDA layer assignment: best k, w, n over the k-candidates (drop-in for the reference)."""
    Ks = _k_list(model, k_candidates)
    kv_factor = kv_bits_to_factor(kv_bits)
    sets = assign_sets(devs)
    fl = lower_fleet(devs, model, kv_factor=kv_factor, sets=sets)
    batch, refs = assemble([fl], [Ks], mip_gap)
    res = get_context(device).solve(batch)
    per_k = _results_for([fl], refs, res)[0]

    if debug:
        print("Objectives by k")
        for k, r in per_k:
            print("k: " + str(k))
            if r is None:
                print(f"  k={k:<4d}  obj=infeasible")
            else:
                print(f"  k={k:<4d}  obj={r.obj_value:.6f}")
    best = _pick(per_k)
    if best is None:
        raise RuntimeError("No feasible MILP found for any k this round.")
    result = HALDAResult(w=list(best.w), n=list(best.n), k=best.k, obj_value=best.obj_value,
                         sets={k: list(v) for k, v in sets.items()})
    if plot:
        from .plotter import plot_k_curve

        plot_k_curve([(k, None if r is None else r.obj_value) for k, r in per_k], k_star=result.k,
                     title="HALDA: k vs objective (final sweep)")
    return result


def halda_solve_batch(
    fleets: Sequence[List[DeviceProfile]],
    model: ModelProfile,
    k_candidates: Optional[Iterable[int]] = None,
    mip_gap: Optional[float] = 1e-4,
    kv_bits: str = "8bit",
    device: int = 0,
) -> List[Optional[HALDAResult]]:
    """Throughput API: many fleets (same model) in one GPU batch.

    Returns one HALDAResult per fleet, or None where no k is feasible (where
    `halda_solve` would raise). Prints nothing."""
    if k_candidates:
        Ks = sorted(set(k_candidates))
    else:
        L = model.L
        Ks = sorted({d for d in range(1, L) if L % d == 0}) if L > 1 else []
    kv_factor = kv_bits_to_factor(kv_bits)
    lowered, sets_all = [], []
    for devs in fleets:
        sets = assign_sets(devs)
        sets_all.append(sets)
        lowered.append(lower_fleet(devs, model, kv_factor=kv_factor, sets=sets))
    batch, refs = assemble(lowered, [Ks] * len(lowered), mip_gap)
    res = get_context(device).solve(batch)
    out: List[Optional[HALDAResult]] = []
    for per_k, sets in zip(_results_for(lowered, refs, res), sets_all):
        best = _pick(per_k)
        out.append(None if best is None else HALDAResult(w=list(best.w), n=list(best.n), k=best.k,
                                                         obj_value=best.obj_value,
                                                         sets={k: list(v) for k, v in sets.items()}))
    return out
