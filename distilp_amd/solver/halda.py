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

What changed: the fleet goes to libhalda as a device-field table; every
k-candidate is lowered on the GPU (bit-identical CSR to lower.lower_fleet, the
host restatement pinned to the reference's arrays) and solved exactly (gap 0)
in ONE halda_solve_fleets call, instead of one scipy/HiGHS call per k. The
objective of each k is then formed here with NumPy from the returned c and x,
exactly as the reference forms it. `halda_solve_batch` runs many fleets through ONE such call and
forms every objective on the host the same way (vectorised offsets, one NumPy dot per feasible
(fleet, k)).
"""

from __future__ import annotations

import numbers
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from ..common import DeviceProfile, ModelProfile
from ._libhalda import STATUS_INFEASIBLE, STATUS_OPTIMAL
from .coefficients import HALDAResult, ILPResult, assign_sets, kappa_constant, valid_factors_of_L
from .fleets import _PACKER, fleet_constants, fleet_table, pack_one, solve_table, sweep_one
from .lower import kv_bits_to_factor


def _as_k(k):
    """A k-candidate as ILPResult(k=...) would store it (pydantic's int coercion,
    dense_common.py:233-237): integers of any integral type (numpy's too) become int; anything
    else is left for the reference's own arithmetic (W = L // k) to reject."""
    return int(k) if isinstance(k, numbers.Integral) else k


def _k_list(model: ModelProfile, k_candidates: Optional[Iterable[int]]) -> List[int]:
    return sorted({_as_k(k) for k in k_candidates}) if k_candidates else valid_factors_of_L(model.L)


def _offset_parts(devs, model: ModelProfile, sets) -> Tuple[float, float, float]:
    """(sum t_comm, sum xi, kappa) in the reference's order (halda_p_solver.py:356-357,
    dense_common.py:100-119, 211-230): the constant part of obj_value."""
    kappa = kappa_constant(devs, model, sets)  # IndexError on an empty fleet, like the reference
    t_comm = 0
    for d in devs:
        t_comm += d.t_comm
    xi_sum = 0
    for d in devs:
        xi_sum += (d.t_ram2vram + d.t_vram2ram) * (0.0 if d.is_unified_mem else 1.0)
    return t_comm, xi_sum, kappa


def _construct(cls, **fields):
    """cls.model_construct(**fields) for a model whose fields are all given, already typed: the field
    dict, its own fields-set, no extra / private state (what model_construct sets), without its
    per-call field walk."""
    o = _new(cls)
    _setattr(o, "__dict__", fields)
    _setattr(o, "__pydantic_fields_set__", set(fields))
    _setattr(o, "__pydantic_extra__", None)
    _setattr(o, "__pydantic_private__", None)
    return o


_new, _setattr = object.__new__, object.__setattr__


def _sweep_on_gpu(devs, model: ModelProfile, sets, Ks: List[int], kv_factor: float, device: int,
                  debug: bool, _cls_out: Optional[list] = None) -> List[Tuple[int, Optional[ILPResult]]]:
    """Every k of one fleet lowered, solved and returned by ONE halda_solve_fleets call (the CSR is
    built on the GPU, bit-identical to lower.lower_fleet); obj_value = c.x + offsets formed here with
    NumPy on the returned c and x, exactly as the reference forms it (halda_p_solver.py:347-357).

    Errors surface where the reference's k loop (halda_p_solver.py:391-412) raises them: k = 0 at
    W = L // k (:72), then the k-independent coefficient errors (b_1 missing, zero T_cpu / s_disk,
    empty fleet) at the first k, after that k's debug line. `sets` is not read (the reference's sets
    come from the same device classes the packer writes); _cls_out, when given, receives a copy of the
    packed device classes (halda_solve builds the result's sets from them)."""
    pos = [k for k in Ks if k > 0]  # k < 0: W < 0, HiGHS reports infeasible
    # the C packer's single-fleet workspace (no per-call allocation), else a FleetTable
    one = bool(pos) and _PACKER is not None and hasattr(_PACKER, "sets")
    try:
        ws = pack_one(devs, model, pos) if one else fleet_table([devs], model)  # the reference's errors
        err = None
    except Exception as e:  # noqa: BLE001 -- re-raised at the first k, as the reference raises it
        err = e
    M, N = len(devs), 7 * len(devs) + 1
    swept = False
    status = X = C = None
    st_list: List[int] = []
    xrow: List[int] = []
    out: List[Tuple[int, Optional[ILPResult]]] = []
    j = -1  # k's index in pos (Ks ascending and distinct)
    for k in Ks:
        if debug:
            print("k: " + str(k))
        if k == 0:
            raise ZeroDivisionError("integer division or modulo by zero")
        if err is not None:
            raise err
        r: Optional[ILPResult] = None
        if k > 0:
            j += 1
            if not swept:
                swept = True
                if one:
                    sweep_one(ws, model, kv_factor, device)
                    status, X, C, xrow = ws.status, ws.x, ws.c, ws.xrow
                    t_comm, xi_sum, kappa = ws.consts.tolist()
                    cls_row = ws.u8[0]
                else:
                    res = solve_table(ws, model, pos, kv_factor, device, want_x=True)
                    status, X, C = res.status[0], res.x[0], res.c[0]
                    xrow = list(range(len(pos)))
                    # sum t_comm, sum xi, kappa in the reference's order (the packer's C loops)
                    t_comm, xi_sum, kappa = (float(v[0]) for v in fleet_constants(ws, model))
                    cls_row = ws.os_class
                if _cls_out is not None:
                    _cls_out.append(cls_row.tobytes())
                st_list = status.tolist()
            st = st_list[j]
            if st == STATUS_OPTIMAL:
                # views of the rows (the workspace is read before this thread's next call): c.dot(x) is
                # numpy's 1-D dot on the same contiguous rows, the reference's float(c @ x) bits
                q = xrow[j]  # an optimal k has L // k >= M (each device takes a layer): its row came back
                if q < 0:  # never another k's row (w >= 1 bounds today, halda_p_solver.py:117)
                    raise RuntimeError(f"libhalda returned k={k} optimal without its x / c row (L // k < M)")
                x = X[q, :N]
                obj = float(C[q, :N].dot(x)) + t_comm + xi_sum + kappa
                wn = np.rint(x[:2 * M]).astype(np.int64).tolist()  # int(round(v)): both round half to even
                r = _construct(ILPResult, k=k, w=wn[:M], n=wn[M:], obj_value=obj)  # fields already typed
            elif st != STATUS_INFEASIBLE:
                raise RuntimeError(f"libhalda rejected the k={k} MILP with status {st}: "
                                   "the lowered MILP does not have the HALDA structure")
        out.append((k, r))
        if debug:
            print(f"  k={k:<4d}  obj=infeasible" if r is None else f"  k={k:<4d}  obj={r.obj_value:.6f}")
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
    devs = list(devs)
    if debug:
        print("Objectives by k")
    cls: list = []
    per_k = _sweep_on_gpu(devs, model, None, Ks, kv_factor, device, debug, cls) if Ks else []
    best = _pick(per_k)
    if best is None:
        raise RuntimeError("No feasible MILP found for any k this round.")
    # the device sets (dense_common.py:149-167) from the classes the packer wrote
    sets = _PACKER.sets(cls[0]) if cls and _PACKER is not None and hasattr(_PACKER, "sets") else assign_sets(devs)
    result = _construct(HALDAResult, w=list(best.w), n=list(best.n), k=best.k, obj_value=best.obj_value, sets=sets)
    if plot:
        from .plotter import plot_k_curve

        plot_k_curve([(k, None if r is None else r.obj_value) for k, r in per_k], k_star=result.k,
                     title="HALDA: k vs objective (final sweep)")
    return result


def _batch_on_gpu(fleets: Sequence[List[DeviceProfile]], model: ModelProfile, Ks: List[int], kv_factor: float,
                  device: int, _multi=None) -> List[Optional[HALDAResult]]:
    """Many fleets' k-sweeps in ONE halda_solve_fleets call (the fused sweep from the packed
    device-field table), with every objective formed here exactly as the reference forms it
    (halda_p_solver.py:347-357): per feasible (fleet, k), c.x with NumPy on the returned c and x
    (only the instances with L // k >= M come back: open_x_offsets) -- np.vecdot over the rows of one
    length runs numpy's 1-D dot loop per row, the bits of `float(c.dot(x))` -- + sum t_comm + sum xi +
    kappa in the reference's own order (fleets.fleet_constants); best k by ascending k and strict "<"
    (:407, the first minimum); w, n = int(round(x)) of the winner. None where no k is feasible."""
    if any(k == 0 for k in Ks):
        raise ZeroDivisionError("integer division or modulo by zero")  # W = L // k (halda_p_solver.py:72)
    fleets = fleets if isinstance(fleets, list) else list(fleets)
    if not fleets:
        return []
    pos = [k for k in Ks if k > 0]  # k < 0: W < 0, HiGHS reports infeasible
    # the table and the results are this thread's reusable workspace: everything returned is built from
    # them below (Python ints / floats), nothing keeps a view
    table = fleet_table(fleets, model, _reuse=True)
    if not pos:
        return [None] * len(fleets)
    res = solve_table(table, model, pos, kv_factor, device, want_x="open", _multi=_multi, _reuse=True)
    st = res.status
    bad = (st != STATUS_OPTIMAL) & (st != STATUS_INFEASIBLE)
    if bad.any():
        f, j = map(int, np.argwhere(bad)[0])
        raise RuntimeError(f"libhalda rejected the (fleet {f}, k={pos[j]}) MILP with status {int(st[f, j])}: "
                           "the lowered MILP does not have the HALDA structure")
    t_sum, x_sum, kappa = fleet_constants(table, model)
    nf, nk = table.n_fleets, len(pos)
    sizes = table.sizes()
    opt = st == STATUS_OPTIMAL
    obj = np.full((nf, nk), np.inf)
    xo = res.x_off.reshape(nf, nk)
    ms = np.unique(sizes)
    for M in ms:  # one vectorised dot per row length N = 7 M + 1
        N = 7 * int(M) + 1
        fi, ji = np.nonzero(opt & (sizes == M)[:, None])
        if len(fi) == 0:
            continue
        if len(ms) == 1:
            # one fleet size: the open instances' rows lie back to back from 0 (open_x_offsets), so the
            # rows are a strided view of x / c, no gather
            n_open = int((xo >= 0).sum())
            X, C = res.x[:n_open * N].reshape(n_open, N), res.c[:n_open * N].reshape(n_open, N)
            cx = np.vecdot(C, X)[xo[fi, ji] // N]
        else:
            idx = xo[fi, ji][:, None] + np.arange(N)[None, :]
            cx = np.vecdot(res.c[idx], res.x[idx])
        obj[fi, ji] = ((cx + t_sum[fi]) + x_sum[fi]) + kappa[fi]
    feas = opt.any(axis=1)
    bj = np.argmin(obj, axis=1)  # the first minimum: ascending k, strict "<"
    best_obj = obj[np.arange(nf), bj]
    best_a = xo[np.arange(nf), bj]
    if _PACKER is not None and hasattr(_PACKER, "results"):
        # every HALDAResult built in C (w, n = rint of the winner's x; sets from the device classes)
        row = np.where(feas, best_a, -1).astype(np.int64)
        kk = np.asarray(pos, np.int64)[bj]
        return _PACKER.results(HALDAResult, res.x, row, kk, np.ascontiguousarray(best_obj), table.dev_off,
                               np.ascontiguousarray(table.os_class))
    out: List[Optional[HALDAResult]] = [None] * nf
    cls = table.os_class
    for M in ms:
        M = int(M)
        fs = np.flatnonzero(feas & (sizes == M))
        if len(fs) == 0:
            continue
        wn = np.rint(res.x[best_a[fs][:, None] + np.arange(2 * M)[None, :]]).astype(np.int64).tolist()
        cm = cls[table.dev_off[fs][:, None] + np.arange(M)[None, :]]
        sets = {s: [r.tolist() for r in np.split(np.nonzero(cm == s)[1], np.cumsum((cm == s).sum(axis=1))[:-1])]
                for s in (1, 2, 3)}
        ks_f, ob_f = [pos[j] for j in bj[fs].tolist()], best_obj[fs].tolist()
        for q, f in enumerate(fs.tolist()):
            row = wn[q]
            out[f] = HALDAResult.model_construct(w=row[:M], n=row[M:], k=ks_f[q], obj_value=ob_f[q],
                                                 sets={"M1": sets[1][q], "M2": sets[2][q], "M3": sets[3][q]})
    return out


def halda_solve_batch(
    fleets: Sequence[List[DeviceProfile]],
    model: ModelProfile,
    k_candidates: Optional[Iterable[int]] = None,
    mip_gap: Optional[float] = 1e-4,
    kv_bits: str = "8bit",
    device: int = 0,
) -> List[Optional[HALDAResult]]:
    """Throughput API: many fleets (same model) in ONE GPU k-sweep (halda_solve_fleets, the fused
    sweep), objectives formed on the host exactly as the reference forms them.

    Returns one HALDAResult per fleet, or None where no k is feasible (where
    `halda_solve` would raise). Prints nothing."""
    if k_candidates:
        Ks = sorted({_as_k(k) for k in k_candidates})
    else:
        L = model.L
        Ks = sorted({d for d in range(1, L) if L % d == 0}) if L > 1 else []
    kv_factor = kv_bits_to_factor(kv_bits)
    if not Ks:
        return [None] * len(fleets)
    return _batch_on_gpu(fleets, model, Ks, kv_factor, device)
