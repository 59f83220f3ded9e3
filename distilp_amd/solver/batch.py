"""Assemble lowered fleets into one libhalda batch (host arrays, halda.h layout).

Every fleet contributes ONE CSR segment (the constraint matrix is k-invariant,
SURVEY.md finding 3); each (fleet, k) instance points at its fleet's segment
through csr_off and owns only its c / bounds / row-bound vectors.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from ._libhalda import HostBatch
from .lower import FleetMILP


@dataclass
class InstanceRef:
    fleet: int
    k: int
    W: int
    col_off: int
    n_cols: int
    c: np.ndarray


def assemble(fleets: Sequence[FleetMILP], ks: Sequence[Sequence[int]], mip_gap: float = 1e-4
             ) -> Tuple[HostBatch, List[InstanceRef]]:
    """Concatenate (fleet, k) instances; k values are used as given (k=0 raises ZeroDivisionError)."""
    rp_parts, ci_parts, val_parts = [], [], []
    csr_starts = []
    rp_len = 0
    nnz = 0
    for fl in fleets:
        csr_starts.append(rp_len)
        rp_parts.append((fl.row_ptr.astype(np.int64) + nnz).astype(np.int32))
        ci_parts.append(fl.col_idx)
        val_parts.append(fl.val)
        rp_len += fl.n_rows + 1
        nnz += fl.nnz
    if nnz >= 2**31:
        raise ValueError("batch too large for int32 CSR offsets; split it")

    n_cols, n_rows, csr_off, col_off, row_off = [], [], [], [], []
    cs, lbs, ubs, rlbs, rubs, integs = [], [], [], [], [], []
    refs: List[InstanceRef] = []
    coff = roff = 0
    max_cols, max_R1, max_tab, max_tab_kc = 1, 1, 0, 0
    for f, (fl, klist) in enumerate(zip(fleets, ks)):
        integ = fl.integrality()
        for k in klist:
            c, lb, ub, row_lb, row_ub, _, W = fl.instance(k)
            n_cols.append(fl.n_cols)
            n_rows.append(fl.n_rows)
            csr_off.append(csr_starts[f])
            col_off.append(coff)
            row_off.append(roff)
            cs.append(c)
            lbs.append(lb)
            ubs.append(ub)
            rlbs.append(row_lb)
            rubs.append(row_ub)
            integs.append(integ)
            refs.append(InstanceRef(fleet=f, k=k, W=W, col_off=coff, n_cols=fl.n_cols, c=c))
            coff += fl.n_cols
            roff += fl.n_rows
            max_cols = max(max_cols, fl.n_cols)
            R = W - fl.M  # lb(w_i) = 1 for every device
            if R >= 0:
                R1 = R + 1
                max_R1 = max(max_R1, R1)
                if k > 1:
                    max_tab_kc = max(max_tab_kc, fl.M * R1)
                else:
                    max_tab = max(max_tab, fl.M * R1)

    def cat(parts, dtype):
        return np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros(0), dtype=dtype)

    batch = HostBatch(
        n_cols=np.asarray(n_cols, np.int32), n_rows=np.asarray(n_rows, np.int32),
        csr_off=np.asarray(csr_off, np.int64), col_off=np.asarray(col_off, np.int64),
        row_off=np.asarray(row_off, np.int64),
        row_ptr=cat(rp_parts, np.int32), col_idx=cat(ci_parts, np.int32), val=cat(val_parts, np.float64),
        c=cat(cs, np.float64), col_lb=cat(lbs, np.float64), col_ub=cat(ubs, np.float64),
        row_lb=cat(rlbs, np.float64), row_ub=cat(rubs, np.float64), integrality=cat(integs, np.uint8),
        max_cols=max_cols, max_R1=max_R1, max_tab=max_tab, max_tab_kc=max_tab_kc, mip_rel_gap=float(mip_gap or 0.0),
    )
    return batch, refs


def settled_instances(b: HostBatch) -> np.ndarray:
    """The bound-infeasible instances of a host batch, one byte each (1 = settled), for
    halda_solve_batch_device_settled: instance i is settled when it is a HALDA instance (N = 7M + 1
    columns, the last row an equality sum_j w_j = W with integral W in [0, 1e6), its entries the first M
    columns with coefficient 1) and its w lower bounds prove infeasibility -- a bound below 0, a ceil above
    W, or ceilings summing past W (NaN bounds count 0, as on the GPU). That is the screen's own verdict
    (HiGHS's presolve answer for M > W = L / k, res.success == False in halda_p_solver.py:369-436), so the
    settled call writes the same results while reading none of these instances' rows."""
    n = b.n_inst
    N = b.n_cols.astype(np.int64)
    m = b.n_rows.astype(np.int64)
    ok = (N >= 1) & ((N - 1) % 7 == 0) & (m >= 1)
    M = np.where(ok, (N - 1) // 7, 0)
    eq = np.where(ok, b.row_off + m - 1, 0)
    W = b.row_ub[eq]
    Wl = b.row_lb[eq]
    with np.errstate(invalid="ignore"):
        ok &= (Wl == W) & (W >= 0.0) & (W < 1e6) & (W == np.floor(W))
    rs = b.row_ptr[np.where(ok, b.csr_off + m - 1, 0)].astype(np.int64)
    re = b.row_ptr[np.where(ok, b.csr_off + m, 0)].astype(np.int64)
    ok &= (re - rs == M) & (M > 0)
    Mo = np.where(ok, M, 0)
    inst = np.repeat(np.arange(n), Mo)
    j = np.arange(int(Mo.sum())) - np.repeat(np.cumsum(Mo) - Mo, Mo)
    e = rs[inst] + j
    bad = (b.col_idx[e] != j) | (b.val[e] != 1.0)
    ok &= np.bincount(inst, weights=bad, minlength=n) == 0
    lb = b.col_lb[b.col_off[inst] + j]
    with np.errstate(invalid="ignore"):
        up = np.ceil(lb)
        nan = np.isnan(lb)
        hit = ~nan & ((lb < 0.0) | (up > W[inst]))
        up = np.where(nan, 0.0, up)
    infeas = (np.bincount(inst, weights=hit, minlength=n) > 0) | (np.bincount(inst, weights=up, minlength=n) > W)
    return (ok & infeas).astype(np.uint8)
