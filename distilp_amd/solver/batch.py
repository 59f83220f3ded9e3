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
