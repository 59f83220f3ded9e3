"""Host lowering: (fleet, model, kv_bits) -> one k-invariant CSR MILP + per-k vectors.

This replaces the reference's dense-row construction in
`solve_fixed_k_milp` (`src/distilp/solver/halda_p_solver.py:59-338`) and the
scipy CSC conversion it triggers (`scipy/optimize/_milp.py:11-73`).

Column layout (halda_p_solver.py:81-106), N = 7M + 1:
    x = [ w(M) | n(M) | s1(M) | s2(M) | s3(M) | t(M) | z(M) | C ]

Row order is the reference's A_ub order followed by the single equality row
(scipy stacks ub rows before eq rows, _milp.py:60-71):
    1. n_i - w_i <= 0                       for every i       (:177-182)
    2. M1 RAM cap  b'w - b's1 <= rhs        i in M1           (:227-233)
    3. M2 Metal cap b'w - b's2 <= rhs       i in M2, metal    (:236-246)
    4. M3 RAM cap  b'w - b'n - b's3 <= rhs  i in M3           (:249-258)
    5. VRAM caps   b'n - b't <= rhs         cuda, then metal  (:261-277)
    6. cycle rows  busy + z - C <= -const ; busy + F - z - C <= -const (:281-297)
    7. sum_i w_i = W                                          (:185-189)
Zero coefficients are not stored (scipy builds its CSC from the dense rows).

Finding 3 of the survey: A does not depend on k. Only W (bounds, eq rhs) and
the objective coefficient of C (k - 1) change, so one CSR per fleet serves
every k-candidate; `FleetMILP.instance(k)` yields the per-k vectors.

All coefficient arithmetic is scalar Python float (same operation order as
the reference) so the arrays are bit-identical to the reference's; the CSR
assembly itself is vectorised NumPy.
"""

from __future__ import annotations

import operator
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import numpy as np

from ..common import DeviceProfile, ModelProfile
from .coefficients import (
    assign_sets,
    b_prime,
    gpu_flops_table,
    gpu_load_throughput,
    kappa_constant,
    objective_vectors,
    sum_f_over_s,
)

# variable blocks
VAR_W, VAR_N, VAR_S1, VAR_S2, VAR_S3, VAR_T, VAR_Z = range(7)


def kv_bits_to_factor(kv_bits: str) -> float:
    """'4bit' -> 0.5, '8bit' -> 1.0, 'fp16'/'bf16' -> 2.0 (halda_p_solver.py:39-56)."""
    key = kv_bits.strip().lower()
    table = {"4bit": 0.5, "8bit": 1.0, "fp16": 2.0, "bf16": 2.0}
    if key not in table:
        raise ValueError(f"Unsupported kv_bits '{kv_bits}'. Use one of: 4bit, 8bit, fp16, bf16")
    return table[key]


@dataclass
class FleetMILP:
    """The k-invariant part of one fleet's HALDA MILP."""

    M: int
    L: int
    n_cols: int
    n_rows: int  # ub rows + 1 eq row
    row_ptr: np.ndarray  # int32 [n_rows + 1]
    col_idx: np.ndarray  # int32 [nnz]
    val: np.ndarray  # float64 [nnz]
    b_ub: np.ndarray  # float64 [n_rows - 1]
    c_base: np.ndarray  # float64 [n_cols], c[C] = 0
    gpu: np.ndarray  # bool [M]  (n/t columns allowed)
    in_set: np.ndarray  # bool [3, M]  (s1/s2/s3 columns allowed)
    obj_offset_parts: tuple  # (sum t_comm, sum xi, kappa) added to c.x in reference order
    sets: Dict[str, List[int]] = field(default_factory=dict)

    @property
    def nnz(self) -> int:
        return int(self.val.shape[0])

    def _bound_templates(self):
        t = getattr(self, "_tpl", None)
        if t is None:
            M = self.M
            lb = np.zeros(self.n_cols)
            lb[:M] = 1.0
            scale = np.zeros(self.n_cols)  # ub = W * scale on the integer columns
            scale[:M] = 1.0
            scale[M:2 * M] = self.gpu
            for s in range(3):
                scale[(2 + s) * M:(3 + s) * M] = self.in_set[s]
            scale[5 * M:6 * M] = self.gpu
            integ = np.ones(self.n_cols, dtype=np.uint8)
            integ[6 * M:] = 0
            t = self._tpl = (lb, scale, integ)
        return t

    def col_bounds(self, W: int):
        lb, scale, _ = self._bound_templates()
        ub = scale * W
        ub[6 * self.M:] = np.inf
        return lb.copy(), ub

    def integrality(self) -> np.ndarray:
        return self._bound_templates()[2].copy()

    def instance(self, k: int):
        """(c, col_lb, col_ub, row_lb, row_ub, integrality, W) for one k."""
        W = self.L // k
        c = self.c_base.copy()
        c[7 * self.M] = float(k - 1)
        lb, ub = self.col_bounds(W)
        row_lb = np.full(self.n_rows, -np.inf)
        row_ub = np.empty(self.n_rows)
        row_ub[:-1] = self.b_ub
        row_lb[-1] = row_ub[-1] = float(W)
        return c, lb, ub, row_lb, row_ub, self.integrality(), W

    def objective_value(self, c: np.ndarray, x: np.ndarray) -> float:
        """obj_value exactly as the reference forms it (halda_p_solver.py:356-357)."""
        t_comm, xi_sum, kappa = self.obj_offset_parts
        return float(c.dot(x)) + t_comm + xi_sum + kappa

    def dense(self) -> np.ndarray:
        """Dense copy of A (tests only)."""
        A = np.zeros((self.n_rows, self.n_cols))
        for r in range(self.n_rows):
            s, e = self.row_ptr[r], self.row_ptr[r + 1]
            A[r, self.col_idx[s:e]] = self.val[s:e]
        return A


_FIELD_NAMES = ("Tc", "tkc", "tkg", "r2v", "v2r", "uma", "tcomm", "sdisk", "ram", "ccpu", "cgpu", "head", "has_cuda",
                "cuda", "has_metal", "metal")
_FIELDS = operator.attrgetter("T_cpu", "t_kvcpy_cpu", "t_kvcpy_gpu", "t_ram2vram", "t_vram2ram", "is_unified_mem",
                              "t_comm", "s_disk", "d_avail_ram", "c_cpu", "c_gpu", "is_head", "has_cuda",
                              "d_avail_cuda", "has_metal", "d_avail_metal")


def _device_arrays(devs: Sequence[DeviceProfile], model: ModelProfile, sets, kv_factor: float):
    """Per-device coefficients as NumPy arrays, element-wise in the reference's
    operation order (dense_common.py:100-126, halda_p_solver.py:195-224), so every
    value is bit-identical to the scalar restatement in coefficients.py.

    Returns None when a device would make the reference raise (T_cpu == 0): the
    caller then runs the scalar path, which raises the same exception."""
    bp = b_prime(model, kv_bits_k=kv_factor)
    Q = model.Q
    cpu, gpu, has_beta, tg, swap = [], [], [], [], []
    for d in devs:
        c = sum_f_over_s(model.f_q, d.scpu, Q)  # raises ValueError like the reference
        table, t_gpu = gpu_flops_table(d), gpu_load_throughput(d)
        hb = table is not None and t_gpu is not None
        cpu.append(c)
        gpu.append(sum_f_over_s(model.f_q, table, Q) if hb else 0.0)
        has_beta.append(hb)
        tg.append(float(t_gpu) if hb else 1.0)
        swap.append(min(d.d_bytes_can_swap, d.d_swap_avail) if d.os_type == "android" else 0)
    cols = list(zip(*map(_FIELDS, devs))) if devs else [[] for _ in _FIELD_NAMES]
    f = dict(zip(_FIELD_NAMES, cols))
    f["swap"] = swap
    f["cuda_ok"] = [bool(h and v is not None) for h, v in zip(f["has_cuda"], f["cuda"])]
    f["metal_ok"] = [bool(h and v is not None) for h, v in zip(f["has_metal"], f["metal"])]
    f["cuda"] = [0 if v is None else v for v in f["cuda"]]
    f["metal"] = [0 if v is None else v for v in f["metal"]]
    Tc = np.asarray(f["Tc"], dtype=np.float64)
    if not np.all(Tc != 0.0):
        return None
    M = len(devs)
    cpu = np.asarray(cpu, dtype=np.float64)
    gpu = np.asarray(gpu, dtype=np.float64)
    hb = np.asarray(has_beta, dtype=bool)
    tg = np.asarray(tg, dtype=np.float64)
    tkc = np.asarray(f["tkc"], dtype=np.float64)
    tkg = np.asarray(f["tkg"], dtype=np.float64)
    alpha = (cpu + tkc) + (bp / Tc)
    beta = np.where(hb, ((gpu - cpu) + (tkg - tkc)) + (bp / tg - bp / Tc), 0.0)
    m1 = np.zeros(M, dtype=bool)
    m1[sets["M1"]] = True
    m2 = np.zeros(M, dtype=bool)
    m2[sets["M2"]] = True
    b = np.where(m1, 0.0, beta)
    xi = (np.asarray(f["r2v"], dtype=np.float64) + np.asarray(f["v2r"], dtype=np.float64)) * np.where(
        np.asarray(f["uma"], dtype=bool), 0.0, 1.0)
    head = np.where(np.asarray(f["head"], dtype=bool), 1.0, 0.0)
    bcio = ((model.b_in / model.V) + model.b_out) * head + np.asarray(f["ccpu"], dtype=np.int64)
    sd = np.maximum(1.0, np.asarray(f["sdisk"], dtype=np.float64))
    pen_bp = bp / sd
    pen_b = model.b_layer / sd
    pen_v = np.where(m2, pen_b, pen_bp)
    const = xi + np.asarray(f["tcomm"], dtype=np.float64)
    S = np.stack([alpha, b, pen_bp, pen_b, pen_bp, pen_v, pen_bp, const], axis=1)
    ram = np.asarray(f["ram"], dtype=np.int64)
    cgpu = np.asarray(f["cgpu"], dtype=np.int64).astype(np.float64)
    metal = np.asarray(f["metal"], dtype=np.int64).astype(np.float64)
    rhs = {
        "M1": ram.astype(np.float64) - bcio,
        "M2": metal - bcio - cgpu,
        "M3": (ram + np.asarray(f["swap"], dtype=np.int64)).astype(np.float64) - bcio,
        "cuda": np.asarray(f["cuda"], dtype=np.int64).astype(np.float64) - cgpu,
        "metal": metal - cgpu - float(model.b_out) * head,
        "cuda_ok": np.asarray(f["cuda_ok"], dtype=bool),
        "metal_ok": np.asarray(f["metal_ok"], dtype=bool),
        "tcomm": f["tcomm"],
    }
    return bp, xi, S, rhs


def _device_scalars(devs: Sequence[DeviceProfile], model: ModelProfile, sets, kv_factor: float):
    """Scalar restatement (raises the reference's exceptions on degenerate inputs)."""
    bp = b_prime(model, kv_bits_k=kv_factor)
    a, b, xi = objective_vectors(list(devs), model, sets, kv_factor)
    m2 = set(sets["M2"])
    rows = []
    for i, d in enumerate(devs):
        sd = max(1.0, float(d.s_disk))
        pen_bp = bp / sd
        pen_b = model.b_layer / sd
        pen_v = pen_b if i in m2 else pen_bp
        rows.append((float(a[i]), float(b[i]), pen_bp, pen_b, pen_bp, pen_v, pen_bp,
                     float(xi[i]) + float(d.t_comm)))
    return bp, a, b, xi, np.array(rows, dtype=np.float64).reshape(len(devs), 8)


def lower_fleet(devs: Sequence[DeviceProfile], model: ModelProfile, kv_bits: str = "8bit",
                kv_factor: float | None = None, sets=None) -> FleetMILP:
    """Build the k-invariant CSR MILP for one fleet."""
    if kv_factor is None:
        kv_factor = kv_bits_to_factor(kv_bits)
    devs = list(devs)
    M = len(devs)
    if sets is None:
        sets = assign_sets(devs)
    kappa = kappa_constant(devs, model, sets)  # IndexError on an empty fleet, like the reference
    arrays = _device_arrays(devs, model, sets, kv_factor)
    if arrays is None:  # degenerate device: the scalar path raises like the reference
        _device_scalars(devs, model, sets, kv_factor)
        raise AssertionError("unreachable: degenerate device did not raise")
    bp, xi, S, R = arrays
    bpf = float(bp)
    N = 7 * M + 1
    iC = 7 * M
    idx = np.arange(M)

    # -- per-row templates: (cols, vals, rhs); rows of one block share a width
    blocks = []

    def add(cols, vals, rhs):
        blocks.append((np.asarray(cols, dtype=np.int64).reshape(len(rhs), -1),
                       np.asarray(vals, dtype=np.float64).reshape(len(rhs), -1),
                       np.asarray(rhs, dtype=np.float64)))

    add(np.stack([idx, M + idx], 1), np.tile([-1.0, 1.0], (M, 1)), np.zeros(M))
    m1 = np.asarray(sets["M1"], dtype=np.int64)
    if len(m1):
        add(np.stack([m1, 2 * M + m1], 1), np.tile([bpf, -bpf], (len(m1), 1)), R["M1"][m1])
    m2 = np.asarray([i for i in sets["M2"] if devs[i].d_avail_metal is not None], dtype=np.int64)
    if len(m2):
        add(np.stack([m2, 3 * M + m2], 1), np.tile([bpf, -bpf], (len(m2), 1)), R["M2"][m2])
    m3 = np.asarray(sets["M3"], dtype=np.int64)
    if len(m3):
        add(np.stack([m3, M + m3, 4 * M + m3], 1), np.tile([bpf, -bpf, -bpf], (len(m3), 1)), R["M3"][m3])
    # VRAM rows: per device the cuda row, then the metal row
    vr_dev = np.concatenate([idx[R["cuda_ok"]], idx[R["metal_ok"]]])
    vr_rhs = np.concatenate([R["cuda"][R["cuda_ok"]], R["metal"][R["metal_ok"]]])
    vr_key = np.concatenate([2 * idx[R["cuda_ok"]], 2 * idx[R["metal_ok"]] + 1])
    order = np.argsort(vr_key, kind="stable")
    if len(vr_dev):
        ii = vr_dev[order]
        add(np.stack([M + ii, 5 * M + ii], 1), np.tile([bpf, -bpf], (len(ii), 1)), vr_rhs[order])

    # cycle rows, interleaved (row1_i, row2_i); busy coefficients = objective coefficients
    busy = S[:, :6]  # a, b, p1, p2, p3, pV
    cyc_cols = np.concatenate([idx[:, None] + M * np.arange(7)[None, :], np.full((M, 1), iC)], 1)
    r1 = np.concatenate([busy, np.ones((M, 1)), -np.ones((M, 1))], 1)
    r2 = r1.copy()
    r2[:, 0] = busy[:, 0] + S[:, 6]  # rowB + rowF on the w column
    r2[:, 6] = -1.0
    cyc_vals = np.stack([r1, r2], 1).reshape(2 * M, 8)
    cyc_cols = np.repeat(cyc_cols, 2, axis=0)
    cyc_rhs = np.repeat(-S[:, 7], 2)
    add(cyc_cols, cyc_vals, cyc_rhs)

    # equality row
    add(idx[None, :], np.ones((1, M)), np.zeros(1))

    cols = [blk[0] for blk in blocks]
    vals = [blk[1] for blk in blocks]
    rhs = np.concatenate([blk[2] for blk in blocks])
    counts, flat_c, flat_v = [], [], []
    for cc, vv in zip(cols, vals):
        keep = vv != 0.0
        counts.append(keep.sum(1))
        flat_c.append(cc[keep])
        flat_v.append(vv[keep])
    counts = np.concatenate(counts)
    row_ptr = np.zeros(len(counts) + 1, dtype=np.int32)
    np.cumsum(counts, out=row_ptr[1:])

    c_base = np.zeros(N)
    c_base[:6 * M] = busy.T.reshape(-1)

    in_set = np.zeros((3, M), dtype=bool)
    for s, key in enumerate(("M1", "M2", "M3")):
        in_set[s, sets[key]] = True
    gpu = R["cuda_ok"] | R["metal_ok"]

    t_comm = 0
    for v in R["tcomm"]:
        t_comm += v
    xi_sum = 0
    for v in xi.tolist():
        xi_sum += v

    return FleetMILP(
        M=M, L=model.L, n_cols=N, n_rows=len(counts),
        row_ptr=row_ptr,
        col_idx=np.concatenate(flat_c).astype(np.int32),
        val=np.concatenate(flat_v),
        b_ub=rhs[:-1].copy(),
        c_base=c_base, gpu=gpu, in_set=in_set,
        obj_offset_parts=(t_comm, xi_sum, kappa), sets=sets,
    )
