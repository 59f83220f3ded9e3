"""CPU oracle for the HALDA k-sweep — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (distilp_amd) never does.

What it restates (reference = firstbatchxyz/distilp 0.1.6):
  * the fixed-k MILP lowering of `solve_fixed_k_milp`
    (src/distilp/solver/halda_p_solver.py:59-338), written here as explicit
    dense rows built from a per-device record, independent of the product's
    vectorised CSR lowering (distilp_amd/solver/lower.py);
  * the MILP solve itself, which in the reference lives in the third-party
    dependency scipy.optimize.milp -> HiGHS (halda_p_solver.py:340-346). The
    oracle calls the same library: scipy 1.15.3 bundling HiGHS 1.8.0
    (git 222cce7), options {time_limit: 3600, mip_rel_gap: mip_gap};
  * result extraction and the k-sweep argmin (halda_p_solver.py:347-436).
  * `exact_solve` wraps oracle/halda_exact.c, an independent exact solver of
    the same dense MILP (brute-force pair enumeration + 2-best DP) that also
    returns the uniqueness margin.

Pinned against tests/golden/*.json and tests/golden/lowered.npz, which were
produced by running the reference itself in the build container
(tests/golden/gen_golden.py).
"""

from __future__ import annotations

import ctypes
import math
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np

HERE = Path(__file__).resolve().parent
EXACT_LIB = HERE / "build" / "libhalda_exact.so"

# The coefficient helpers (alpha/beta/xi, b', kappa, sets) are pure scalar
# restatements of dense_common.py; the oracle re-derives them independently.


def _kv_factor(kv_bits: str) -> float:  # halda_p_solver.py:39-56
    s = kv_bits.strip().lower()
    if s == "4bit":
        return 0.5
    if s == "8bit":
        return 1.0
    if s in ("fp16", "bf16"):
        return 2.0
    raise ValueError(f"Unsupported kv_bits '{kv_bits}'. Use one of: 4bit, 8bit, fp16, bf16")


def _bprime(model, kv: float) -> int:  # dense_common.py:25-46
    elems_k = model.hk * model.ek * model.n_kv
    elems_v = model.hv * model.ev * model.n_kv
    nominal = kv * elems_k + kv * elems_v
    return int((1.0 + 0.15) * float(model.b_layer) + (1.0 + 2.0 / 64.0) * nominal)


def _ratio(f: Dict, S: Optional[Dict], q) -> float:  # dense_common.py:49-75
    if S is None or "b_1" not in f or q not in S:
        return 0.0
    if "b_1" not in S[q]:
        raise ValueError(f"Batch size 1 (key 'b_1') not found in S_by_q[{q}]")
    s = S[q]["b_1"]
    return 0.0 + f["b_1"] / s if s > 0 else 0.0


def _device_record(d, model, kv: float, in_m1: bool, in_m2: bool) -> Dict:
    """dense_common.py:100-126 (alpha, beta, xi, bcio) + the penalty terms of halda_p_solver.py:195-224."""
    bp = _bprime(model, kv)
    cpu = _ratio(model.f_q, d.scpu, model.Q)
    alpha = cpu + d.t_kvcpy_cpu + (bp / d.T_cpu)
    if d.has_metal and d.sgpu_metal:
        S_gpu = d.sgpu_metal
    elif d.has_cuda and d.sgpu_cuda:
        S_gpu = d.sgpu_cuda
    else:
        S_gpu = None
    if d.has_metal and d.T_metal:
        T_gpu = d.T_metal
    elif d.has_cuda and d.T_cuda:
        T_gpu = d.T_cuda
    else:
        T_gpu = None
    beta = 0.0
    if S_gpu is not None and T_gpu is not None:
        beta = (_ratio(model.f_q, S_gpu, model.Q) - cpu) + (d.t_kvcpy_gpu - d.t_kvcpy_cpu) + (bp / T_gpu - bp / d.T_cpu)
    xi = (d.t_ram2vram + d.t_vram2ram) * (0 if d.is_unified_mem else 1)
    sd = max(1.0, float(d.s_disk))
    head = 1.0 if d.is_head else 0.0
    return {
        "bp": bp, "a": alpha, "b": 0.0 if in_m1 else beta, "xi": xi,
        "bcio": ((model.b_in / model.V) + model.b_out) * head + d.c_cpu,
        "p1": bp / sd, "p2": model.b_layer / sd, "p3": bp / sd,
        "pV": (model.b_layer / sd) if in_m2 else (bp / sd), "F": bp / sd,
    }


def _kappa(devs, model, sets) -> float:  # dense_common.py:211-230
    hi = 0
    for i, d in enumerate(devs):
        if d.is_head:
            hi = i
            break
    h = devs[hi]
    parts = [
        _ratio(model.f_out, h.scpu, model.Q),
        (model.b_in / model.V + model.b_out) / h.T_cpu,
        model.b_in / (model.V * h.s_disk),
        model.b_out / h.s_disk,
    ]
    acc = parts[0]
    for p in parts[1:]:
        acc = acc + p
    tail = 0.0
    for i in sets["M1"] + sets["M3"]:
        d = devs[i]
        sw = min(d.d_bytes_can_swap, d.d_swap_avail) if d.os_type == "android" else 0
        tail += (d.c_cpu - d.d_avail_ram - sw) / d.s_disk
    return acc + tail


def sets_of(devs) -> Dict[str, List[int]]:  # dense_common.py:129-167
    out = {"M1": [], "M2": [], "M3": []}
    for i, d in enumerate(devs):
        out["M1" if d.os_type == "mac_no_metal" else "M2" if d.os_type == "mac_metal" else "M3"].append(i)
    return out


def lower_dense(devs, model, k: int, kv: float, sets=None):
    """Dense (c, integrality, lb, ub, A_ub, b_ub, A_eq, b_eq, const) for one (fleet, k)."""
    M = len(devs)
    sets = sets or sets_of(devs)
    kappa = _kappa(devs, model, sets)
    W = model.L // k
    N = 7 * M + 1
    col = {name: (lambda i, b=b: b * M + i) for b, name in enumerate(["w", "n", "s1", "s2", "s3", "t", "z"])}
    iC = 7 * M
    recs = [_device_record(d, model, kv, i in sets["M1"], i in sets["M2"]) for i, d in enumerate(devs)]
    bp = float(_bprime(model, kv))

    lb, ub = np.zeros(N), np.zeros(N)
    integ = np.ones(N, dtype=np.uint8)
    for i, d in enumerate(devs):
        gpu = bool(d.has_cuda and d.d_avail_cuda is not None) or bool(d.has_metal and d.d_avail_metal is not None)
        lb[col["w"](i)], ub[col["w"](i)] = 1, W
        ub[col["n"](i)] = W if gpu else 0
        ub[col["t"](i)] = W if gpu else 0
        for s, key in (("s1", "M1"), ("s2", "M2"), ("s3", "M3")):
            ub[col[s](i)] = W if i in sets[key] else 0
        ub[col["z"](i)] = np.inf
        integ[col["z"](i)] = 0
    ub[iC] = np.inf
    integ[iC] = 0

    rows, rhs = [], []

    def row(entries, r):
        v = np.zeros(N)
        for j, val in entries:
            v[j] += val
        rows.append(v)
        rhs.append(r)

    for i in range(M):
        row([(col["n"](i), 1.0), (col["w"](i), -1.0)], 0.0)
    for i in sets["M1"]:
        row([(col["w"](i), bp), (col["s1"](i), -bp)], float(devs[i].d_avail_ram) - float(recs[i]["bcio"]))
    for i in sets["M2"]:
        if devs[i].d_avail_metal is None:
            continue
        row([(col["w"](i), bp), (col["s2"](i), -bp)],
            float(devs[i].d_avail_metal) - float(recs[i]["bcio"]) - float(devs[i].c_gpu))
    for i in sets["M3"]:
        d = devs[i]
        sw = min(d.d_bytes_can_swap, d.d_swap_avail) if d.os_type == "android" else 0
        row([(col["w"](i), bp), (col["n"](i), -bp), (col["s3"](i), -bp)],
            float(d.d_avail_ram + sw) - float(recs[i]["bcio"]))
    for i, d in enumerate(devs):
        if d.has_cuda and d.d_avail_cuda is not None:
            row([(col["n"](i), bp), (col["t"](i), -bp)], float(d.d_avail_cuda) - float(d.c_gpu))
        if d.has_metal and d.d_avail_metal is not None:
            hd = 1.0 if d.is_head else 0.0
            row([(col["n"](i), bp), (col["t"](i), -bp)],
                float(d.d_avail_metal) - float(d.c_gpu) - float(model.b_out * hd))
    for i, d in enumerate(devs):
        r = recs[i]
        busy = [(col["w"](i), float(r["a"])), (col["n"](i), float(r["b"])), (col["s1"](i), r["p1"]),
                (col["s2"](i), r["p2"]), (col["s3"](i), r["p3"]), (col["t"](i), r["pV"])]
        const = float(r["xi"]) + float(d.t_comm)
        row(busy + [(col["z"](i), 1.0), (iC, -1.0)], -const)
        # row 2 = busy + fetch (F on w) - z - C; the w entry is a + F in one rounding
        busy2 = [(j, v + (r["F"] if j == col["w"](i) else 0.0)) for j, v in busy]
        row(busy2 + [(col["z"](i), -1.0), (iC, -1.0)], -const)

    c = np.zeros(N)
    c[iC] = float(k - 1)
    for i in range(M):
        r = recs[i]
        for name, key in (("w", "a"), ("n", "b"), ("s1", "p1"), ("s2", "p2"), ("s3", "p3"), ("t", "pV")):
            c[col[name](i)] = float(r[key])
    A_eq = np.zeros((1, N))
    A_eq[0, :M] = 1.0
    t_comm = 0
    for d in devs:
        t_comm += d.t_comm
    xi_sum = 0
    for r in recs:
        xi_sum += float(r["xi"])
    A_ub = np.vstack(rows) if rows else np.zeros((0, N))
    return {
        "c": c, "integrality": integ, "lb": lb, "ub": ub, "A_ub": A_ub, "b_ub": np.asarray(rhs, dtype=float),
        "A_eq": A_eq, "b_eq": np.array([float(W)]), "const": (t_comm, xi_sum, kappa), "W": W, "M": M,
    }


def objective_value(prob, x) -> float:  # halda_p_solver.py:356-357
    t_comm, xi_sum, kappa = prob["const"]
    return float(prob["c"].dot(x)) + t_comm + xi_sum + kappa


def highs_solve(prob, mip_gap: Optional[float] = 1e-4, relax: bool = False):
    """scipy.optimize.milp (HiGHS 1.8.0) on the dense problem, as the reference calls it."""
    from scipy.optimize import Bounds, LinearConstraint, milp

    cons = []
    if prob["A_ub"].shape[0]:
        cons.append(LinearConstraint(prob["A_ub"], -np.inf, prob["b_ub"]))
    cons.append(LinearConstraint(prob["A_eq"], prob["b_eq"], prob["b_eq"]))
    opts = {"time_limit": 3600.0}
    if mip_gap is not None:
        opts["mip_rel_gap"] = float(mip_gap)
    integ = np.zeros_like(prob["integrality"]) if relax else prob["integrality"]
    return milp(c=prob["c"], integrality=integ, bounds=Bounds(prob["lb"], prob["ub"]), constraints=cons, options=opts)


def halda_solve_oracle(devs, model, k_candidates=None, mip_gap=1e-4, kv_bits="8bit", solver="highs"):
    """k-sweep (halda_p_solver.py:369-436) with either HiGHS or the exact C solver.

    Returns (best dict or None, per_k list). Prints nothing."""
    if k_candidates:
        Ks = sorted(set(k_candidates))
    else:
        L = model.L
        Ks = sorted({d for d in range(1, L) if L % d == 0})
    kv = _kv_factor(kv_bits)
    sets = sets_of(devs)
    best, per_k = None, []
    for k in Ks:
        prob = lower_dense(devs, model, k, kv, sets)
        M = prob["M"]
        if solver == "highs":
            res = highs_solve(prob, mip_gap)
            ok, x, extra = res.success, (res.x if res.success else None), {}
        else:
            st, x, b1, b2, nodes = exact_solve(prob)
            ok, extra = st == 0, {"margin": b2 - b1, "nodes": nodes}
        if not ok:
            per_k.append({"k": k, "success": False})
            continue
        w = [int(round(v)) for v in x[:M]]
        n = [int(round(v)) for v in x[M:2 * M]]
        obj = objective_value(prob, x)
        rec = {"k": k, "success": True, "w": w, "n": n, "obj_value": obj, **extra}
        per_k.append(rec)
        if best is None or obj < best["obj_value"]:
            best = {"w": w, "n": n, "k": k, "obj_value": obj, "sets": {s: list(v) for s, v in sets.items()}}
    return best, per_k


# ---------------------------------------------------------------- exact solver
_lib = None


def _load_exact():
    global _lib
    if _lib is None:
        if not EXACT_LIB.exists():
            raise FileNotFoundError(f"{EXACT_LIB} missing: run `make -C oracle` (or __graft_entry__.build())")
        lib = ctypes.CDLL(str(EXACT_LIB))
        dp = ctypes.POINTER(ctypes.c_double)
        lib.halda_exact_solve.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, dp,
                                          ctypes.POINTER(ctypes.c_uint8), ctypes.c_double, dp, dp, dp,
                                          ctypes.POINTER(ctypes.c_int64)]
        lib.halda_exact_solve.restype = ctypes.c_int
        _lib = lib
    return _lib


def exact_solve(prob, eps: float = 1e-9):
    """(status, x, best_obj_lin, second_best_obj_lin, dp_runs). status 0 ok, 2 infeasible, <0 unsupported."""
    lib = _load_exact()
    A = np.ascontiguousarray(np.vstack([prob["A_ub"], prob["A_eq"]]), dtype=np.float64)
    m, n = A.shape
    bl = np.concatenate([np.full(prob["A_ub"].shape[0], -np.inf), prob["b_eq"]]).astype(np.float64)
    bu = np.concatenate([prob["b_ub"], prob["b_eq"]]).astype(np.float64)

    def p(a):
        return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))

    keep = [A, bl, bu]
    c, lb, ub = (np.ascontiguousarray(prob[k], dtype=np.float64) for k in ("c", "lb", "ub"))
    integ = np.ascontiguousarray(prob["integrality"], dtype=np.uint8)
    x = np.zeros(n)
    b1, b2 = ctypes.c_double(), ctypes.c_double()
    nodes = ctypes.c_int64()
    st = lib.halda_exact_solve(n, m, p(A), p(bl), p(bu), p(c), p(lb), p(ub),
                               integ.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), eps,
                               x.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(b1), ctypes.byref(b2),
                               ctypes.byref(nodes))
    del keep
    return st, x, b1.value, b2.value, nodes.value


def uniqueness_margin_ok(best: float, second: float, rel: float = 1e-7) -> bool:
    """True when the optimum is unique by more than `rel` (relative, floor 1e-9 absolute)."""
    if not math.isfinite(second):
        return True
    return (second - best) > rel * max(1.0, abs(best))
