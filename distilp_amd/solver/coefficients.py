"""Per-device HALDA model coefficients (host side, exact FP64 scalar arithmetic).

Restates `src/distilp/solver/components/dense_common.py` of the reference.
Every formula keeps the reference's operation order so that the lowered
MILP is bit-identical to the one the reference hands to HiGHS; errors the
reference raises on bad inputs (ZeroDivisionError on T_cpu == 0, ValueError
on a missing batch key, IndexError on an empty fleet) surface the same way.

  valid_factors_of_L   dense_common.py:9-22   (prints "L [factors...]")
  b_prime              dense_common.py:25-46  (int-truncated bytes/layer)
  sum_f_over_s         dense_common.py:49-75
  gpu_flops_table      dense_common.py:78-86
  gpu_load_throughput  dense_common.py:89-97
  alpha_beta_xi        dense_common.py:100-119
  b_cio_b              dense_common.py:122-126
  classify_device_case dense_common.py:129-146
  assign_sets          dense_common.py:149-167
  objective_vectors    dense_common.py:170-208
  kappa_constant       dense_common.py:211-230
  ILPResult/HALDAResult dense_common.py:233-279
"""

from __future__ import annotations

import math
import sys
from typing import Dict, List, Optional, Tuple

from pydantic import BaseModel

from ..common import DeviceProfile, ModelProfile


_FACTORS: Dict[int, Tuple[str, List[int]]] = {}


def valid_factors_of_L(L: int) -> List[int]:
    """Divisors of L other than L, sorted. Prints the unsorted discovery list
    exactly like the reference (dense_common.py:21), which the CLI shows (the printed line and the
    list are remembered per integer L: the same text, written in one call)."""
    hit = _FACTORS.get(L) if type(L) is int else None
    if hit is not None:
        sys.stdout.write(hit[0])
        return list(hit[1])
    found: List[int] = []
    for d in range(1, int(math.sqrt(L)) + 1):
        if L % d:
            continue
        if d != L:
            found.append(d)
        q = L // d
        if q != d and q != L:
            found.append(q)
    print(L, found)
    out = sorted(set(found))
    if type(L) is int:
        _FACTORS[L] = (f"{L} {found}\n", out)
    return out


def b_prime(model: ModelProfile, kv_bits_k: float = 1.0, kv_bits_v: Optional[float] = None,
            *, rho_w: float = 0.15, kv_group: int = 64) -> int:
    """Bytes per resident layer incl. KV cache and per-group scales, truncated to int."""
    kv_v = kv_bits_k if kv_bits_v is None else kv_bits_v
    kv_nominal = kv_bits_k * (model.hk * model.ek * model.n_kv) + kv_v * (model.hv * model.ev * model.n_kv)
    kv_bytes = (1.0 + (2.0 / float(max(1, kv_group)))) * kv_nominal
    return int((1.0 + float(rho_w)) * float(model.b_layer) + kv_bytes)


def sum_f_over_s(f_by_q: Dict[str, float], s_by_q, q, batch_size: int = 1) -> float:
    """f_q[b] / S[q][b], or 0 when the batch key / quant level is absent or S <= 0."""
    key = f"b_{batch_size}"
    if key not in f_by_q or q not in s_by_q:
        return 0.0
    table = s_by_q[q]
    if key not in table:
        raise ValueError(f"Batch size {batch_size} (key '{key}') not found in S_by_q[{q}]")
    s_val = table[key]
    f_val = f_by_q[key]
    return 0.0 + f_val / s_val if s_val > 0 else 0.0


def gpu_flops_table(dev: DeviceProfile):
    """Metal table preferred over CUDA; None when neither is present/truthy."""
    if dev.has_metal and dev.sgpu_metal:
        return dev.sgpu_metal
    if dev.has_cuda and dev.sgpu_cuda:
        return dev.sgpu_cuda
    return None


def gpu_load_throughput(dev: DeviceProfile) -> Optional[float]:
    if dev.has_metal and dev.T_metal:
        return dev.T_metal
    if dev.has_cuda and dev.T_cuda:
        return dev.T_cuda
    return None


def alpha_beta_xi(dev: DeviceProfile, model: ModelProfile, kv_factor: float = 1.0,
                  bp: Optional[int] = None) -> Tuple[float, float, float]:
    """(alpha, beta, xi): CPU s/layer, GPU-minus-CPU s/layer, fixed transfer s.
    `bp` = b_prime(model, kv_factor) when the caller already has it."""
    if bp is None:
        bp = b_prime(model, kv_bits_k=kv_factor)
    cpu_comp = sum_f_over_s(model.f_q, dev.scpu, model.Q)
    alpha = cpu_comp + dev.t_kvcpy_cpu + (bp / dev.T_cpu)
    table, t_gpu = gpu_flops_table(dev), gpu_load_throughput(dev)
    beta = 0.0
    if table is not None and t_gpu is not None:
        delta_comp = sum_f_over_s(model.f_q, table, model.Q) - cpu_comp
        beta = delta_comp + (dev.t_kvcpy_gpu - dev.t_kvcpy_cpu) + (bp / t_gpu - bp / dev.T_cpu)
    xi = (dev.t_ram2vram + dev.t_vram2ram) * (0 if dev.is_unified_mem else 1)
    return alpha, beta, xi


def b_cio_b(dev: DeviceProfile, model: ModelProfile) -> float:
    """Head-device I/O layer bytes plus the CPU compute buffer."""
    return ((model.b_in / model.V) + model.b_out) * (1.0 if dev.is_head else 0.0) + dev.c_cpu


_CASE = {"mac_no_metal": 1, "mac_metal": 2}


def classify_device_case(dev: DeviceProfile) -> int:
    """1 = macOS without Metal, 2 = macOS with Metal, 3 = everything else."""
    return _CASE.get(dev.os_type, 3)


def assign_sets(devs: List[DeviceProfile]) -> Dict[str, List[int]]:
    m1: List[int] = []
    m2: List[int] = []
    m3: List[int] = []
    case = _CASE.get
    for i, d in enumerate(devs):
        c = case(d.os_type, 3)
        (m1 if c == 1 else m2 if c == 2 else m3).append(i)
    return {"M1": m1, "M2": m2, "M3": m3}


def objective_vectors(devs: List[DeviceProfile], model: ModelProfile, sets: Dict[str, List[int]],
                      kv_factor: float = 1.0) -> Tuple[List[float], List[float], List[float]]:
    """a = alpha, b = beta (0 for M1 devices), c = xi."""
    m1 = set(sets["M1"])
    bp = b_prime(model, kv_bits_k=kv_factor)
    a: List[float] = []
    b: List[float] = []
    c: List[float] = []
    for i, d in enumerate(devs):
        alpha, beta, xi = alpha_beta_xi(d, model, kv_factor, bp)
        a.append(alpha)
        b.append(0.0 if i in m1 else beta)
        c.append(xi)
    return a, b, c


def kappa_constant(devs: List[DeviceProfile], model: ModelProfile, sets: Dict[str, List[int]]) -> float:
    """Constant objective part: head-device I/O layers + M1/M3 RAM headroom term.

    The head is the first is_head device (index 0 when none); s_disk is NOT
    floored here (ZeroDivisionError on 0, as in the reference)."""
    hi = next((i for i, d in enumerate(devs) if d.is_head), 0)
    head = devs[hi]
    total = sum_f_over_s(model.f_out, head.scpu, model.Q)
    total += (model.b_in / model.V + model.b_out) / head.T_cpu
    total += model.b_in / (model.V * head.s_disk)
    total += (model.b_out / head.s_disk) if hi not in sets.get("M4", []) else 0.0
    tail = 0.0
    for i in sets.get("M1", []) + sets.get("M3", []):
        d = devs[i]
        swap = min(d.d_bytes_can_swap, d.d_swap_avail) if d.os_type == "android" else 0
        tail += (d.c_cpu - d.d_avail_ram - swap) / d.s_disk
    return total + tail


class ILPResult(BaseModel):
    k: int
    w: List[int]
    n: List[int]
    obj_value: float


class HALDAResult(BaseModel):
    w: List[int]
    n: List[int]
    k: int
    obj_value: float
    sets: Dict[str, List[int]]

    def print_solution(self, devices: List[DeviceProfile]) -> None:
        """Formatted report; line formats match dense_common.py:247-279."""
        bar = "=" * 60
        print(f"\n{bar}")
        print("HALDA Solution")
        print(bar)
        print(f"\nOptimal k: {self.k}")
        print(f"Objective value: {self.obj_value:.6f}")
        print("\nLayer distribution (w):")
        total = sum(self.w)
        for dev, wi in zip(devices, self.w):
            print(f"  {dev.name:40s}: {wi:3d} layers ({(wi / total) * 100:5.1f}%)")
        print("\nGPU assignments (n):")
        for dev, ni in zip(devices, self.n):
            if ni > 0:
                print(f"  {dev.name:40s}: {ni:3d} layers on GPU")
            else:
                print(f"  {dev.name:40s}: CPU only")
        print("\nDevice sets:")
        for name in ("M1", "M2", "M3"):
            if self.sets[name]:
                print(f"  {name}: {', '.join(devices[i].name for i in self.sets[name])}")
