"""Seeded synthetic heterogeneous fleets.

The reference ships no generator; this one defines the benchmark workloads:
  C2  M=16 fleets, seeds 0..N
  C3  M=64 fleets, seeds 0..4095 (4096 scenarios x 9 k = 36,864 instances)
  C5  perturbation stream around fleet seed 0 (every numeric field x LU(0.9, 1.1))

Templates are the three committed device profiles (hermes_70b/m3_air,
llama_3_70b/online/m1, m2). Model: llama_3_70b/online (L=80, Q4_K), kv "4bit".
LU(lo, hi) is log-uniform. Output is plain dicts in the DeviceProfile JSON
schema, so fleets can be committed as JSON and validated by either package.
"""

from __future__ import annotations

import copy
import json
import math
from pathlib import Path
from typing import Dict, List

import numpy as np

REPO = Path(__file__).resolve().parent.parent
PROFILES = REPO / "test" / "profiles"
TEMPLATE_FILES = ("hermes_70b/m3_air.json", "llama_3_70b/online/m1.json", "llama_3_70b/online/m2.json")
MODEL_FILE = "llama_3_70b/online/model_profile.json"
KINDS = ("mac_metal", "mac_no_metal", "linux_cuda", "linux_cpu", "android")


def load_templates() -> List[Dict]:
    return [json.loads((PROFILES / f).read_text()) for f in TEMPLATE_FILES]


def load_model_dict() -> Dict:
    return json.loads((PROFILES / MODEL_FILE).read_text())


def _lu(rng: np.random.Generator, lo: float, hi: float) -> float:
    return float(math.exp(rng.uniform(math.log(lo), math.log(hi))))


def _scale_table(table: Dict, f: float) -> Dict:
    return {q: {b: float(v) * f for b, v in per_b.items()} for q, per_b in table.items()}


def synth_device(rng: np.random.Generator, i: int, templates: List[Dict]) -> Dict:
    tpl = templates[int(rng.integers(len(templates)))]
    kind = "mac_metal" if i == 0 else KINDS[int(rng.integers(len(KINDS)))]
    d = copy.deepcopy(tpl)
    d["name"] = f"dev{i:03d}-{kind}"
    d["is_head"] = i == 0
    d["scpu"] = _scale_table(tpl["scpu"], _lu(rng, 0.25, 4.0))
    d["T_cpu"] = float(tpl["T_cpu"]) * _lu(rng, 0.5, 2.0)
    d["s_disk"] = float(tpl["s_disk"]) * _lu(rng, 0.25, 2.0)
    d["d_avail_ram"] = int(_lu(rng, 4e9, 64e9))
    d["t_comm"] = _lu(rng, 0.005, 0.1)
    for key in ("sgpu_cuda", "sgpu_metal", "T_cuda", "T_metal", "d_avail_cuda", "d_avail_metal"):
        d[key] = None
    d["t_ram2vram"] = d["t_vram2ram"] = 0.0
    d["has_cuda"] = d["has_metal"] = False
    if kind == "mac_metal":
        d.update(os_type="mac_metal", has_metal=True, is_unified_mem=True)
        d["sgpu_metal"] = _scale_table(tpl["sgpu_metal"], _lu(rng, 0.5, 4.0))
        d["T_metal"] = float(tpl["T_metal"]) * _lu(rng, 0.5, 3.0)
        d["d_avail_metal"] = d["d_avail_ram"]
    elif kind == "linux_cuda":
        d.update(os_type="linux", has_cuda=True, is_unified_mem=False)
        d["sgpu_cuda"] = _scale_table(tpl["sgpu_metal"], _lu(rng, 2.0, 20.0))
        d["T_cuda"] = _lu(rng, 3e11, 3e12)
        d["d_avail_cuda"] = int(_lu(rng, 8e9, 80e9))
        d["t_ram2vram"] = _lu(rng, 1e-5, 1e-4)
        d["t_vram2ram"] = _lu(rng, 1e-5, 1e-4)
    elif kind == "mac_no_metal":
        d.update(os_type="mac_no_metal", is_unified_mem=True)
    elif kind == "linux_cpu":
        d.update(os_type="linux", is_unified_mem=False)
    else:
        d.update(os_type="android", is_unified_mem=False)
    return d


def synth_fleet(seed: int, M: int, templates: List[Dict] | None = None) -> List[Dict]:
    """M device dicts; device 0 is the mac_metal head."""
    templates = templates or load_templates()
    rng = np.random.default_rng(seed)
    return [synth_device(rng, i, templates) for i in range(M)]


def _perturb(value, rng, lo=0.9, hi=1.1):
    if isinstance(value, bool) or value is None or isinstance(value, str):
        return value
    if isinstance(value, int):
        return int(value * _lu(rng, lo, hi))
    if isinstance(value, float):
        return value * _lu(rng, lo, hi)
    if isinstance(value, dict):
        return {k: _perturb(v, rng, lo, hi) for k, v in value.items()}
    return value


def perturbed_fleet(base: List[Dict], i: int) -> List[Dict]:
    """C5 stream element i: every numeric field of every device x LU(0.9, 1.1), seed 10_000 + i."""
    rng = np.random.default_rng(10_000 + i)
    return [{k: _perturb(v, rng) for k, v in d.items()} for d in base]
