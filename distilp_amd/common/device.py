"""DeviceProfile: the per-device solver input.

Field names, types, defaults and optionality follow the reference schema
(`src/distilp/common/device.py:12-93`) so that every profile JSON the
reference accepts validates here unchanged. Symbols in the trailing comments
are the HALDA paper's notation.
"""

from __future__ import annotations

from typing import Dict, Optional

from pydantic import BaseModel, Field

from .types import QuantizationLevel

FlopsTable = Dict[QuantizationLevel, Dict[str, float]]


class DeviceProfile(BaseModel):
    """One device of a fleet (profiler output == solver input)."""

    # identification / capability flags
    name: str = ""
    os_type: str = ""  # mac_no_metal | mac_metal | linux | android (anything else -> M3)
    is_head: bool = True  # I_{m=1}
    is_unified_mem: bool = False  # I_UMA
    has_cuda: bool = False
    has_metal: bool = False

    # CPU path
    scpu: FlopsTable = Field(default_factory=dict)  # s^cpu_{m,q}[b_x], FLOP/s
    T_cpu: float = 0.0  # register-load throughput, B/s

    # KV-cache copy time (s)
    t_kvcpy_cpu: float = 0.0
    t_kvcpy_gpu: float = 0.0

    # host<->device and inter-device transfer times (s)
    t_ram2vram: float = 0.0
    t_vram2ram: float = 0.0
    t_comm: float = 0.0

    s_disk: float = 0.0  # disk read throughput, B/s
    d_avail_ram: int = 0  # bytes

    # GPU path (absent on CPU-only devices)
    sgpu_cuda: Optional[FlopsTable] = None
    sgpu_metal: Optional[FlopsTable] = None
    T_cuda: Optional[float] = None
    T_metal: Optional[float] = None
    d_avail_cuda: Optional[int] = None
    d_avail_metal: Optional[int] = None

    # compute buffers (bytes)
    c_cpu: int = 0
    c_gpu: int = 0

    # swap (android)
    d_bytes_can_swap: int = 0
    d_swap_avail: int = 0

    def print_summary(self) -> None:
        """Human-readable summary (same lines as the reference, device.py:78-93)."""
        gib = 1024**3
        print(f"   OS Type: {self.os_type}")
        print(f"   RAM: {self.d_avail_ram / gib:.1f} GB")
        print(f"   Is Head: {self.is_head}")
        print(f"   Unified Memory: {self.is_unified_mem}")
        if self.has_cuda and self.d_avail_cuda:
            print(f"   CUDA: {self.d_avail_cuda / gib:.1f} GB")
        if self.has_metal and self.d_avail_metal:
            print(f"   Metal: {self.d_avail_metal / gib:.1f} GB")
        print(f"   Disk Speed: {self.s_disk / (1024**2):.1f} MB/s")
