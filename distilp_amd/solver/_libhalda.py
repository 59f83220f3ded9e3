"""ctypes binding of libhalda (include/halda.h).

The product path has exactly one engine: distilp_amd/libhalda.so on a gfx950
GPU. If the library is missing or no MI355X is visible, every call raises
`HaldaUnavailable` — there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Optional

import numpy as np

LIB_PATH = Path(os.environ.get("HALDA_LIB", Path(__file__).resolve().parent.parent / "libhalda.so"))

ABI_VERSION = 3  # include/halda.h HALDA_ABI_VERSION (2: halda_fleet_result.x_off; 3: byte counts as double)

STATUS_OPTIMAL = 0
STATUS_LIMIT = 1
STATUS_INFEASIBLE = 2
STATUS_UNSUPPORTED = -1
STATUS_TOO_LARGE = -2

_c_i32p = ctypes.POINTER(ctypes.c_int32)
_c_i64p = ctypes.POINTER(ctypes.c_int64)
_c_dp = ctypes.POINTER(ctypes.c_double)
_c_u8p = ctypes.POINTER(ctypes.c_uint8)


class HaldaUnavailable(RuntimeError):
    """libhalda.so is not built or no gfx950 device is present."""


class HaldaBatchC(ctypes.Structure):
    _fields_ = [
        ("n_inst", ctypes.c_int32),
        ("max_cols", ctypes.c_int32),
        ("max_R1", ctypes.c_int32),
        ("max_tab", ctypes.c_int32),
        ("max_tab_kc", ctypes.c_int32),
        ("n_cols", ctypes.c_void_p),
        ("n_rows", ctypes.c_void_p),
        ("csr_off", ctypes.c_void_p),
        ("col_off", ctypes.c_void_p),
        ("row_off", ctypes.c_void_p),
        ("row_ptr", ctypes.c_void_p),
        ("col_idx", ctypes.c_void_p),
        ("val", ctypes.c_void_p),
        ("c", ctypes.c_void_p),
        ("col_lb", ctypes.c_void_p),
        ("col_ub", ctypes.c_void_p),
        ("row_lb", ctypes.c_void_p),
        ("row_ub", ctypes.c_void_p),
        ("integrality", ctypes.c_void_p),
        ("mip_rel_gap", ctypes.c_double),
        ("mip_abs_gap", ctypes.c_double),
        ("time_limit", ctypes.c_double),
        ("x0", ctypes.c_void_p),
        ("y0", ctypes.c_void_p),
    ]


class HaldaResultC(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_void_p),
        ("x", ctypes.c_void_p),
        ("obj_lin", ctypes.c_void_p),
        ("dual_bound", ctypes.c_void_p),
        ("gap", ctypes.c_void_p),
        ("nodes", ctypes.c_void_p),
    ]


EXPORTS = ("halda_version", "halda_init", "halda_solve_batch", "halda_solve_batch_device",
           "halda_solve_batch_device_settled", "halda_last_kernel_ms",
           "halda_last_solve_kernel_ms", "halda_last_phase_ms", "halda_lds_bytes", "halda_last_error", "halda_free",
           "halda_solve_fleets", "halda_solve_fleets_host", "halda_last_lowered", "halda_set_timing",
           "halda_last_fleet_ms", "halda_set_fleets_path", "halda_init_multi", "halda_solve_fleets_multi",
           "halda_free_multi", "halda_comm_unique_id", "halda_comm_init", "halda_comm_destroy",
           "halda_solve_fleets_sharded", "halda_fleets_plan_create", "halda_fleets_plan_launch",
           "halda_fleets_plan_free", "halda_solve_fleets_sharded_emulated", "halda_fleets_plan_launch_many",
           "halda_fleets_group_create", "halda_fleets_group_launch", "halda_fleets_group_free",
           "halda_resident_release", "halda_host_alloc", "halda_host_free")

_lib = None
_lib_lock = threading.Lock()


def _torch_runtime_first() -> None:
    """PyTorch-ROCm bundles its own HIP runtime, libhalda links /opt/rocm's: when libhalda's
    initialises the GPU first, torch's then finds no device in this process ("No HIP GPUs are
    available"; the other order works, tools/probe_runtime_order.py). So when torch is already
    imported, its runtime is initialised before libhalda is loaded. (A program that imports torch only
    after its first libhalda call must initialise torch's CUDA itself first: INTEGRATION.md.)"""
    import sys

    torch = sys.modules.get("torch")
    if torch is None:
        return
    try:
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except Exception:  # noqa: BLE001 -- no GPU / CPU-only torch: nothing to order
        pass


def load_library(path: Path | str | None = None):
    """dlopen libhalda and declare the prototypes. Raises HaldaUnavailable if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = Path(path) if path is not None else LIB_PATH
        _torch_runtime_first()
        if not p.exists():
            raise HaldaUnavailable(f"{p} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                                   "or `make -C distilp_amd/csrc`")
        lib = ctypes.CDLL(str(p))
        lib.halda_version.restype = ctypes.c_int
        if lib.halda_version() != ABI_VERSION:
            raise HaldaUnavailable(f"{p} has ABI {lib.halda_version()}, this binding needs {ABI_VERSION}: rebuild it")
        lib.halda_init.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        lib.halda_init.restype = ctypes.c_int
        lib.halda_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(HaldaBatchC), ctypes.POINTER(HaldaResultC)]
        lib.halda_solve_batch.restype = ctypes.c_int
        lib.halda_solve_batch_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(HaldaBatchC),
                                                 ctypes.POINTER(HaldaResultC), ctypes.c_void_p]
        lib.halda_solve_batch_device.restype = ctypes.c_int
        lib.halda_solve_batch_device_settled.argtypes = [ctypes.c_void_p, ctypes.POINTER(HaldaBatchC),
                                                         ctypes.POINTER(HaldaResultC), ctypes.c_void_p,
                                                         ctypes.c_void_p]
        lib.halda_solve_batch_device_settled.restype = ctypes.c_int
        lib.halda_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.halda_last_kernel_ms.restype = ctypes.c_int
        lib.halda_last_solve_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.halda_last_solve_kernel_ms.restype = ctypes.c_int
        lib.halda_last_phase_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.halda_last_phase_ms.restype = ctypes.c_int
        lib.halda_set_fleets_path.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.halda_set_fleets_path.restype = ctypes.c_int
        lib.halda_last_fleet_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.halda_last_fleet_ms.restype = ctypes.c_int
        lib.halda_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.halda_set_timing.restype = ctypes.c_int
        lib.halda_lds_bytes.argtypes = [ctypes.c_int32] * 4
        lib.halda_lds_bytes.restype = ctypes.c_int64
        lib.halda_last_error.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        lib.halda_last_error.restype = ctypes.c_int
        lib.halda_free.argtypes = [ctypes.c_void_p]
        lib.halda_free.restype = None
        lib.halda_resident_release.argtypes = [ctypes.c_void_p]
        lib.halda_resident_release.restype = ctypes.c_int
        lib.halda_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        lib.halda_host_alloc.restype = ctypes.c_int
        lib.halda_host_free.argtypes = [ctypes.c_void_p]
        lib.halda_host_free.restype = None
        if path is None:
            _lib = lib
        return lib


def last_error(lib) -> str:
    buf = ctypes.create_string_buffer(1024)
    lib.halda_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


@dataclass
class HostBatch:
    """A batch of lowered instances in host memory (NumPy, C-contiguous)."""

    n_cols: np.ndarray  # int32 [n]
    n_rows: np.ndarray  # int32 [n]
    csr_off: np.ndarray  # int64 [n]
    col_off: np.ndarray  # int64 [n]
    row_off: np.ndarray  # int64 [n]
    row_ptr: np.ndarray  # int32
    col_idx: np.ndarray  # int32
    val: np.ndarray  # float64
    c: np.ndarray
    col_lb: np.ndarray
    col_ub: np.ndarray
    row_lb: np.ndarray
    row_ub: np.ndarray
    integrality: np.ndarray  # uint8
    max_cols: int
    max_R1: int
    max_tab: int
    max_tab_kc: int
    mip_rel_gap: float = 1e-4

    @property
    def n_inst(self) -> int:
        return int(self.n_cols.shape[0])

    @property
    def total_cols(self) -> int:
        return int(self.c.shape[0])

    def nbytes(self) -> int:
        return sum(getattr(self, f).nbytes for f in ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr",
                                                     "col_idx", "val", "c", "col_lb", "col_ub", "row_lb", "row_ub",
                                                     "integrality"))


@dataclass
class BatchResult:
    status: np.ndarray
    x: np.ndarray
    obj_lin: np.ndarray
    dual_bound: np.ndarray
    gap: np.ndarray
    nodes: np.ndarray


def _ptr(a: np.ndarray) -> int:
    return int(a.ctypes.data)


class HaldaContext:
    """One libhalda context bound to one GPU (halda_init / halda_free)."""

    def __init__(self, device: int = 0, lib=None):
        self.lib = lib or load_library()
        ctx = ctypes.c_void_p()
        rc = self.lib.halda_init(int(device), ctypes.byref(ctx))
        if rc != 0:
            raise HaldaUnavailable(f"halda_init({device}) failed ({rc}): {last_error(self.lib)}")
        self.ctx = ctx
        self.device = device
        self._lock = threading.Lock()

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.halda_free(self.ctx)
            self.ctx = None

    def release_resident(self):
        """Let the context's resident single-fleet wave go now (halda_resident_release) instead of after
        its 2 ms idle limit: for a caller about to wait on the whole device through libhalda's runtime."""
        with self._lock:
            rc = self.lib.halda_resident_release(self.ctx)
        if rc != 0:
            raise RuntimeError(f"halda_resident_release failed ({rc}): {last_error(self.lib)}")

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def _batch_struct(self, b: HostBatch) -> HaldaBatchC:
        s = HaldaBatchC()
        s.n_inst = b.n_inst
        s.max_cols, s.max_R1, s.max_tab, s.max_tab_kc = b.max_cols, b.max_R1, b.max_tab, b.max_tab_kc
        for f in ("n_cols", "n_rows", "csr_off", "col_off", "row_off", "row_ptr", "col_idx", "val", "c", "col_lb",
                  "col_ub", "row_lb", "row_ub", "integrality"):
            setattr(s, f, _ptr(getattr(b, f)))
        s.mip_rel_gap = b.mip_rel_gap
        s.mip_abs_gap = 1e-6
        s.time_limit = 3600.0
        s.x0 = s.y0 = None
        return s

    def solve(self, b: HostBatch) -> BatchResult:
        """halda_solve_batch on host arrays (synchronous)."""
        n = b.n_inst
        out = BatchResult(status=np.empty(n, np.int32), x=np.zeros(b.total_cols), obj_lin=np.empty(n),
                          dual_bound=np.empty(n), gap=np.empty(n), nodes=np.empty(n, np.int64))
        r = HaldaResultC(_ptr(out.status), _ptr(out.x), _ptr(out.obj_lin), _ptr(out.dual_bound), _ptr(out.gap),
                         _ptr(out.nodes))
        s = self._batch_struct(b)
        with self._lock:
            rc = self.lib.halda_solve_batch(self.ctx, ctypes.byref(s), ctypes.byref(r))
        if rc != 0:
            raise RuntimeError(f"halda_solve_batch failed ({rc}): {last_error(self.lib)}")
        return out

    def solve_device(self, dev_ptrs: Dict[str, int], b: HostBatch, out_ptrs: Dict[str, int],
                     stream: Optional[int] = None, settled: Optional[int] = None) -> None:
        """halda_solve_batch_device: arrays already resident in HBM (e.g. torch tensors). `settled`: the
        device address of n_inst bytes marking instances the caller proved bound-infeasible
        (halda_solve_batch_device_settled; batch.settled_instances computes them from a host batch)."""
        s = HaldaBatchC()
        s.n_inst = b.n_inst
        s.max_cols, s.max_R1, s.max_tab, s.max_tab_kc = b.max_cols, b.max_R1, b.max_tab, b.max_tab_kc
        for f, p in dev_ptrs.items():
            setattr(s, f, int(p))
        s.mip_rel_gap = b.mip_rel_gap
        s.time_limit = 3600.0
        r = HaldaResultC(**{k: int(v) for k, v in out_ptrs.items()})
        with self._lock:  # one launch at a time per context (verdict bytes, hand-back flag)
            st = ctypes.c_void_p(stream) if stream else None
            if settled:
                rc = self.lib.halda_solve_batch_device_settled(self.ctx, ctypes.byref(s), ctypes.byref(r),
                                                               ctypes.c_void_p(int(settled)), st)
            else:
                rc = self.lib.halda_solve_batch_device(self.ctx, ctypes.byref(s), ctypes.byref(r), st)
        if rc != 0:
            raise RuntimeError(f"halda_solve_batch_device failed ({rc}): {last_error(self.lib)}")

    def last_kernel_ms(self, solve_only: bool = False) -> float:
        """Device time of the last launch sequence (or of halda_solve_kernel alone)."""
        ms = ctypes.c_double()
        fn = self.lib.halda_last_solve_kernel_ms if solve_only else self.lib.halda_last_kernel_ms
        rc = fn(self.ctx, ctypes.byref(ms))
        if rc != 0:
            raise RuntimeError(f"halda_last_kernel_ms failed ({rc}): {last_error(self.lib)}")
        return ms.value

    FLEET_PATHS = {"csr": 0, "fused": 1, "wave": 2, "dp": 3, "seg": 4, "kslot_unsplit": 5, "kslot_sequential": 6}

    def set_fleets_path(self, path) -> None:
        """halda_solve_fleets on the fused sweep ("fused" / True, default: fleets of at most 16 devices
        four per wave, one wave per open k -- the k-slot kernel), the same with the segment kernel
        (four fleets per wave, every k in turn: "seg"), the fused sweep one fleet per wave ("wave"), the CSR
        pipeline ("csr" / False), or (test paths) the fused sweep with every k = 1 solve of its
        register launch done by the exact DP it falls back to ("dp"), with the k-slot kernel's
        k = 2 threshold scan unsplit ("kslot_unsplit"; the default splits it over two waves), or split
        in sequential order ("kslot_sequential": part 1 makes its leaf checks and phase 0 itself)."""
        code = self.FLEET_PATHS[path] if isinstance(path, str) else int(bool(path))
        rc = self.lib.halda_set_fleets_path(self.ctx, code)
        if rc != 0:
            raise RuntimeError(f"halda_set_fleets_path failed ({rc}): {last_error(self.lib)}")

    def set_timing(self, on: bool) -> None:
        """Record (or not) the per-launch HIP events behind last_kernel_ms / last_phase_ms."""
        self.lib.halda_set_timing(self.ctx, int(bool(on)))

    def last_fleet_ms(self) -> Dict[str, float]:
        """Device time of each launch of the last halda_solve_fleets call (zero entries dropped)."""
        ms = (ctypes.c_double * 9)()
        rc = self.lib.halda_last_fleet_ms(self.ctx, ms)
        if rc != 0:
            raise RuntimeError(f"halda_last_fleet_ms failed ({rc}): {last_error(self.lib)}")
        names = ("halda_sweep_kernel", "halda_sweep_tables_kernel", "halda_lower_kernel", "halda_screen_kernel",
                 "halda_solve_k1_kernel", "halda_solve_kernel", "halda_pick_kernel", "halda_sweep_seg_kernel",
                 "halda_sweep_kslot_kernel")
        return {n: float(v) for n, v in zip(names, ms) if v > 0.0}

    def last_phase_ms(self) -> Dict[str, float]:
        """Device time of each launch of the last solve: screen, k = 1 fast path, general kernel. A settled
        batch has no screen launch: its k = 1 kernel is halda_solve_k1_settled_kernel (include/halda.h)."""
        ms = (ctypes.c_double * 3)()
        rc = self.lib.halda_last_phase_ms(self.ctx, ms)
        if rc != 0:
            raise RuntimeError(f"halda_last_phase_ms failed ({rc}): {last_error(self.lib)}")
        if ms[0] == 0.0:
            return {"halda_solve_k1_settled_kernel": ms[1], "halda_solve_kernel": ms[2]}
        return {"halda_screen_kernel": ms[0], "halda_solve_k1_kernel": ms[1], "halda_solve_kernel": ms[2]}


_contexts: Dict[int, HaldaContext] = {}
_ctx_lock = threading.Lock()


def get_context(device: int = 0) -> HaldaContext:
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = HaldaContext(device)
            _contexts[device] = ctx
        return ctx
