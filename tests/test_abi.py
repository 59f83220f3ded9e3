"""C-ABI surface of libhalda (CPU-only: loads the library, checks exports; no GPU compute)."""

import ctypes
import re

import pytest

from distilp_amd.solver import _libhalda as lh

from .conftest import REPO

HEADER = REPO / "include" / "halda.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void)\s+\**(halda_\w+)\s*\(", text, re.M)))


def test_header_declares_the_binding_exports():
    assert declared_functions() == sorted(lh.EXPORTS)


@pytest.fixture(scope="module")
def lib():
    if not lh.LIB_PATH.exists():
        pytest.fail(f"{lh.LIB_PATH} not built (run __graft_entry__.build())")
    return lh.load_library()


def test_library_exports_every_declared_symbol(lib):
    raw = ctypes.CDLL(str(lh.LIB_PATH))
    for name in declared_functions():
        assert hasattr(raw, name), name


def test_version_and_lds_budget(lib):
    assert lib.halda_version() == 3
    # C3 shape: M = 64 (449 cols), R + 1 = 17 extra-layer states -> well under 160 KiB
    b = lib.halda_lds_bytes(449, 17, 64 * 17, 0)
    assert 0 < b < 64 * 1024
    assert lib.halda_lds_bytes(449, 81, 64 * 81, 40 * 41) > b


def test_struct_layout_matches_header():
    # halda_batch: 5 int32 then 8-byte aligned pointers/doubles
    assert lh.HaldaBatchC.n_cols.offset == 24
    assert ctypes.sizeof(lh.HaldaBatchC) == 24 + 14 * 8 + 3 * 8 + 2 * 8
    assert ctypes.sizeof(lh.HaldaResultC) == 6 * 8


def test_init_without_gpu_fails_loudly(lib):
    """No silent CPU fallback: without a gfx950 device halda_init returns an error code."""
    ctx = ctypes.c_void_p()
    rc = lib.halda_init(0, ctypes.byref(ctx))
    if rc == 0:  # running on a GPU box
        lib.halda_free(ctx)
        pytest.skip("GPU present")
    assert rc < 0
    assert "device" in lh.last_error(lib) or "gfx950" in lh.last_error(lib)


def test_product_path_has_no_oracle_import():
    """The shipped package never imports the oracle (test infrastructure only)."""
    for p in (REPO / "distilp_amd").rglob("*.py"):
        src = p.read_text()
        assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, re.M), p


def test_lds_bytes_beyond_the_old_128_state_cap(lib):
    """R + 1 > 128 is legal (the reference has no cap, halda_p_solver.py:72); shapes beyond the LDS
    budget are reported as such (the library then runs the global-table launch)."""
    assert 0 < lib.halda_lds_bytes(7 * 8 + 1, 249, 8 * 249, 8 * 121) < 160 * 1024
    assert lib.halda_lds_bytes(7 * 100 + 1, 157, 100 * 157, 100 * 29) > 160 * 1024


def test_integration_md_stub_is_the_committed_file():
    """INTEGRATION.md path B shows integration/halda_milp.py verbatim (the GPU suite runs that file)."""
    md = (REPO / "INTEGRATION.md").read_text()
    code = (REPO / "integration" / "halda_milp.py").read_text()
    assert "```python\n" + code + "```" in md


def test_plan_entry_points_reject_bad_arguments(lib):
    """The plan / path entry points validate their arguments before any HIP call (HALDA_E_ARG = -22,
    include/halda.h:56), so a binding's mistakes fail loudly on any host."""
    raw = ctypes.CDLL(str(lh.LIB_PATH))
    P = ctypes.c_void_p
    many = raw.halda_fleets_plan_launch_many
    many.argtypes = [ctypes.POINTER(P), ctypes.c_int32, ctypes.POINTER(P), ctypes.c_int32, ctypes.c_int64,
                     ctypes.c_int32]
    many.restype = ctypes.c_int
    plans, streams = (P * 1)(None), (P * 1)(None)
    assert many(None, 1, streams, 1, 0, 1) == -22
    assert "launch_many" in lh.last_error(lib)
    assert many(plans, 0, streams, 1, 0, 1) == -22
    assert many(plans, 1, streams, 0, 0, 1) == -22
    assert many(plans, 1, streams, 1, -1, 1) == -22
    assert many(plans, 1, streams, 1, 0, -1) == -22
    assert many(plans, 1, streams, 1, 0, 0) == 0  # no steps: nothing launched
    assert many(plans, 1, streams, 1, 0, 1) == -22  # the NULL plan, from halda_fleets_plan_launch
    assert "NULL plan" in lh.last_error(lib)
    raw.halda_fleets_plan_launch.argtypes = [P, P]
    assert raw.halda_fleets_plan_launch(None, None) == -22
    raw.halda_set_fleets_path.argtypes = [P, ctypes.c_int]
    assert raw.halda_set_fleets_path(None, 1) == -22


LLVM = __import__("pathlib").Path("/opt/rocm/lib/llvm/bin")


def kernel_resources(tmp_path):
    """Per kernel of libhalda's gfx950 code object: the AMDGPU metadata the compiler wrote (scratch bytes
    per lane, VGPRs, spills), read from the .hip_fatbin bundle with the ROCm LLVM tools."""
    import subprocess

    tools = [LLVM / t for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(t.exists() for t in tools):
        pytest.skip("ROCm LLVM tools not found")
    fat, co = tmp_path / "fatbin.bin", tmp_path / "gfx950.co"
    subprocess.run([str(tools[0]), f"--dump-section=.hip_fatbin={fat}", str(lh.LIB_PATH), str(tmp_path / "host.so")],
                   check=True, capture_output=True)
    subprocess.run([str(tools[1]), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    notes = subprocess.run([str(tools[2]), "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    out = {}
    for item in re.split(r"(?m)^  - \.agpr_count:", notes)[1:]:
        kv = dict(re.findall(r"(?m)^    \.(\w+):\s+(\S+)", item))
        out[re.search(r"halda_\w+?_kernel", kv["name"]).group(0)] = {
            k: int(kv[k]) for k in ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count")}
    return out


def test_hot_kernels_use_no_scratch_at_their_occupancy(lib, tmp_path):
    """The kernels the bench times keep every value in registers (no scratch) within the VGPR budget of
    the occupancy DESIGN.md states: the C3 group launch at seven waves per SIMD (<= 72), the C2 k-slot
    group launch at five four-wave workgroups per CU (<= 96), path B's k = 1 kernels at four (<= 128)."""
    res = kernel_resources(tmp_path)
    budget = {"halda_sweep_steps_kernel": 72, "halda_sweep_kslot_steps_kernel": 96,
              "halda_solve_k1_settled_kernel": 128, "halda_solve_k1_kernel": 128, "halda_sweep_kernel": 128,
              "halda_screen_kernel": 128, "halda_resident_kernel": 128}
    for name, vgprs in budget.items():
        r = res[name]
        assert r["private_segment_fixed_size"] == 0 and r["vgpr_spill_count"] == 0, (name, r)
        assert r["vgpr_count"] <= vgprs, (name, r)
