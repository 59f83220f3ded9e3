"""The resident single-fleet solver (halda_resident_kernel): halda_solve's latency path, where one wave
stays resident between calls and takes each fleet from a pinned mailbox instead of a kernel launch per
call (halda_solve_fleets_host with one fleet). Every answer must be the bits of the launch-per-call path
(a context made with HALDA_RESIDENT=0) on the same fleet -- statuses, per-k objectives, x and c of every
k, best k, obj_value, w, n -- including after the wave has left for lack of requests and is relaunched,
and a context must be freed promptly while its wave is resident. Reference: halda_p_solver.py:369-436."""

import contextlib
import ctypes
import io
import os
import time

import numpy as np
import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver._libhalda import HaldaContext, get_context
from distilp_amd.solver.fleets import HaldaFleetResultC, _bind, _host_struct, fleet_table, model_struct
from distilp_amd.synth import synth_fleet

pytestmark = pytest.mark.gpu


def _call(ctx, table, model, ks):
    """halda_solve_fleets_host on `ctx` for a one-fleet table, x / c of every k (dense layout)."""
    lib = _bind(ctx.lib)
    fs, keep = _host_struct(table)
    nd, nk = table.n_devices, len(ks)
    xs = 7 * nd + 1
    out = {"best_k": np.zeros(1, np.int32), "obj_value": np.zeros(1), "w": np.zeros(nd, np.int32),
           "n": np.zeros(nd, np.int32), "obj_by_k": np.zeros(nk), "status": np.zeros(nk, np.int32),
           "x": np.zeros(nk * xs), "c": np.zeros(nk * xs)}
    r = HaldaFleetResultC(*(out[k].ctypes.data for k in ("best_k", "obj_value", "w", "n", "obj_by_k", "status",
                                                         "x", "c")), None)
    karr = np.asarray(ks, np.int32)
    m = model_struct(model, 0.5)
    with ctx._lock:
        rc = lib.halda_solve_fleets_host(ctx.ctx, ctypes.byref(m), ctypes.byref(fs), karr.ctypes.data, nk,
                                         ctypes.byref(r))
    assert rc == 0
    return out


@pytest.fixture(scope="module")
def launch_ctx():
    os.environ["HALDA_RESIDENT"] = "0"
    try:
        ctx = HaldaContext(0)
    finally:
        os.environ.pop("HALDA_RESIDENT", None)
    yield ctx
    ctx.close()


def test_resident_answers_equal_launch_per_call(llama_online_model, launch_ctx):
    """60 one-fleet calls (1..64 devices, two k lists, L = 80 and L = 48), some separated by pauses longer
    than the wave's idle limit (2 ms) so that it leaves and is relaunched: the resident context's answers
    equal the launch-per-call context's bit for bit."""
    ctx = get_context(0)
    rng = np.random.default_rng(3)
    for i in range(60):
        M = int(rng.integers(1, 65)) if i % 5 else 64
        model = llama_online_model if i % 3 else llama_online_model.model_copy(update={"L": 48})
        L = model.L
        ks = [d for d in range(1, L) if L % d == 0] if i % 2 else [1, 2, 4]
        table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(40000 + i, M)]], model)
        got = _call(ctx, table, model, ks)
        want = _call(launch_ctx, table, model, ks)
        for k in want:
            assert np.array_equal(got[k], want[k]), (i, M, k)
        if i % 7 == 0:
            time.sleep(0.01)


def test_halda_solve_through_the_resident_wave(llama_online_model):
    """halda_solve (the unchanged API) on a C3-shaped fleet, back to back and after idle pauses: the
    same HALDAResult every time."""
    from distilp_amd.solver import halda_solve

    devs = [DeviceProfile.model_validate(d) for d in synth_fleet(0, 64)]
    outs = []
    for i in range(12):
        with contextlib.redirect_stdout(io.StringIO()):
            outs.append(halda_solve(devs, llama_online_model, mip_gap=1e-4, plot=False, kv_bits="4bit"))
        if i % 4 == 3:
            time.sleep(0.005)
    assert all(o == outs[0] for o in outs)


def test_context_with_a_resident_wave_is_freed_promptly(llama_online_model):
    """halda_free while the wave is resident: it sets `stop` and waits for the wave, well within the
    idle limit's order of magnitude; a freed context's plans fail cleanly (no use of freed memory)."""
    ctx = HaldaContext(0)
    table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(41000, 64)]], llama_online_model)
    for _ in range(3):
        _call(ctx, table, llama_online_model, [1, 2, 4, 5, 8, 10, 16, 20, 40])
    t0 = time.perf_counter()
    ctx.close()
    assert time.perf_counter() - t0 < 1.0


def test_resident_timeout_stops_the_wave_and_launches(llama_online_model, launch_ctx):
    """A resident wave that gives no answer in time (fault injection: HALDA_RESIDENT_TEST=drop never posts
    the request, so the wave idles while the host waits 20 ms): the call stops the wave, waits until it
    has left -- so it can never write a stale answer into the pinned buffer later -- and answers by a
    launch instead of failing; the context keeps working (launch per call from then on), bit for bit."""
    os.environ["HALDA_RESIDENT_TEST"] = "drop"
    try:
        ctx = HaldaContext(0)
    finally:
        os.environ.pop("HALDA_RESIDENT_TEST", None)
    try:
        ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
        for i, M in enumerate((64, 17, 64, 3)):
            table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(42000 + i, M)]],
                                llama_online_model)
            got = _call(ctx, table, llama_online_model, ks)
            want = _call(launch_ctx, table, llama_online_model, ks)
            for k in want:
                assert np.array_equal(got[k], want[k]), (i, M, k)
    finally:
        t0 = time.perf_counter()
        ctx.close()
        assert time.perf_counter() - t0 < 1.0


def test_resident_release_lets_the_wave_go_at_once(llama_online_model, launch_ctx):
    """halda_resident_release right after a resident call returns within a fraction of the wave's 2 ms idle
    limit (it stops the wave instead of waiting it out), is a no-op when repeated, and the next call
    relaunches the wave with the same answers."""
    ctx = get_context(0)
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    table = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(43000, 64)]], llama_online_model)
    want = _call(launch_ctx, table, llama_online_model, ks)
    took = []
    for _ in range(5):
        got = _call(ctx, table, llama_online_model, ks)
        for k in want:
            assert np.array_equal(got[k], want[k]), k
        t0 = time.perf_counter()
        ctx.release_resident()
        took.append(time.perf_counter() - t0)
        ctx.release_resident()  # nothing resident now
    assert sorted(took)[2] < 1.5e-3, took
