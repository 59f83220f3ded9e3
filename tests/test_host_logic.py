"""Host-side restatement of dense_common.py / halda_p_solver.py helpers (CPU only).

Each helper is compared against the oracle's independent restatement and against
behaviours the reference exhibits (prints, error types)."""

import math

import pytest

from distilp_amd.common import DeviceProfile
from distilp_amd.solver import coefficients as co
from distilp_amd.solver.lower import kv_bits_to_factor, lower_fleet
from oracle import milp_oracle as mo

from .helpers import fixture_fleet, synth_devices


def test_valid_factors_print_and_order(capsys):
    assert co.valid_factors_of_L(80) == [1, 2, 4, 5, 8, 10, 16, 20, 40]
    assert capsys.readouterr().out == "80 [1, 2, 40, 4, 20, 5, 16, 8, 10]\n"
    assert co.valid_factors_of_L(64) == [1, 2, 4, 8, 16, 32]
    assert capsys.readouterr().out == "64 [1, 2, 32, 4, 16, 8]\n"
    assert co.valid_factors_of_L(1) == []
    assert co.valid_factors_of_L(49) == [1, 7]


@pytest.mark.parametrize("s,f", [("4bit", 0.5), (" 8BIT ", 1.0), ("fp16", 2.0), ("bf16", 2.0)])
def test_kv_factor(s, f):
    assert kv_bits_to_factor(s) == f == mo._kv_factor(s)


def test_b_prime_truncates(llama_online_model):
    for kv in (0.5, 1.0, 2.0):
        bp = co.b_prime(llama_online_model, kv)
        assert isinstance(bp, int) and bp == mo._bprime(llama_online_model, kv)


@pytest.mark.parametrize("M", [1, 3, 8, 16])
def test_coefficients_match_oracle(llama_online_model, M):
    for seed in range(3):
        devs = synth_devices(M, seed)
        sets = co.assign_sets(devs)
        assert sets == mo.sets_of(devs)
        a, b, c = co.objective_vectors(devs, llama_online_model, sets, 0.5)
        for i, d in enumerate(devs):
            rec = mo._device_record(d, llama_online_model, 0.5, i in sets["M1"], i in sets["M2"])
            assert (a[i], b[i], c[i]) == (rec["a"], rec["b"], rec["xi"])
            assert co.b_cio_b(d, llama_online_model) == rec["bcio"]
        assert co.kappa_constant(devs, llama_online_model, sets) == mo._kappa(devs, llama_online_model, sets)


def test_error_paths_match_reference_types(llama_online_model):
    devs = synth_devices(2, 0)
    bad = [d.model_copy(update={"T_cpu": 0.0}) for d in devs]
    with pytest.raises(ZeroDivisionError):
        lower_fleet(bad, llama_online_model, "4bit")
    no_disk = [d.model_copy(update={"s_disk": 0.0}) for d in devs]
    with pytest.raises(ZeroDivisionError):  # kappa uses the raw s_disk (dense_common.py:221-228)
        lower_fleet(no_disk, llama_online_model, "4bit")
    with pytest.raises(IndexError):  # empty fleet: kappa_constant indexes devs[0]
        lower_fleet([], llama_online_model, "4bit")
    missing = devs[0].model_copy(update={"scpu": {"Q4_K": {"b_2": 1e11}}})
    with pytest.raises(ValueError, match="b_1"):
        lower_fleet([missing], llama_online_model, "4bit")


def test_s_disk_floor_in_rows_not_in_kappa(llama_online_model):
    """s_disk < 1 is floored at 1.0 in the penalties (halda_p_solver.py:196) but not in kappa."""
    devs = synth_devices(2, 1)
    slow = [devs[0], devs[1].model_copy(update={"s_disk": 0.5})]
    fl = lower_fleet(slow, llama_online_model, "4bit")
    bp = co.b_prime(llama_online_model, 0.5)
    assert fl.c_base[2 * 2 + 1] == bp / 1.0  # s1 price of device 1 uses max(1, s_disk)
    p = mo.lower_dense(slow, llama_online_model, 1, 0.5)
    assert fl.objective_value(p["c"], 0 * p["c"]) == mo.objective_value(p, 0 * p["c"])


def test_multiple_heads_and_android_swap(llama_online_model):
    """Several is_head devices each pay b_out in their metal row; android swap enters M3 rhs and kappa."""
    devs = synth_devices(4, 2)
    tweaked = [d.model_copy(update={"is_head": True}) for d in devs]
    for k in (1, 2):
        p = mo.lower_dense(tweaked, llama_online_model, k, 0.5)
        fl = lower_fleet(tweaked, llama_online_model, "4bit")
        A = fl.dense()
        assert (A[:-1] == p["A_ub"]).all() and (fl.instance(k)[4][:-1] == p["b_ub"]).all()


def test_fixture_device_schema_roundtrip():
    devs, model = fixture_fleet("llama_3_70b/online")
    for d in devs:
        again = DeviceProfile.model_validate_json(d.model_dump_json())
        assert again == d
    assert math.isclose(model.b_layer, 454557696)


def _raises(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001
        return type(e)
    return None


@pytest.mark.parametrize("f_q_b1,f_out_b1,head", [(True, True, 0), (False, True, 0), (False, True, 1),
                                                  (True, False, 1), (False, False, 0)])
def test_fleet_table_b1_rule_matches_reference(llama_online_model, f_q_b1, f_out_b1, head):
    """_sum_f_over_S raises only when "b_1" is in f AND q is in S AND S[q] lacks "b_1"
    (dense_common.py:62-64): alpha reads f_q with every device's scpu, kappa f_out with the head's.
    fleet_table must raise exactly when the host restatement (coefficients.py) does."""
    from distilp_amd.solver.fleets import fleet_table

    model = llama_online_model.model_copy(update={
        "f_q": {} if not f_q_b1 else dict(llama_online_model.f_q),
        "f_out": {} if not f_out_b1 else dict(llama_online_model.f_out)})
    devs = [d.model_copy(update={"is_head": False}) for d in synth_devices(3, 0)]
    devs[head] = devs[head].model_copy(update={"is_head": True})
    devs[head] = devs[head].model_copy(update={"scpu": {model.Q: {"b_2": 1e11}}})
    sets = co.assign_sets(devs)

    def host():
        co.objective_vectors(devs, model, sets, 0.5)
        co.kappa_constant(devs, model, sets)

    assert _raises(lambda: fleet_table([devs], model)) == _raises(host)


def test_halda_solve_raises_where_the_reference_loop_does(llama_online_model, capsys):
    """k = 0 raises at W = L // k (halda_p_solver.py:72) before anything else; an empty k list is
    RuntimeError (:413-414) without touching the fleet; coefficient errors surface at the first k,
    after its debug line. None of these reach the GPU."""
    from distilp_amd.solver import halda_solve

    devs = synth_devices(2, 0)
    with pytest.raises(ZeroDivisionError):
        halda_solve(devs, llama_online_model, k_candidates=[0, 1], plot=False)
    one_layer = llama_online_model.model_copy(update={"L": 1})
    with pytest.raises(RuntimeError, match="No feasible MILP found for any k this round."):
        halda_solve([], one_layer, plot=False)  # valid_factors_of_L(1) == []: the empty fleet is never read
    assert capsys.readouterr().out == "1 []\n"
    bad = [devs[0].model_copy(update={"scpu": {llama_online_model.Q: {"b_2": 1e11}}}), devs[1]]
    with pytest.raises(ValueError, match="b_1"):
        halda_solve(bad, llama_online_model, k_candidates=[-1, 1], plot=False, debug=True)
    assert capsys.readouterr().out == "Objectives by k\nk: -1\n"


def test_c_packer_equals_python_packer(llama_online_model):
    """fleet_table (the C packer, distilp_amd/csrc/fleetpack.c) against fleet_table_py (the Python
    restatement of the reference's field reads and truthiness tests): every field of 300 synthetic
    fleets of 1..70 devices bit for bit, and the same exception type and message on bad input."""
    import numpy as np

    from distilp_amd.common import DeviceProfile
    from distilp_amd.solver import fleets as fleets_mod
    from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS, _host_struct, fleet_table, fleet_table_py
    from distilp_amd.synth import synth_fleet

    assert fleets_mod._PACKER is not None, "the C packer is not built for this interpreter"
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(500 + s, 1 + (s * 7) % 70)] for s in range(300)]
    a, b = fleet_table(fleets, llama_online_model), fleet_table_py(fleets, llama_online_model)
    # a field reassigned on a packed table is what the C struct points at (the blocks are dropped)
    t = fleet_table(fleets[:3], llama_online_model)
    t.T_cpu = t.T_cpu * 2
    s, keep = _host_struct(t)
    assert not hasattr(t, "_blocks") and s.T_cpu == keep["T_cpu"].ctypes.data
    for f in ("dev_off", "os_class", "flags") + F64_FIELDS + BYTE_FIELDS:
        assert getattr(a, f).dtype == getattr(b, f).dtype and np.array_equal(getattr(a, f), getattr(b, f)), f

    def err(fn):
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            return type(e), str(e)
        return None

    devs = fleets[5]
    m = llama_online_model
    cases = [
        [devs, []],                                                           # empty fleet (kappa's IndexError)
        [[devs[0].model_copy(update={"T_cpu": 0.0})] + devs[1:]],            # alpha: b' / T_cpu
        [[d.model_copy(update={"s_disk": 0.0}) for d in devs]],              # kappa: s_disk
        [[devs[0].model_copy(update={"scpu": {m.Q: {"b_2": 1.0}}})] + devs[1:]],  # b_1 missing
        [[d.model_copy(update={"os_type": "android", "d_bytes_can_swap": 7, "d_swap_avail": 5}) for d in devs]],
    ]
    for fl in cases:
        assert err(lambda: fleet_table(fl, m)) == err(lambda: fleet_table_py(fl, m)), fl
    # the packer's parallel pass (several threads reading the profiles, forced on here by
    # HALDA_PACK_THREADS; by default it runs from 8,192 devices): the same table, and the same
    # exception through its serial fallback
    import subprocess
    import sys

    code = (
        "import sys, numpy as np; sys.path.insert(0, '.');"
        "from tests.conftest import *; from distilp_amd.common import DeviceProfile;"
        "from distilp_amd.solver.fleets import F64_FIELDS, BYTE_FIELDS, fleet_table, fleet_table_py;"
        "from distilp_amd.synth import synth_fleet, load_model_dict;"
        "from distilp_amd.common import ModelProfileSplit;"
        "m = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile();"
        "fl = [[DeviceProfile.model_validate(d) for d in synth_fleet(900 + s, 1 + (s * 5) % 64)] for s in range(200)];"
        "fl[7] = [d.model_copy(update={'os_type': 'android', 'd_bytes_can_swap': 7, 'd_swap_avail': 5}) for d in fl[7]];"
        "a, b = fleet_table(fl, m), fleet_table_py(fl, m);"
        "assert all(np.array_equal(getattr(a, f), getattr(b, f)) for f in ('dev_off', 'os_class', 'flags') + F64_FIELDS + BYTE_FIELDS);"
        "bad = fl[:50] + [[fl[50][0].model_copy(update={'T_cpu': 0.0})] + fl[50][1:]];"
        "e = None\ntry: fleet_table(bad, m)\nexcept ZeroDivisionError as x: e = x\nassert e is not None;"
        "miss = fl[:9] + [[fl[9][0].model_copy(update={'scpu': {m.Q: {'b_2': 1.0}}})] + fl[9][1:]];"
        "e = None\ntry: fleet_table(miss, m)\nexcept ValueError as x: e = x\nassert 'b_1' in str(e);"
        "print('ok')")
    env = dict(__import__("os").environ, HALDA_PACK_THREADS="4")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                       cwd=str(__import__("pathlib").Path(__file__).resolve().parent.parent))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
    ok = fleet_table(cases[-1], m)
    assert np.array_equal(ok.swap, fleet_table_py(cases[-1], m).swap) and (ok.swap == 5).all()


def test_bench_gpus_mismatch_fails_loudly():
    """`bench.py --gpus 2` inside a one-rank launch exits with an error (before any GPU call), instead
    of reporting n_gpus: 1."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "--gpus 2 but the launcher started 1 rank" in p.stderr
    assert p.stdout.strip() == ""


def test_fleet_constants_equal_reference_order(llama_online_model):
    """fleets.fleet_constants (NumPy column sweeps over all fleets) == the reference-order scalar loops
    (halda._offset_parts: sum t_comm, sum xi, kappa of dense_common.py:211-230) bit for bit, on ragged
    fleets with android swap, unified memory, no head and a head that is not device 0."""
    import numpy as np

    from distilp_amd.common import DeviceProfile
    from distilp_amd.solver.coefficients import assign_sets
    from distilp_amd.solver.fleets import fleet_constants, fleet_constants_np, fleet_table
    from distilp_amd.solver.halda import _offset_parts
    from distilp_amd.synth import synth_fleet

    fleets = []
    for s in range(120):
        devs = [DeviceProfile.model_validate(d) for d in synth_fleet(700 + s, 1 + (s * 11) % 67)]
        if s % 5 == 1:
            devs = [d.model_copy(update={"is_head": False}) for d in devs]
        if s % 5 == 2 and len(devs) > 2:
            devs = [d.model_copy(update={"is_head": i == 2}) for i, d in enumerate(devs)]
        if s % 7 == 3:
            devs = [d.model_copy(update={"os_type": "android", "d_bytes_can_swap": 3 << 30,
                                         "d_swap_avail": 1 << 30}) if i % 2 else d for i, d in enumerate(devs)]
        if s % 4 == 0:
            devs = [d.model_copy(update={"is_unified_mem": True}) if i % 3 == 0 else d for i, d in enumerate(devs)]
        fleets.append(devs)
    t = fleet_table(fleets, llama_online_model)
    assert hasattr(t, "_heads")  # the C packer's table: fleet_constants runs its C loops
    ts, xs, ks = fleet_constants(t, llama_online_model)
    tn, xn, kn = fleet_constants_np(t, llama_online_model)
    for f, devs in enumerate(fleets):
        want = _offset_parts(devs, llama_online_model, assign_sets(devs))
        assert (ts[f], xs[f], ks[f]) == want, f
        assert (tn[f], xn[f], kn[f]) == want, f
    # a uniform batch takes the reshape path
    same = fleets[7:8] * 5
    t2 = fleet_table(same, llama_online_model)
    want = _offset_parts(same[0], llama_online_model, assign_sets(same[0]))
    assert all(tuple(v[f] for v in fleet_constants(t2, llama_online_model)) == want for f in range(5))
    assert np.all(np.isfinite(ks))


def test_open_x_offsets_layout(llama_online_model):
    """Compact x / c layout: only instances with W = L // k >= M (and W < 1e6) get a slot, slots are
    contiguous in (fleet, k) order, each 7 M + 1 long."""
    import numpy as np

    from distilp_amd.common import DeviceProfile
    from distilp_amd.solver.fleets import fleet_table, open_x_offsets
    from distilp_amd.synth import synth_fleet

    sizes = [1, 16, 64, 3, 40]
    t = fleet_table([[DeviceProfile.model_validate(d) for d in synth_fleet(s, m)] for s, m in enumerate(sizes)],
                    llama_online_model)
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    off = open_x_offsets(t, llama_online_model, ks).reshape(len(sizes), len(ks))
    nxt = 0
    for f, M in enumerate(sizes):
        for j, k in enumerate(ks):
            if 80 // k >= M:
                assert off[f, j] == nxt
                nxt += 7 * M + 1
            else:
                assert off[f, j] == -1
    assert (off >= 0).sum() == sum(sum(80 // k >= M for k in ks) for M in sizes)
    assert np.array_equal(open_x_offsets(t, llama_online_model, []), np.zeros(0, np.int64))


@pytest.mark.parametrize("sizes", [[64] * 40, [16, 64, 3, 1, 40, 16, 7]])
def test_batch_results_c_builder_equals_python(llama_online_model, monkeypatch, sizes):
    """halda._batch_on_gpu's host half on a stand-in GPU answer (solve_table replaced): the objectives
    through the strided-row dot (one fleet size) or the gather (mixed sizes), and the HALDAResult list
    built in C (_fleetpack.results) equal the Python construction (model_construct per fleet) field for
    field -- w / n rounded half to even, k, obj_value, sets -- with None where no k is feasible; each
    object owns its fields-set."""
    import types

    import numpy as np

    from distilp_amd.common import DeviceProfile
    from distilp_amd.solver import halda as H
    from distilp_amd.solver.fleets import FleetSolve, fleet_table, open_x_offsets
    from distilp_amd.synth import synth_fleet

    m = llama_online_model
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(40 + s, M)] for s, M in enumerate(sizes)]
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    table = fleet_table(fleets, m)
    xo = open_x_offsets(table, m, ks)
    nf, nk = len(fleets), len(ks)
    ext = int(np.max(xo + np.repeat(7 * table.sizes() + 1, nk)))
    rng = np.random.default_rng(1)
    st = np.where(xo.reshape(nf, nk) >= 0, 0, 2).astype(np.int32)
    st[3 % nf, :] = 2  # a fleet without a feasible k
    x = rng.integers(0, 9, 2 * ext).astype(np.float64) + np.where(rng.random(2 * ext) < 0.3, 0.5, 0.0)
    # values beyond the builder's small-int table and below 0, integral and half-way
    odd = np.array([255.5, 256.0, 256.5, 257.0, 300.5, 1e6, -0.5, -2.5, -3.0, 2.0 ** 40 + 0.5])
    x[:ext] = np.where(rng.random(ext) < 0.05, rng.choice(odd, ext), x[:ext])
    x[ext:] = rng.normal(size=ext)
    res = FleetSolve(best_k=None, obj_value=None, w=None, n=None, obj_by_k=None, status=st, ks=ks, x=x[:ext],
                     c=x[ext:], x_off=xo)
    monkeypatch.setattr(H, "solve_table", lambda *a, **k: res)
    got = H._batch_on_gpu(fleets, m, ks, 0.5, 0)
    monkeypatch.setattr(H, "_PACKER", types.SimpleNamespace())  # no `results`: the Python construction
    want = H._batch_on_gpu(fleets, m, ks, 0.5, 0)
    assert len(got) == len(want) == nf and got[3 % nf] is None and want[3 % nf] is None
    for g, w in zip(got, want):
        if w is None:
            assert g is None
            continue
        assert type(g) is type(w) and g.model_dump() == w.model_dump() and g == w
        assert all(type(v) is int for v in g.w + g.n) and type(g.k) is int and type(g.obj_value) is float
        assert g.model_fields_set == w.model_fields_set
    # the objective of every fleet against the reference's own formula on the same c and x
    from distilp_amd.solver.fleets import fleet_constants

    t_sum, x_sum, kap = fleet_constants(table, m)
    sz = table.sizes()
    for f, g in enumerate(got):
        if g is None:
            continue
        N = 7 * int(sz[f]) + 1
        objs = [float(res.c[xo[f * nk + j]:xo[f * nk + j] + N].dot(res.x[xo[f * nk + j]:xo[f * nk + j] + N]))
                + t_sum[f] + x_sum[f] + kap[f] if st[f, j] == 0 else np.inf for j in range(nk)]
        assert g.obj_value == min(objs) and g.k == ks[int(np.argmin(objs))], f
    live = [g for g in got if g is not None]
    live[0].k = 99
    assert live[1].k != 99 and "k" in live[1].model_fields_set


def test_bench_gpus_n_spawns_one_rank_per_gpu(monkeypatch):
    """`python bench.py --gpus 8` (no WORLD_SIZE yet) starts its ranks itself before touching the GPU:
    torch.distributed.run with one process per GPU on 127.0.0.1, the same bench arguments (RCCL
    backend by default), and relays the launcher's exit code."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(repo))
    import bench

    seen = {}

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5"])
    assert bench.main() == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")
    assert "--backend" not in cmd  # nccl (RCCL) is the default backend of the ranks


def test_k_candidates_are_stored_as_int(llama_online_model):
    """k-candidates of any integral type (numpy's too) are deduplicated, sorted and kept as int, as
    ILPResult(k=...) coerces them in the reference (dense_common.py:233-237)."""
    import numpy as np

    from distilp_amd.solver.halda import _k_list

    ks = _k_list(llama_online_model, [np.int64(4), 2, np.int32(2), 1])
    assert ks == [1, 2, 4] and all(type(k) is int for k in ks)
