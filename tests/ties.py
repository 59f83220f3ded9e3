"""Fleets with repeated devices (exact ties between devices' increments and cycle times), shared by the
CPU oracle test and the GPU k-slot parity test.

The reference solves such a fleet itself: test/test_integration.py:88 loads the same device profile
twice (cli/solver.py:43-54 marks the first as head). Homogeneous clusters give the same shape at any
size. Kinds (all at most 16 devices, so a batch of more than 64 of them takes the k-slot kernel):
  twice   one device profile twice, the first marked head (the reference's own case);
  copies  16 copies of one synthetic device;
  two     8 + 8 copies of two synthetic devices;
  half    8 distinct synthetic devices, each twice.
"""

import copy

from .conftest import REPO

FIXTURE_FOLDERS = ("hermes_70b", "llama_3_70b/4bit", "llama_3_70b/online", "qwen3_32b/bf16")


def _validate(dicts):
    from distilp_amd.common import DeviceProfile

    return [DeviceProfile.model_validate(copy.deepcopy(d)) for d in dicts]


def fixture_twice(folder):
    """(devices, model) of test_integration.py:88's shape: the folder's first device profile loaded
    twice, through this package's cli loader (load_devices_and_model, the reference's head rule)."""
    from distilp_amd.cli.solver import load_devices_and_model

    base = REPO / "test" / "profiles" / folder
    dev = sorted(p for p in base.glob("*.json") if p.name != "model_profile.json")[0]
    return load_devices_and_model([str(dev), str(dev)], str(base / "model_profile.json"))


def tied_fleets(n_each=20, seed0=21000):
    """[(kind, devices)] -- n_each synthetic fleets of each kind but 'twice'."""
    from distilp_amd.synth import load_templates, synth_fleet

    tpl = load_templates()
    out = []
    for s in range(n_each):
        src = synth_fleet(seed0 + s, 16, tpl)
        one = src[s % 2]  # the head device (s even) or a non-head one
        out.append(("copies", _validate([one] * 16)))
        out.append(("two", _validate([src[1]] * 8 + [src[2 + s % 14]] * 8)))
        out.append(("half", _validate(src[:8] + src[:8])))
    return out


# ---------------------------------------------------------------- reference-run goldens for ties
# tests/golden/ties.json (tests/golden/gen_golden.py `ties`): the reference's halda_solve on the
# "same device twice" shape (its own cli loader) for every folder x kv_bits x mip_gap, and on
# tied_fleets(20) under two models; per k the HiGHS status, obj_value, fun and dual bound.
TIE_MODELS = ("llama_3_70b/online", "qwen3_32b/bf16")


def tie_golden():
    import json

    return json.loads((REPO / "tests" / "golden" / "ties.json").read_text())


def twice_cases():
    """[(key, devices, model, kv_bits, mip_gap, golden entry)] of the golden's twice cases."""
    from distilp_amd.cli.solver import load_devices_and_model

    out = []
    for key, g in tie_golden()["twice"].items():
        base = REPO / "test" / "profiles" / g["folder"]
        dev = str(base / g["device_file"])
        devs, model = load_devices_and_model([dev, dev], str(base / "model_profile.json"))
        out.append((key, devs, model, g["kv_bits"], g["mip_gap"], g))
    return out


def tie_model(name):
    """The model a tied-fleet golden was made with: the synthetic llama_3_70b/online profile, or the
    qwen3_32b/bf16 folder's (loaded as the reference CLI loads it)."""
    from distilp_amd.common import ModelProfileSplit
    from distilp_amd.synth import load_model_dict

    if name == "llama_3_70b/online":
        return ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    from distilp_amd.cli.solver import load_devices_and_model

    base = REPO / "test" / "profiles" / name
    dev = sorted(p for p in base.glob("*.json") if p.name != "model_profile.json")[0]
    return load_devices_and_model([str(dev)], str(base / "model_profile.json"))[1]


def _eps(v):
    return 1e-9 * max(1.0, abs(v))


def check_sweep_against_golden(g, ours_per_k, ours_k, ours_obj):
    """One k-sweep against the reference's: g = {"result", "per_k"}; ours_per_k = {k: obj_value or None
    (infeasible)}. Per k the same status and an objective inside the interval HiGHS proved
    [obj_value - (fun - dual_bound), obj_value] (a point when HiGHS closed the gap); the best objective no
    worse than the reference's, and the same best k wherever every k was closed and the reference's best
    is unique by more than 1e-9. Returns True when the golden is exact (every gap closed)."""
    exact = True
    objs = []
    for r in g["per_k"]:
        o = ours_per_k[r["k"]]
        if not r["success"]:
            assert o is None, (r["k"], o)
            continue
        assert o is not None, r["k"]
        hi = r["obj_value"]
        gap = r["fun"] - r["dual_bound"]
        exact = exact and gap <= _eps(r["fun"])
        assert hi - max(gap, 0.0) - _eps(hi) <= o <= hi + _eps(hi), (r["k"], o, hi, gap)
        objs.append(hi)
    res = g["result"]
    assert res is not None and ours_k > 0
    assert ours_obj <= res["obj_value"] + _eps(res["obj_value"]), (ours_obj, res["obj_value"])
    objs.sort()
    if exact and (len(objs) < 2 or objs[1] - objs[0] > _eps(objs[0])):
        assert ours_k == res["k"], (ours_k, res["k"])
        assert abs(ours_obj - res["obj_value"]) <= _eps(res["obj_value"])
    return exact
