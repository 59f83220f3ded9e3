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
