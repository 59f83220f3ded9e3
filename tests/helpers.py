"""Shared test helpers: load fixture fleets and golden arrays."""

import glob
import json
from functools import lru_cache

import numpy as np

from .conftest import GOLDEN, REPO


def fixture_fleet(folder):
    """Devices + model of a test/profiles folder, loaded like cli/solver.py:57-86."""
    from distilp_amd.common import DeviceProfile, ModelProfileSplit

    base = REPO / "test" / "profiles" / folder
    files = sorted(f for f in glob.glob(str(base / "*.json")) if not f.endswith("model_profile.json"))
    devs = [DeviceProfile.model_validate(json.loads(open(f).read())) for f in files]
    devs[0].is_head = True
    model = ModelProfileSplit.model_validate(json.loads((base / "model_profile.json").read_text())).to_model_profile()
    return devs, model


@lru_cache(maxsize=None)
def _synth_json(M):
    return json.loads((GOLDEN / f"synthetic_M{M}.json").read_text())


def synth_devices(M, seed, dicts=None):
    from distilp_amd.common import DeviceProfile

    if dicts is None:
        dicts = _synth_json(M)["fleets"][seed]["devices"]
    return [DeviceProfile.model_validate(d) for d in dicts]


def golden_lowered_keys(z):
    keys = {}
    for f in z.files:
        if f.endswith("_c"):
            key = f[:-2]
            m, s, k = key.split("_")
            keys[key] = (int(m[1:]), int(s[1:]), int(k[1:]))
    return keys


def load_golden_lowered(z, key):
    A = np.zeros(tuple(z[key + "_Aub_shape"]))
    A[z[key + "_Aub_row"], z[key + "_Aub_col"]] = z[key + "_Aub_val"]
    return {
        "c": z[key + "_c"], "lb": z[key + "_lb"], "ub": z[key + "_ub"], "integrality": z[key + "_integrality"],
        "b_ub": z[key + "_bub"], "A_eq": z[key + "_Aeq"], "b_eq": z[key + "_beq"], "A_ub": A,
    }
