import json
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the built libhalda.so")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def pytest_collection_modifyitems(config, items):
    # GPU runs: PyTorch's bundled HIP runtime must initialise before libhalda's (see
    # distilp_amd.solver._libhalda._torch_runtime_first), whichever test file comes first
    if any(item.get_closest_marker("gpu") for item in items):
        import torch  # noqa: F401


def load_json(name):
    return json.loads((GOLDEN / name).read_text())


@pytest.fixture(scope="session")
def fixtures_golden():
    return load_json("fixtures.json")


@pytest.fixture(scope="session")
def synth_golden():
    out = {}
    for p in sorted(GOLDEN.glob("synthetic_M*.json")):
        d = json.loads(p.read_text())
        out[d["M"]] = d
    return out


@pytest.fixture(scope="session")
def llama_online_model():
    from distilp_amd.common import ModelProfileSplit
    from distilp_amd.synth import load_model_dict

    return ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
