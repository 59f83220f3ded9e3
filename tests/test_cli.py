"""`solver` CLI (reference src/cli/solver.py): loaders on CPU, full stdout parity on the GPU."""

import contextlib
import io
import json
import os

import pytest

from .conftest import REPO


@pytest.fixture
def in_repo(monkeypatch):
    monkeypatch.chdir(REPO)


def test_loaders_resolve_reference_fixture_paths(in_repo):
    from cli.solver import load_from_profile_folder
    from distilp.common import DeviceProfile, ModelProfile

    for folder, n_dev, L in [("hermes_70b", 1, 80), ("llama_3_70b/online", 2, 80), ("qwen3_32b/bf16", 1, 64)]:
        devs, model = load_from_profile_folder(folder)  # falls back to test/profiles/<folder>
        assert len(devs) == n_dev and model.L == L
        assert isinstance(devs[0], DeviceProfile) and isinstance(model, ModelProfile)
        assert devs[0].is_head
    devs, _ = load_from_profile_folder("llama_3_70b/online")
    assert [d.name for d in devs] == ["Mac", "Omers-MBP-32193"]  # sorted file order m1, m2
    with pytest.raises(FileNotFoundError):
        load_from_profile_folder("no_such_profile")


def test_split_model_reduction_matches_fixture(in_repo):
    from distilp_amd.cli.solver import load_model_profile

    m = load_model_profile("test/profiles/llama_3_70b/online/model_profile.json")
    raw = json.loads((REPO / "test/profiles/llama_3_70b/online/model_profile.json").read_text())
    assert m.b_layer == raw["b"][1] and m.b_in == raw["b_i"][1] and m.b_out == raw["b_o"][1]
    assert m.f_q == {k: v[1] for k, v in raw["f_q"]["decode"].items()}
    assert m.f_out == raw["f_out"]["decode"] and m.Q == raw["quantization"]


def test_legacy_model_profile_is_rejected(in_repo):
    """model_profile_qwen3_4b_8bit.json is the reference's legacy format; it fails validation there too."""
    from pydantic import ValidationError

    from distilp_amd.cli.solver import load_model_profile

    with pytest.raises(ValidationError):
        load_model_profile("test/profiles/model_profile_qwen3_4b_8bit.json")


def test_argparse_errors(in_repo):
    from distilp_amd.cli.solver import main

    with pytest.raises(SystemExit):
        with contextlib.redirect_stderr(io.StringIO()):
            main(["--devices", "test/profiles/hermes_70b/m3_air.json"])


@pytest.mark.gpu
def test_cli_stdout_matches_reference(in_repo, fixtures_golden):
    from distilp_amd.cli.solver import main

    for name, case in fixtures_golden["cli"].items():
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert main(case["argv"]) == case["code"]
        assert buf.getvalue() == case["stdout"], name


@pytest.mark.gpu
def test_cli_save_solution(in_repo, tmp_path):
    from distilp_amd.cli.solver import main

    out = tmp_path / "sol.json"
    with contextlib.redirect_stdout(io.StringIO()):
        main(["--profile", "llama_3_70b/online", "--no-plot", "--save-solution", str(out)])
    sol = json.loads(out.read_text())
    assert sol["k"] == 2
    assert sol["layer_distribution"] == {"Mac": {"w": 13, "n": 13}, "Omers-MBP-32193": {"w": 27, "n": 27}}
    assert sol["sets"] == {"M1": [], "M2": ["Mac", "Omers-MBP-32193"], "M3": []}
    assert abs(sol["objective_value"] - 1.9349421818288455) < 1e-9
