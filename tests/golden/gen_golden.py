"""Generate golden vectors from the REFERENCE implementation (this container only).

Run:  python tests/golden/gen_golden.py          (needs /root/reference; ~1-2 min)

The reference (distilp 0.1.6, /root/reference/src) is imported read-only via the
3.10 shim of SURVEY.md §8c (PEP 695 `type` aliases pre-registered), with
bytecode writing disabled. Its `scipy.optimize.milp` call site
(halda_p_solver.py:340-346) is wrapped to record every fixed-k MILP it issues
and HiGHS's answer. Nothing from the reference is copied into the repo; only
inputs and outputs (data) are written:

  tests/golden/fixtures.json         per profile folder x kv_bits x mip_gap:
                                     HALDAResult + per-k (status, w, n, obj, nodes,
                                     dual bound, LP-relaxation objective) + CLI stdout
  tests/golden/synthetic_M{M}.json   seeded fleets (device dicts) + per-k results
  tests/golden/lowered.npz           the exact MILP arrays (c, A_ub CSR, b_ub, A_eq,
                                     bounds, integrality) for a few (fleet, k)
  tests/golden/ties.json             fleets of repeated devices (exact ties): the
                                     reference's own "same device twice" shape
                                     (test/test_integration.py:88, loaded by its
                                     cli.solver.load_devices_and_model) for every
                                     profile folder x kv_bits x mip_gap, and the tied
                                     synthetic fleets of tests/ties.py (copies / two /
                                     half) under two models: HALDAResult + per-k

Run `python tests/golden/gen_golden.py ties` to (re)write ties.json alone.

Solver: scipy 1.15.3 / HiGHS 1.8.0 (git 222cce7), the version present here.
"""

from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import time
import types
import typing
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF_SRC = Path("/root/reference/src")
REF_ROOT = Path("/root/reference")

FOLDERS = ["hermes_70b", "llama_3_70b/4bit", "llama_3_70b/online", "qwen3_32b/bf16"]
KV = ["4bit", "8bit", "fp16"]
GAPS = [1e-4, 1e-9]
SYNTH = {1: 24, 2: 24, 3: 24, 4: 24, 8: 24, 16: 24, 32: 12, 64: 16}
LOWERED = [(1, 0, 40), (2, 3, 2), (3, 1, 4), (4, 0, 1), (4, 2, 5), (8, 5, 2), (16, 1, 1), (16, 2, 4),
           (64, 0, 1), (64, 0, 2)]


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF_SRC))
    shim = types.ModuleType("distilp.common.types")
    shim.ModelPhase = typing.Literal["merged", "prefill", "decode"]
    shim.QuantizationLevel = typing.Literal["Q4_K", "Q5_K", "Q6_K", "Q8_0", "BF16", "F16", "F32"]
    sys.modules["distilp.common.types"] = shim
    import distilp.solver.halda_p_solver as hp  # noqa: E402
    import cli.solver as cli  # noqa: E402
    from distilp.common import DeviceProfile, ModelProfileSplit  # noqa: E402
    return hp, cli, DeviceProfile, ModelProfileSplit


class MilpSpy:
    """Wraps scipy.optimize.milp inside the reference module; records each call."""

    def __init__(self, hp, keep_arrays=False):
        self.hp = hp
        self.real = hp.milp
        self.calls = []
        self.keep_arrays = keep_arrays

    def __call__(self, c, integrality, bounds, constraints, options):
        res = self.real(c=c, integrality=integrality, bounds=bounds, constraints=constraints, options=options)
        lp = self.real(c=c, integrality=np.zeros_like(integrality), bounds=bounds, constraints=constraints)
        M = (len(c) - 1) // 7
        rec = {
            "k": int(round(c[-1])) + 1,
            "status": int(res.status),
            "success": bool(res.success),
            "lp_status": int(lp.status),
            "lp_obj": float(lp.fun) if lp.success else None,
        }
        if res.success:
            x = np.asarray(res.x)
            rec.update(
                w=[int(round(v)) for v in x[:M]], n=[int(round(v)) for v in x[M:2 * M]],
                x=[float(v) for v in x], fun=float(res.fun), nodes=int(getattr(res, "mip_node_count", -1)),
                dual_bound=float(getattr(res, "mip_dual_bound", np.nan)), gap=float(getattr(res, "mip_gap", np.nan)),
            )
        if self.keep_arrays:
            rec["arrays"] = (np.array(c), np.array(integrality), bounds, constraints)
        self.calls.append(rec)
        return res

    def fixed_k(self, *args, **kwargs):
        """Wraps solve_fixed_k_milp to record the per-k obj_value (halda_p_solver.py:356-366)."""
        r = self.real_fixed_k(*args, **kwargs)
        self.calls[-1]["obj_value"] = float(r.obj_value)
        return r

    def __enter__(self):
        self.real_fixed_k = self.hp.solve_fixed_k_milp
        self.hp.milp = self
        self.hp.solve_fixed_k_milp = self.fixed_k
        return self

    def __exit__(self, *exc):
        self.hp.milp = self.real
        self.hp.solve_fixed_k_milp = self.real_fixed_k


def run_solve(hp, devs, model, kv, gap, keep_arrays=False):
    with MilpSpy(hp, keep_arrays) as spy:
        buf = io.StringIO()
        err = None
        with contextlib.redirect_stdout(buf):
            try:
                r = hp.halda_solve(devs, model, mip_gap=gap, plot=False, kv_bits=kv)
                result = {"w": r.w, "n": r.n, "k": r.k, "obj_value": r.obj_value, "sets": r.sets}
            except Exception as e:  # noqa: BLE001
                result, err = None, f"{type(e).__name__}: {e}"
    return result, err, spy.calls, buf.getvalue()


def cli_stdout(cli, argv):
    buf = io.StringIO()
    old = sys.argv
    sys.argv = ["solver"] + argv
    try:
        with contextlib.redirect_stdout(buf):
            code = cli.main()
    finally:
        sys.argv = old
    return code, buf.getvalue()


def strip_arrays(calls):
    return [{k: v for k, v in c.items() if k != "arrays"} for c in calls]


def main():
    hp, cli, DeviceProfile, ModelProfileSplit = import_reference()
    sys.path.append(str(REPO))
    from distilp_amd.synth import load_model_dict, synth_fleet  # our generator (data only)

    os.chdir(REF_ROOT)  # the reference CLI resolves "test/profiles/<name>" from cwd
    t0 = time.time()

    # ---- 1. profile-folder fixtures
    fixtures = {}
    for folder in FOLDERS:
        devs, model = cli.load_from_profile_folder(f"test/profiles/{folder}")
        for kv in KV:
            for gap in GAPS:
                res, err, calls, out = run_solve(hp, devs, model, kv, gap)
                fixtures[f"{folder}|{kv}|{gap:g}"] = {
                    "folder": folder, "kv_bits": kv, "mip_gap": gap, "result": res, "error": err,
                    "per_k": strip_arrays(calls), "stdout": out,
                }
    cli_cases = {}
    for name, argv in {
        "hermes_default": ["--profile", "hermes_70b", "--no-plot"],
        "online_default": ["--profile", "llama_3_70b/online", "--no-plot"],
        "online_quiet": ["--profile", "llama_3_70b/online", "--no-plot", "--quiet"],
        "qwen_verbose": ["--profile", "qwen3_32b/bf16", "--no-plot", "--verbose"],
        "online_gap": ["--profile", "llama_3_70b/online", "--no-plot", "--mip-gap", "1e-9"],
    }.items():
        code, out = cli_stdout(cli, argv)
        cli_cases[name] = {"argv": argv, "code": code, "stdout": out}
    (HERE / "fixtures.json").write_text(json.dumps({"fixtures": fixtures, "cli": cli_cases}, indent=1))
    print(f"fixtures done {time.time() - t0:.1f}s", file=sys.stderr)

    # ---- 2. synthetic fleets
    model_dict = load_model_dict()
    model = ModelProfileSplit.model_validate(model_dict).to_model_profile()
    lowered = {}
    for M, count in SYNTH.items():
        fleets = []
        for seed in range(count):
            devd = synth_fleet(seed, M)
            devs = [DeviceProfile.model_validate(d) for d in devd]
            want_arrays = {(M, seed, k) for (m_, s_, k) in LOWERED if m_ == M and s_ == seed for _ in [0]}
            res, err, calls, _ = run_solve(hp, devs, model, "4bit", 1e-4, keep_arrays=bool(want_arrays))
            for rec in calls:
                if (M, seed, rec["k"]) in want_arrays:
                    c, integ, bounds, cons = rec["arrays"]
                    key = f"M{M}_s{seed}_k{rec['k']}"
                    A_ub = np.asarray(cons[0].A)
                    nz = np.nonzero(A_ub)
                    lowered[key + "_c"] = c
                    lowered[key + "_integrality"] = integ.astype(np.uint8)
                    lowered[key + "_lb"] = np.asarray(bounds.lb, dtype=float)
                    lowered[key + "_ub"] = np.asarray(bounds.ub, dtype=float)
                    lowered[key + "_Aub_shape"] = np.array(A_ub.shape)
                    lowered[key + "_Aub_row"] = nz[0].astype(np.int32)
                    lowered[key + "_Aub_col"] = nz[1].astype(np.int32)
                    lowered[key + "_Aub_val"] = A_ub[nz]
                    lowered[key + "_bub"] = np.asarray(cons[0].ub, dtype=float)
                    lowered[key + "_Aeq"] = np.asarray(cons[1].A, dtype=float)
                    lowered[key + "_beq"] = np.asarray(cons[1].ub, dtype=float)
            fleets.append({"seed": seed, "devices": devd, "result": res, "error": err,
                           "per_k": strip_arrays(calls)})
        (HERE / f"synthetic_M{M}.json").write_text(json.dumps(
            {"M": M, "model": "llama_3_70b/online", "kv_bits": "4bit", "mip_gap": 1e-4, "fleets": fleets}))
        print(f"M={M} done {time.time() - t0:.1f}s", file=sys.stderr)
    np.savez_compressed(HERE / "lowered.npz", **lowered)


TIE_SEED0, TIE_N_EACH = 21000, 20  # tests/ties.py tied_fleets(20): 60 fleets
TIE_MODELS = {"llama_3_70b/online": None, "qwen3_32b/bf16": "test/profiles/qwen3_32b/bf16/model_profile.json"}


def tied_fleet_dicts(synth_fleet, tpl):
    """[(kind, seed, device dicts)] built exactly as tests/ties.py tied_fleets() builds its fleets."""
    import copy

    out = []
    for s in range(TIE_N_EACH):
        src = synth_fleet(TIE_SEED0 + s, 16, tpl)
        one = src[s % 2]
        out.append(("copies", s, [copy.deepcopy(one) for _ in range(16)]))
        out.append(("two", s, [copy.deepcopy(src[1]) for _ in range(8)] + [copy.deepcopy(src[2 + s % 14]) for _ in range(8)]))
        out.append(("half", s, copy.deepcopy(src[:8] + src[:8])))
    return out


def gen_ties():
    hp, cli, DeviceProfile, ModelProfileSplit = import_reference()
    sys.path.append(str(REPO))
    from distilp_amd.synth import load_model_dict, load_templates, synth_fleet  # our generator (data only)

    os.chdir(REF_ROOT)
    t0 = time.time()
    twice = {}
    for folder in FOLDERS:
        base = Path("test/profiles") / folder
        dev = sorted(p for p in base.glob("*.json") if p.name != "model_profile.json")[0]
        devs, model = cli.load_devices_and_model([str(dev), str(dev)], str(base / "model_profile.json"))
        for kv in KV:
            for gap in GAPS:
                res, err, calls, _ = run_solve(hp, devs, model, kv, gap)
                twice[f"{folder}|{kv}|{gap:g}"] = {"folder": folder, "device_file": dev.name, "kv_bits": kv,
                                                   "mip_gap": gap, "result": res, "error": err,
                                                   "per_k": strip_arrays(calls)}
    print(f"twice done {time.time() - t0:.1f}s", file=sys.stderr)
    tpl = load_templates()
    fleets = tied_fleet_dicts(synth_fleet, tpl)
    tied = {}
    for mname, mfile in TIE_MODELS.items():
        if mfile is None:
            model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
        else:
            model = cli.load_model_profile(mfile)
        rows = []
        for kind, seed, dicts in fleets:
            devs = [DeviceProfile.model_validate(d) for d in dicts]
            res, err, calls, _ = run_solve(hp, devs, model, "4bit", 1e-4)
            rows.append({"kind": kind, "seed": seed, "result": res, "error": err, "per_k": strip_arrays(calls)})
        tied[mname] = {"model": mname, "kv_bits": "4bit", "mip_gap": 1e-4, "fleets": rows}
        print(f"tied {mname} done {time.time() - t0:.1f}s", file=sys.stderr)
    (HERE / "ties.json").write_text(json.dumps({"twice": twice, "tied": tied, "seed0": TIE_SEED0,
                                                "n_each": TIE_N_EACH}))


if __name__ == "__main__":
    if sys.argv[1:] == ["ties"]:
        gen_ties()
    else:
        main()
