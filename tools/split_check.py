"""Diagnostic (GPU): the k-slot launch against the one-fleet-per-wave sweep on a mixed-size batch;
prints every (fleet, k) whose obj_by_k differs, with the fleet size.
  python tools/split_check.py [--sizes mixed|c2]"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from distilp_amd.common import DeviceProfile, ModelProfileSplit  # noqa: E402
from distilp_amd.solver._libhalda import get_context  # noqa: E402
from distilp_amd.solver.fleets import fleet_table, solve_table  # noqa: E402
from distilp_amd.synth import load_model_dict, synth_fleet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="mixed")
    a = ap.parse_args()
    sizes = [1 + (s * 7) % 16 for s in range(300)] if a.sizes == "mixed" else [16] * 200 + [12] * 57
    model = ModelProfileSplit.model_validate(load_model_dict()).to_model_profile()
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    fleets = [[DeviceProfile.model_validate(d) for d in synth_fleet(11000 + s, M)] for s, M in enumerate(sizes)]
    table = fleet_table(fleets, model)
    ctx = get_context(0)
    ctx.set_fleets_path("fused")
    seg = solve_table(table, model, ks, 0.5, want_x=True)
    ctx.set_fleets_path("wave")
    wave = solve_table(table, model, ks, 0.5, want_x=True)
    ctx.set_fleets_path("fused")
    d = np.argwhere(seg.obj_by_k != wave.obj_by_k)
    print(f"{len(d)} differing (fleet, k) of {seg.obj_by_k.size}")
    for f, j in d[:40]:
        print(f"fleet {f} M {sizes[f]} k {ks[j]} kslot {seg.obj_by_k[f, j]!r} wave {wave.obj_by_k[f, j]!r} "
              f"seg-in-wg {f % 4}")


if __name__ == "__main__":
    main()
