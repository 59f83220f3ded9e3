"""Diagnostic driver for rocprofv3 passes over the C3 headline's launches (library HALDA_LIB or the
in-tree one): `--groups` group launches of `--steps` batches each (halda_sweep_steps_kernel) and `--single`
per-batch launches on one stream (halda_sweep_kernel), on the bench's 4096 C3 fleets and 16 resident
copies. Every group launch has the same K, so per-dispatch counters divide by K x 4096 items.
    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 tools/steps_profile.py --steps 20"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--groups", type=int, default=3)
    ap.add_argument("--single", type=int, default=20)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--ks", type=str, default="", help="comma-separated k-candidates instead of L = 80's")
    ap.add_argument("--path", type=str, default="", help="HaldaContext.set_fleets_path name (test paths)")
    a = ap.parse_args()
    ks = [int(k) for k in a.ks.split(",")] if a.ks else KS
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_timing(False)
    if a.path:
        ctx.set_fleets_path(a.path)
    s = torch.cuda.Stream(dev)
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(4096), a.M), model)
    dts = [DeviceFleetTable(table, model, ks, 0.5, dev) for _ in range(16)]
    group = PlanGroup(dts, ctx)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {"steps": a.steps, "persistent": group.persistent, "group_us": [], "single_us": None}
    for g in range(a.groups):
        torch.cuda.synchronize(dev)
        e0.record(s)
        group.launch(g * a.steps, a.steps, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize(dev)
        out["group_us"].append(e0.elapsed_time(e1) * 1e3)
    e0.record(s)
    for i in range(a.single):
        dts[i % 16].launch(ctx, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize(dev)
    out["single_us"] = e0.elapsed_time(e1) * 1e3 / max(a.single, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
