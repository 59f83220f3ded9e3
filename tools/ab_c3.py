"""Diagnostic: C3 k-sweep timings of the library HALDA_LIB points at -- one launch (HIP events around 200
back-to-back launches on one stream), the two-stream step (200 and 20 steps, wall), and the group launch
of bench.py's headline (K batches in one halda_fleets_group_launch: wall per step at K = 200 and 20, and
the launch's own HIP-event time) -- for A/B runs of build variants:
    HALDA_LIB=build/variants/x.so python tools/ab_c3.py [--M 64]"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [int(k) for k in os.environ.get("HALDA_AB_KS", "1,2,4,5,8,10,16,20,40").split(",")]  # (diagnostic override)


def main():
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, PlanGroup, fleet_table

    M = int(sys.argv[sys.argv.index("--M") + 1]) if "--M" in sys.argv else 64
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_timing(False)
    ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(4096), M), model)
    dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(16)]
    for i in range(8):
        dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(ss[0])
    for i in range(200):
        dts[i % 16].launch(ctx, ss[0].cuda_stream)
    e1.record(ss[0])
    torch.cuda.synchronize(dev)
    out = {"lib": os.environ.get("HALDA_LIB", "default"), "M": M, "ks": KS, "one_launch_us": e0.elapsed_time(e1) / 200 * 1e3}
    for steps in (200, 20, 200, 20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(steps):
            dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        out.setdefault(f"two_stream_{steps}_us", []).append((time.perf_counter() - t0) / steps * 1e6)
    group = PlanGroup(dts, ctx)
    out["persistent"] = group.persistent
    group.launch(0, 20, ss[0].cuda_stream)
    for steps in (200, 20, 200, 20):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        group.launch(0, steps, ss[0].cuda_stream)
        torch.cuda.synchronize(dev)
        out.setdefault(f"group_{steps}_us", []).append((time.perf_counter() - t0) / steps * 1e6)
        e0.record(ss[0])
        group.launch(0, steps, ss[0].cuda_stream)
        e1.record(ss[0])
        torch.cuda.synchronize(dev)
        out.setdefault(f"group_{steps}_event_us_per_step", []).append(e0.elapsed_time(e1) / steps * 1e3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
