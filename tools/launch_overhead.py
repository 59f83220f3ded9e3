"""Diagnostic: host time per k-sweep enqueue -- the prepared plan (DeviceFleetTable.launch ->
halda_fleets_plan_launch) against halda_solve_fleets per call (launch_unplanned) and a bare ctypes call
(halda_version) -- and the wall time per C3 / C2 step, one stream and two alternating streams.
   python tools/launch_overhead.py"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_timing(False)
    model = bench.load_model()
    lib = ctx.lib
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        lib.halda_version()
    print(f"bare ctypes call (halda_version): {(time.perf_counter() - t0) / n * 1e6:.2f} us", flush=True)
    for M in (64, 16):
        table = fleet_table(bench.build_fleets(range(4096), M), model)
        dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(16)]
        ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        for how in ("plan", "unplanned", "plan", "unplanned"):
            for nstreams in (1, 2):
                go = [(d.launch if how == "plan" else d.launch_unplanned) for d in dts]
                for i in range(2 * len(ss)):
                    go[i % 16](ctx, ss[i % nstreams].cuda_stream)
                torch.cuda.synchronize(dev)
                for steps in (20, 200):
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for i in range(steps):
                        go[i % 16](ctx, ss[i % nstreams].cuda_stream)
                    t1 = time.perf_counter()
                    torch.cuda.synchronize(dev)
                    t2 = time.perf_counter()
                    print(f"M={M} {how:9s} streams {nstreams} steps {steps:3d}: host enqueue "
                          f"{(t1 - t0) / steps * 1e6:.2f} us/launch, wall {(t2 - t0) / steps * 1e6:.2f} us/step",
                          flush=True)


if __name__ == "__main__":
    main()
