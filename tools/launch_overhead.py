"""Diagnostic: host time per halda_solve_fleets enqueue (DeviceFleetTable.launch) vs device time per
C3 k-sweep, one stream and two alternating streams.   python tools/launch_overhead.py"""
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
    table = fleet_table(bench.build_fleets(range(4096), 64), model)
    dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(16)]
    ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for nstreams in (1, 2, 1, 2):
        for i in range(5):
            dts[i % 16].launch(ctx, ss[i % nstreams].cuda_stream)
        torch.cuda.synchronize(dev)
        n = 200
        t0 = time.perf_counter()
        for i in range(n):
            dts[i % 16].launch(ctx, ss[i % nstreams].cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        print(f"streams {nstreams}: host enqueue {(t1 - t0) / n * 1e6:.2f} us/launch, "
              f"wall {(t2 - t0) / n * 1e6:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
