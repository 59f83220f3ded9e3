"""Diagnostic: where a short timed region's fixed cost goes (bench.py's headline at --steps 20): host
wall vs the GPU span (a HIP event before the first launch, events after the last launch on both streams)
vs steps x the steady-state step.   python tools/ramp.py"""
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
    ss = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(4096), 64), model)
    dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(16)]
    for i in range(8):
        dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    for steps in (20, 200, 20, 200, 20):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev[0].record(ss[0])
        ss[1].wait_event(ev[0])  # (a no-op wait: keeps both streams' spans from the same start)
        t1 = time.perf_counter()
        for i in range(steps):
            dts[i % 16].launch(ctx, ss[i % 2].cuda_stream)
        t2 = time.perf_counter()
        ev[1].record(ss[0])
        ev[2].record(ss[1])
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        gpu = max(ev[0].elapsed_time(ev[1]), ev[0].elapsed_time(ev[2])) * 1e3
        print(f"steps {steps:3d}: host wall {(t3 - t0) * 1e6:8.1f} us  (events {(t1 - t0) * 1e6:.1f}, enqueue "
              f"{(t2 - t1) * 1e6:.1f})  GPU span {gpu:8.1f} us = {gpu / steps:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
