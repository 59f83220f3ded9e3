"""Diagnostic: one M = 64 fleet's k-sweep through halda_solve_fleets_host (the single halda_solve
path: zero-copy pinned table, polled completion), per output variant, host wall time and the
kernel's HIP-event time; plus the same fleet from a device-resident table (no PCIe in the kernel).
   python tools/one_fleet_time.py"""
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, n=300):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts)


def main():
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table, solve_table

    model = bench.load_model()
    devs = bench.build_fleets([0], 64)[0]
    ks = bench.KS_L80
    table = fleet_table([devs], model)
    ctx = get_context(0)
    for name, wx in (("no x", False), ("x all k (dense)", True), ("x open k only", "open")):
        us = timeit(lambda: solve_table(table, model, ks, 0.5, want_x=wx))
        ctx.set_timing(True)
        solve_table(table, model, ks, 0.5, want_x=wx)
        ms = ctx.last_fleet_ms()
        ctx.set_timing(False)
        print(f"solve_table {name:18s} {us:7.1f} us wall; launches {ms}")
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    dt = DeviceFleetTable(table, model, ks, 0.5, dev)

    def dev_one():
        dt.launch(ctx, s.cuda_stream)
        s.synchronize()

    us = timeit(dev_one)
    ctx.set_timing(True)
    dev_one()
    print(f"device-resident table, stream sync {us:7.1f} us wall; launches {ctx.last_fleet_ms()}")
    ctx.set_timing(False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(100):
        dt.launch(ctx, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize(dev)
    print(f"device-resident table, 100 back-to-back launches: {e0.elapsed_time(e1) * 10:.1f} us each")


if __name__ == "__main__":
    main()
