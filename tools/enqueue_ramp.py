"""Diagnostic: the host time of each enqueue in a bench-like timed region (C3 k-sweep, resident tables
rotating over copies, two streams), to see whether the first steps after the synchronize cost more.
  python tools/enqueue_ramp.py [--steps 20] [--warmup 5]"""
import argparse
import math
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--pin", action="store_true", help="pin this process to one core, GC off")
    ap.add_argument("--spin-flags", action="store_true", help="hipSetDeviceFlags(hipDeviceScheduleSpin) first")
    ap.add_argument("--hot-us", type=float, default=0.0, help="busy-wait this long on the host before each region")
    args = ap.parse_args()
    if args.spin_flags:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(1))
    if args.pin:
        import gc
        import os
        gc.disable()
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(4096), 64), model)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    srefs = [s1.cuda_stream, s2.cuda_stream]
    n_sw = max(2, min(32, math.ceil(2 * bench.MALL_BYTES / DeviceFleetTable(table, model, bench.KS_L80, 0.5, dev).nbytes())))
    sweeps = [DeviceFleetTable(table, model, bench.KS_L80, 0.5, dev) for _ in range(n_sw)]
    for t in sweeps:
        t.plan(ctx)
    turn = [0]

    def step():
        sweeps[turn[0] % n_sw].launch(ctx, srefs[turn[0] % 2])
        turn[0] += 1

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    for r in range(args.rounds):
        torch.cuda.synchronize(dev)
        if args.hot_us:
            th = time.perf_counter_ns() + int(args.hot_us * 1e3)
            while time.perf_counter_ns() < th:
                pass
        ts = []
        t0 = time.perf_counter_ns()
        for _ in range(args.steps):
            step()
            ts.append(time.perf_counter_ns())
        t_enq = time.perf_counter_ns()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter_ns()
        d = [(b - a) / 1e3 for a, b in zip([t0] + ts[:-1], ts)]
        print(f"round {r}: n_sw {n_sw}; enqueue us per step {[round(x, 1) for x in d]}; "
              f"enqueue total {(t_enq - t0) / 1e3:.1f} us, wall {(t1 - t0) / 1e3:.1f} us = {(t1 - t0) / 1e3 / args.steps:.2f} us/step")


if __name__ == "__main__":
    main()
