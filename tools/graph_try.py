"""Diagnostic: the C3 k-sweep steps captured into one HIP graph (torch.cuda.CUDAGraph over the library's
launches, the two streams as forked branches) against the same steps launched one by one.
  python tools/graph_try.py [--steps 20]"""
import argparse
import math
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, PlanRotation, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(4096), 64), model)
    sa = torch.cuda.Stream(dev)
    sb = torch.cuda.Stream(dev)
    n_sw = max(2, min(32, math.ceil(2 * bench.MALL_BYTES / DeviceFleetTable(table, model, bench.KS_L80, 0.5, dev).nbytes())))
    sweeps = [DeviceFleetTable(table, model, bench.KS_L80, 0.5, dev) for _ in range(n_sw)]
    for t in sweeps:
        t.plan(ctx)
    rot = PlanRotation(sweeps, ctx, [sa.cuda_stream, sb.cuda_stream])
    ctx.set_timing(False)
    for i in range(4):
        rot.launch(i, 1)
    torch.cuda.synchronize(dev)
    K = args.steps

    def loop():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rot.launch(0, K)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / K * 1e6

    # capture: branch A (even steps) on sa, branch B (odd steps) on sb, forked from sa and joined back
    g = torch.cuda.CUDAGraph()
    ra = PlanRotation(sweeps, ctx, [sa.cuda_stream])
    rb = PlanRotation(sweeps, ctx, [sb.cuda_stream])
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(g, stream=sa):
        fork = torch.cuda.Event()
        fork.record(sa)
        sb.wait_event(fork)
        for i in range(K):
            (ra if i % 2 == 0 else rb).launch(i, 1)
        join = torch.cuda.Event()
        join.record(sb)
        sa.wait_event(join)
    torch.cuda.synchronize(dev)

    def replay():
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / K * 1e6

    for r in range(args.rounds):
        print(f"round {r}: launches {loop():.2f} us/step   graph {replay():.2f} us/step")


if __name__ == "__main__":
    main()
