"""Device time of halda_solve_fleets on the fused sweep vs the CSR pipeline for C2 / C3 shapes
(and any --M / --fleets), from resident device tables; prints one JSON line per (shape, path).

  python tools/sweep_time.py [--M 64,16] [--fleets 4096] [--iters 20]
"""

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=str, default="64,16")
    ap.add_argument("--fleets", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--paths", type=str, default="fused,wave,csr")
    args = ap.parse_args()
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    model = bench.load_model()
    for M in [int(m) for m in args.M.split(",")]:
        table = fleet_table(bench.build_fleets(range(args.fleets), M), model)
        dts = [DeviceFleetTable(table, model, KS, 0.5, dev) for _ in range(4)]
        ref = None
        for path in args.paths.split(","):
            ctx.set_fleets_path(path)
            for i in range(3):
                dts[i % 4].launch(ctx, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            got = (dts[2].out["best_k"].cpu().numpy(), dts[2].out["w"].cpu().numpy())
            if ref is None:
                ref = got
            same = bool((ref[0] == got[0]).all() and (ref[1] == got[1]).all())
            ctx.set_timing(False)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(args.iters):
                dts[i % 4].launch(ctx, stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ctx.set_timing(True)
            per = []
            for i in range(5):
                dts[i % 4].launch(ctx, stream.cuda_stream)
                torch.cuda.synchronize(dev)
                per.append(ctx.last_fleet_ms())
            launch = {k: statistics.mean(p.get(k, 0.0) for p in per) for k in per[0]}
            ms = e0.elapsed_time(e1) / args.iters
            print(json.dumps({"M": M, "fleets": args.fleets, "path": path, "ms_per_sweep": ms,
                              "instances_per_s": args.fleets * len(KS) / (ms * 1e-3), "launch_ms": launch,
                              "same_as_first_path": same}), flush=True)
        ctx.set_fleets_path(True)


if __name__ == "__main__":
    main()
