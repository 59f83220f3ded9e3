"""Diagnostic: median time of each step of halda_solve_batch on the 4096 C3 fleets (host and GPU parts).
   python tools/batch_parts.py [--fleets 4096] [--M 64]"""
import argparse
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, n=5):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fleets", type=int, default=4096)
    ap.add_argument("--M", type=int, default=64)
    args = ap.parse_args()
    import bench
    from distilp_amd.solver import halda as H
    from distilp_amd.solver.fleets import fleet_constants, fleet_table, solve_table

    model = bench.load_model()
    fleets = bench.build_fleets(range(args.fleets), args.M)
    ks = bench.KS_L80
    table = fleet_table(fleets, model)
    out = {}
    out["fleet_table (C packer)"] = timeit(lambda: fleet_table(fleets, model))
    out["fleet_constants"] = timeit(lambda: fleet_constants(table, model))
    out["solve_table (PCIe in, sweep, PCIe out)"] = timeit(lambda: solve_table(table, model, ks, 0.5, want_x="open"))
    out["halda_solve_batch total"] = timeit(lambda: H.halda_solve_batch(fleets, model, kv_bits="4bit"))
    for k, v in out.items():
        print(f"{k:40s} {v:8.2f} ms")


if __name__ == "__main__":
    main()
