"""Diagnostic: greedy rounds of the k = 1 solves of the C3 fleets (CSR pipeline: nodes = rounds).
   python tools/k1_rounds.py [--fleets 4096] [--M 64]"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fleets", type=int, default=4096)
    ap.add_argument("--M", type=int, default=64)
    args = ap.parse_args()
    import bench
    from distilp_amd.solver._libhalda import get_context

    model, lowered, batch, refs = bench.build_workload(0, args.fleets, args.M)
    res = get_context(0).solve(batch)
    ks = np.array([r.k for r in refs])
    sel = (ks == 1) & (res.status == 0)
    nd = res.nodes[sel]
    print(f"k=1 solves {sel.sum()}: rounds mean {nd.mean():.2f} p50 {np.median(nd):.0f} p90 "
          f"{np.percentile(nd, 90):.0f} max {nd.max()}; histogram {np.bincount(nd)[:20].tolist()}")


if __name__ == "__main__":
    main()
