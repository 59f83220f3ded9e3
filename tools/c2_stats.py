"""Diagnostic: C2-shape batch (M=16 fleets, all k of L=80): per-k DP passes (nodes) and general-kernel time."""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fleets", type=int, default=1024)
    ap.add_argument("--M", type=int, default=16)
    args = ap.parse_args()
    import bench
    from distilp_amd.solver._libhalda import get_context

    model, lowered, batch, refs = bench.build_workload(0, args.fleets, args.M)
    ctx = get_context(0)
    for _ in range(2):
        res = ctx.solve(batch)
    ph = ctx.last_phase_ms()
    ks = np.array([r.k for r in refs])
    for k in sorted(set(ks)):
        sel = ks == k
        st = res.status[sel]
        nd = res.nodes[sel][st == 0]
        if len(nd):
            print(f"k={k:3d} feasible {len(nd):5d}  nodes mean {nd.mean():7.1f}  p50 {np.median(nd):6.0f}  "
                  f"p99 {np.percentile(nd, 99):6.0f}  max {nd.max():6d}")
        else:
            print(f"k={k:3d} feasible     0")
    print("launch ms", ph)


if __name__ == "__main__":
    main()
