"""Diagnostic: per-phase cycle shares of halda_solve_kernel from a -DHALDA_STAMPS build.

  hipcc ... -DHALDA_STAMPS -o build/variants/libhalda_stamps.so distilp_amd/csrc/halda.hip
  HALDA_LIB=build/variants/libhalda_stamps.so python tools/phase_stamps.py [--fleets 4096]

Read SHARES, not absolute time (stamps are s_memtime, shader clock)."""

import argparse
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fleets", type=int, default=4096)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--k", type=int, default=0, help="only instances of this k (0 = all)")
    ap.add_argument("--dp", action="store_true", help="library built with -DHALDA_STAMPS_DP (stamps 1..5 inside dp_pass)")
    args = ap.parse_args()
    import bench
    from distilp_amd.solver._libhalda import get_context, load_library

    model, lowered, batch, refs = bench.build_workload(0, args.fleets, args.M)
    ctx = get_context(0)
    for _ in range(3):
        res = ctx.solve(batch)
    lib = load_library()
    n = min(batch.n_inst, 65536)
    K = 12  # kStamps in halda.hip
    buf = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    got = lib.halda_debug_stamps(buf, n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, K).astype(np.int64)
    ok = res.status[:n] == 0
    if args.k:
        ok &= np.array([r.k == args.k for r in refs[:n]])
    st = st[ok]
    names = ["device", "rows", "check", "tables", "dp", "output"]
    if args.dp:  # 0 start, 1 phase-0 DP call, 2 hmax, 3 scan entry, 4 scan's first allocation, 5 scan done, 6 output done
        names = ["decode+tables+dp0", "hmax", "scan setup", "scan alloc0", "scan events", "output"]
    d = np.diff(st[:, :7], axis=1)
    d[:, 2] = st[:, 3] - st[:, 2]
    tot = st[:, 6] - st[:, 0]
    nodes = res.nodes[:n][ok]
    print("nodes (DP passes / greedy rounds): median", np.median(nodes), "max", nodes.max(), "mean", nodes.mean())
    print(f"instances {len(st)}  median total {np.median(tot):.0f} cycles")
    for j, nm in enumerate(names):
        print(f"  {nm:8s} median {np.median(d[:, j]):9.0f}  mean {d[:, j].mean():9.0f}  share {d[:, j].sum() / tot.sum():.3f}")


if __name__ == "__main__":
    main()
