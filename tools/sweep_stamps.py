"""Diagnostic: per-phase shader-clock shares of the fused sweep kernel (C3 shape) from a
-DHALDA_STAMPS build, plus the wave timeline (constant 100 MHz clock).

  HALDA_LIB=build/variants/libhalda_stamps.so python tools/sweep_stamps.py [--M 64] [--fleets 4096]
"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
KS = [1, 2, 4, 5, 8, 10, 16, 20, 40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--fleets", type=int, default=4096)
    args = ap.parse_args()
    import torch

    import bench
    from distilp_amd.solver._libhalda import get_context, load_library
    from distilp_amd.solver.fleets import DeviceFleetTable, fleet_table

    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    stream = torch.cuda.Stream(dev)
    model = bench.load_model()
    table = fleet_table(bench.build_fleets(range(args.fleets), args.M), model)
    dt = DeviceFleetTable(table, model, KS, 0.5, dev)
    for _ in range(3):
        dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    lib = load_library()
    K = 12
    n = args.fleets
    buf = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.halda_debug_stamps(buf, n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, K).astype(np.int64)
    names = ["loads+records+offsets", "to k=1", "k1_alloc", "k=1 output", "k>1 + writes", "final writes"]
    d = np.diff(st[:, :7], axis=1)
    tot = st[:, 6] - st[:, 0]
    print(f"fleets {n}  median wave life {np.median(tot):.0f} shader cycles")
    for j, nm in enumerate(names):
        print(f"  {nm:24s} median {np.median(d[:, j]):8.0f}  share {d[:, j].sum() / tot.sum():.3f}")
    t0, t1, tr = st[:, 7], st[:, 8], st[:, 9]
    base = t0.min()
    q = [0, 10, 50, 90, 99, 100]
    print(f"timeline (100 MHz ticks = 10 ns), percentiles {q}:")
    print(f"  wave start      {np.percentile(t0 - base, q)}")
    print(f"  records done    {np.percentile(tr - base, q)}")
    print(f"  wave end        {np.percentile(t1 - base, q)}")
    print(f"  records phase   {np.percentile(tr - t0, q)}")
    print(f"  after records   {np.percentile(t1 - tr, q)}")


if __name__ == "__main__":
    main()
