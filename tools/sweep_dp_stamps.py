"""Diagnostic: per-k phase costs (shader cycles) of the fused sweep's table path from a
-DHALDA_STAMPS -DHALDA_STAMPS_DP build (per-instance stamps, instance = fleet * n_k + j).

  HALDA_LIB=build/variants/libhalda_stamps_dp.so python tools/sweep_dp_stamps.py [--M 16] [--fleets 4096]
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
    ap.add_argument("--M", type=int, default=16)
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
    dt = DeviceFleetTable(table, model, KS, 0.5, dev, want_per_k=True)
    lib = load_library()
    K = 12
    n = min(args.fleets * len(KS), 65536)
    buf = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(3):
        dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    lib.halda_debug_stamps(buf, n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, K).astype(np.int64)
    status = dt.out["status"].cpu().numpy()[:n]
    for j, k in enumerate(KS):
        sel = (np.arange(n) % len(KS) == j) & (status == 0) & (st[:, 0] > 0) & (st[:, 8] > st[:, 0])
        if not sel.any():
            continue
        s = st[sel]
        ph = {"table": s[:, 6] - s[:, 0], "dp": s[:, 7] - s[:, 6], "output": s[:, 8] - s[:, 7],
              "total": s[:, 8] - s[:, 0]}
        kc = (s[:, 5] > s[:, 6])
        if kc.any():
            t = s[kc]
            ph.update({"phase0": t[:, 1] - t[:, 6], "hmax": t[:, 2] - t[:, 1], "scan_setup": t[:, 3] - t[:, 2],
                       "alloc0": t[:, 4] - t[:, 3], "events": t[:, 5] - t[:, 4]})
        print(f"k={k:3d} n={sel.sum():5d} " + "  ".join(f"{a}={np.median(b):.0f}" for a, b in ph.items()))


if __name__ == "__main__":
    main()
