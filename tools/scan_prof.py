"""Diagnostic: where an event of the k-slot kernel's split threshold scan spends its cycles (C2 shape),
from a -DHALDA_STAMPS build (kc_scan_incremental's HALDA_SCANPROF sites, part 1 = the k = 2 wave).

  HALDA_LIB=build/variants/libhalda_stamps.so python tools/scan_prof.py [--fleets 4096]

Per segment (fleet) of the k = 2 wave: shader cycles summed over its scan events, split into the
steps of an event: (0) the useful-opening test + min reduction + stop test, (1) the pick (lowest) +
broadcast of its unit, (2) the LDS round trip of li / lj, (3) the max reduction (lam) + highest,
(4) the objective update; per event and in total, percentiles over the fleets."""
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
    dt = DeviceFleetTable(table, model, KS, 0.5, dev)
    for _ in range(3):
        dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    lib = load_library()
    slots = [k for k in KS if 80 // k >= args.M]
    groups = (args.fleets + 3) // 4
    n = groups * len(slots)
    buf = (ctypes.c_ulonglong * (64 * n))()
    lib.halda_debug_scanprof.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.halda_debug_scanprof(buf, n)
    pr = np.frombuffer(buf, dtype=np.uint64).reshape(groups, len(slots), 4, 16).astype(np.int64)
    j = slots.index(2)
    q = [10, 50, 90, 99]
    names = ["min reduction + tests", "lowest + bcast", "LDS round trip", "max reduction + highest", "update"]
    pre = ["T0 + caps at T0", "split cut", "greedy at T0", "S / openings / lam", "loop exit", "helper wait"]
    # per wave: the segment with the most events (the wave runs its segments in lockstep)
    ev = pr[:, j, :, 15]
    top = ev.argmax(axis=1)
    p = pr[np.arange(groups), j, top]
    ok = p[:, 15] > 0
    p = p[ok]
    e = p[:, 15]
    print(f"k = 2 part-1 waves with events: {len(p)}; events of the longest segment {np.percentile(e, q)}")
    tot = p[:, :11].sum(axis=1)
    print(f"  scan cycles (longest segment) {np.percentile(tot, q)}")
    for t, nm in enumerate(names):
        print(f"  event: {nm:26s} per event: median {np.median(p[:, t] / e):7.0f}  p90 {np.percentile(p[:, t] / e, 90):7.0f}"
              f"   total median {np.median(p[:, t]):7.0f}")
    for t, nm in enumerate(pre):
        print(f"  {nm:33s} median {np.median(p[:, 5 + t]):7.0f}  p90 {np.percentile(p[:, 5 + t], 90):7.0f}")
    for t, nm in ((11, "leaf scan (dp_pass_lanes)"), (12, "leaf checks (ballots)"), (13, "phase-0 greedy")):
        print(f"  {nm:33s} median {np.median(p[:, t]):7.0f}  p90 {np.percentile(p[:, t], 90):7.0f}")
    # barrier -> dp_pass_lanes entry, from the kernel's own stamp 11 (after the tables barrier)
    K = 12
    sb = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.halda_debug_stamps(sb, n)
    st = np.frombuffer(sb, dtype=np.uint64).reshape(groups, len(slots), K).astype(np.int64)
    gap = p[:, 14] - st[np.arange(groups), j, 11][ok]
    print(f"  {'barrier -> dp_pass_lanes entry':33s} median {np.median(gap):7.0f}  p90 {np.percentile(gap, 90):7.0f}")

if __name__ == "__main__":
    main()
