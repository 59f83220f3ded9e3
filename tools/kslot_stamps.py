"""Diagnostic: per-slot phase times of the k-slot kernel (C2 shape) from a -DHALDA_STAMPS build.

  HALDA_LIB=build/variants/libhalda_stamps.so python tools/kslot_stamps.py [--M 16] [--fleets 4096]

Per k-slot wave (one k for four fleets): records (field loads, records, constants), solve (the k's
greedy / tables + threshold scan, outputs), the wait at the workgroup barrier, and the pick (slot 0);
shader-clock cycles, percentiles over the workgroups; plus the wave-start spread (100 MHz clock).
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
    dt = DeviceFleetTable(table, model, KS, 0.5, dev)
    for _ in range(3):
        dt.launch(ctx, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ms = ctx.last_fleet_ms() if False else None
    lib = load_library()
    slots = [k for k in KS if 80 // k >= args.M]
    groups = (args.fleets + 3) // 4
    n = groups * len(slots)
    K = 12
    buf = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.halda_debug_stamps(buf, n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(groups, len(slots), K).astype(np.int64)
    q = [10, 50, 90, 99]
    print(f"{groups} workgroups x {len(slots)} k-slots {slots}; shader-clock cycles, percentiles {q}")
    for j, k in enumerate(slots):
        s = st[:, j]
        print(f"  k={k:3d} records {np.percentile(s[:, 1] - s[:, 0], q)}  table share {np.percentile(s[:, 6] - s[:, 1], q)}"
              f"  wait for tables {np.percentile(s[:, 11] - s[:, 6], q)}  solve {np.percentile(s[:, 2] - s[:, 11], q)}"
              f"  barrier wait {np.percentile(s[:, 3] - s[:, 2], q)}")
    for j, k in enumerate(slots):
        s = st[:, j]
        if (s[:, 9] > 0).all():
            print(f"  k={k:3d} leaf scan {np.percentile(s[:, 9] - s[:, 11], q)}"
                  f"  phase-0 greedy {np.percentile(s[:, 10] - s[:, 9], q)}  threshold scan "
                  f"{np.percentile(s[:, 7] - s[:, 10], q)}  output {np.percentile(s[:, 2] - s[:, 7], q)}  "
                  f"scan events (segment 0) {np.percentile(s[:, 8], q)}")
    s0 = st[:, 0]
    print(f"  pick (slot 0) {np.percentile(s0[:, 4] - s0[:, 3], q)}")
    life = st[:, :, 4].max(axis=1) - st[:, :, 0].min(axis=1)
    print(f"  workgroup life {np.percentile(life, q)}")
    # the slowest workgroups (they set the launch): each slot wave's phases, and the k = 2 wave's steps
    t0 = st[:, :, 0].min(axis=1)
    for g in np.argsort(life)[-6:][::-1]:
        parts = []
        for j, k in enumerate(slots):
            s = st[g, j] - t0[g]
            parts.append(f"k={k}: rec {s[1]} tab {s[6]} bar {s[11]} solved {s[2]}")
        line = f"  wg {g} life {life[g]}: " + " | ".join(parts)
        if 2 in slots:
            s = st[g, slots.index(2)]
            line += (f" || k=2 leaf {s[9] - s[11]} ph0 {s[10] - s[9]} scan {s[7] - s[10]} ev {s[8]}"
                     f" out {s[2] - s[7]}")
        print(line)
    t0 = st[:, :, 5] & ((1 << 40) - 1)
    print(f"  wave start spread (10 ns ticks) {np.percentile(t0 - t0.min(), [0, 10, 50, 90, 100])}")
    hw = (st[:, :, 5] >> 40) & 0xFFFF  # HW_ID[15:0]: wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]
    xcc = (st[:, :, 5] >> 56) & 0xF
    simd = (hw >> 4) & 3
    for j, k in enumerate(slots):
        print(f"  k={k:3d} waves per SIMD id {np.bincount(simd[:, j], minlength=4).tolist()}")
    same = (simd[:, :, None] == simd[:, None, :]).sum(axis=(1, 2)) - len(slots)
    print(f"  workgroups whose slot waves share a SIMD: {int((same > 0).sum())} of {groups}")
    # chip-wide SIMD key (XCC, SE, SH, CU, SIMD): how many waves of each k-slot share one SIMD
    key = (xcc << 16) | (hw >> 4)
    for j, k in enumerate(slots):
        _, cnt = np.unique(key[:, j], return_counts=True)
        print(f"  k={k:3d} waves sharing one SIMD: {np.bincount(cnt).tolist()} (index = waves on the SIMD)")
    _, cnt = np.unique(key.ravel(), return_counts=True)
    print(f"  all slot waves per SIMD: {np.bincount(cnt).tolist()}; SIMDs used {len(cnt)}")


if __name__ == "__main__":
    main()
