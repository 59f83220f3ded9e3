"""Diagnostic: wave timeline of halda_screen_k1_kernel from a -DHALDA_STAMPS build.

  hipcc ... -DHALDA_STAMPS [-DHALDA_STAMPS_DECODE] -o build/variants/libhalda_stamps.so distilp_amd/csrc/halda.hip
  HALDA_LIB=build/variants/libhalda_stamps.so python tools/k1_timeline.py [--fleets 4096] [--ks 1,2,...]

Per wave (= instance): slot 7 shader clock and slot 8 constant 100 MHz clock at wave start, slot 9
100 MHz clock at wave end; k = 1 survivors also stamp slots 0..6 inside solve_k1 (shader clock:
0 start, 1 decode done [or decode round trips with HALDA_STAMPS_DECODE], 4/5 around k1_alloc,
6 output written). Prints the kernel span, wave lifetimes of settled and solved instances, the
phase split of a solve (converted to µs with the measured shader clock), and when waves start."""

import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def pct(a, ps=(10, 50, 90)):
    return " ".join(f"p{p} {np.percentile(a, p):8.2f}" for p in ps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fleets", type=int, default=4096)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--ks", type=str, default="")
    ap.add_argument("--decode", action="store_true", help="library built with -DHALDA_STAMPS_DECODE")
    args = ap.parse_args()
    import bench
    from distilp_amd.solver._libhalda import get_context, load_library

    ks = [int(k) for k in args.ks.split(",")] if args.ks else None
    model, lowered, batch, refs = bench.build_workload(0, args.fleets, args.M, ks)
    ctx = get_context(0)
    for _ in range(3):
        res = ctx.solve(batch)
    lib = load_library()
    n = min(batch.n_inst, 65536)
    K = 12
    buf = (ctypes.c_ulonglong * (K * n))()
    lib.halda_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.halda_debug_stamps(buf, n)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, K).astype(np.int64)
    solved = (res.status[:n] == 0) & (np.array([r.k for r in refs[:n]]) == 1)
    t0 = st[:, 8].min()
    start_us = (st[:, 8] - t0) / 100.0
    end_us = (st[:, 9] - t0) / 100.0
    life = end_us - start_us
    print(f"instances {n}: solved k=1 {solved.sum()}, settled/other {(~solved).sum()}")
    print(f"kernel span (first wave start -> last wave end) {end_us.max():.2f} us")
    if (~solved).any():
        print(f"settled wave lifetime us: {pct(life[~solved])}")
    print(f"solved  wave lifetime us: {pct(life[solved])}")
    if (~solved).any():
        print(f"settled wave start us:    {pct(start_us[~solved], (0, 10, 50, 90, 100))}")
    print(f"solved  wave start us:    {pct(start_us[solved], (0, 10, 50, 90, 100))}")
    s = st[solved]
    cyc = s[:, 6] - s[:, 7]
    rt = (s[:, 9] - s[:, 8]) / 100.0
    ghz = np.median(cyc / np.maximum(rt, 1e-3)) / 1e3
    print(f"shader clock ~{ghz:.2f} GHz (median cycles / realtime)")
    to_us = 1.0 / (ghz * 1e3)
    if args.decode:
        parts = [("screen", 7, 0), ("decode RT1", 0, 1), ("decode RT2..", 1, 2), ("cap rows", 2, 3),
                 ("cycle half 1", 3, 4), ("cycle half 2", 4, 5), ("alloc+out", 5, 6)]
    else:
        parts = [("screen", 7, 0), ("decode", 0, 1), ("alloc", 4, 5), ("output", 5, 6)]
    for nm, a, b in parts:
        d = (s[:, b] - s[:, a]) * to_us
        print(f"  {nm:13s} us: {pct(d)}   share {d.sum() / (cyc * to_us).sum():.3f}")
    # concurrency: how many waves are alive at time t (sampled)
    ts = np.linspace(0, end_us.max(), 12)
    alive = [int(((start_us <= t) & (end_us > t)).sum()) for t in ts]
    alive_s = [int(((start_us <= t) & (end_us > t) & solved).sum()) for t in ts]
    print("alive waves over time (t us: all/solved): " +
          ", ".join(f"{t:.0f}: {a}/{b}" for t, a, b in zip(ts, alive, alive_s)))


if __name__ == "__main__":
    main()
