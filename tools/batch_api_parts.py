"""Diagnostic: where the public batch API's time goes (halda_solve_batch on the bench's 4,096 C3 fleets):
each call's total and its parts -- fleet_table (the C packer over the DeviceProfile objects), solve_table
(the GPU k-sweep with PCIe in / out), fleet_constants, the C result builder and the NumPy rest -- median of
`--runs` warm calls.  python tools/batch_api_parts.py [--runs 5] [--threads N]"""
import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--fleets", type=int, default=4096)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    import bench
    from distilp_amd.solver import halda as H
    from distilp_amd.solver import fleets as FL

    model = bench.load_model()
    fleets = bench.build_fleets(range(a.fleets), 64)
    parts = {}

    def timed(name, fn):
        def wrap(*args, **kw):
            t0 = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                parts.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)
        return wrap

    H.fleet_table = timed("pack", H.fleet_table)
    H.solve_table = timed("gpu_sweep", H.solve_table)
    H.fleet_constants = timed("constants", H.fleet_constants)
    if H._PACKER is not None and hasattr(H._PACKER, "results"):
        real = H._PACKER

        class P:
            def __getattr__(self, k):
                return getattr(real, k)

        p = P()
        p.results = timed("results", real.results)
        H._PACKER = p
    tot = []
    for _ in range(a.runs + 1):
        t0 = time.perf_counter()
        H.halda_solve_batch(fleets, model, mip_gap=1e-4, kv_bits="4bit")
        tot.append((time.perf_counter() - t0) * 1e3)
    out = {"fleets": a.fleets, "threads": os.environ.get("HALDA_PACK_THREADS", "default"),
           "total_ms": statistics.median(tot[1:])}
    for k, v in parts.items():
        out[k + "_ms"] = statistics.median(v[1:])
    out["rest_ms"] = out["total_ms"] - sum(out[k + "_ms"] for k in parts)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
