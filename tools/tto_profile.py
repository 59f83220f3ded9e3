"""Diagnostic: where the time of one M = 64 halda_solve goes (cProfile over 200 calls + the GPU
launch times of the last call).   python tools/tto_profile.py"""
import contextlib
import cProfile
import io
import pstats
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import bench
    from distilp_amd.solver import halda_solve
    from distilp_amd.solver._libhalda import get_context

    model = bench.load_model()
    devs = bench.build_fleets([0], 64)[0]
    for _ in range(10):
        with contextlib.redirect_stdout(io.StringIO()):
            halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits="4bit")
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits="4bit")
        ts.append((time.perf_counter() - t0) * 1e3)
    print("median ms", statistics.median(ts))
    print("launch ms", get_context(0).last_fleet_ms())
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        with contextlib.redirect_stdout(io.StringIO()):
            halda_solve(devs, model, mip_gap=1e-4, plot=False, kv_bits="4bit")
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
