"""Diagnostic: median time of each step of one M = 64 halda_solve (host and GPU parts).
   python tools/tto_parts.py"""
import contextlib
import io
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, n=300):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(ts)


def main():
    import numpy as np

    import bench
    from distilp_amd.solver import halda as H
    from distilp_amd.solver.coefficients import HALDAResult, ILPResult, assign_sets
    from distilp_amd.solver.fleets import fleet_table, solve_table
    from distilp_amd.solver._libhalda import get_context

    model = bench.load_model()
    devs = bench.build_fleets([0], 64)[0]
    ks = [1, 2, 4, 5, 8, 10, 16, 20, 40]
    sets = assign_sets(devs)
    table = fleet_table([devs], model)
    res = solve_table(table, model, ks, 0.5, want_x=True)
    out = {}
    out["valid_factors+kv+sets"] = timeit(lambda: (H._k_list(model, ks), H.kv_bits_to_factor("4bit"), assign_sets(devs)))
    out["offset_parts(kappa)"] = timeit(lambda: H._offset_parts(devs, model, sets))
    out["fleet_table"] = timeit(lambda: fleet_table([devs], model))
    out["solve_table(GPU round trip)"] = timeit(lambda: solve_table(table, model, ks, 0.5, want_x=True))
    ctx = get_context(0)
    out["  of which C call"] = 0.0

    def post():
        M, N = 64, 449
        x = np.array(res.x[0, 0, :N])
        c = np.array(res.c[0, 0, :N])
        obj = float(c.dot(x))
        wn = np.rint(x[:2 * M]).astype(np.int64).tolist()
        return ILPResult(k=1, w=wn[:M], n=wn[M:], obj_value=obj)

    out["per-k result (1 feasible k)"] = timeit(post)
    r = post()
    out["HALDAResult"] = timeit(lambda: HALDAResult(w=list(r.w), n=list(r.n), k=1, obj_value=r.obj_value,
                                                    sets={k: list(v) for k, v in sets.items()}))
    with contextlib.redirect_stdout(io.StringIO()):
        out["halda_solve total"] = timeit(lambda: H.halda_solve(devs, model, k_candidates=ks, plot=False, kv_bits="4bit"))
    for k, v in out.items():
        print(f"{k:32s} {v:8.1f} us")
    print("launch ms", ctx.last_fleet_ms())


if __name__ == "__main__":
    main()
