"""Diagnostic (CPU): the k > 1 tables G_i(e), H_i(e) of one fleet restated from the dense lowering
(oracle/milp_oracle.py lower_dense: least slacks per (w, n), least-cost n with ties to the smallest n,
least cycle time H = max(P, (P + Q) / 2) at it), and the scan model (tools/scan_model.py) on them.
Wrote tests/golden/tie_tables_qwen3_half_k2.npz (fleet 15 of test_gpu_ties.py's qwen3_32b batch, k = 2):
   python tools/tie_tables.py [out.npz]"""
import math
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))


def tables(p, M, W):
    A, b, c, lb, ub = p["A_ub"], p["b_ub"], p["c"], p["lb"], p["ub"]
    iC, R1 = 7 * M, W - M + 1
    G, H = np.full((M, R1), np.inf), np.full((M, R1), np.inf)
    for i in range(M):
        rows = [r for r in range(A.shape[0]) if any(A[r, blk * M + i] != 0 for blk in range(7))]
        cyc = [r for r in rows if A[r, iC] != 0]
        cap = [r for r in rows if A[r, iC] == 0]
        for e in range(R1):
            w, best = 1 + e, None
            for n in range(0, min(w, int(ub[M + i])) + 1):
                x = np.zeros(A.shape[1])
                x[i], x[M + i] = w, n
                ok = True
                for r in cap:
                    sl = [blk for blk in range(2, 6) if A[r, blk * M + i] != 0]
                    act = A[r, i] * w + A[r, M + i] * n
                    if not sl:
                        ok = ok and act <= b[r] + 1e-9 * max(1, abs(b[r]))
                        continue
                    j = sl[0] * M + i
                    x[j] = max(x[j], math.ceil((act - b[r]) / -A[r, j] - 1e-9))
                for blk in range(2, 6):
                    j = blk * M + i
                    x[j] = max(x[j], lb[j])
                    ok = ok and x[j] <= ub[j]
                if ok:
                    g = sum(c[blk * M + i] * x[blk * M + i] for blk in range(6))
                    if best is None or g < best[0]:
                        best = (g, x.copy())
            if best is None:
                continue
            g, x = best
            P, Q = (sum(A[r, blk * M + i] * x[blk * M + i] for blk in range(6)) - b[r] for r in cyc)
            if A[cyc[0], 6 * M + i] < 0:
                P, Q = Q, P
            G[i, e], H[i, e] = g, max(P, (P + Q) / 2)
    return G, H


def main(out=None):
    import scan_model as sm
    from oracle import milp_oracle as mo
    from tests.ties import fixture_twice, tied_fleets

    twice, model = fixture_twice("qwen3_32b/bf16")
    devs = ([twice] + [d for _, d in tied_fleets(24)])[15]
    k, M = 2, len(devs)
    W = model.L // k
    p = mo.lower_dense(devs, model, k, 0.5)
    st, _, b1, _, _ = mo.exact_solve(p)
    G, H = tables(p, M, W)
    print("exact oracle", st, b1, "scan model", sm.model(G, H, k - 1, W))
    if out:
        np.savez(out, G=G, H=H)


if __name__ == "__main__":
    main(*sys.argv[1:])
