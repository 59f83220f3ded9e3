"""Diagnostic (CPU): a Python model of the k > 1 solve of the k-slot kernel on dumped tables
(tools/kslot_tables.py -> gpurun_out/c2_tables.npz): the phase-0 greedy, the incremental threshold
scan (kc_scan_incremental, its event count) and a brute-force min over T of kc T + S(T), to study
the scan's sequential length offline.   python tools/scan_model.py [gpurun_out/c2_tables.npz]"""
import sys

import numpy as np

INF = float("inf")


def capped_sum(G, lo, cap, need):
    """S at caps: every device at lo, then the `need` smallest increments below the caps (convex rows)."""
    inc = []
    for i in range(len(G)):
        for e in range(lo[i], cap[i]):
            inc.append(G[i][e + 1] - G[i][e])
    if len(inc) < need:
        return INF
    inc.sort()
    return sum(G[i][lo[i]] for i in range(len(G))) + sum(inc[:need])


def model(G, H, kc, W):
    M, R1 = G.shape
    fin = np.isfinite(G)
    lo = [int(np.argmax(fin[i])) for i in range(M)]
    hi = [int(R1 - 1 - np.argmax(fin[i][::-1])) for i in range(M)]
    need = (R1 - 1) - sum(lo)
    # phase 0: unconstrained
    s_inf = capped_sum(G, lo, hi, need)
    # unconstrained allocation (greedy, ties to the lowest device)
    e = list(lo)
    for _ in range(need):
        best, bi = INF, -1
        for i in range(M):
            if e[i] < hi[i]:
                d = G[i][e[i] + 1] - G[i][e[i]]
                if d < best:
                    best, bi = d, i
        e[bi] += 1
    hmax = max(max(0.0, H[i][e[i]]) for i in range(M))
    best0 = kc * hmax + s_inf
    # brute force over candidate T
    Ts = sorted(set(float(H[i][k]) for i in range(M) for k in range(lo[i], hi[i] + 1)))
    T0 = max(H[i][lo[i]] for i in range(M))
    bestF, bestT, nT = best0, None, 0
    for T in Ts:
        if T < T0:
            continue
        if kc * T + s_inf >= bestF:
            break
        nT += 1
        cap = [max(k for k in range(lo[i], hi[i] + 1) if H[i][k] <= T) for i in range(M)]
        S = capped_sum(G, lo, cap, need)
        if kc * T + S < bestF:
            bestF, bestT = kc * T + S, T
    # incremental scan events (useful openings), as kc_scan_incremental
    T = T0
    cap = [lo[i] for i in range(M)]
    for i in range(M):
        while cap[i] < hi[i] and H[i][cap[i] + 1] <= T:
            cap[i] += 1
    # optimal capped allocation at T0
    e = list(lo)
    nd = need
    avail = sum(cap[i] - lo[i] for i in range(M))
    if avail <= nd:
        e = list(cap)
        nd -= avail
    else:
        for _ in range(nd):
            best, bi = INF, -1
            for i in range(M):
                if e[i] < cap[i]:
                    d = G[i][e[i] + 1] - G[i][e[i]]
                    if d < best:
                        best, bi = d, i
            e[bi] += 1
        nd = 0
    S = sum(G[i][e[i]] for i in range(M))
    best = best0
    events = 0

    def lam_of():
        v = [G[i][e[i]] - G[i][e[i] - 1] if e[i] > lo[i] else -INF for i in range(M)]
        m = max(v)
        return m, max(i for i in range(M) if v[i] == m)

    lam, lj = (lam_of() if nd == 0 else (-INF, -1))
    if nd == 0 and kc * T + S < best:
        best = kc * T + S
    while True:
        cands = [(H[i][cap[i] + 1], i) for i in range(M)
                 if e[i] == cap[i] and cap[i] < hi[i] and (nd > 0 or G[i][cap[i] + 1] - G[i][cap[i]] < lam)]
        if not cands:
            break
        Tn, li = min(cands)
        if not (kc * Tn + s_inf < best):
            break
        events += 1
        d = G[li][cap[li] + 1] - G[li][cap[li]]
        if nd == 0:
            S += d - lam
            e[lj] -= 1
        else:
            S += d
            nd -= 1
        cap[li] += 1
        e[li] += 1
        if nd == 0:
            lam, lj = lam_of()
        T = Tn
        if nd == 0 and kc * T + S < best:
            best = kc * T + S
    return {"best": best, "brute": bestF, "events": events, "nT": nT, "n_cand": len(Ts), "need": need,
            "T0": T0, "hmax": hmax, "s_inf": s_inf}


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c2_tables.npz"
    z = np.load(path)
    G, H = z["G"], z["H"]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    rows = [model(G[f], H[f], 1.0, 40) for f in range(n)]
    ev = np.array([r["events"] for r in rows])
    nT = np.array([r["nT"] for r in rows])
    ok = np.array([abs(r["best"] - r["brute"]) <= 1e-9 * abs(r["brute"]) for r in rows])
    print(f"{n} fleets: incremental == brute force: {ok.mean():.3f}; events p50/p90/p99/max "
          f"{np.percentile(ev, [50, 90, 99]).tolist()} {ev.max()}; candidate T in range p50/p90/max "
          f"{np.percentile(nT, [50, 90]).tolist()} {nT.max()}; candidates {np.median([r['n_cand'] for r in rows])}")


if __name__ == "__main__":
    main()
