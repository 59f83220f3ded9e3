"""Diagnostic (CPU): a Python model of the k > 1 solve of the k-slot kernel on dumped tables
(tools/kslot_tables.py -> gpurun_out/c2_tables.npz): the phase-0 greedy, the incremental threshold
scan (kc_scan_incremental, its event count) and a brute-force min over T of kc T + S(T), to study
the scan's sequential length offline, and (--split) the k-slot kernel's split of that scan over waves.
  python tools/scan_model.py [gpurun_out/c2_tables.npz] [n_fleets] [--split]"""
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


def scan_range(G, H, kc, t_start=None, t_stop=INF):
    """kc_scan_incremental on one fleet's tables, from the optimal capped allocation at max(T0, t_start)
    to the openings T <= t_stop (ScanSplit parts): (best objective bound found, its T or None, events)."""
    M, R1 = G.shape
    fin = np.isfinite(G)
    lo = [int(np.argmax(fin[i])) for i in range(M)]
    hi = [int(R1 - 1 - np.argmax(fin[i][::-1])) for i in range(M)]
    need = (R1 - 1) - sum(lo)
    e = list(lo)
    for _ in range(need):  # phase 0
        best, bi = INF, -1
        for i in range(M):
            if e[i] < hi[i] and G[i][e[i] + 1] - G[i][e[i]] < best:
                best, bi = G[i][e[i] + 1] - G[i][e[i]], i
        e[bi] += 1
    s_inf = sum(G[i][e[i]] for i in range(M))
    best = kc * max(max(0.0, H[i][e[i]]) for i in range(M)) + s_inf
    T = max(H[i][lo[i]] for i in range(M))
    if t_start is not None:
        T = max(T, t_start)
    cap = list(lo)
    for i in range(M):
        while cap[i] < hi[i] and H[i][cap[i] + 1] <= T:
            cap[i] += 1
    e, nd = list(lo), need
    avail = sum(cap[i] - lo[i] for i in range(M))
    if avail <= nd:
        e, nd = list(cap), nd - avail
    else:
        for _ in range(nd):
            b, bi = INF, -1
            for i in range(M):
                if e[i] < cap[i] and G[i][e[i] + 1] - G[i][e[i]] < b:
                    b, bi = G[i][e[i] + 1] - G[i][e[i]], i
            e[bi] += 1
        nd = 0
    S = sum(G[i][e[i]] for i in range(M))

    def lam_of():
        v = [G[i][e[i]] - G[i][e[i] - 1] if e[i] > lo[i] else -INF for i in range(M)]
        m = max(v)
        return m, max(i for i in range(M) if v[i] == m)

    lam, lj = lam_of() if nd == 0 else (-INF, -1)
    bestT = None
    if nd == 0 and kc * T + S < best:
        best = kc * T + S
        bestT = T if t_start is None else None  # a helper's start only bounds its pruning
    events = 0
    while True:
        c = [(H[i][cap[i] + 1], i) for i in range(M)
             if e[i] == cap[i] and cap[i] < hi[i] and (nd > 0 or G[i][cap[i] + 1] - G[i][cap[i]] < lam)]
        if not c:
            break
        Tn, li = min(c)
        Te = max(T, Tn)  # T never decreases (see kc_scan_incremental)
        if not (kc * Te + s_inf < best) or Te > t_stop:
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
        T = Te
        if nd == 0 and kc * T + S < best:
            best, bestT = kc * T + S, T
    return best, bestT, events


def split_cuts(G, H, n_parts):
    """ScanSplit's cuts: H at cap(T0) + 2 (and + 3) over the devices with an opening past T0; two parts:
    the value of rank (n - 1) * 5 / 8 of the first (the kernel's), three: its lower quartile and the
    lower median of the second."""
    M, R1 = G.shape
    fin = np.isfinite(G)
    lo = [int(np.argmax(fin[i])) for i in range(M)]
    hi = [int(R1 - 1 - np.argmax(fin[i][::-1])) for i in range(M)]
    T0 = max(H[i][lo[i]] for i in range(M))
    cap = list(lo)
    for i in range(M):
        while cap[i] < hi[i] and H[i][cap[i] + 1] <= T0:
            cap[i] += 1
    has = [i for i in range(M) if cap[i] < hi[i]]
    if not has:
        return [INF] * (n_parts - 1)
    v2 = sorted(H[i][min(cap[i] + 2, hi[i])] for i in has)
    if n_parts == 2:
        return [v2[(len(v2) - 1) * 5 // 8]]
    v3 = sorted(H[i][min(cap[i] + 3, hi[i])] for i in has)
    a, b = v2[(len(v2) - 1) // 4], v3[(len(v3) - 1) // 2]
    return [min(a, b), max(a, b)]


def split_report(G, H, n, kc=1.0):
    """Longest scan chain per wave (events) unsplit / in two / three parts, and that the parts' merged
    optimum equals the one scan's."""
    out = {}
    for parts in (1, 2, 3):
        longest, agree = [], True
        for f in range(n):
            best1, _, ev1 = scan_range(G[f], H[f], kc)
            if parts == 1:
                longest.append(ev1)
                continue
            cuts = split_cuts(G[f], H[f], parts)
            bounds = [None] + cuts
            stops = cuts + [INF]
            res = [scan_range(G[f], H[f], kc, t_start=bounds[p], t_stop=stops[p]) for p in range(parts)]
            merged = res[0][0]
            for p in range(1, parts):
                if res[p][1] is not None and res[p][0] < merged:
                    merged = res[p][0]
            agree = agree and abs(merged - best1) <= 1e-9 * abs(best1)
            longest.append(max(r[2] for r in res))
        a = np.array(longest)
        out[parts] = (int(a.max()), float(np.percentile(a, 99)), agree)
    return out


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
        Te = max(T, Tn)
        if not (kc * Te + s_inf < best):
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
        T = Te
        if nd == 0 and kc * T + S < best:
            best = kc * T + S
    return {"best": best, "brute": bestF, "events": events, "nT": nT, "n_cand": len(Ts), "need": need,
            "T0": T0, "hmax": hmax, "s_inf": s_inf}


def main():
    split = "--split" in sys.argv
    argv = [a for a in sys.argv[1:] if a != "--split"]
    path = argv[0] if argv else "gpurun_out/c2_tables.npz"
    z = np.load(path)
    G, H = z["G"], z["H"]
    n = int(argv[1]) if len(argv) > 1 else 256
    if split:  # the ScanSplit cuts (halda_solve.hpp): longest chain per wave, merged optimum == one scan
        for parts, (mx, p99, agree) in split_report(G, H, n).items():
            print(f"{n} fleets, {parts} part(s): longest scan per wave max {mx} p99 {p99:.1f} events; "
                  f"merged optimum == one scan: {agree}")
        return
    rows = [model(G[f], H[f], 1.0, 40) for f in range(n)]
    ev = np.array([r["events"] for r in rows])
    nT = np.array([r["nT"] for r in rows])
    ok = np.array([abs(r["best"] - r["brute"]) <= 1e-9 * abs(r["brute"]) for r in rows])
    print(f"{n} fleets: incremental == brute force: {ok.mean():.3f}; events p50/p90/p99/max "
          f"{np.percentile(ev, [50, 90, 99]).tolist()} {ev.max()}; candidate T in range p50/p90/max "
          f"{np.percentile(nT, [50, 90]).tolist()} {nT.max()}; candidates {np.median([r['n_cand'] for r in rows])}")


if __name__ == "__main__":
    main()
