"""The k-slot kernel's split threshold scan (ScanSplit, distilp_amd/csrc/halda_solve.hpp), as an
algorithm: on random tables of the shape the scan accepts (convex G rows, nondecreasing H rows), the
parts cut at the kernel's T_a (T_b) and merged the kernel's way (a later part only when strictly
better) find the one scan's optimum, which is the brute-force min over T of kc T + S(T)
(tools/scan_model.py restates the kernel's scan; the GPU kernel itself is checked bit for bit against
the unsplit sweep in test_gpu_sweep.py)."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
import scan_model as sm  # noqa: E402


def _tables(rng, M, R1):
    """Convex G rows (increasing increments) and nondecreasing H rows, some rows with a finite prefix."""
    G = np.full((M, R1), np.inf)
    H = np.full((M, R1), np.inf)
    for i in range(M):
        n = R1 if rng.random() < 0.8 else int(rng.integers(R1 // 2, R1))
        inc = np.sort(rng.uniform(0.01, 1.0, n - 1))
        G[i, :n] = rng.uniform(0.0, 1.0) + np.concatenate([[0.0], np.cumsum(inc)])
        H[i, :n] = rng.uniform(0.05, 0.3) + np.cumsum(rng.uniform(0.0, 0.1, n))
    return G, H


@pytest.mark.parametrize("seed", range(6))
def test_split_parts_merge_to_the_one_scan(seed):
    rng = np.random.default_rng(seed)
    Gs, Hs = [], []
    for _ in range(24):
        g, h = _tables(rng, 12, 20)
        Gs.append(g)
        Hs.append(h)
    G, H = np.array(Gs), np.array(Hs)
    rep = sm.split_report(G, H, len(Gs), kc=1.0)
    for parts, (longest, _, agree) in rep.items():
        assert agree, parts
    assert rep[1][0] > 0 and rep[2][0] <= rep[1][0] and rep[3][0] <= rep[1][0]  # the scans do run
    for f in range(len(Gs)):  # the one scan is the brute-force optimum
        r = sm.model(G[f], H[f], 1.0, 0)
        assert abs(r["best"] - r["brute"]) <= 1e-9 * max(1.0, abs(r["brute"]))


def _tied_tables(rng, M, R1, kind):
    """Tables with exact ties, as fleets of repeated devices produce them (the reference's own "same
    device twice", test/test_integration.py:88, and homogeneous clusters): `kind` "copies" -- every row
    one device's; "two" -- two devices, each M / 2 times; "half" -- half the rows duplicates of the
    other half; "grid" -- distinct rows whose increments and cycle times come from a coarse grid
    (ties across different devices); "linear" -- rows whose increments are constant over stretches
    (summed in floating point, so equal increments differ by rounding), each row twice."""
    def row(grid=False, linear=False):
        if linear:
            inc = np.repeat(np.sort(rng.uniform(0.001, 0.05, 3)), [R1 // 3, R1 // 3, R1 - 1 - 2 * (R1 // 3)])
            h = rng.uniform(0.1, 0.2) + np.cumsum(np.full(R1, rng.uniform(0.05, 0.15)))
            return rng.uniform(0.0, 1.0) + np.concatenate([[0.0], np.cumsum(inc)]), h
        if grid:
            inc = np.sort(rng.integers(1, 4, R1 - 1).astype(float)) / 4
            h = 0.25 + np.cumsum(rng.integers(0, 2, R1).astype(float)) / 8
        else:
            inc = np.sort(rng.uniform(0.01, 1.0, R1 - 1))
            h = rng.uniform(0.05, 0.3) + np.cumsum(rng.uniform(0.0, 0.1, R1))
        return np.concatenate([[0.0], np.cumsum(inc)]) + (0.0 if grid else rng.uniform(0.0, 1.0)), h

    if kind == "copies":
        rows = [row()] * M
    elif kind == "two":
        a, b = row(), row()
        rows = [a] * (M // 2) + [b] * (M - M // 2)
    elif kind == "half":
        base = [row() for _ in range(M // 2)]
        rows = base + base[: M - M // 2]
    elif kind == "linear":
        base = [row(linear=True) for _ in range(M // 2)]
        rows = base + base[: M - M // 2]
    else:
        rows = [row(grid=True) for _ in range(M)]
    return np.array([r[0] for r in rows]), np.array([r[1] for r in rows])


@pytest.mark.parametrize("kind", ["copies", "two", "half", "grid", "linear"])
@pytest.mark.parametrize("M", [2, 16])
def test_split_parts_exact_under_increment_ties(kind, M):
    """The helper parts start from the greedy's optimal capped allocation at their cut, which under ties
    need not be the allocation the one scan holds there. The exchange step keeps ANY optimal capped
    allocation optimal (its largest taken increment lam and the set of useful openings are the same for
    every optimal allocation), so the merged optimum must still be the brute-force one. Linear
    stretches make equal increments differ by rounding, which can make an opening useful only after T
    passed its H: the scan then takes it at the current T (T never decreases) -- without that, the qwen3
    "half" fleet of test_gpu_ties.py recorded an objective below the brute-force optimum."""
    rng = np.random.default_rng(1000 + M)
    R1 = 2 * M + 6
    Gs, Hs = [], []
    for _ in range(16):
        g, h = _tied_tables(rng, M, R1, kind)
        Gs.append(g)
        Hs.append(h)
    G, H = np.array(Gs), np.array(Hs)
    for kc in (0.5, 1.0, 4.0):
        rep = sm.split_report(G, H, len(Gs), kc=kc)
        for parts, (_, _, agree) in rep.items():
            assert agree, (parts, kc)
        for f in range(len(Gs)):
            r = sm.model(G[f], H[f], kc, 0)
            assert abs(r["best"] - r["brute"]) <= 1e-9 * max(1.0, abs(r["brute"])), (f, kc)


def _linear_twins(rng, M, R1):
    """M / 2 devices, each twice, whose costs are linear in the layer count (every increment the same
    value, summed in floating point) and whose cycle times grow linearly: the shape of a fleet of
    repeated devices whose capacity slacks never bind."""
    base = []
    for _ in range(M // 2):
        g = rng.uniform(0, 0.1) + np.cumsum(np.concatenate([[0.0], np.full(R1 - 1, rng.uniform(0.001, 0.05))]))
        h = rng.uniform(0.1, 0.2) + np.cumsum(np.full(R1, rng.uniform(0.05, 0.15)))
        base.append((g, h))
    rows = base + base
    return np.array([r[0] for r in rows]), np.array([r[1] for r in rows])


def test_scan_takes_late_openings_at_the_current_threshold():
    """Equal increments that differ by rounding can make an opening useful only after the scan's T has
    passed its H; taken at its own (lower) H, the recorded kc T + S priced an allocation whose largest
    cycle time exceeds T -- an objective below the true optimum (tests/golden/tie_tables_qwen3_half_k2.npz:
    the k = 2 tables of test_gpu_ties.py's qwen3_32b "half" fleet 15, made by tools/tie_tables.py, where
    the GPU returned an allocation costing 1.0910 against the optimum 0.9790). With T never decreasing the
    scan is the brute-force optimum there and on 300 random fleets of linear twins (2 of which the old
    rule got wrong)."""
    from tests.conftest import GOLDEN

    z = np.load(GOLDEN / "tie_tables_qwen3_half_k2.npz")
    r = sm.model(z["G"], z["H"], 1.0, 0)
    assert abs(r["brute"] - 0.9790121232082947) <= 1e-12 and abs(r["best"] - r["brute"]) <= 1e-12
    for parts, (_, _, agree) in sm.split_report(z["G"][None], z["H"][None], 1, kc=1.0).items():
        assert agree, parts
    for seed in range(300):
        G, H = _linear_twins(np.random.default_rng(seed), 16, 17)
        r = sm.model(G, H, 1.0, 0)
        assert abs(r["best"] - r["brute"]) <= 1e-9 * max(1.0, abs(r["brute"])), seed
