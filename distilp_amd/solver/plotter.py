"""k-vs-objective plot of the last sweep (reference: solver/components/plotter.py:4-58).

A UI side effect only: prints and returns quietly when matplotlib is missing or
no k is feasible; never affects the solve.
"""

from __future__ import annotations

from typing import List, Optional, Tuple


def plot_k_curve(per_k_objs: List[Tuple[int, Optional[float]]], k_star: Optional[int] = None,
                 title: str = "HALDA: k vs objective", save_path: Optional[str] = None) -> None:
    try:
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available; skipping plot.")
        return
    points = sorted(((k, v) for k, v in per_k_objs if v is not None), key=lambda kv: kv[0])
    if not points:
        print("No feasible k values to plot.")
        return
    ks = [k for k, _ in points]
    plt.figure()
    plt.plot(ks, [v for _, v in points], marker="o")
    plt.xlabel("k (number of segments)")
    plt.xticks(ks)
    plt.ylabel("Objective (estimated latency)")
    plt.title(title)
    plt.tight_layout()
    if save_path:
        plt.savefig(save_path, dpi=150)
        print(f"Saved plot to {save_path}")
    try:
        plt.show()
    except Exception:
        pass
    finally:
        plt.close()
