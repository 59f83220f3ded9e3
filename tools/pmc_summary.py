"""Summarise a profiles/run_round.sh run into profiles/<round>_*.

Writes:
  profiles/<R>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<R>_pmc.json           per-launch FETCH_SIZE / WRITE_SIZE of halda_solve_kernel and
                                  halda_screen_kernel, the 8-B/lane FETCH_SIZE calibration and the
                                  corrected HBM bytes per launch (read by bench.py as roofline.traffic)
"""

import csv
import json
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def short(name):
    """'(anonymous namespace)::halda_sweep_kernel((anonymous namespace)::SweepArgs)' -> 'halda_sweep_kernel'."""
    import re

    m = re.search(r"(halda_\w+)\(", name)
    return m.group(1) if m else name.split("(")[0]


def per_kernel(csv_path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(csv_path)):
        if r["Counter_Name"] == counter:
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def by_grid(trace_csv, out_csv):
    """Per (kernel, grid size x, y) launch statistics: separates the C3 launches from the bench's small
    time-to-optimal launches, and a group launch's K (grid y) from its warm-up's (the --stats summary
    averages over all of them)."""
    d = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        if "halda" in r["Kernel_Name"]:
            d[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r.get("Grid_Size_Y") or 1))].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(out_csv, "w") as f:
        f.write('"Name","Grid_Size_X","Grid_Size_Y","Calls","AverageNs","MinNs","MaxNs"\n')
        for (k, g, gy), v in sorted(d.items()):
            f.write(f'"{k}",{g},{gy},{len(v)},{statistics.mean(v):.1f},{min(v)},{max(v)}\n')


def main(R):
    src = REPO / "gpurun_out" / f"prof_{R}"
    dst = REPO / "profiles"
    shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / f"{R}_kernel_stats.csv")
    shutil.copy(src / "trace_bench.json", dst / f"{R}_bench_under_rocprof.json")
    by_grid(src / "trace" / "run_kernel_trace.csv", dst / f"{R}_kernel_by_grid.csv")
    fetch = per_kernel(src / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(src / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE")
    cal = per_kernel(src / "calib" / "run_counter_collection.csv", "FETCH_SIZE")
    calib_bytes = 1 << 30
    def pick(prefix):
        return statistics.median(next(v for k, v in cal.items() if k.startswith(prefix))) * 1024 / calib_bytes

    f8, f16 = pick("read8"), pick("read16")
    sha = (src / "lib_sha256").read_text().strip() if (src / "lib_sha256").exists() else None
    out = {"libhalda_sha256": sha, "fetch_size_over_bytes_8B_per_lane": f8,
           "fetch_size_over_bytes_16B_per_lane": f16, "kernels": {}}
    for name in fetch:
        if "halda" not in name:
            continue
        # the big C3 launches only (the bench also runs small time-to-optimal batches)
        fk = max(fetch[name])
        wk = max(write.get(name, [0.0]))
        out["kernels"][name] = {
            "FETCH_SIZE_KB": fk, "WRITE_SIZE_KB": wk,
            "hbm_bytes_per_launch": fk * 1024 / f8 + wk * 1024,
        }
        if name in ("halda_sweep_steps_kernel", "halda_sweep_kslot_steps_kernel"):  # one launch = K batches
            e = out["kernels"][name]
            e["steps"] = STEPS
            e["hbm_bytes_per_batch"] = e["hbm_bytes_per_launch"] / STEPS
    solve = out["kernels"].get("halda_sweep_kernel") or out["kernels"].get("halda_solve_k1_kernel")
    out["hbm_bytes_per_launch"] = solve["hbm_bytes_per_launch"] if solve else None
    out["note"] = ("FETCH_SIZE corrected by the measured FETCH_SIZE/bytes ratio of an 8-B-per-lane "
                   "coalesced read (tools/hbm_calib.hip), the solve kernel's dominant access width; "
                   "WRITE_SIZE taken as bytes. Largest launch per kernel = the C3 batch.")
    (dst / f"{R}_pmc.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))



STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 20  # the --steps of run_round.sh's PMC passes

if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
