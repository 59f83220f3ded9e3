"""Per-kernel, per-grid mean of every counter in rocprofv3 counter_collection CSVs.

  python tools/pmc_table.py gpurun_out/prof_r02/pmc_sweep1/run_counter_collection.csv [...]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    import re

    m = re.search(r"(halda_\w+)\(", name)
    return m.group(1) if m else name.split("(")[0]


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]) if "Grid_Size" in r else int(r.get("Grid_Size_X", 0)))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (k, g), cs in sorted(acc.items()):
        if "halda" not in k:
            continue
        print(f"{k} grid={g}")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
