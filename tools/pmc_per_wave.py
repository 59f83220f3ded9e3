"""Per-dispatch mean of rocprofv3 SQ counters of one kernel, per wave (diagnostic):
   python tools/pmc_per_wave.py gpurun_out/pmc_v3 [kernel substring, default halda_sweep_kernel]"""
import collections
import csv
import sys


def main(d, kernel="halda_sweep_kernel"):
    per = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if kernel in r["Kernel_Name"]:
            per.setdefault(r["Dispatch_Id"], collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
    ds = list(per.values())
    avg = {k: sum(x[k] for x in ds) / len(ds) for k in ds[0]}
    w = avg.get("SQ_WAVES", 1.0)
    print(d, kernel, f"dispatches={len(ds)}",
          " ".join(f"{k}={v:.0f}({v / w:.1f}/wave)" for k, v in sorted(avg.items())))


if __name__ == "__main__":
    main(*sys.argv[1:])
