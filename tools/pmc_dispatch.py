"""Per-kernel means of rocprofv3 counter-collection CSVs (one or more passes), per dispatch and per
item where the caller gives items per dispatch of a kernel:
    python tools/pmc_dispatch.py out1/run_counter_collection.csv [out2/...] [--items halda_sweep_steps_kernel=81920]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    cut = args.index("--items") if "--items" in args else len(args)
    paths = args[:cut]
    items = {}
    if "--items" in sys.argv:
        for kv in sys.argv[sys.argv.index("--items") + 1:]:
            if "=" in kv:
                k, v = kv.split("=")
                items[k] = float(v)
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> dispatch -> counter
    for p in paths:
        for r in csv.DictReader(open(p)):
            m = re.search(r"(halda_\w+)", r["Kernel_Name"])
            if not m:
                continue
            per[m.group(1)][(p, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, ds in per.items():
        cnt = defaultdict(list)
        for d in ds.values():
            for c, v in d.items():
                cnt[c].append(v)
        mean = {c: sum(v) / len(v) for c, v in cnt.items()}
        print(k, "dispatches", len(ds))
        for c, v in sorted(mean.items()):
            extra = f"  per item {v / items[k]:.2f}" if k in items else ""
            print(f"   {c:24s} {v:16.1f}{extra}")
        w = mean.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
                if c in mean:
                    print(f"   {c} per wave {mean[c] / w:.1f}")
        cyc = mean.get("SQ_WAVE_CYCLES")
        if cyc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in mean:
                    print(f"   {c} / WAVE_CYCLES {mean[c] / cyc:.3f}")


if __name__ == "__main__":
    main()
