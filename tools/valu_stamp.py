"""Record the VALU count per wave of the fused-sweep kernels for THIS libhalda.so build.

Run on the GPU box right after the counter passes (same snapshot, so the hashed library is the one
profiled), e.g. via profiles/run_round.sh:

  python tools/valu_stamp.py r03 c3=gpurun_out/valu_c3/run_counter_collection.csv \
                                 c2=gpurun_out/valu_c2/run_counter_collection.csv

Writes gpurun_out/<R>_valu.json (copied to profiles/ afterwards): {"libhalda_sha256": ..., "workloads": {"c3": {kernel: {...}}, ...}}
with, per kernel, the largest launch's SQ_INSTS_VALU / SQ_WAVES (valu_per_wave), SQ_WAVES (waves),
SQ_WAIT_ANY / SQ_WAVE_CYCLES (wait_any_frac), SALU and LDS instructions per wave. bench.py reads
it for the VALU-issue roof only when the hash matches the library it loads.
"""

import csv
import hashlib
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def short(name):
    m = re.search(r"(halda_\w+)\(", name)
    return m.group(1) if m else name.split("(")[0]


def per_dispatch(path):
    """{kernel: [{counter: value} per dispatch]}"""
    d = defaultdict(lambda: defaultdict(dict))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if "halda" not in k:
            continue
        d[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    return {k: list(v.values()) for k, v in d.items()}


def summarise(path):
    out = {}
    for k, ds in per_dispatch(path).items():
        waves = max(x.get("SQ_WAVES", 0.0) for x in ds)
        big = [x for x in ds if x.get("SQ_WAVES", 0.0) == waves and waves > 0]
        if not big:
            continue

        def mean(c):
            v = [x[c] for x in big if c in x]
            return sum(v) / len(v) if v else None

        valu, cyc, wait = mean("SQ_INSTS_VALU"), mean("SQ_WAVE_CYCLES"), mean("SQ_WAIT_ANY")
        salu, lds = mean("SQ_INSTS_SALU"), mean("SQ_INSTS_LDS")
        out[k] = {"valu_per_wave": valu / waves, "waves": int(waves), "dispatches": len(big),
                  "wait_any_frac": (wait / cyc) if (wait is not None and cyc) else None,
                  "salu_per_wave": salu / waves if salu is not None else None,
                  "lds_per_wave": lds / waves if lds is not None else None}
    return out


def main():
    R = sys.argv[1]
    lib = REPO / "distilp_amd" / "libhalda.so"
    res = {"libhalda_sha256": hashlib.sha256(lib.read_bytes()).hexdigest(), "workloads": {},
           "note": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS "
                   "over tools/sweep_time.py (fused path); largest launch per kernel"}
    for arg in sys.argv[2:]:
        # name=path[:items] -- items: (batch, fleet) items per dispatch of a steps launch (K x fleets)
        name, rest = arg.split("=", 1)
        path, _, items = rest.partition(":")
        res["workloads"][name] = summarise(path)
        if items:
            for e in res["workloads"][name].values():
                e["items"] = int(items)
    # written under gpurun_out/ on the GPU box (merged back), then copied to profiles/ by the builder
    dst = REPO / "gpurun_out" / f"{R}_valu.json"
    dst.parent.mkdir(exist_ok=True)
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
