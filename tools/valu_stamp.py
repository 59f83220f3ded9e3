"""Record the VALU count per wave of the fused-sweep kernels for THIS libhalda.so build.

Run on the GPU box right after the counter passes (same snapshot, so the hashed library is the one
profiled), e.g. via profiles/run_round.sh:

  python tools/valu_stamp.py r03 c3=gpurun_out/valu_c3/run_counter_collection.csv \
                                 c2=gpurun_out/valu_c2/run_counter_collection.csv

Writes gpurun_out/<R>_valu.json (copied to profiles/ afterwards): {"libhalda_sha256": ..., "workloads": {"c3": {kernel: {...}}, ...}}
with, per kernel, the largest launch's SQ_INSTS_VALU / SQ_WAVES (valu_per_wave), SQ_WAVES (waves),
SQ_WAIT_ANY / SQ_WAVE_CYCLES (wait_any_frac), SALU and LDS instructions per wave. bench.py reads
it for the VALU-issue roof only when the hash matches the library it loads.

A workload may name several counter CSVs joined by '+' (one rocprofv3 pass each: at most 8 SQ counters
fit one pass); their per-kernel means are merged. With the per-type pass (SQ_INSTS_VALU_{ADD,MUL,FMA,
TRANS}_F64, INT32, INT64, CVT) each kernel also gets `valu_types` (instructions per wave by type), from
which bench.py prices FP64 arithmetic at 4 cycles per wave64 instruction (16 FP64 lanes per cycle per
SIMD), FP64 transcendentals at 8 and every other VALU at 2 (32 lanes per cycle, MI355X_MICROARCH.md:54).
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

        out[k] = {"waves": int(waves), "dispatches": len(big),
                  "means": {c: mean(c) for c in set().union(*big) if c != "SQ_WAVES"}}
    return out


TYPES = ("ADD_F64", "MUL_F64", "FMA_F64", "TRANS_F64", "INT32", "INT64", "CVT")


def finish(e):
    """Per-wave figures of one kernel from its merged counter means."""
    waves, m = e["waves"], e.pop("means")

    def per(c):
        return m[c] / waves if m.get(c) is not None else None

    cyc, wait = m.get("SQ_WAVE_CYCLES"), m.get("SQ_WAIT_ANY")
    e.update({"valu_per_wave": per("SQ_INSTS_VALU"),
              "wait_any_frac": (wait / cyc) if (wait is not None and cyc) else None,
              "salu_per_wave": per("SQ_INSTS_SALU"), "lds_per_wave": per("SQ_INSTS_LDS")})
    if all(f"SQ_INSTS_VALU_{t}" in m for t in TYPES):
        e["valu_types"] = {t.lower(): per(f"SQ_INSTS_VALU_{t}") for t in TYPES}
    return e


def merge(paths):
    out = {}
    for p in paths:
        for k, e in summarise(p).items():
            if k not in out:
                out[k] = e
            elif e["waves"] == out[k]["waves"]:
                out[k]["means"].update(e["means"])
    return {k: finish(e) for k, e in out.items()}


def main():
    R = sys.argv[1]
    lib = REPO / "distilp_amd" / "libhalda.so"
    res = {"libhalda_sha256": hashlib.sha256(lib.read_bytes()).hexdigest(), "workloads": {},
           "note": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS "
                   "(+ a per-type pass: SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, INT32, INT64, CVT) over "
                   "tools/sweep_time.py (fused path) and tools/steps_profile.py; largest launch per kernel"}
    for arg in sys.argv[2:]:
        # name=path[:items] -- items: (batch, fleet) items per dispatch of a steps launch (K x fleets)
        name, rest = arg.split("=", 1)
        path, _, items = rest.partition(":")
        res["workloads"][name] = merge(path.split("+"))
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
