#!/bin/bash
# VALU / SALU per wave of the C3 register sweep up to each phase (diagnostic exit builds, make exits):
# exit1 = loads + records + offsets, exit2 = + the bookkeeping before the k = 1 greedy, exit3 = + the
# greedy, full = the product build. Run on the GPU box:  bash tools/valu_phases.sh
set -euo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/valu_phases
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY"
for v in exit1 exit2 exit3 full; do
  L=build/variants/libhalda_$v.so
  [ $v = full ] && L=distilp_amd/libhalda.so
  HALDA_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$v" -o run -- \
      python3 tools/sweep_time.py --M 64 --paths fused --iters 3 > "$OUT/$v.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, sys, collections
out = sys.argv[1]
for v in ("exit1", "exit2", "exit3", "full"):
    d = collections.defaultdict(dict)
    for r in csv.DictReader(open(f"{out}/{v}/run_counter_collection.csv")):
        if "halda_sweep_kernel" in r["Kernel_Name"]:
            d[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    big = [x for x in d.values() if x.get("SQ_WAVES", 0) == 4096]
    n = len(big)
    f = lambda c: sum(x[c] for x in big) / n / 4096
    print(f"{v:6s} dispatches {n}: VALU/wave {f('SQ_INSTS_VALU'):.1f}  SALU/wave {f('SQ_INSTS_SALU'):.1f}  "
          f"wait_any/cycles {sum(x['SQ_WAIT_ANY'] for x in big) / sum(x['SQ_WAVE_CYCLES'] for x in big):.3f}")
PY
