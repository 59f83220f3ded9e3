#!/bin/bash
# SQ instruction counts of the fused sweep kernel (C3 shape) for each libhalda build given, one counter
# pass per build:  bash profiles/run_pmc_variants.sh out_dir lib1.so lib2.so ...
set -euo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  HALDA_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM \
      --kernel-trace --output-format csv -d "$OUT/$n" -o run -- \
      python3 tools/sweep_time.py --M 64 --paths fused --iters 3 > "$OUT/$n.log" 2>&1
  echo "== $n"
  python3 tools/pmc_table.py "$OUT/$n/run_counter_collection.csv" | grep -A9 "halda_sweep_kernel"
done
