#!/bin/bash
# SQ instruction-mix / stall counters for the solve kernel (diagnostic; one counter pass).
#   bash profiles/run_pmc_sq.sh r01
set -euo pipefail
R=${1:-r01}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --kernel-trace -T --output-format csv -d "$OUT/pmc_sq" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_sq.json" 2> "$OUT/pmc_sq.err"
