#!/bin/bash
# VALU / wait counters of the fused-sweep kernels for the current build -> profiles/<R>_valu.json
# (read by bench.py for the VALU-issue roof; keyed by the libhalda.so hash).
#   bash profiles/run_valu.sh r05
set -euo pipefail
R=${1:-r03}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/valu_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/c3" -o run -- \
    python3 tools/sweep_time.py --M 64 --paths fused --iters 3 > "$OUT/c3.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/c2" -o run -- \
    python3 tools/sweep_time.py --M 16 --paths fused --iters 3 > "$OUT/c2.log" 2>&1
# the headline's group launch: K = 20 batches of the 4096 C3 fleets per dispatch (81,920 items)
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/c3_steps" -o run -- \
    python3 tools/steps_profile.py --steps 20 --single 0 > "$OUT/c3_steps.log" 2>&1
python3 tools/valu_stamp.py "$R" c3="$OUT/c3/run_counter_collection.csv" c2="$OUT/c2/run_counter_collection.csv" \
    c3_steps="$OUT/c3_steps/run_counter_collection.csv:81920"
