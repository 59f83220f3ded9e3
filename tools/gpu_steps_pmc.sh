#!/bin/bash
# rocprofv3 passes over tools/steps_profile.py (C3 group launches of K = 20 vs per-batch launches):
# SQ issue/wait counters, then GRBM (effective clock), each pass its own run.  bash tools/gpu_steps_pmc.sh r05a
set -euo pipefail
R=${1:-r05}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/steps_pmc_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/steps_profile.py --steps 20 > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$OUT/sq" -o run -- python3 tools/steps_profile.py --steps 20 > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_INSTS_SMEM \
    --output-format csv -d "$OUT/grbm" -o run -- python3 tools/steps_profile.py --steps 20 > "$OUT/grbm.log" 2>&1
python3 tools/pmc_dispatch.py "$OUT/sq/run_counter_collection.csv" "$OUT/grbm/run_counter_collection.csv" \
    --items halda_sweep_steps_kernel=81920 halda_sweep_kernel=4096 > "$OUT/summary.txt"
