#!/bin/bash
# SQ instruction-mix / stall counters of the fused sweep kernel (C3 and C2 shapes), two passes.
#   bash profiles/run_pmc_sweep.sh r02
set -euo pipefail
R=${1:-r02}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d "$OUT/pmc_sweep1" -o run -- \
    python3 tools/sweep_time.py --paths fused --iters 3 > "$OUT/pmc_sweep1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/pmc_sweep2" -o run -- \
    python3 tools/sweep_time.py --paths fused --iters 3 > "$OUT/pmc_sweep2.log" 2>&1
