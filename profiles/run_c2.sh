#!/bin/bash
# Config C2 (M = 16 fleets, every k of L = 80): bench line, rocprofv3 kernel stats of the fused sweep
# and of the CSR pipeline, SQ issue/stall counters of the sweep kernels.   bash profiles/run_c2.sh r02
set -euo pipefail
R=${1:-r02}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_${R}_c2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --M 16 --no-cpu-baseline --no-tto --streams 1 > "$OUT/c2_bench.json" 2> "$OUT/c2_bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/sweep_time.py --M 16,64 --iters 10 > "$OUT/trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d "$OUT/pmc_sq1" -o run -- \
    python3 tools/sweep_time.py --M 16,64 --paths fused --iters 3 > "$OUT/pmc_sq1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/pmc_sq2" -o run -- \
    python3 tools/sweep_time.py --M 16,64 --paths fused --iters 3 > "$OUT/pmc_sq2.log" 2>&1
