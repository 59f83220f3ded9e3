#!/bin/bash
# Memory-pipeline counters of the solve kernels (diagnostic; separate passes, kernel trace only).
#   bash profiles/run_pmc_mem.sh r01
set -euo pipefail
R=${1:-r01}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run pmc_ta TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run pmc_tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
run pmc_tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
run pmc_tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
