#!/bin/bash
# instruction-fetch / wait counters of the k-slot (C2) and register (C3) sweep kernels
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/icache; mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
P3="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
for M in 16 64; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/m${M}_p$i -o run -- \
      python3 tools/sweep_time.py --M $M --paths fused --iters 3 > $O/m${M}_p$i.log 2>&1 || exit 1
  done
done
