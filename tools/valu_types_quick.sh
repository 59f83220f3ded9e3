#!/bin/bash
# The steps launches' SQ pass and per-type VALU pass alone (a subset of profiles/run_round.sh), for a
# quick look at the VALU-issue pricing of a build: bash tools/valu_types_quick.sh <R>
set -euo pipefail
R=${1:-r06pre}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
TYPES="SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
for M in 64 16; do
  echo "[prof] sq steps M=$M"
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS \
      --kernel-trace --output-format csv -d "$OUT/valu_steps$M" -o run -- \
      python3 tools/steps_profile.py --steps 20 --single 0 --M $M > "$OUT/valu_steps$M.log" 2>&1
  echo "[prof] valu types steps M=$M"
  timeout -s KILL 180 rocprofv3 --pmc $TYPES \
      --kernel-trace --output-format csv -d "$OUT/types_steps$M" -o run -- \
      python3 tools/steps_profile.py --steps 20 --single 0 --M $M > "$OUT/types_steps$M.log" 2>&1
done
python3 tools/valu_stamp.py "$R" \
    c3_steps="$OUT/valu_steps64/run_counter_collection.csv+$OUT/types_steps64/run_counter_collection.csv:81920" \
    c2_steps="$OUT/valu_steps16/run_counter_collection.csv+$OUT/types_steps16/run_counter_collection.csv:81920"
