#!/bin/bash
# One round's profile set, run on the GPU box from the repo root (build beforehand, in this tree):
#   bash profiles/run_round.sh r06
# 1) rocprofv3 kernel trace + stats of the bench (--streams 1: each dispatch's begin..end is its own)
# 2) PMC passes, one counter group per run (MI355X_MICROARCH.md): FETCH_SIZE, WRITE_SIZE, the
#    FETCH_SIZE calibration binary, and the SQ instruction counts of the fused-sweep kernels on C3 and
#    C2 (tools/valu_stamp.py keys them to this libhalda.so build; bench.py reads them for the VALU roof)
# Summaries: python tools/pmc_summary.py <R> 20; python tools/valu_stamp.py <R> c3=... c2=... (below)
set -euo pipefail
R=${1:-r03}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
# the library these passes profile (pmc_summary.py / valu_stamp.py key the summaries to it)
sha256sum distilp_amd/libhalda.so | cut -d' ' -f1 > "$OUT/lib_sha256"
echo "[prof] trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-tto --streams 1 > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
echo "[prof] fetch"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-tto --no-latency > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
echo "[prof] write"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-tto --no-latency > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
echo "[prof] calib"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/calib" -o run -- \
    ./build/hbm_calib > "$OUT/calib.json" 2> "$OUT/calib.err"
for M in 64 16; do
  echo "[prof] sq M=$M"
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS \
      --kernel-trace --output-format csv -d "$OUT/valu_m$M" -o run -- \
      python3 tools/sweep_time.py --M $M --paths fused --iters 3 > "$OUT/valu_m$M.log" 2>&1
done
# the steps launches (the headline's and C2's): the SQ pass, then the per-type VALU pass (FP64 arithmetic
# apart from the rest, for the VALU-issue roof's pricing; 8 SQ counters, one pass)
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
python3 tools/valu_stamp.py "$R" c3="$OUT/valu_m64/run_counter_collection.csv" c2="$OUT/valu_m16/run_counter_collection.csv" \
    c3_steps="$OUT/valu_steps64/run_counter_collection.csv+$OUT/types_steps64/run_counter_collection.csv:81920" \
    c2_steps="$OUT/valu_steps16/run_counter_collection.csv+$OUT/types_steps16/run_counter_collection.csv:81920" > /dev/null
echo "[prof] done"
