#!/bin/bash
# Profiling recipe used for profiles/<round>_*: run on the GPU box from the repo root.
#   bash profiles/run_profile.sh r05
# 1) rocprofv3 kernel trace + stats of the bench (same command as the bench line, fewer steps, and
#    --streams 1 so that every dispatch's begin..end is its own: with two streams in flight the
#    dispatches of consecutive batches overlap and their durations include each other)
# 2) two separate PMC passes (FETCH_SIZE, WRITE_SIZE) with kernel trace only, per MI355X_MICROARCH.md
set -euo pipefail
R=${1:-r02}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
# the library these passes profile (pmc_summary.py keys the summary to it; bench.py uses a summary
# only for the libhalda.so it loads)
sha256sum distilp_amd/libhalda.so | cut -d' ' -f1 > "$OUT/lib_sha256"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-latency --streams 1 > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-tto --no-latency > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --no-tto --no-latency > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
# FETCH_SIZE calibration for 8-B and 16-B per-lane coalesced reads of a known byte count
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/calib" -o run -- \
    ./build/hbm_calib > "$OUT/calib.json" 2> "$OUT/calib.err"
