#!/bin/bash
# A/B of steps-kernel builds with tools/ab_c3.py (per-launch and group-launch timings), one line per library:
#   bash tools/gpu_ab_steps.sh out.log lib1.so lib2.so ...
set -e
OUT=$1; shift
for L in "$@"; do
  HALDA_LIB=$L timeout -k 10 200 python -u tools/ab_c3.py >> "$OUT" 2>&1
done
