#!/bin/bash
# A/B of build variants on the C3 (and C2) k-sweep, alternating:  bash tools/ab_libs.sh lib1 lib2 ...
mkdir -p gpurun_out
for round in 1 2; do
  for L in "$@"; do
    HALDA_LIB=$L timeout -k 10 120 python -u tools/ab_c3.py --M 64 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for L in "$@"; do
  HALDA_LIB=$L timeout -k 10 120 python -u tools/ab_c3.py --M 16 2>&1 | grep -v amdgpu.ids || exit 1
done
