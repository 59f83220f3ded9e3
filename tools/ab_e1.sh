#!/bin/bash
# A/B of fused-sweep library variants (build/variants/libhalda_<v>.so) on the C3 and C2 shapes
# (diagnostic):  VARS="head v2" bash tools/ab_e1.sh
set -e
for r in 1 2; do
for v in ${VARS:-head v2}; do
  HALDA_LIB=build/variants/libhalda_$v.so timeout -k 10 120 python tools/sweep_time.py --M ${MS:-64,16} --paths fused --iters 50 | grep '{' | cut -c1-100 | sed "s/^/$v /"
done
done
