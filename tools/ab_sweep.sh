#!/bin/bash
# A/B of libhalda variants on the fused sweep (C3 and C2 shapes): bash tools/ab_sweep.sh lib1.so lib2.so ...
for lib in "$@"; do
  echo "== $lib"
  HALDA_LIB=$lib timeout -k 10 120 python tools/sweep_time.py --paths fused --iters 30 | grep '{' | cut -c1-160
done
