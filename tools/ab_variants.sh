#!/bin/bash
# A/B over library variants, run on the GPU box from the repo root (bash tools/ab_variants.sh [bench args])
# A/B over library variants (build/variants/libhalda_<v>.so; "new" = the in-tree build,
# "new:ENV=VAL" = the in-tree build with an environment setting), 3 rounds
set -e
VARS=${VARS:-"head new"}
for r in $(seq ${ROUNDS:-3}); do
  for v in $VARS; do
    unset HALDA_LIB; envset=""
    case $v in
      new) ;;
      new:*) envset=${v#new:} ;;
      *) export HALDA_LIB=$PWD/build/variants/libhalda_$v.so ;;
    esac
    tag=$(echo $v | tr ':=' '__')
    env $envset timeout -k 10 100 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${tag}_$r.json 2>/dev/null
    echo "$v $(grep -o "\"ms_per_step\": [0-9.]*\|\"launch_ms\": {[^}]*}" gpurun_out/ab_${tag}_$r.json | tr "\n" " ")"
  done
done
