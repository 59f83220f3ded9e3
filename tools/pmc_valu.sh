#!/bin/bash
# SQ instruction counts of the fused sweep kernel (C3) per library variant (diagnostic):
#   VARS="v2 v3" bash tools/pmc_valu.sh
export TMPDIR=/tmp
for v in ${VARS:-head}; do
  HALDA_LIB=$PWD/build/variants/libhalda_$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/pmc_$v -o run -- python3 tools/sweep_time.py --M 64 --paths fused --iters 3 > gpurun_out/pmc_$v.log 2>&1 || exit 1
done
