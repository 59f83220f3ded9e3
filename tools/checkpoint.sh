#!/bin/bash
# Round-end measurement on the GPU box (development): GPU suite, the bench at the driver's 20 steps
# and at 200, the rocprofv3 kernel-trace / PMC passes and the VALU counters of this build.
#   bash tools/checkpoint.sh r04
set -o pipefail
R=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cp_tests.log 2>&1 || { echo tests failed; tail -5 gpurun_out/cp_tests.log; exit 1; }
tail -1 gpurun_out/cp_tests.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/cp_b20.json 2> gpurun_out/cp_b20.err || { echo bench20 failed; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 > gpurun_out/cp_b200.json 2> gpurun_out/cp_b200.err || { echo bench200 failed; exit 1; }
echo bench ok
timeout -k 10 1000 bash profiles/run_profile.sh $R || { echo profile failed; exit 1; }
timeout -k 10 500 bash profiles/run_valu.sh $R || { echo valu failed; exit 1; }
echo all ok
