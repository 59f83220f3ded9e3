#!/bin/bash
# One GPU iteration (development): the parity tests of the sweep paths, then an A/B of the previous
# build (build/variants/libhalda_prev.so) against the current one on the C2 / C3 sweeps, then the scan
# profile of the stamps build.   bash tools/gpu_iter.sh [tests...]
set -o pipefail
mkdir -p gpurun_out
T=${@:-tests/test_gpu_ties.py tests/test_gpu_sweep.py tests/test_gpu_configs.py}
timeout -k 10 900 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread > gpurun_out/it_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/it_tests.log
[ $rc -eq 0 ] || exit 1
for v in prev cur prev cur; do
  if [ $v = prev ]; then L=build/variants/libhalda_prev.so; else L=distilp_amd/libhalda.so; fi
  HALDA_LIB=$L timeout -k 10 120 python -u tools/sweep_time.py --M 16,64 --paths fused --iters 100 > gpurun_out/it_st_$v.log 2>&1 || exit 1
  echo $v; grep -v amdgpu.ids gpurun_out/it_st_$v.log
done
if [ -f build/variants/libhalda_stamps.so ]; then
  HALDA_LIB=build/variants/libhalda_stamps.so timeout -k 10 120 python -u tools/scan_prof.py > gpurun_out/it_sp.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/it_sp.log
fi
