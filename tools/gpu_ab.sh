mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ties.py tests/test_gpu_sweep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/t3.log
for v in prev cur prev cur; do
  if [ $v = prev ]; then L=build/variants/libhalda_prev.so; else L=distilp_amd/libhalda.so; fi
  HALDA_LIB=$L timeout -k 10 120 python -u tools/sweep_time.py --M 16,64 --paths fused --iters 100 > gpurun_out/st_$v.log 2>&1 || exit 1
  echo $v; cat gpurun_out/st_$v.log | grep -v amdgpu.ids
done
HALDA_LIB=build/variants/libhalda_stamps.so timeout -k 10 200 python -u tools/sweep_stamps.py > gpurun_out/ss.log 2>&1
timeout -k 10 200 python -u tools/k1_rounds.py > gpurun_out/k1r.log 2>&1
cat gpurun_out/ss.log gpurun_out/k1r.log
