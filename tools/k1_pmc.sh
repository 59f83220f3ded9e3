export TMPDIR=/tmp
mkdir -p gpurun_out/k1pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/k1pmc/a -o run -- python3 tools/sweep_time.py --M 64 --paths csr --iters 3 > gpurun_out/k1pmc/a.log 2>&1
