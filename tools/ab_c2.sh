#!/bin/bash
# A/B of library variants on the C2 k-sweep (k-slot kernel launch time), two alternating rounds:
#   bash tools/ab_c2.sh lib1 lib2 ...
mkdir -p gpurun_out
for round in 1 2 3; do
  for L in "$@"; do
    HALDA_LIB=$L timeout -k 10 120 python -u tools/sweep_time.py --M 16 --paths fused --iters 300 2>&1 | grep -v amdgpu.ids \
      | python3 -c "import sys, json; [print('$L', json.loads(l)['launch_ms'].get('halda_sweep_kslot_kernel'), json.loads(l)['ms_per_sweep']) for l in sys.stdin if l.startswith('{')]" || exit 1
  done
done
