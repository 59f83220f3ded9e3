#!/bin/bash
# A/B of library variants on path B's k = 1 kernel (C3 fleets through the CSR pipeline):
#   bash tools/ab_k1.sh lib1 lib2 ...
for round in 1 2; do
  for L in "$@"; do
    HALDA_LIB=$L timeout -k 10 120 python -u tools/sweep_time.py --M 64 --paths csr --iters 30 2>&1 | grep -v amdgpu.ids \
      | python3 -c "import sys, json; [print('$L', json.loads(l)['launch_ms'].get('halda_solve_k1_kernel')) for l in sys.stdin if l.startswith('{')]" || exit 1
  done
done
