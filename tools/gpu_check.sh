#!/bin/bash
# GPU check used during development: parity tests, phase stamps, short bench.
set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -3
HALDA_LIB=build/variants/libhalda_stamps.so timeout -k 10 300 python tools/phase_stamps.py
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_cur.json
python -c "import json;d=json.load(open('gpurun_out/bench_cur.json'));print('cur', d['ms_per_step'], d['roofline']['kernel_ms'], d['time_to_optimal_ms'])"
