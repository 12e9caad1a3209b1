#!/bin/bash
# round 3: nat64 map rework (hot index, ADDR_MAP values, reset), bench modes
source scripts/lib_steps.sh
step nat64_tests 700 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py -x -v --timeout 300 --timeout-method thread
step b_nat64 300 python bench.py --config nat64 --only --cpu-seconds 2
step b_4to6 300 python bench.py --config nat64_4to6 --only --cpu-seconds 2
step b_cold 300 python bench.py --config nat64_cold --only --cpu-seconds 2 --steps 200
step bench_modes 900 python -u -m pytest tests/test_bench_modes_gpu.py -x -v --timeout 300 --timeout-method thread
