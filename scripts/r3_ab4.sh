#!/bin/bash
source scripts/lib_steps.sh
step nat64_tests 400 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py -x -v --timeout 100 --timeout-method thread
step parse_tests 400 python -u -m pytest tests/test_parse_gpu.py -x -q --timeout 100 --timeout-method thread
step ab_nat 600 bash scripts/ab_variants.sh "nat64 nat64_cold nat64_4to6 imix_csum" "-" cur
export CFG=nat64_cold
step stats_cold 300 bash scripts/ab_stats.sh cur
