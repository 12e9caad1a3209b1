#!/bin/bash
source scripts/lib_steps.sh
step parse_tests 600 python -u -m pytest tests/test_parse_gpu.py -x -q --timeout 300 --timeout-method thread
step nat64_tests 700 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 300 --timeout-method thread
step ab_nat 600 bash scripts/ab_variants.sh "nat64 nat64_cold" "-" cur tail1024
step ab_parse 300 bash scripts/ab_variants.sh "imix_csum parse256" "-" cur su3
export CFG=nat64_cold
step stats_cold 300 bash scripts/ab_stats.sh cur tail1024
