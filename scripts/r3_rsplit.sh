#!/bin/bash
# ADDR_MAP split into address / port arrays: nat64 parity, A/B with FETCH_SIZE
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread
step ab 900 bash scripts/ab_variants.sh "nat64_4to6" "FETCH_SIZE" base rsplit
step ab2 600 bash scripts/ab_variants.sh "nat64_4to6 nat64" "-" rsplit base rsplit base
