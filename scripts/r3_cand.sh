#!/bin/bash
# first-packet candidates marked by the fused kernel: nat64 parity, cold/steady A/B
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread
export CFG=nat64_cold
step stats 600 bash scripts/ab_stats.sh base cand
step ab 600 bash scripts/ab_variants.sh "nat64 nat64_cold" "-" cand base cand base
