#!/bin/bash
# round 4 (w): late claims in the rows path: parity, then cold and steady A/B against early claims
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -q --timeout 300 --timeout-method thread
export CFG=nat64_cold
step cold 300 bash scripts/ab_stats.sh early late
export AB_STEPS=2000
step ab 300 bash scripts/ab_variants.sh "nat64 nat64_cold" "-" early late early late
