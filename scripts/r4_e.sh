#!/bin/bash
# round 4 (e): batched order pass + parallel scan; the steady-state cost of
# the two tail launches (notail ablation: fused kernel alone, stop event).
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -v --timeout 120 --timeout-method thread
export CFG=nat64_cold
step cold_stats 170 bash scripts/ab_stats.sh new
export AB_STEPS=2000
step steady_ab 170 bash scripts/ab_variants.sh "nat64" "-" new notail new
step cold_ab 170 bash scripts/ab_variants.sh "nat64_cold" "-" new
