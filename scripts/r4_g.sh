#!/bin/bash
# round 4 (g): the order launch's chunk phase by clock: U = 4 / 1 chunks per
# workgroup, without the stash verification.
source scripts/lib_steps.sh
export AB_STEPS=600
for v in clock clock_u1 clock_nov; do
  step cold_$v 170 bash scripts/ab_variants.sh "nat64_cold" "-" $v
  grep "order clock" gpurun_out/ab_${v}_nat64_cold.log | head -3
done
export CFG=nat64_cold
step cold_new 170 bash scripts/ab_stats.sh new
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -q --timeout 120 --timeout-method thread
