#!/bin/bash
# round 4 (l): 16-B slot loads in the verify, vector scan loads; parity, clocks, cold stats, e2e phases
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -q --timeout 120 --timeout-method thread
export AB_STEPS=600
step cold_clock 170 bash scripts/ab_variants.sh "nat64_cold" "-" clock
grep "order clock" gpurun_out/ab_clock_nat64_cold.log | head -2
export CFG=nat64_cold
step cold_new 170 bash scripts/ab_stats.sh new
for c in nat64 nat64_4to6; do
  step e2e_$c 170 python bench.py --e2e --config $c --steps 300 --warmup 50
done
