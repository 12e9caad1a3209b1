#!/bin/bash
# round 4 (h): the order launch's chunk phase: which access is slow
source scripts/lib_steps.sh
export AB_STEPS=600
for v in clock_nov clock_plain clock_noslot clock_both; do
  step cold_$v 170 bash scripts/ab_variants.sh "nat64_cold" "-" $v
  grep "order clock" gpurun_out/ab_${v}_nat64_cold.log | head -2
done
step launch_gap 120 tools/launch_gap
for c in nat64 nat64_4to6 nat64 nat64_4to6; do
  step e2e_$c 170 python bench.py --e2e --config $c --steps 300 --warmup 50
  tail -1 gpurun_out/e2e_$c.log >> gpurun_out/e2e_alternating.log
done
export AB_STEPS=2000
step wait_ab 170 bash scripts/ab_variants.sh "nat64 nat64_4to6" "-" new alwayswait
bash scripts/r4_j.sh
