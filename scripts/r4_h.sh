#!/bin/bash
# round 4 (h): the order launch's chunk phase: which access is slow
source scripts/lib_steps.sh
export AB_STEPS=600
for v in clock_nov clock_plain clock_noslot clock_both; do
  step cold_$v 170 bash scripts/ab_variants.sh "nat64_cold" "-" $v
  grep "order clock" gpurun_out/ab_${v}_nat64_cold.log | head -2
done
