#!/bin/bash
# round 4 (k): the order launch by per-workgroup clocks (no atomics of the
# instrument's own), with the verify / slot reads ablated, and without chunks.
source scripts/lib_steps.sh
export AB_STEPS=600
for v in clock clock_nov clock_noslot; do
  step cold_$v 170 bash scripts/ab_variants.sh "nat64_cold" "-" $v
  grep "order clock" gpurun_out/ab_${v}_nat64_cold.log | head -2
done
export CFG=nat64_cold
step cold_nochunks 170 bash scripts/ab_stats.sh nochunks
for c in nat64 nat64_4to6; do
  step e2e_$c 170 python bench.py --e2e --config $c --steps 300 --warmup 50
done
