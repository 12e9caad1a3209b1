#!/bin/bash
# round 4 (j): does the order launch wait behind the fused kernel's write-back?
source scripts/lib_steps.sh
export AB_STEPS=600
export CFG=nat64_cold
step cold_gap 170 bash scripts/ab_stats.sh clock_gap
grep "order clock" gpurun_out/abstats_clock_gap.log | head -3
