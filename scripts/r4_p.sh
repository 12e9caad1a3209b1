#!/bin/bash
# round 4 (p): does the deferred flag's single-address store cost the cold fused kernel?
source scripts/lib_steps.sh
export CFG=nat64_cold
step cold_new 170 bash scripts/ab_stats.sh new
step cold_noflag 170 bash scripts/ab_stats.sh noflag
step cold_new2 170 bash scripts/ab_stats.sh new
