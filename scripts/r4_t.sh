#!/bin/bash
# round 4 (t): steady-state tail launches with the flag line left clean
source scripts/lib_steps.sh
export CFG=nat64
step stats 300 bash scripts/ab_stats.sh lazy lazy_clean
export AB_STEPS=2000
step ab 170 bash scripts/ab_variants.sh "nat64" "-" lazy lazy_clean lazy lazy_clean
