#!/bin/bash
# where the cold pass's tail time goes: the deferred-frame patch ablated (timing only)
source scripts/lib_steps.sh
export CFG=nat64_cold
step stats 600 bash scripts/ab_stats.sh base nopatch
