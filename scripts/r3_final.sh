#!/bin/bash
# final round-3 check: smoke, every GPU test, driver + default bench, then the
# nat64 family's stats/PMC sweep on the final nat64 sources
bash scripts/gpu_check.sh || exit $?
bash scripts/all_configs.sh r3 nat64 nat64_4to6 nat64_cold || exit $?
