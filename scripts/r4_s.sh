#!/bin/bash
# round 4 (s): the 6to4 fused kernel's steady state against round 3's: lazy claim tag, stash store
source scripts/lib_steps.sh
R=$GRAFT_REPO_ROOT
step r3_stats 170 bash -c "cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/st_r3 -o s --output-format csv -- python3 $R/capsule_amd/var/r3tree/bench.py --config nat64 --only --no-cpu --steps 1000 --warmup 500"
export CFG=nat64
step stats 300 bash scripts/ab_stats.sh eager lazy lazy_nostash
f=$(find gpurun_out/st_r3 -name '*kernel_stats.csv' | head -1); echo "== r3"; cut -d, -f1-4 "$f" | head -3
