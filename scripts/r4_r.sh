#!/bin/bash
# round 4 (r): rocprof kernel stats of the nat64 steady state, round-3 tree vs this tree, same box
source scripts/lib_steps.sh
R=$GRAFT_REPO_ROOT
step r3_stats 170 bash -c "cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/st_r3 -o s --output-format csv -- python3 $R/capsule_amd/var/r3tree/bench.py --config nat64 --only --no-cpu --steps 1000 --warmup 500"
step r4_stats 170 bash -c "cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/st_r4 -o s --output-format csv -- python3 $R/bench.py --config nat64 --only --no-cpu --steps 1000 --warmup 500"
for d in st_r3 st_r4; do echo "== $d"; f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); cut -d, -f1-4,6,7 "$f" | head -5; done
