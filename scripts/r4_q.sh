#!/bin/bash
# round 4 (q): round-3 tree vs this tree, same box, nat64 configs (is 6to4's
# steady state slower than round 3's?)
source scripts/lib_steps.sh
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for c in nat64 nat64_4to6; do
    step r3_${c}_$rep 170 bash -c "cd $R/capsule_amd/var/r3tree && python bench.py --config $c --only --no-cpu --steps 2000"
    step r4_${c}_$rep 170 python bench.py --config $c --only --no-cpu --steps 2000
  done
done
for f in gpurun_out/r[34]_*.log; do echo "$f $(grep '^{' $f | python3 -c 'import json,sys; r=json.loads(sys.stdin.readline()); print(r["roofline"]["kernel_us"])')"; done
