#!/bin/bash
# round 4 (n): e2e with two pipeline streams (upload + kernel, download) vs three
source scripts/lib_steps.sh
for c in nat64_4to6 nat64 parse64 imix_csum; do
  step e2e2_$c 170 python bench.py --e2e --config $c --steps 300 --warmup 50
  step e2e3_$c 170 env CGPU_E2E_STREAMS=3 python bench.py --e2e --config $c --steps 300 --warmup 50
done
grep -h '^{' gpurun_out/e2e[23]_*.log
step launch_gap 120 tools/launch_gap
