#!/bin/bash
# round 4 (m): why 4to6 end to end runs at 60 % of 6to4's PCIe rate: stream
# creation order and hardware-queue sharing
source scripts/lib_steps.sh
for c in nat64 nat64_4to6; do
  step e2e_$c 170 python bench.py --e2e --config $c --steps 300 --warmup 50
  step e2e_late_$c 170 env CGPU_E2E_STREAMS_LATE=1 python bench.py --e2e --config $c --steps 300 --warmup 50
  step e2e_hwq8_$c 170 env GPU_MAX_HW_QUEUES=8 CGPU_E2E_STREAMS_LATE=1 python bench.py --e2e --config $c --steps 300 --warmup 50
done
grep -h '^{' gpurun_out/e2e_*nat64*.log
