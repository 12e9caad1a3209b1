#!/bin/bash
# round-3 sweep, nat64 family + end-to-end rates
bash scripts/all_configs.sh r3 nat64 nat64_4to6 nat64_cold || exit $?
for c in nat64 nat64_4to6 parse64 imix_csum; do
  timeout -k 10 300 python bench.py --e2e --config $c --steps 300 --warmup 30 > gpurun_out/e2e_$c.log 2>&1
  rc=$?; echo "e2e $c rc=$rc"; tail -1 gpurun_out/e2e_$c.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for c in nat64 nat64_4to6; do
  timeout -k 10 300 python bench.py --e2e --ingress frames --config $c --burst 1048576 --steps 30 > gpurun_out/e2e_frames_$c.log 2>&1
  rc=$?; echo "e2e frames $c rc=$rc"; tail -1 gpurun_out/e2e_frames_$c.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
