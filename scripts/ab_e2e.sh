#!/bin/bash
# A/B of the mbuf ingress across variant libraries
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $REPO/gpurun_out
for v in "$@"; do
  for ing in zero_copy; do
    for cfg in parse64 imix_csum; do
      CAPSULE_GPU_LIB=$REPO/capsule_amd/var/$v.so timeout -k 10 200 python $REPO/bench.py --e2e --ingress $ing --config $cfg --burst 1048576 --steps 100 > $REPO/gpurun_out/abe2e_${v}_$cfg.log 2>&1 || { echo "$v $cfg failed"; tail -3 $REPO/gpurun_out/abe2e_${v}_$cfg.log; exit 1; }
      echo "$v $ing $cfg $(tail -1 $REPO/gpurun_out/abe2e_${v}_$cfg.log | cut -c100-200)"
    done
  done
done
