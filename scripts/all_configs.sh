#!/bin/bash
# bench + rocprofv3 (stats, FETCH_SIZE, WRITE_SIZE) for every config.
# usage: bash scripts/all_configs.sh <tag> [configs...]
TAG=${1:-r03}; shift
CONFIGS=${*:-parse64 parse256 parse1500 imix imix_csum nat64 nat64_4to6}
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in $CONFIGS; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 5 --only > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 gpurun_out/bench_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  bash scripts/profile.sh ${TAG}_$c --config $c --steps 1000 --warmup 1000 || exit $?
done
