#!/bin/bash
# One gpurun call: bench + rocprofv3 (stats, FETCH_SIZE, WRITE_SIZE) for every
# config, then the end-to-end (host-resident, PCIe-inclusive) rates.
# usage: bash scripts/round_sweep.sh <tag> [configs...]
TAG=${1:-round1}; shift
CONFIGS=${*:-parse64 parse256 parse1500 imix imix_csum nat64 nat64_4to6}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/all_configs.sh "$TAG" $CONFIGS || exit $?
for c in parse64 imix_csum nat64; do
  timeout -k 10 300 python bench.py --e2e --config $c --steps 300 --warmup 30 > gpurun_out/e2e_$c.log 2>&1
  rc=$?; echo "e2e $c rc=$rc"; tail -1 gpurun_out/e2e_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
