#!/bin/bash
# GPU tests of the rte_mbuf ingress + end-to-end mbuf burst rates.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ingress_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ingress_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/ingress_tests.log
[ $rc -ne 0 ] && exit $rc
for cfg in parse64 imix_csum; do
  for ing in zero_copy stage; do
    for b in 65536 1048576; do
      timeout -k 10 200 python bench.py --e2e --ingress $ing --config $cfg --burst $b --steps 100 > gpurun_out/e2e_mbuf_${cfg}_${ing}_$b.log 2>&1 || { echo "e2e $cfg $ing $b failed"; tail -5 gpurun_out/e2e_mbuf_${cfg}_${ing}_$b.log; exit 1; }
      tail -1 gpurun_out/e2e_mbuf_${cfg}_${ing}_$b.log
    done
  done
done
