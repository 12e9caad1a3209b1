#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nat64_mbufs_gpu.py tests/test_ingress_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_nat64_frames.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_nat64_frames.log; [ $rc -ne 0 ] && exit $rc
for b in 65536 1048576; do
  for ing in zero_copy frames; do
    timeout -k 10 200 python bench.py --e2e --ingress $ing --config nat64 --burst $b --steps 100 > gpurun_out/e2e_nat64_${ing}_$b.log 2>&1 || { echo "$ing $b failed"; tail -3 gpurun_out/e2e_nat64_${ing}_$b.log; exit 1; }
    echo "nat64 burst $b $ing: $(tail -1 gpurun_out/e2e_nat64_${ing}_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mpps", d["us_per_burst"], "us/burst", d["act_frac"])')"
  done
done
