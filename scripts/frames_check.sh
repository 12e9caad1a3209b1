#!/bin/bash
# cgpu_parse_frames: GPU parity tests, then end-to-end rates of the three
# ingress shapes (mbufs staged / mbufs zero-copy / frame pairs zero-copy)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ingress_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_frames.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_frames.log; [ $rc -ne 0 ] && exit $rc
for cfg in parse64 imix_csum; do
  for b in 65536 1048576; do
    for ing in zero_copy frames; do
      timeout -k 10 200 python bench.py --e2e --ingress $ing --config $cfg --burst $b --steps 100 > gpurun_out/e2e_${ing}_${cfg}_$b.log 2>&1 || { echo "$ing $cfg $b failed"; tail -3 gpurun_out/e2e_${ing}_${cfg}_$b.log; exit 1; }
      echo "$cfg burst $b $ing: $(tail -1 gpurun_out/e2e_${ing}_${cfg}_$b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mpps", d["us_per_burst"], "us/burst")')"
    done
  done
done
