#!/bin/bash
# nat64 4to6 end to end over rte_mbuf bursts and frame pairs (tests + 1 Mi bursts)
source scripts/lib_steps.sh
step modes 600 python -u -m pytest tests/test_bench_modes_gpu.py -x -q --timeout 200 --timeout-method thread -k "ingress"
for ing in zero_copy frames; do
  for b in 65536 1048576; do
    step e2e_${ing}_nat64_4to6_$b 300 python bench.py --e2e --ingress $ing --config nat64_4to6 --burst $b --steps 30
    step e2e_${ing}_nat64_$b 300 python bench.py --e2e --ingress $ing --config nat64 --burst $b --steps 30
  done
done
