#!/bin/bash
# nat64 6to4 per-call time against the port map's capacity (50,000 keys)
export TMPDIR=/tmp
mkdir -p gpurun_out
for lg in ${SIZES:-16 17 18 20 16 20}; do
  CGPU_BENCH_PORTMAP_LOG2=$lg timeout -k 10 200 python3 bench.py --config nat64 --only --no-cpu --steps 2000 --warmup 1000 > gpurun_out/pm_$lg.log 2>&1 || { echo "log2 $lg failed"; tail -5 gpurun_out/pm_$lg.log; exit 1; }
  python3 - gpurun_out/pm_$lg.log $lg <<'PY'
import json, sys
r = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]
print("log2", sys.argv[2], "Mpps", r["value"], "kernel_us", r["roofline"]["kernel_us"])
PY
done
