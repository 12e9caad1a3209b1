#!/bin/bash
# nat64 GPU tests + smoke + short benches of the nat64 configs and parse64.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_nat64 300 python -u -m pytest tests/test_nat64_gpu.py -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for c in nat64 nat64_4to6 parse64; do
  step bench_$c 300 python bench.py --config $c --steps 300 --warmup 30 --cpu-seconds 3
done
