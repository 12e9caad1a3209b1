#!/bin/bash
# GPU-box validation: smoke, GPU tests, the default bench and the driver's
# short bench.  Each GPU step has its own time limit; a failure stops the
# script (rc 1 = test failures, still reported; >= 124 or a signal = stop).
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 400 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python bench.py
