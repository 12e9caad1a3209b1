#!/bin/bash
# GPU-box validation: smoke, GPU tests, a short bench.  Each GPU step has its
# own time limit; a crash/abort/timeout (rc >= 124 or signal) stops the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q
step bench 400 python bench.py --steps 500 --cpu-seconds 5
