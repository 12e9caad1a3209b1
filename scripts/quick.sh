#!/bin/bash
# quick GPU iteration: GPU tests (TESTS, default all) then benches of the given configs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${TESTS:-tests} -q -m gpu -x > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -4 gpurun_out/quick_tests.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/quick_tests.log | head -20; exit $rc; fi
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 300 --warmup 30 --no-cpu --only > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 3; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], 'Mpps', d['roofline'])"
done
