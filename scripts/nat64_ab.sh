#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py tests/test_bench_parity_gpu.py tests/test_threads_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_nat64.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_nat64.log; [ $rc -ne 0 ] && exit $rc
AB_STEPS=2000 bash scripts/ab_variants.sh "nat64" "-" ${AB_VARS:-old new old new}
