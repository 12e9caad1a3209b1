#!/bin/bash
# correctness of a variant library: the GPU nat64 tests against it
V=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
CAPSULE_GPU_LIB=$REPO/capsule_amd/var/$V.so timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $REPO/gpurun_out/abtest_$V.log 2>&1
rc=$?; echo "test $V rc=$rc"; tail -3 $REPO/gpurun_out/abtest_$V.log; exit $rc
