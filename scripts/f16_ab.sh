export TMPDIR=/tmp
CAPSULE_GPU_LIB=$PWD/capsule_amd/var/f16.so timeout -k 10 300 python -u -m pytest tests/test_nat64_gpu.py tests/test_nat64_mbufs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_f16.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_f16.log; [ $rc -ne 0 ] && exit $rc
AB_STEPS=2000 bash scripts/ab_variants.sh "nat64" "-" old f16 old f16
