#!/bin/bash
# round 4: cgpu_reconcile on the GPU -- its parity tests, smoke, both bench
# configs, and rocprof kernel stats + HBM bytes for each
source scripts/lib_steps.sh
step recon_tests 600 python -u -m pytest tests/test_reconcile_gpu.py -x -v --timeout 120 --timeout-method thread
step nat64_new 600 python -u -m pytest tests/test_nat64_gpu.py -x -v --timeout 300 --timeout-method thread -k "rows_path_mixed or bench_nat64_4to6"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_recon64 300 python bench.py --config reconcile64 --only --no-cpu --steps 300
step bench_recon_imix 300 python bench.py --config reconcile_imix --only --no-cpu --steps 300
step launch_gap 120 tools/launch_gap
bash scripts/profile.sh r4_reconcile64 --config reconcile64 --steps 100 || exit $?
bash scripts/profile.sh r4_reconcile_imix --config reconcile_imix --steps 100 || exit $?
