#!/bin/bash
# round 4 (c): the two-launch nat64 tail (sharded arrivals, no polling) and
# the plain deferred flag: parity first, then cold/steady kernel stats, the
# event/wait A/B, the reconcile store A/B, and the TAGJOIN=0 variant last.
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -v --timeout 120 --timeout-method thread
step recon_tests 400 python -u -m pytest tests/test_reconcile_gpu.py -x -q --timeout 120 --timeout-method thread
export CFG=nat64_cold
step cold_stats 170 bash scripts/ab_stats.sh new
export CFG=nat64
step steady_stats 170 bash scripts/ab_stats.sh new
step gap_ab 170 bash scripts/ab_variants.sh "nat64 nat64_4to6" "-" new new_rec new_nowait
export AB_STEPS=300
step recon_ab 170 bash scripts/ab_variants.sh "reconcile64 reconcile_imix" "FETCH_SIZE;WRITE_SIZE" recon_fields recon_whole
export CFG=nat64_cold
step cold_verify 120 bash scripts/ab_stats.sh new_verify
