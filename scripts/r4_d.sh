#!/bin/bash
# round 4 (d): the tail without frame reads (stashed checksums), grid-stride
# tail launches with per-XCD arrival shards: parity, cold/steady stats, and
# the fused kernel's SQ and HBM counters (steady state).
source scripts/lib_steps.sh
step nat64_tests 600 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -v --timeout 120 --timeout-method thread
export CFG=nat64_cold
step cold_stats 170 bash scripts/ab_stats.sh new
cp -r gpurun_out/abstats_new gpurun_out/abstats_new_cold
export CFG=nat64
step steady_stats 170 bash scripts/ab_stats.sh new
export AB_STEPS=1000
step steady_pmc 170 bash scripts/ab_variants.sh "nat64" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;FETCH_SIZE;WRITE_SIZE" new
step cold_pmc 170 bash scripts/ab_variants.sh "nat64_cold" "FETCH_SIZE;WRITE_SIZE" new
