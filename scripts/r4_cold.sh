#!/bin/bash
# round 4: the redesigned cold port map (claim tags + published keys in the
# fused kernel, a ticketed two-phase tail): nat64 parity first, then the
# old design (base), its representative-read ablation (norep) and the new
# design (new) timed and counted on the cold and steady configs
source scripts/lib_steps.sh
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1) || true
step launch_gap 120 tools/launch_gap
step nat64_tests 900 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -v --timeout 300 --timeout-method thread
export CFG=nat64_cold
step cold_stats 600 bash scripts/ab_stats.sh base norep new
export CFG=nat64
step steady_stats 600 bash scripts/ab_stats.sh base new
export AB_STEPS=300
step cold_pmc 900 bash scripts/ab_variants.sh nat64_cold "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;FETCH_SIZE" base norep new
