#!/bin/bash
# round 4 (b): parity of the new cold port map and of the whole-64-B
# reconcile stores, then A/B timings + counters:
#   nat64_cold / nat64: base (round-3 map), norep (base without the
#   representative read, timing only), new (claim tags, two-phase tail)
#   reconcile64 / reconcile_imix: recon_fields (2-B field stores) vs
#   recon_whole (first 64 B rewritten whole)
source scripts/lib_steps.sh
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1) || true
step launch_gap 120 tools/launch_gap
step recon_tests 600 python -u -m pytest tests/test_reconcile_gpu.py -x -q --timeout 120 --timeout-method thread
step nat64_tests 900 python -u -m pytest tests/test_nat64_gpu.py tests/test_bench_parity_gpu.py tests/test_nat64_mbufs_gpu.py -x -v --timeout 300 --timeout-method thread
export CFG=nat64_cold
step cold_stats 600 bash scripts/ab_stats.sh base norep new new_verify
export CFG=nat64
step steady_stats 600 bash scripts/ab_stats.sh base new new_verify
export AB_STEPS=300
step recon_ab 600 bash scripts/ab_variants.sh "reconcile64 reconcile_imix" "FETCH_SIZE;WRITE_SIZE" recon_fields recon_whole
step cold_pmc 900 bash scripts/ab_variants.sh nat64_cold "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;FETCH_SIZE" base norep new
step gap_ab 900 bash scripts/ab_variants.sh "nat64 nat64_4to6" "-" base new new_rec new_nowait
