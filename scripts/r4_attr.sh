#!/bin/bash
# round 4: where the cold port map's fused-kernel time goes (the
# representative-frame read of a batch-local join, ablated for timing only),
# what an empty launch / an event record costs, and the counter list
source scripts/lib_steps.sh
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1) || true
step launch_gap 120 tools/launch_gap
export CFG=nat64_cold
step cold_stats 600 bash scripts/ab_stats.sh base norep
export AB_STEPS=300
step cold_pmc 900 bash scripts/ab_variants.sh nat64_cold "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;FETCH_SIZE" base norep
