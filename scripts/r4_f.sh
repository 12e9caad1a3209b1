#!/bin/bash
# round 4 (f): where the cold tail's time goes: in-kernel clock of the order
# launch's phases, patch without frame stores, tail PMC counters.
source scripts/lib_steps.sh
export AB_STEPS=600
step cold_clock 170 bash scripts/ab_variants.sh "nat64_cold" "-" clock
grep "order clock" gpurun_out/ab_clock_nat64_cold.log | head -5
export CFG=nat64_cold
step cold_nps 170 bash scripts/ab_stats.sh nopatchstore
step cold_pmc 300 bash scripts/ab_variants.sh "nat64_cold" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU;FETCH_SIZE;WRITE_SIZE" new
