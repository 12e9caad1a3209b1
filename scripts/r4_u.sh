#!/bin/bash
# round 4 (u): SQ breakdown of reconcile64 against parse64 (same frames)
source scripts/lib_steps.sh
export AB_STEPS=300
step sq 300 bash scripts/ab_variants.sh "reconcile64 parse64" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS" cur
