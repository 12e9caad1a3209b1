#!/bin/bash
# round 4 (i): counters the verdict asked for: IMIX-with-checksums L2 hits /
# misses against its read bytes (three runs on one box), the 6to4 fused
# kernel's SQ breakdown, the 4to6 read bytes.
source scripts/lib_steps.sh
export AB_STEPS=300
for r in 1 2 3; do
  step imix_pmc_$r 170 bash scripts/ab_variants.sh "imix_csum" "TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" new
done
step nat64_sq 170 bash scripts/ab_variants.sh "nat64" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD;SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR;FETCH_SIZE;WRITE_SIZE" new
step n4to6_pmc 170 bash scripts/ab_variants.sh "nat64_4to6" "FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" new
