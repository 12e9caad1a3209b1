#!/bin/bash
# round 4 (z): reconcile kernels with their own occupancy target: whole-64-B
# stores from registers at 6 workgroups per CU (no spill) vs the coalesced
# re-read stores; parse64 as the control for the refactor (pre = before it)
source scripts/lib_steps.sh
export AB_STEPS=1000
step ab 400 bash scripts/ab_variants.sh "reconcile64 reconcile_imix parse64" "-" pre w0c1w8 w1c0w6 w0c1w6 pre w1c0w6
