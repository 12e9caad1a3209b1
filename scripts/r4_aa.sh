#!/bin/bash
# round 4 (aa): the reconcile window variant's occupancy target, 4 / 5 / 6 workgroups per CU
source scripts/lib_steps.sh
export AB_STEPS=1000
step ab 300 bash scripts/ab_variants.sh "reconcile64" "-" rw6 rw5 rw4 rw6 rw5 rw4
